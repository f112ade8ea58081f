/*
 * End-to-end host batch benchmark: keys start in host memory (as in an
 * mbuf), are copied into pinned staging, moved H2D, hashed, and the hashes
 * moved D2H into the caller's array -- the path nc_gpuhash_submit() takes
 * for a proxy that hashes on the host side (BASELINE.json
 * configs[4]: pipelined GET replay, mbuf-size 16384, mixed-length keys).
 *
 * For each batch shape and in-flight depth (context slots) it reports keys/s,
 * key GB/s and the mean submit-to-done time per batch (at depth 1 the
 * round-trip latency; deeper, it includes waiting behind earlier batches). Every batch's
 * hashes are checked against the per-key host hash_fnv1a_64().
 *
 *   tools/nc_e2e_bench [seconds-per-point]     (one JSON line per point)
 */
#define _GNU_SOURCE
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "nc_gpuhash.h"
#include "nc_gpuhash_synth.h"

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

struct batch {
    uint64_t first; /* first key of the batch in the corpus */
    uint32_t nkeys;
};

/* Split the corpus into batches: either a byte budget (an mbuf's worth of
 * keys) or a fixed key count. */
static uint32_t plan_batches(const uint64_t *off, uint64_t n, uint64_t byte_budget, uint32_t key_count,
                             struct batch *b, uint32_t maxb)
{
    uint32_t nb = 0;
    uint64_t i = 0;
    while (i < n && nb < maxb) {
        uint64_t j = i;
        if (byte_budget) {
            while (j < n && off[j + 1] - off[i] <= byte_budget) j++;
            if (j == i) j = i + 1;
        } else {
            j = i + key_count;
            if (j > n) break;
        }
        b[nb].first = i;
        b[nb].nkeys = (uint32_t)(j - i);
        nb++;
        i = j;
    }
    return nb;
}

static int run_point(const uint8_t *keys, const uint64_t *off, const struct batch *b, uint32_t nb,
                     int nslots, double seconds, const char *shape, uint64_t max_keys, uint64_t max_bytes,
                     int zero_copy)
{
    nc_gpuhash_ctx_t *ctx = nc_gpuhash_ctx_create(0, max_keys, max_bytes, nslots);
    if (!ctx) {
        fprintf(stderr, "ctx_create failed\n");
        return 1;
    }
    nc_gpuhash_ctx_set_zero_copy(ctx, zero_copy ? UINT64_MAX : 0); /* both paths measured */
    uint32_t maxk = 0;
    for (uint32_t i = 0; i < nb; i++)
        if (b[i].nkeys > maxk) maxk = b[i].nkeys;
    uint32_t *outs = malloc((size_t)nslots * maxk * sizeof(uint32_t));
    int *tick = malloc((size_t)nslots * sizeof(int));
    uint32_t *which = malloc((size_t)nslots * sizeof(uint32_t));
    double *t_sub = malloc((size_t)nslots * sizeof(double));
    if (!outs || !tick || !which || !t_sub) return 1;

    /* warm-up: one pass over a few batches */
    for (uint32_t i = 0; i < nb && i < 16; i++) {
        int t;
        if (nc_gpuhash_submit(ctx, NC_GPUHASH_FNV1A_64, keys, off + b[i].first, b[i].nkeys, outs, &t) != NC_OK ||
            nc_gpuhash_wait(ctx, t) != NC_OK) {
            fprintf(stderr, "warm-up failed\n");
            return 1;
        }
    }

    uint64_t done_keys = 0, done_bytes = 0, batches = 0, bad = 0;
    double lat_sum = 0.0;
    int inflight = 0, head = 0;
    uint32_t next = 0;
    const double t0 = now_s();
    double tend = t0 + seconds;
    for (;;) {
        const int stop = now_s() >= tend;
        if (inflight == nslots || (stop && inflight > 0)) {
            /* retire the oldest */
            const int s = head;
            if (nc_gpuhash_wait(ctx, tick[s]) != NC_OK) {
                fprintf(stderr, "wait failed\n");
                return 1;
            }
            lat_sum += now_s() - t_sub[s];
            const struct batch *bb = &b[which[s]];
            const uint32_t *o = outs + (size_t)s * maxk;
            /* check a stride of the batch against the host per-key hash */
            for (uint32_t k = 0; k < bb->nkeys; k += 1 + bb->nkeys / 64) {
                const uint64_t ks = off[bb->first + k], ke = off[bb->first + k + 1];
                if (o[k] != hash_fnv1a_64((const char *)keys + ks, (size_t)(ke - ks))) bad++;
            }
            done_keys += bb->nkeys;
            done_bytes += off[bb->first + bb->nkeys] - off[bb->first];
            batches++;
            head = (head + 1) % nslots;
            inflight--;
            continue;
        }
        if (stop) break;
        const int s = (head + inflight) % nslots;
        const uint32_t bi = next;
        next = (next + 1) % nb;
        t_sub[s] = now_s();
        if (nc_gpuhash_submit(ctx, NC_GPUHASH_FNV1A_64, keys, off + b[bi].first, b[bi].nkeys,
                              outs + (size_t)s * maxk, &tick[s]) != NC_OK) {
            fprintf(stderr, "submit failed\n");
            return 1;
        }
        which[s] = bi;
        inflight++;
    }
    const double el = now_s() - t0;
    printf("{\"path\": \"%s\", \"shape\": \"%s\", \"slots\": %d, "
           "\"batches\": %" PRIu64 ", \"keys_per_batch\": %.1f, \"bytes_per_batch\": %.1f, "
           "\"mkeys_s\": %.3f, \"gbs\": %.4f, \"submit_to_done_us\": %.1f, \"mismatches\": %" PRIu64 "}\n",
           zero_copy ? "host->pinned(mapped)->kernel->host" : "host->pinned->H2D->kernel->D2H->host", shape, nslots,
           batches, (double)done_keys / (double)batches, (double)done_bytes / (double)batches,
           (double)done_keys / el / 1e6, (double)done_bytes / el / 1e9, lat_sum / (double)batches * 1e6, bad);
    fflush(stdout);
    nc_gpuhash_ctx_destroy(ctx);
    free(outs);
    free(tick);
    free(which);
    free(t_sub);
    return bad ? 2 : 0;
}

int main(int argc, char **argv)
{
    const double seconds = argc > 1 ? atof(argv[1]) : 2.0;
    /* C5 corpus: Zipf 8-64 B printable keys (SURVEY.md §8d seed 5) */
    const struct nc_synth_spec spec = {5, NC_SYNTH_ZIPF, 8, 64, NC_SYNTH_BYTES_PRINTABLE, 1.0};
    const uint64_t n = 1u << 22;
    uint64_t *off = malloc((n + 1) * sizeof(uint64_t));
    if (!off || nc_synth_offsets_host(&spec, 0, n, off) != NC_OK) return 1;
    uint8_t *keys = malloc(off[n] + NC_GPUHASH_PAD);
    if (!keys || nc_synth_fill_host(&spec, 0, n, off, keys) != NC_OK) return 1;
    const uint32_t maxb = 1u << 20;
    struct batch *b = malloc(maxb * sizeof(struct batch));
    if (!b) return 1;

    static const struct {
        const char *name;
        uint64_t bytes;
        uint32_t keys;
    } shapes[] = {
        {"mbuf16384", 16384, 0}, /* one mbuf of keys: the pipelined GET replay batch */
        {"keys8192", 0, 8192},   /* SURVEY.md C5 batch: 64 conns x 128 pipelined GETs */
        {"keys65536", 0, 65536},
        {"keys1048576", 0, 1u << 20},
    };
    static const int depths[] = {1, 2, 4, 8};
    int rc = 0;
    for (size_t si = 0; si < sizeof(shapes) / sizeof(shapes[0]); si++) {
        const uint32_t nb = plan_batches(off, n, shapes[si].bytes, shapes[si].keys, b, maxb);
        uint32_t mk = 0;
        uint64_t mb = 0;
        for (uint32_t i = 0; i < nb; i++) {
            if (b[i].nkeys > mk) mk = b[i].nkeys;
            const uint64_t by = off[b[i].first + b[i].nkeys] - off[b[i].first];
            if (by > mb) mb = by;
        }
        for (int zc = 0; zc < 2; zc++) {
            for (size_t di = 0; di < sizeof(depths) / sizeof(depths[0]); di++) {
                const int r = run_point(keys, off, b, nb, depths[di], seconds, shapes[si].name, mk, mb, zc);
                if (r) rc = r;
                if (r == 1) return 1;
            }
        }
    }
    free(b);
    free(keys);
    free(off);
    return rc;
}
