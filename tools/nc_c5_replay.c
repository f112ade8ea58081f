/*
 * C5: pipelined GET replay (BASELINE.json configs[4]; the
 * shape of /root/reference/scripts/pipelined_read.sh:7-23).
 *
 * 64 connections each pipeline 128 "get <key>\r\n" requests; keys are C5's
 * printable Zipf 8-64 B keys (seed 5). The connections' request streams are
 * read into mbufs of 16,384 bytes (16,336 data bytes after the 48-byte
 * header, src/nc_mbuf.c:270-271) with the reference's repair semantics: a
 * request whose key would straddle the end of an mbuf moves whole into the
 * next one (src/proto/nc_memcache.c:746-749), so no key is ever split. One
 * batch = the keys of one mbuf, handed to nc_gpuhash_submit_spans() as
 * keypos-style spans pointing INTO the mbuf (no packing by the caller), the
 * way the fragment loop would.
 *
 * For in-flight depths 1, 2 and 4 (context slots), copy and zero-copy paths,
 * and depths 1, 2, 4, 8 and 16 of the batch ring (nc_gpuhash_ring: a resident
 * worker polls mapped host memory, no HIP call per batch),
 * it reports submit->done latency per mbuf and keys/s, and beside them the
 * per-key host hash of the same spans through a hash_t pointer (one core, as
 * the reference's event loop does, src/nc_server.c:643). Every batch is
 * checked against that host hash.
 *
 *   tools/nc_c5_replay [seconds-per-point]        (one JSON line per point)
 *   tools/nc_c5_replay SECONDS timeline           (the ring at one batch in
 *       flight with its device timeline: where a batch's submit -> done goes)
 */
#define _GNU_SOURCE
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "nc_gpuhash.h"
#include "nc_gpuhash_probe.h"
#include "nc_gpuhash_synth.h"

#define NCONN 64
#define DEPTH 128
#define MBUF_DATA 16336u /* 16384 - sizeof(struct mbuf) */

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

struct mbuf {
    uint8_t data[MBUF_DATA + NC_GPUHASH_PAD];
    uint32_t len;
    uint32_t nkeys;
    struct nc_keyspan *spans;
};

typedef uint32_t (*hash_t)(const char *, size_t);

static uint32_t *first_of(const struct mbuf *mb, uint32_t nmb)
{
    uint32_t *first = malloc((nmb + 1) * sizeof(uint32_t));
    if (!first) exit(1);
    first[0] = 0;
    for (uint32_t i = 0; i < nmb; i++) first[i + 1] = first[i] + mb[i].nkeys;
    return first;
}

static int cmp_d(const void *a, const void *b)
{
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

/* one batch in flight through the batch ring, with the worker's timeline:
 * host submit call; device found -> staged (the batch fetched across PCIe
 * into LDS) -> issued (hashes computed, stores issued) -> stored (stores
 * acknowledged) -> released (the release, or the write-through drain, before
 * the done word; its stamp may land just after the done word, and then the
 * batch counts 0 here); and the host's submit -> done.
 * Medians in microseconds. */
static int ring_timeline(double seconds, struct mbuf *mb, uint32_t nmb, uint32_t maxk, const uint32_t *ref,
                         const uint32_t *first)
{
    nc_gpuhash_ring_t *ring = nc_gpuhash_ring_create_ex(0, 1, maxk, MBUF_DATA, 1, 0);
    if (!ring || nc_gpuhash_ring_debug_timeline(ring, 1, 0, NULL) != NC_OK) return 1;
    uint32_t *outs = malloc(maxk * sizeof(uint32_t));
    enum { NMAX = 200000, NV = 10 };
    double *v[NV];
    for (int i = 0; i < NV; i++) v[i] = malloc(NMAX * sizeof(double));
    if (!outs) return 1;
    uint64_t bad = 0;
    int n = 0;
    const double tend = now_s() + seconds;
    for (uint32_t i = 0; n < NMAX && now_s() < tend; i++) {
        const uint32_t bi = i % nmb;
        int tk;
        const double a = now_s();
        if (nc_gpuhash_ring_submit_spans(ring, NC_GPUHASH_FNV1A_64, mb[bi].spans, mb[bi].nkeys, outs, &tk) != NC_OK)
            return 1;
        const double b = now_s();
        if (nc_gpuhash_ring_wait(ring, tk) != NC_OK) return 1;
        const double c = now_s();
        for (uint32_t k = 0; k < mb[bi].nkeys; k++) bad += outs[k] != ref[first[bi] + k];
        uint64_t tl[8];
        if (nc_gpuhash_ring_debug_timeline(ring, -1, 0, tl) != NC_OK) return 1;
        const uint64_t stored = tl[3], released = tl[5] == (uint64_t)i + 1u ? tl[4] : 0; /* may land late: then 0 */
        if (i >= nmb) { /* past the warm-up (the first launch) */
            v[0][n] = (b - a) * 1e6;
            v[1][n] = (c - a) * 1e6;
            v[2][n] = (double)(tl[1] - tl[0]) * 0.01;
            v[3][n] = (double)(tl[2] - tl[1]) * 0.01;
            v[4][n] = (double)(tl[3] - tl[2]) * 0.01;
            v[5][n] = (double)(tl[3] - tl[0]) * 0.01;
            v[6][n] = released > stored ? (double)(released - stored) * 0.01 : 0.0;
            v[7][n] = v[1][n] - v[0][n] - v[5][n] - v[6][n];
            v[8][n] = (double)tl[6]; /* the shader clock over the hash phase, MHz */
            v[9][n] = tl[7] > tl[1] ? (double)(tl[7] - tl[1]) * 0.01 : 0.0; /* wave 0's own keys */
            n++;
        }
    }
    double med[NV];
    for (int i = 0; i < NV; i++) {
        qsort(v[i], (size_t)n, sizeof(double), cmp_d);
        med[i] = n ? v[i][n / 2] : 0.0;
    }
    printf("{\"point\": \"ring_timeline\", \"staging\": \"%s\", \"depth\": 1, \"threads\": %d, \"batches\": %d, \"median_us\": "
           "{\"host_submit_call\": %.2f, \"submit_to_done\": %.2f, \"dev_fetch\": %.2f, \"dev_hash\": %.2f, "
           "\"dev_store_ack\": %.2f, \"dev_found_to_stored\": %.2f, \"dev_release\": %.2f, "
           "\"rest_detect_done_reap\": %.2f}, \"hash_clock_mhz_median\": %.0f, \"wave0_own_hash_us\": %.2f, \"mismatches\": %" PRIu64 "}\n",
           nc_gpuhash_ring_debug_staging(ring) == 1 ? "device" : "host", NC_GPUHASH_RING_DEFAULT_THREADS, n, med[0], med[1], med[2], med[3], med[4], med[5], med[6], med[7], med[8], med[9], bad);
    nc_gpuhash_ring_destroy(ring);
    return bad ? 2 : 0;
}

int main(int argc, char **argv)
{
    const double seconds = argc > 1 ? atof(argv[1]) : 1.0;
    const struct nc_synth_spec spec = {5, NC_SYNTH_ZIPF, 8, 64, NC_SYNTH_BYTES_PRINTABLE, 1.0};
    const uint64_t n = NCONN * DEPTH;
    uint64_t *off = malloc((n + 1) * sizeof(uint64_t));
    if (!off || nc_synth_offsets_host(&spec, 0, n, off) != NC_OK) return 1;
    uint8_t *keys = malloc(off[n] + NC_GPUHASH_PAD);
    if (!keys || nc_synth_fill_host(&spec, 0, n, off, keys) != NC_OK) return 1;

    /* the request stream, connection after connection, read into mbufs with
     * repair: a request that does not fit the current mbuf opens the next */
    struct mbuf *mb = calloc(n, sizeof(struct mbuf));
    struct nc_keyspan *spans = malloc(n * sizeof(struct nc_keyspan));
    if (!mb || !spans) return 1;
    uint32_t nmb = 0, nsp = 0;
    mb[0].spans = spans;
    for (uint64_t k = 0; k < n; k++) {
        const uint32_t klen = (uint32_t)(off[k + 1] - off[k]);
        const uint32_t req = 4u + klen + 2u; /* "get " key "\r\n" */
        if (mb[nmb].len + req > MBUF_DATA) { /* repair: the whole request moves on */
            nmb++;
            mb[nmb].spans = spans + nsp;
        }
        struct mbuf *m = &mb[nmb];
        memcpy(m->data + m->len, "get ", 4);
        memcpy(m->data + m->len + 4, keys + off[k], klen);
        memcpy(m->data + m->len + 4 + klen, "\r\n", 2);
        m->spans[m->nkeys].start = m->data + m->len + 4;
        m->spans[m->nkeys].end = m->data + m->len + 4 + klen;
        m->nkeys++;
        nsp++;
        m->len += req;
    }
    nmb++;
    uint32_t maxk = 0;
    uint64_t sum_len = 0;
    for (uint32_t i = 0; i < nmb; i++) {
        if (mb[i].nkeys > maxk) maxk = mb[i].nkeys;
        sum_len += mb[i].len;
    }

    /* host per-key hash of the same spans, one core, through a hash_t */
    volatile hash_t fn = hash_fnv1a_64;
    uint32_t *ref = malloc(n * sizeof(uint32_t));
    if (!ref) return 1;
    double host_s = 1e30;
    for (int rep = 0; rep < 5; rep++) {
        const double a = now_s();
        int reps = 0;
        do {
            uint32_t *r = ref;
            for (uint32_t i = 0; i < nmb; i++)
                for (uint32_t j = 0; j < mb[i].nkeys; j++)
                    *r++ = fn((const char *)mb[i].spans[j].start,
                              (size_t)(mb[i].spans[j].end - mb[i].spans[j].start));
            reps++;
        } while (now_s() - a < 0.05);
        const double s = (now_s() - a) / reps;
        if (s < host_s) host_s = s;
    }
    printf("{\"point\": \"host_per_key\", \"mbufs\": %u, \"keys\": %" PRIu64 ", \"keys_per_mbuf\": %.1f, "
           "\"mbuf_fill_bytes\": %.1f, \"us_per_mbuf\": %.3f, \"mkeys_s\": %.2f, \"threads\": 1}\n",
           nmb, n, (double)n / nmb, (double)sum_len / nmb, host_s / nmb * 1e6, (double)n / host_s / 1e6);
    fflush(stdout);

    if (argc > 2 && strcmp(argv[2], "timeline") == 0) return ring_timeline(seconds, mb, nmb, maxk, ref, first_of(mb, nmb));

    static const int depths[] = {1, 2, 4};
    int rc = 0;
    uint32_t *first = malloc((nmb + 1) * sizeof(uint32_t));
    if (!first) return 1;
    first[0] = 0;
    for (uint32_t i = 0; i < nmb; i++) first[i + 1] = first[i] + mb[i].nkeys;
    for (int zc = 0; zc < 2; zc++) {
        for (size_t di = 0; di < sizeof(depths) / sizeof(depths[0]); di++) {
            const int nslots = depths[di];
            nc_gpuhash_ctx_t *ctx = nc_gpuhash_ctx_create(0, maxk, MBUF_DATA, nslots);
            if (!ctx) {
                fprintf(stderr, "ctx_create failed\n");
                return 1;
            }
            nc_gpuhash_ctx_set_zero_copy(ctx, zc ? UINT64_MAX : 0);
            uint32_t *outs = malloc((size_t)nslots * maxk * sizeof(uint32_t));
            int tick[8];
            uint32_t which[8];
            double t_sub[8];
            if (!outs) return 1;
            for (uint32_t i = 0; i < nmb; i++) { /* warm-up */
                int t;
                if (nc_gpuhash_submit_spans(ctx, NC_GPUHASH_FNV1A_64, mb[i].spans, mb[i].nkeys, outs, &t) != NC_OK ||
                    nc_gpuhash_wait(ctx, t) != NC_OK)
                    return 1;
            }
            uint64_t done_keys = 0, batches = 0, bad = 0;
            double lat_sum = 0.0;
            int inflight = 0, head = 0;
            uint32_t next = 0;
            const double t0 = now_s(), tend = t0 + seconds;
            for (;;) {
                const int stop = now_s() >= tend;
                if (inflight == nslots || (stop && inflight > 0)) {
                    const int s = head;
                    if (nc_gpuhash_wait(ctx, tick[s]) != NC_OK) return 1;
                    lat_sum += now_s() - t_sub[s];
                    const uint32_t *o = outs + (size_t)s * maxk;
                    for (uint32_t k = 0; k < mb[which[s]].nkeys; k++) bad += o[k] != ref[first[which[s]] + k];
                    done_keys += mb[which[s]].nkeys;
                    batches++;
                    head = (head + 1) % nslots;
                    inflight--;
                    continue;
                }
                if (stop) break;
                const int s = (head + inflight) % nslots;
                const uint32_t bi = next;
                next = (next + 1) % nmb;
                t_sub[s] = now_s();
                if (nc_gpuhash_submit_spans(ctx, NC_GPUHASH_FNV1A_64, mb[bi].spans, mb[bi].nkeys,
                                            outs + (size_t)s * maxk, &tick[s]) != NC_OK) {
                    fprintf(stderr, "submit failed\n");
                    return 1;
                }
                which[s] = bi;
                inflight++;
            }
            const double el = now_s() - t0;
            printf("{\"point\": \"gpu\", \"path\": \"%s\", \"depth\": %d, \"batches\": %" PRIu64
                   ", \"keys_per_batch\": %.1f, \"submit_to_done_us\": %.2f, \"mkeys_s\": %.2f, "
                   "\"mismatches\": %" PRIu64 "}\n",
                   zc ? "zero-copy (mapped pinned staging)" : "copy (pinned staging, H2D, D2H)", nslots, batches,
                   (double)done_keys / (double)batches, lat_sum / (double)batches * 1e6,
                   (double)done_keys / el / 1e6, bad);
            fflush(stdout);
            if (bad) rc = 2;
            nc_gpuhash_ctx_destroy(ctx);
            free(outs);
        }
    }
    /* the batch ring: the same loop over nc_gpuhash_ring_*, one lane per
     * batch in flight (up to 8), lane workgroups of 256 and 1024 threads */
    static const int rdepths[] = {1, 2, 4, 8, 16};
    static const uint32_t rthreads[] = {256, 1024};
    for (size_t ti = 0; ti < sizeof(rthreads) / sizeof(rthreads[0]); ti++) {
    for (size_t di = 0; di < sizeof(rdepths) / sizeof(rdepths[0]); di++) {
        const int nslots = rdepths[di];
        nc_gpuhash_ring_t *ring = nc_gpuhash_ring_create_ex(0, (uint32_t)nslots, maxk, MBUF_DATA, 0, rthreads[ti]);
        if (!ring) {
            fprintf(stderr, "ring_create failed\n");
            return 1;
        }
        uint32_t *outs = malloc((size_t)nslots * maxk * sizeof(uint32_t));
        int tick[16];
        uint32_t which[16];
        double t_sub[16];
        if (!outs) return 1;
        for (uint32_t i = 0; i < nmb; i++) { /* warm-up (the first submit launches the workers) */
            int tk;
            if (nc_gpuhash_ring_submit_spans(ring, NC_GPUHASH_FNV1A_64, mb[i].spans, mb[i].nkeys, outs, &tk) != NC_OK ||
                nc_gpuhash_ring_wait(ring, tk) != NC_OK)
                return 1;
        }
        uint64_t done_keys = 0, batches = 0, bad = 0;
        double lat_sum = 0.0;
        int inflight = 0, head = 0;
        uint32_t next = 0;
        const double t0 = now_s(), tend = t0 + seconds;
        for (;;) {
            const int stop = now_s() >= tend;
            if (inflight == nslots || (stop && inflight > 0)) {
                const int s = head;
                if (nc_gpuhash_ring_wait(ring, tick[s]) != NC_OK) return 1;
                lat_sum += now_s() - t_sub[s];
                const uint32_t *o = outs + (size_t)s * maxk;
                for (uint32_t k = 0; k < mb[which[s]].nkeys; k++) bad += o[k] != ref[first[which[s]] + k];
                done_keys += mb[which[s]].nkeys;
                batches++;
                head = (head + 1) % nslots;
                inflight--;
                continue;
            }
            if (stop) break;
            const int s = (head + inflight) % nslots;
            const uint32_t bi = next;
            next = (next + 1) % nmb;
            t_sub[s] = now_s();
            if (nc_gpuhash_ring_submit_spans(ring, NC_GPUHASH_FNV1A_64, mb[bi].spans, mb[bi].nkeys,
                                             outs + (size_t)s * maxk, &tick[s]) != NC_OK) {
                fprintf(stderr, "ring submit failed\n");
                return 1;
            }
            which[s] = bi;
            inflight++;
        }
        const double el = now_s() - t0;
        printf("{\"point\": \"gpu\", \"path\": \"ring (resident worker)\", \"staging\": \"%s\", \"depth\": %d, "
               "\"lanes\": %u, \"threads\": %u, "
               "\"batches\": %" PRIu64 ", \"keys_per_batch\": %.1f, \"submit_to_done_us\": %.2f, \"mkeys_s\": %.2f, "
               "\"mismatches\": %" PRIu64 ", \"worker_launches\": %" PRIu64 "}\n",
               nc_gpuhash_ring_debug_staging(ring) == 1 ? "device" : "host", nslots, nc_gpuhash_ring_lanes(ring),
               rthreads[ti], batches, (double)done_keys / (double)batches,
               lat_sum / (double)batches * 1e6, (double)done_keys / el / 1e6, bad, nc_gpuhash_ring_launches(ring));
        fflush(stdout);
        if (bad) rc = 2;
        nc_gpuhash_ring_destroy(ring);
        free(outs);
    }
    }
    free(first);
    free(ref);
    free(spans);
    free(mb);
    free(keys);
    free(off);
    return rc;
}
