/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Thin driver linked against the REAL reference hashkit, compiled from the
 * sources where they lie under /root/reference (see oracle/Makefile, target
 * `ref`; output only into oracle/_ref/). Nothing here re-implements a hash: it
 * only calls the reference's own functions so that
 *   - tests/golden/make_golden.py can emit golden vectors from the reference,
 *   - bench.py can time the reference itself as the CPU baseline
 *     (cpu_baseline.kind = "reference").
 * The batch loop calls each key through a hash_t pointer, exactly as
 * server_pool_hash does (src/nc_server.c:643).
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <nc_core.h>
#include <nc_server.h>
#include <nc_hashkit.h>

/* hash_algos[] order, src/nc_conf.c:30-35 (HASH_CODEC, src/hashkit/nc_hashkit.h:24-36). */
#define DEFINE_ACTION(_hash, _name) hash_##_name,
static hash_t ref_algos[] = { HASH_CODEC(DEFINE_ACTION) NULL };
#undef DEFINE_ACTION

int ref_nmodes(void) { return HASH_SENTINEL; }

uint32_t ref_hash(int mode, const char *key, size_t len)
{
    if (mode < 0 || mode >= HASH_SENTINEL) return 0;
    return ref_algos[mode](key, len);
}

uint32_t ref_ketama_hash(const char *key, size_t len, uint32_t alignment)
{
    return ketama_hash(key, len, alignment);
}

struct ref_job {
    hash_t fn;
    const char *keys;
    const uint64_t *offsets;
    uint64_t lo, hi;
    uint32_t *out;
};

static void *ref_run(void *arg)
{
    struct ref_job *j = arg;
    hash_t volatile fn = j->fn;
    for (uint64_t i = j->lo; i < j->hi; i++) {
        uint64_t s = j->offsets[i];
        j->out[i] = fn(j->keys + s, (size_t)(j->offsets[i + 1] - s));
    }
    return NULL;
}

static uint64_t ref_lower_bound(const uint64_t *off, uint64_t n, uint64_t t)
{
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        uint64_t mid = lo + (hi - lo) / 2;
        if (off[mid] < t) lo = mid + 1; else hi = mid;
    }
    return lo;
}

int ref_hash_batch(int mode, const char *keys, const uint64_t *offsets,
                   uint64_t nkeys, uint32_t *out, int nthreads)
{
    if (mode < 0 || mode >= HASH_SENTINEL) return -1;
    if (nthreads <= 1 || nkeys < 1024) {
        struct ref_job j = { ref_algos[mode], keys, offsets, 0, nkeys, out };
        ref_run(&j);
        return 0;
    }
    if (nthreads > 256) nthreads = 256;
    struct ref_job jobs[256];
    pthread_t tids[256];
    uint64_t total = offsets[nkeys] - offsets[0], prev = 0;
    for (int t = 0; t < nthreads; t++) {
        uint64_t cut = (t == nthreads - 1) ? nkeys
            : ref_lower_bound(offsets, nkeys, offsets[0] + total * (uint64_t)(t + 1) / (uint64_t)nthreads);
        if (total == 0) cut = nkeys * (uint64_t)(t + 1) / (uint64_t)nthreads;
        if (cut < prev) cut = prev;
        jobs[t] = (struct ref_job){ ref_algos[mode], keys, offsets, prev, cut, out };
        prev = cut;
    }
    for (int t = 0; t < nthreads; t++) pthread_create(&tids[t], NULL, ref_run, &jobs[t]);
    for (int t = 0; t < nthreads; t++) pthread_join(tids[t], NULL);
    return 0;
}

double ref_time_batch(int mode, const char *keys, const uint64_t *offsets,
                      uint64_t nkeys, uint32_t *out, int nthreads, int reps)
{
    double best = 1e30;
    ref_hash_batch(mode, keys, offsets, nkeys, out, nthreads);
    for (int r = 0; r < (reps > 0 ? reps : 1); r++) {
        struct timespec a, b;
        clock_gettime(CLOCK_MONOTONIC, &a);
        if (ref_hash_batch(mode, keys, offsets, nkeys, out, nthreads) != 0) return -1.0;
        clock_gettime(CLOCK_MONOTONIC, &b);
        double s = (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
        if (s < best) best = s;
    }
    return best;
}

/*
 * Build a continuum with the reference's own ketama_update / modula_update
 * (src/hashkit/nc_ketama.c:58, src/hashkit/nc_modula.c:29) over a pool whose
 * servers are all live. dist: 0 ketama, 1 modula. Returns the number of
 * points copied out, or -1.
 */
int ref_build_continuum(int dist, const char *const *names, const uint32_t *name_lens,
                        const uint32_t *weights, uint32_t nserver,
                        uint32_t *values, uint32_t *indices, uint32_t cap)
{
    struct server_pool pool;
    memset(&pool, 0, sizeof(pool));
    if (array_init(&pool.server, nserver, sizeof(struct server)) != NC_OK) return -1;
    for (uint32_t s = 0; s < nserver; s++) {
        struct server *srv = array_push(&pool.server);
        memset(srv, 0, sizeof(*srv));
        srv->idx = s;
        srv->owner = &pool;
        srv->name.data = (uint8_t *)names[s];
        srv->name.len = name_lens[s];
        srv->weight = weights[s];
        srv->next_retry = 0;
    }
    pool.auto_eject_hosts = 0;
    rstatus_t st = (dist == 0) ? ketama_update(&pool) : modula_update(&pool);
    int ret = -1;
    if (st == NC_OK && pool.ncontinuum <= cap) {
        for (uint32_t i = 0; i < pool.ncontinuum; i++) {
            values[i] = pool.continuum[i].value;
            indices[i] = pool.continuum[i].index;
        }
        ret = (int)pool.ncontinuum;
    }
    free(pool.continuum);
    array_deinit(&pool.server);
    return ret;
}

uint32_t ref_dispatch(int dist, const uint32_t *values, const uint32_t *indices,
                      uint32_t n, uint32_t hash)
{
    struct continuum *c = malloc((size_t)n * sizeof(*c));
    if (c == NULL) return UINT32_MAX;
    for (uint32_t i = 0; i < n; i++) { c[i].value = values[i]; c[i].index = indices[i]; }
    uint32_t r = (dist == 0) ? ketama_dispatch(c, n, hash) : modula_dispatch(c, n, hash);
    free(c);
    return r;
}
