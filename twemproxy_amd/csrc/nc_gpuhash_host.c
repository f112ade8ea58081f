/*
 * Host side of the batched hasher, in C like the rest of twemproxy.
 *
 *  - hash: selector (src/nc_conf.c:1738-1764 conf_set_hash over
 *    hash_strings[] :23-27, HASH_CODEC src/hashkit/nc_hashkit.h:24-36);
 *  - contexts: nslots batches in flight, each with pinned host staging, its
 *    own HIP stream and device buffers. submit() packs (copies) keys out of the
 *    caller's mbuf spans into pinned staging — mbufs are recycled once the
 *    message is released (src/nc_mbuf.c:118-128) — and enqueues H2D, the
 *    kernel (nc_gpuhash_batch_device) and D2H without blocking; poll() is the
 *    completion check the event loop (src/nc_core.c:356 core_loop) would call;
 *  - byte-balanced shard planning for multi-GPU runs.
 *
 * There is no CPU fallback anywhere in this file: without a usable GPU every
 * batched call fails with NC_ERROR / errno ENODEV.
 */
#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "nc_gpuhash.h"

/* ---------------- hash: selector ---------------- */

static const char *const nc_mode_names[NC_GPUHASH_NMODES] = {
    "one_at_a_time", "md5", "crc16", "crc32", "crc32a", "fnv1_64",
    "fnv1a_64", "fnv1_32", "fnv1a_32", "hsieh", "murmur", "jenkins",
};

int nc_gpuhash_mode_from_name(const char *name, size_t len)
{
    if (name != NULL) {
        for (int m = 0; m < NC_GPUHASH_NMODES; m++) {
            /* string_compare: equal length and bytes (src/nc_string.c) */
            if (strlen(nc_mode_names[m]) == len && memcmp(nc_mode_names[m], name, len) == 0) {
                return m;
            }
        }
    }
    errno = EINVAL; /* "is not a valid hash" */
    return -1;
}

const char *nc_gpuhash_mode_name(int mode)
{
    if (mode < 0 || mode >= NC_GPUHASH_NMODES) {
        return NULL;
    }
    return nc_mode_names[mode];
}

const char *nc_gpuhash_version(void) { return "nc_gpuhash 0.1.0 (gfx950)"; }

int nc_gpuhash_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        return 0;
    }
    return n;
}

/* ---------------- shard planning ---------------- */

int nc_gpuhash_frag_plan(const uint32_t *sidx, uint32_t nkeys, uint32_t nserver, uint32_t *frag_seq,
                         uint32_t *frag_server, uint32_t *frag_nkeys)
{
    if ((nkeys != 0 && (sidx == NULL || frag_seq == NULL || frag_server == NULL || frag_nkeys == NULL)) ||
        nserver == 0) {
        errno = EINVAL;
        return -1;
    }
    /* the distinct servers, kept sorted in frag_server (at most
     * min(nkeys, nserver) of them: a request's keys touch few servers) */
    uint32_t nf = 0;
    for (uint32_t i = 0; i < nkeys; i++) {
        const uint32_t s = sidx[i];
        if (s >= nserver) {
            errno = EINVAL;
            return -1;
        }
        uint32_t lo = 0, hi = nf;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) / 2;
            if (frag_server[mid] < s) lo = mid + 1; else hi = mid;
        }
        if (lo == nf || frag_server[lo] != s) {
            memmove(frag_server + lo + 1, frag_server + lo, (size_t)(nf - lo) * sizeof(*frag_server));
            frag_server[lo] = s;
            nf++;
        }
    }
    for (uint32_t f = 0; f < nf; f++) frag_nkeys[f] = 0;
    for (uint32_t i = 0; i < nkeys; i++) {
        uint32_t lo = 0, hi = nf;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) / 2;
            if (frag_server[mid] < sidx[i]) lo = mid + 1; else hi = mid;
        }
        frag_seq[i] = lo;
        frag_nkeys[lo]++;
    }
    return (int)nf;
}

rstatus_t nc_gpuhash_shard_bounds(const uint64_t *offsets, uint64_t nkeys, uint32_t nshards,
                                  uint64_t *key_bounds)
{
    if (offsets == NULL || key_bounds == NULL || nshards == 0) {
        errno = EINVAL;
        return NC_ERROR;
    }
    const uint64_t base = offsets[0], total = offsets[nkeys] - offsets[0];
    key_bounds[0] = 0;
    for (uint32_t g = 1; g < nshards; g++) {
        /* first key whose start is >= the g-th byte quantile; ranges with no
         * bytes at all (all-empty keys) fall back to an even key split */
        uint64_t cut;
        if (total == 0) {
            cut = nkeys * g / nshards;
        } else {
            unsigned __int128 want = (unsigned __int128)total * g / nshards;
            uint64_t target = base + (uint64_t)want;
            uint64_t lo = 0, hi = nkeys;
            while (lo < hi) {
                uint64_t mid = lo + (hi - lo) / 2;
                if (offsets[mid] < target) lo = mid + 1; else hi = mid;
            }
            cut = lo;
        }
        if (cut < key_bounds[g - 1]) cut = key_bounds[g - 1];
        key_bounds[g] = cut;
    }
    key_bounds[nshards] = nkeys;
    return NC_OK;
}

/* ---------------- contexts ---------------- */

struct nc_slot {
    hipStream_t stream;
    hipEvent_t done;
    uint8_t *h_keys;
    uint64_t *h_off;
    uint32_t *h_out;
    uint8_t *m_keys; /* device addresses of the mapped staging (zero-copy batches) */
    uint64_t *m_off;
    uint32_t *m_out;
    uint8_t *d_keys;
    uint64_t *d_off;
    uint32_t *d_out;
    uint32_t *user_out;
    uint32_t nkeys;
    int busy; /* SLOT_FREE, SLOT_PACKING (owned by one submitter, not yet launched), SLOT_RUNNING */
    int ticket;
};

enum { SLOT_FREE = 0, SLOT_PACKING = 1, SLOT_RUNNING = 2 };

struct nc_gpuhash_ctx {
    int device;
    uint64_t max_keys;
    uint64_t max_key_bytes;
    int nslots;
    int next_gen;
    uint64_t zero_copy_bytes; /* batches with at most this many key bytes skip the copies */
    int unmapped;             /* staging has no device mapping: zero-copy unavailable */
    struct nc_slot *slots;
    /* Slot state (busy, ticket, user_out, next_gen) is shared by every thread
     * that submits to or polls this context (the batch layer
     * must be safe from worker threads). A slot being packed is owned by its
     * submitter alone, so the memcpy into pinned staging runs unlocked. */
    pthread_mutex_t lock;
    int lock_init;
};

static rstatus_t hip_fail(hipError_t e)
{
    if (getenv("NC_GPUHASH_DEBUG") != NULL) fprintf(stderr, "nc_gpuhash: host path: %s\n", hipGetErrorString(e));
    errno = (e == hipErrorNoDevice || e == hipErrorInvalidDevice) ? ENODEV
          : (e == hipErrorOutOfMemory ? ENOMEM : EIO);
    return errno == ENOMEM ? NC_ENOMEM : NC_ERROR;
}

void nc_gpuhash_ctx_destroy(nc_gpuhash_ctx_t *ctx)
{
    if (ctx == NULL) {
        return;
    }
    if (ctx->slots != NULL) {
        hipSetDevice(ctx->device);
        for (int i = 0; i < ctx->nslots; i++) {
            struct nc_slot *s = &ctx->slots[i];
            if (s->stream) hipStreamSynchronize(s->stream);
            if (s->done) hipEventDestroy(s->done);
            if (s->stream) hipStreamDestroy(s->stream);
            if (s->h_keys) hipHostFree(s->h_keys);
            if (s->h_off) hipHostFree(s->h_off);
            if (s->h_out) hipHostFree(s->h_out);
            if (s->d_keys) hipFree(s->d_keys);
            if (s->d_off) hipFree(s->d_off);
            if (s->d_out) hipFree(s->d_out);
        }
        free(ctx->slots);
    }
    if (ctx->lock_init) pthread_mutex_destroy(&ctx->lock);
    free(ctx);
}

nc_gpuhash_ctx_t *nc_gpuhash_ctx_create(int device, uint64_t max_keys, uint64_t max_key_bytes, int nslots)
{
    if (max_keys == 0 || nslots < 1 || nslots > 64) {
        errno = EINVAL;
        return NULL;
    }
    int ndev = nc_gpuhash_device_count();
    if (device < 0 || device >= ndev) {
        errno = ENODEV;
        return NULL;
    }
    nc_gpuhash_ctx_t *ctx = calloc(1, sizeof(*ctx));
    if (ctx == NULL) {
        errno = ENOMEM;
        return NULL;
    }
    if (pthread_mutex_init(&ctx->lock, NULL) != 0) {
        free(ctx);
        errno = ENOMEM;
        return NULL;
    }
    ctx->lock_init = 1;
    ctx->device = device;
    ctx->max_keys = max_keys;
    ctx->max_key_bytes = max_key_bytes;
    ctx->nslots = nslots;
    /* zero-copy up to 1 MiB of keys by default: measured faster for one-mbuf
     * (-25 % latency) and 8K-key (-50 %) batches, even at 1M keys */
    const char *zc = getenv("NC_GPUHASH_ZERO_COPY");
    ctx->zero_copy_bytes = zc ? strtoull(zc, NULL, 0) : (1u << 20);
    ctx->slots = calloc((size_t)nslots, sizeof(struct nc_slot));
    if (ctx->slots == NULL || hipSetDevice(device) != hipSuccess) {
        nc_gpuhash_ctx_destroy(ctx);
        errno = ENOMEM;
        return NULL;
    }
    const size_t kb = (size_t)max_key_bytes + NC_GPUHASH_PAD;
    for (int i = 0; i < nslots; i++) {
        struct nc_slot *s = &ctx->slots[i];
        hipError_t e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&s->done, hipEventDisableTiming);
        if (e == hipSuccess) e = hipHostMalloc((void **)&s->h_keys, kb, hipHostMallocDefault);
        if (e == hipSuccess) e = hipHostMalloc((void **)&s->h_off, (max_keys + 1) * sizeof(uint64_t), hipHostMallocDefault);
        if (e == hipSuccess) e = hipHostMalloc((void **)&s->h_out, max_keys * sizeof(uint32_t), hipHostMallocDefault);
        /* ROCm maps pinned host memory into the device's address space: a
         * zero-copy batch's kernel reads the keys and writes the hashes
         * across PCIe in place. Without the mapping, zero-copy stays off. */
        if (e == hipSuccess && (hipHostGetDevicePointer((void **)&s->m_keys, s->h_keys, 0) != hipSuccess ||
                                hipHostGetDevicePointer((void **)&s->m_off, s->h_off, 0) != hipSuccess ||
                                hipHostGetDevicePointer((void **)&s->m_out, s->h_out, 0) != hipSuccess))
            ctx->unmapped = 1;
        if (e == hipSuccess) e = hipMalloc((void **)&s->d_keys, kb);
        if (e == hipSuccess) e = hipMalloc((void **)&s->d_off, (max_keys + 1) * sizeof(uint64_t));
        if (e == hipSuccess) e = hipMalloc((void **)&s->d_out, max_keys * sizeof(uint32_t));
        if (e != hipSuccess) {
            hip_fail(e);
            int saved = errno;
            nc_gpuhash_ctx_destroy(ctx);
            errno = saved;
            return NULL;
        }
        s->ticket = -1;
    }
    return ctx;
}

rstatus_t nc_gpuhash_ctx_set_zero_copy(nc_gpuhash_ctx_t *ctx, uint64_t max_key_bytes)
{
    if (ctx == NULL) {
        errno = EINVAL;
        return NC_ERROR;
    }
    pthread_mutex_lock(&ctx->lock);
    ctx->zero_copy_bytes = max_key_bytes;
    pthread_mutex_unlock(&ctx->lock);
    return NC_OK;
}

/* Copy a finished slot's hashes to the caller and free the slot (ctx->lock held). */
static void slot_finish(struct nc_slot *s)
{
    memcpy(s->user_out, s->h_out, (size_t)s->nkeys * sizeof(uint32_t));
    s->busy = SLOT_FREE;
}

/* A free slot, reserved for the caller (SLOT_PACKING); finished slots are
 * delivered on the way. NULL when every slot is packing or still running. */
static struct nc_slot *slot_acquire(nc_gpuhash_ctx_t *ctx, int *idx)
{
    struct nc_slot *got = NULL;
    pthread_mutex_lock(&ctx->lock);
    for (int i = 0; i < ctx->nslots; i++) {
        struct nc_slot *s = &ctx->slots[i];
        if (s->busy == SLOT_RUNNING && hipEventQuery(s->done) == hipSuccess) {
            slot_finish(s);
        }
        if (s->busy == SLOT_FREE) {
            s->busy = SLOT_PACKING;
            *idx = i;
            got = s;
            break;
        }
    }
    pthread_mutex_unlock(&ctx->lock);
    return got;
}

static rstatus_t slot_release(nc_gpuhash_ctx_t *ctx, struct nc_slot *s, rstatus_t rc)
{
    pthread_mutex_lock(&ctx->lock);
    s->busy = SLOT_FREE;
    pthread_mutex_unlock(&ctx->lock);
    return rc;
}

/* Enqueue H2D -> kernel -> D2H on the slot's stream; staging already packed by
 * the caller, who owns the slot (SLOT_PACKING). On failure the slot is freed. */
static rstatus_t slot_launch(nc_gpuhash_ctx_t *ctx, struct nc_slot *s, int idx, int mode, uint32_t nkeys,
                             const struct nc_gpuhash_shape *shape, uint32_t *out, int *ticket)
{
    const uint64_t nbytes = s->h_off[nkeys];
    memset(s->h_keys + nbytes, 0, NC_GPUHASH_PAD);
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return slot_release(ctx, s, hip_fail(e));
    pthread_mutex_lock(&ctx->lock);
    const int zero_copy = nbytes <= ctx->zero_copy_bytes && !ctx->unmapped;
    pthread_mutex_unlock(&ctx->lock);
    if (zero_copy) {
        /* zero-copy: one kernel launch over the mapped staging, no DMA */
        if (nc_gpuhash_batch_device_shaped(mode, s->m_keys, s->m_off, nkeys, s->m_out, shape, s->stream) != NC_OK)
            return slot_release(ctx, s, NC_ERROR);
    } else {
        e = hipMemcpyAsync(s->d_keys, s->h_keys, nbytes + NC_GPUHASH_PAD, hipMemcpyHostToDevice, s->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(s->d_off, s->h_off, ((size_t)nkeys + 1) * sizeof(uint64_t), hipMemcpyHostToDevice,
                               s->stream);
        if (e != hipSuccess) return slot_release(ctx, s, hip_fail(e));
        if (nc_gpuhash_batch_device_shaped(mode, s->d_keys, s->d_off, nkeys, s->d_out, shape, s->stream) != NC_OK)
            return slot_release(ctx, s, NC_ERROR);
        e = hipMemcpyAsync(s->h_out, s->d_out, (size_t)nkeys * sizeof(uint32_t), hipMemcpyDeviceToHost, s->stream);
        if (e != hipSuccess) return slot_release(ctx, s, hip_fail(e));
    }
    e = hipEventRecord(s->done, s->stream);
    if (e != hipSuccess) return slot_release(ctx, s, hip_fail(e));
    pthread_mutex_lock(&ctx->lock);
    s->user_out = out;
    s->nkeys = nkeys;
    s->ticket = idx + ctx->nslots * (ctx->next_gen++ & 0xffffff);
    s->busy = SLOT_RUNNING;
    *ticket = s->ticket;
    pthread_mutex_unlock(&ctx->lock);
    return NC_OK;
}

rstatus_t nc_gpuhash_submit(nc_gpuhash_ctx_t *ctx, int mode, const uint8_t *keys, const uint64_t *offsets,
                            uint32_t nkeys, uint32_t *out, int *ticket)
{
    if (ctx == NULL || offsets == NULL || out == NULL || ticket == NULL || mode < 0 || mode >= NC_GPUHASH_NMODES) {
        errno = EINVAL;
        return NC_ERROR;
    }
    const uint64_t nbytes = offsets[nkeys] - offsets[0];
    if (nkeys > ctx->max_keys || nbytes > ctx->max_key_bytes) {
        errno = ENOMEM;
        return NC_ENOMEM;
    }
    int idx;
    struct nc_slot *s = slot_acquire(ctx, &idx);
    if (s == NULL) {
        errno = EAGAIN;
        return NC_EAGAIN;
    }
    if (nbytes) memcpy(s->h_keys, keys + offsets[0], nbytes);
    const uint64_t base = offsets[0];
    /* two plain passes: the rebasing one stays a vector loop of streaming
     * stores into the pinned staging, the shape one reads cached memory */
    for (uint32_t i = 0; i <= nkeys; i++) {
        s->h_off[i] = offsets[i] - base;
    }
    uint64_t lo = UINT64_MAX, hi = 0;
    for (uint32_t i = 0; i < nkeys; i++) {
        const uint64_t len = offsets[i + 1] - offsets[i];
        lo = len < lo ? len : lo;
        hi = len > hi ? len : hi;
    }
    struct nc_gpuhash_shape shape = {nbytes, (uint32_t)(lo > UINT32_MAX ? UINT32_MAX : lo),
                                     (uint32_t)(hi > UINT32_MAX ? UINT32_MAX : hi)};
    return slot_launch(ctx, s, idx, mode, nkeys, &shape, out, ticket);
}

rstatus_t nc_gpuhash_submit_spans(nc_gpuhash_ctx_t *ctx, int mode, const struct nc_keyspan *spans,
                                  uint32_t nkeys, uint32_t *out, int *ticket)
{
    if (ctx == NULL || (spans == NULL && nkeys) || out == NULL || ticket == NULL || mode < 0 ||
        mode >= NC_GPUHASH_NMODES) {
        errno = EINVAL;
        return NC_ERROR;
    }
    if (nkeys > ctx->max_keys) {
        errno = ENOMEM;
        return NC_ENOMEM;
    }
    int idx;
    struct nc_slot *s = slot_acquire(ctx, &idx);
    if (s == NULL) {
        errno = EAGAIN;
        return NC_EAGAIN;
    }
    uint64_t pos = 0;
    struct nc_gpuhash_shape shape = {0, UINT32_MAX, 0};
    s->h_off[0] = 0;
    for (uint32_t i = 0; i < nkeys; i++) {
        const size_t n = (size_t)(spans[i].end - spans[i].start);
        if (pos + n > ctx->max_key_bytes) {
            errno = ENOMEM;
            return slot_release(ctx, s, NC_ENOMEM);
        }
        memcpy(s->h_keys + pos, spans[i].start, n);
        pos += n;
        s->h_off[i + 1] = pos;
        if (n < shape.min_len) shape.min_len = (uint32_t)n;
        if (n > shape.max_len) shape.max_len = (uint32_t)n;
    }
    shape.key_bytes = pos;
    return slot_launch(ctx, s, idx, mode, nkeys, &shape, out, ticket);
}

static struct nc_slot *slot_of(nc_gpuhash_ctx_t *ctx, int ticket)
{
    if (ctx == NULL || ticket < 0) return NULL;
    return &ctx->slots[ticket % ctx->nslots];
}

rstatus_t nc_gpuhash_poll(nc_gpuhash_ctx_t *ctx, int ticket)
{
    struct nc_slot *s = slot_of(ctx, ticket);
    if (s == NULL) {
        errno = EINVAL;
        return NC_ERROR;
    }
    rstatus_t rc = NC_OK;
    pthread_mutex_lock(&ctx->lock);
    if (s->busy == SLOT_RUNNING && s->ticket == ticket) {
        const hipError_t e = hipEventQuery(s->done);
        if (e == hipErrorNotReady) rc = NC_EAGAIN;
        else if (e != hipSuccess) rc = hip_fail(e);
        else slot_finish(s);
    } /* else finished and already delivered */
    pthread_mutex_unlock(&ctx->lock);
    return rc;
}

rstatus_t nc_gpuhash_wait(nc_gpuhash_ctx_t *ctx, int ticket)
{
    struct nc_slot *s = slot_of(ctx, ticket);
    if (s == NULL) {
        errno = EINVAL;
        return NC_ERROR;
    }
    pthread_mutex_lock(&ctx->lock);
    const int pending = s->busy == SLOT_RUNNING && s->ticket == ticket;
    pthread_mutex_unlock(&ctx->lock);
    if (!pending) return NC_OK;
    /* the event stays valid while the ticket's slot is not re-acquired, and a
     * slot is re-acquired only after its event has completed */
    hipError_t e = hipEventSynchronize(s->done);
    if (e != hipSuccess) return hip_fail(e);
    pthread_mutex_lock(&ctx->lock);
    if (s->busy == SLOT_RUNNING && s->ticket == ticket) slot_finish(s);
    pthread_mutex_unlock(&ctx->lock);
    return NC_OK;
}

/* ---------------- process-wide synchronous batch ---------------- */

static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;
static nc_gpuhash_ctx_t *g_ctx;

rstatus_t nc_hashkit_batch(int mode, const uint8_t *keys, const uint64_t *offsets, uint32_t nkeys, uint32_t *out)
{
    if (offsets == NULL || out == NULL || mode < 0 || mode >= NC_GPUHASH_NMODES) {
        errno = EINVAL;
        return NC_ERROR;
    }
    const uint64_t nbytes = offsets[nkeys] - offsets[0];
    pthread_mutex_lock(&g_lock);
    if (g_ctx == NULL || g_ctx->max_keys < nkeys || g_ctx->max_key_bytes < nbytes) {
        uint64_t mk = nkeys < 65536 ? 65536 : nkeys, mb = nbytes < (1u << 22) ? (1u << 22) : nbytes;
        if (g_ctx) {
            if (g_ctx->max_keys > mk) mk = g_ctx->max_keys;
            if (g_ctx->max_key_bytes > mb) mb = g_ctx->max_key_bytes;
            nc_gpuhash_ctx_destroy(g_ctx);
        }
        g_ctx = nc_gpuhash_ctx_create(0, mk, mb, 1);
        if (g_ctx == NULL) {
            int saved = errno;
            pthread_mutex_unlock(&g_lock);
            errno = saved;
            return saved == ENOMEM ? NC_ENOMEM : NC_ERROR;
        }
    }
    int ticket;
    rstatus_t rc = nc_gpuhash_submit(g_ctx, mode, keys, offsets, nkeys, out, &ticket);
    if (rc == NC_OK) rc = nc_gpuhash_wait(g_ctx, ticket);
    pthread_mutex_unlock(&g_lock);
    return rc;
}

/* ---------------- whole batches from caller-pinned memory ---------------- */

#define NC_PIPE_MAX_DEPTH 4

struct nc_gpuhash_pipe {
    int device;
    int depth;
    uint64_t chunk_keys, chunk_bytes;
    hipStream_t s_h2d, s_comp, s_d2h;
    uint8_t *d_keys[NC_PIPE_MAX_DEPTH];
    uint64_t *d_off[NC_PIPE_MAX_DEPTH];
    uint32_t *d_out[NC_PIPE_MAX_DEPTH];
    hipEvent_t h2d_done[NC_PIPE_MAX_DEPTH], kern_done[NC_PIPE_MAX_DEPTH], d2h_done[NC_PIPE_MAX_DEPTH];
};

void nc_gpuhash_pipe_destroy(nc_gpuhash_pipe_t *p)
{
    if (p == NULL) return;
    hipSetDevice(p->device);
    if (p->s_h2d) hipStreamSynchronize(p->s_h2d);
    if (p->s_comp) hipStreamSynchronize(p->s_comp);
    if (p->s_d2h) hipStreamSynchronize(p->s_d2h);
    for (int b = 0; b < NC_PIPE_MAX_DEPTH; b++) {
        if (p->d_keys[b]) hipFree(p->d_keys[b]);
        if (p->d_off[b]) hipFree(p->d_off[b]);
        if (p->d_out[b]) hipFree(p->d_out[b]);
        if (p->h2d_done[b]) hipEventDestroy(p->h2d_done[b]);
        if (p->kern_done[b]) hipEventDestroy(p->kern_done[b]);
        if (p->d2h_done[b]) hipEventDestroy(p->d2h_done[b]);
    }
    if (p->s_h2d) hipStreamDestroy(p->s_h2d);
    if (p->s_comp) hipStreamDestroy(p->s_comp);
    if (p->s_d2h) hipStreamDestroy(p->s_d2h);
    free(p);
}

nc_gpuhash_pipe_t *nc_gpuhash_pipe_create(int device, uint64_t chunk_keys, uint64_t chunk_bytes, int depth)
{
    if (chunk_keys == 0 || chunk_bytes == 0 || depth < 2 || depth > NC_PIPE_MAX_DEPTH || chunk_keys >= (1ull << 32)) {
        errno = EINVAL;
        return NULL;
    }
    if (device < 0 || device >= nc_gpuhash_device_count()) {
        errno = ENODEV;
        return NULL;
    }
    nc_gpuhash_pipe_t *p = calloc(1, sizeof(*p));
    if (p == NULL) {
        errno = ENOMEM;
        return NULL;
    }
    p->device = device;
    p->depth = depth;
    p->chunk_keys = chunk_keys;
    p->chunk_bytes = chunk_bytes;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&p->s_h2d, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&p->s_comp, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&p->s_d2h, hipStreamNonBlocking);
    for (int b = 0; b < depth && e == hipSuccess; b++) {
        e = hipMalloc((void **)&p->d_keys[b], chunk_bytes + NC_GPUHASH_PAD);
        if (e == hipSuccess) e = hipMalloc((void **)&p->d_off[b], (chunk_keys + 1) * sizeof(uint64_t));
        if (e == hipSuccess) e = hipMalloc((void **)&p->d_out[b], chunk_keys * sizeof(uint32_t));
        if (e == hipSuccess) e = hipEventCreateWithFlags(&p->h2d_done[b], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&p->kern_done[b], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&p->d2h_done[b], hipEventDisableTiming);
    }
    if (e != hipSuccess) {
        hip_fail(e);
        int saved = errno;
        nc_gpuhash_pipe_destroy(p);
        errno = saved;
        return NULL;
    }
    return p;
}

/* last key index k1 > k0 such that keys [k0, k1) fit the chunk limits */
static uint64_t pipe_cut(const nc_gpuhash_pipe_t *p, const uint64_t *off, uint64_t k0, uint64_t nkeys)
{
    uint64_t hi = nkeys - k0 < p->chunk_keys ? nkeys : k0 + p->chunk_keys;
    const uint64_t limit = off[k0] + p->chunk_bytes;
    if (off[hi] <= limit) return hi;
    uint64_t lo = k0; /* largest k in [k0, hi) with off[k] <= limit */
    while (hi - lo > 1) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (off[mid] <= limit) lo = mid; else hi = mid;
    }
    return lo;
}

/* every stream of the pipe idle: no DMA still reads the caller's keys or
 * offsets, none still writes its out, no kernel still runs. Every exit of
 * nc_gpuhash_batch_pinned goes through here, so the caller may free or
 * unregister its buffers as soon as the call returns, error or not. errno is
 * kept. */
static hipError_t pipe_drain(nc_gpuhash_pipe_t *p)
{
    const int saved = errno;
    const hipError_t a = hipStreamSynchronize(p->s_h2d);
    const hipError_t b = hipStreamSynchronize(p->s_comp);
    const hipError_t c = hipStreamSynchronize(p->s_d2h);
    errno = saved;
    return a != hipSuccess ? a : (b != hipSuccess ? b : c);
}

rstatus_t nc_gpuhash_batch_pinned(nc_gpuhash_pipe_t *p, int mode, const uint8_t *keys, const uint64_t *offsets,
                                  uint64_t nkeys, uint32_t *out, const struct nc_gpuhash_shape *shape, int flags)
{
    if (p == NULL || offsets == NULL || (out == NULL && nkeys) || (keys == NULL && nkeys) || mode < 0 ||
        mode >= NC_GPUHASH_NMODES) {
        errno = EINVAL;
        return NC_ERROR;
    }
    if (nkeys == 0) return NC_OK;
    hipError_t e = hipSetDevice(p->device);
    if (e != hipSuccess) return hip_fail(e);
    if (flags != 0) { /* no flags are defined */
        errno = EINVAL;
        return NC_ERROR;
    }
    const char *dbgs = getenv("NC_GPUHASH_DEBUG");
    const int dbg = dbgs ? atoi(dbgs) : 0;
    uint64_t k0 = 0;
    for (uint64_t c = 0; k0 < nkeys; c++) {
        const int b = (int)(c % (uint64_t)p->depth);
        const uint64_t k1 = pipe_cut(p, offsets, k0, nkeys);
        if (k1 == k0) { /* one key longer than a chunk buffer */
            pipe_drain(p);
            errno = ENOMEM;
            return NC_ENOMEM;
        }
        const uint64_t b0 = offsets[k0], nb = offsets[k1] - b0;
        /* buffers of chunk c - depth: keys/offsets free once its kernel ran,
         * out free once its hashes are back */
        if (c >= (uint64_t)p->depth) e = hipStreamWaitEvent(p->s_h2d, p->kern_done[b], 0);
        if (e == hipSuccess)
            e = hipMemcpyAsync(p->d_keys[b], keys + b0, nb + NC_GPUHASH_PAD, hipMemcpyHostToDevice, p->s_h2d);
        if (e == hipSuccess)
            e = hipMemcpyAsync(p->d_off[b], offsets + k0, (k1 - k0 + 1) * sizeof(uint64_t), hipMemcpyHostToDevice,
                               p->s_h2d);
        if (e == hipSuccess) e = hipEventRecord(p->h2d_done[b], p->s_h2d);
        if (e == hipSuccess) e = hipStreamWaitEvent(p->s_comp, p->h2d_done[b], 0);
        if (e == hipSuccess && c >= (uint64_t)p->depth) e = hipStreamWaitEvent(p->s_comp, p->d2h_done[b], 0);
        if (e != hipSuccess) break;
        /* the chunk's offsets are absolute: hand the kernel the key base that
         * puts offsets[k0] at the start of the chunk buffer */
        struct nc_gpuhash_shape sh;
        const struct nc_gpuhash_shape *shp = NULL;
        if (shape != NULL) {
            sh = *shape;
            sh.key_bytes = nb;
            shp = &sh;
        }
        if (dbg >= 2) { /* DIAGNOSTIC: each chunk's inputs checked on the host before its launch */
            hipStreamSynchronize(p->s_h2d);
            uint64_t o[2];
            hipMemcpy(o, p->d_off[b], sizeof(o), hipMemcpyDeviceToHost);
            uint64_t ol;
            hipMemcpy(&ol, p->d_off[b] + (k1 - k0), sizeof(ol), hipMemcpyDeviceToHost);
            fprintf(stderr, "nc_gpuhash pipe: mode %d chunk %llu buf %d keys [%llu, %llu) bytes [%llu, +%llu) dev off %llu %llu .. %llu%s\n",
                    mode, (unsigned long long)c, b, (unsigned long long)k0, (unsigned long long)k1,
                    (unsigned long long)b0, (unsigned long long)nb, (unsigned long long)o[0], (unsigned long long)o[1],
                    (unsigned long long)ol, (o[0] != offsets[k0] || ol != offsets[k1]) ? " MISMATCH" : "");
            if (o[0] != offsets[k0] || ol != offsets[k1]) {
                pipe_drain(p);
                errno = EIO;
                return NC_ERROR;
            }
        }
        if (nc_gpuhash_batch_device_shaped(mode, (const uint8_t *)((uintptr_t)p->d_keys[b] - b0), p->d_off[b], k1 - k0, p->d_out[b], shp,
                                           p->s_comp) != NC_OK) {
            pipe_drain(p);
            return NC_ERROR;
        }
        if (dbg >= 2) {
            e = hipStreamSynchronize(p->s_comp);
            fprintf(stderr, "nc_gpuhash pipe: chunk %llu kernel: %s\n", (unsigned long long)c, hipGetErrorString(e));
            if (e != hipSuccess) break;
        }
        e = hipEventRecord(p->kern_done[b], p->s_comp);
        if (e == hipSuccess) e = hipStreamWaitEvent(p->s_d2h, p->kern_done[b], 0);
        if (e == hipSuccess)
            e = hipMemcpyAsync(out + k0, p->d_out[b], (k1 - k0) * sizeof(uint32_t), hipMemcpyDeviceToHost, p->s_d2h);
        if (e == hipSuccess) e = hipEventRecord(p->d2h_done[b], p->s_d2h);
        if (e != hipSuccess) break;
        k0 = k1;
    }
    hipError_t e2 = pipe_drain(p);
    if (e == hipSuccess) e = e2;
    return e == hipSuccess ? NC_OK : hip_fail(e);
}

rstatus_t nc_gpuhash_host_register(void *ptr, size_t bytes)
{
    if (ptr == NULL || bytes == 0) {
        errno = EINVAL;
        return NC_ERROR;
    }
    hipError_t e = hipHostRegister(ptr, bytes, hipHostRegisterMapped);
    return e == hipSuccess ? NC_OK : hip_fail(e);
}

rstatus_t nc_gpuhash_host_unregister(void *ptr)
{
    if (ptr == NULL) {
        errno = EINVAL;
        return NC_ERROR;
    }
    hipError_t e = hipHostUnregister(ptr);
    return e == hipSuccess ? NC_OK : hip_fail(e);
}
