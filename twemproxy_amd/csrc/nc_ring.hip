/*
 * Small batches without a HIP call per batch (the C5 shape:
 * one mbuf's ~600 keys).
 *
 * The context path (nc_gpuhash_submit_spans) spends ~5 µs of host time per
 * batch in hipLaunchKernel and hipEventRecord, and the device idles between
 * batches. Here the batch ring lives in mapped, coherent
 * host memory and resident worker workgroups serve it:
 *
 *   lanes: batch `seq` belongs to lane seq % kLanes, and each lane has its
 *     own worker, so one lane's PCIe round trips (fetch the batch, store the
 *     hashes) overlap the other's; every lane walks the same slots.
 *   host submit: copy the bytes under the spans into the slot's staging —
 *     the mbuf region they cover in ONE memcpy when it fits (the keys of a
 *     read are contiguous in their mbuf, src/nc_mbuf.h:25-40), else key by
 *     key — with one u32 per key (its start and end in the staged image, 16
 *     bits each), then publish the slot with ONE 64-bit store of its
 *     descriptor: sequence number + 1 in the high word, mode / key count /
 *     key bytes packed in the low word (release). No HIP call while the
 *     worker runs.
 *   worker: thread 0 polls the next slot's descriptor (one system-scope
 *     acquire load across PCIe per poll, s_sleep between polls): the load
 *     that finds the slot published also carries the batch's shape. The
 *     workgroup stages the slot's offsets and key bytes into LDS with
 *     coalesced 16-byte reads across PCIe, all of them in flight at once,
 *     every thread hashes
 *     keys from LDS with the per-key functions (nc_hash_key.h: all 12
 *     modes), writes the hashes to the slot's mapped output, fences at system
 *     scope, and thread 0 stores the slot's completion word (release).
 *   host poll: one load of that word; the hashes are copied to the caller.
 *
 * The worker always ends: it returns when `stop` is set, after kIdleTicks of
 * an empty ring, and after kLifeTicks in any case (s_memrealtime, 100 MHz).
 * Leaving is race-free: the worker publishes `exiting`, fences, then looks at
 * the next slot's descriptor once more; the host publishes the descriptor,
 * fences, then looks at `exiting`. At least one of them sees the other, so a batch is either taken
 * by the leaving worker or the host knows to relaunch one (only once the
 * previous launch has completed: never two workers on one lane). A relaunch
 * starts at `processed`, the lane's count of finished batches.
 */
#include <hip/hip_runtime.h>

#include <errno.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "nc_gpuhash.h"
#include "nc_hash_key.h"

namespace {

constexpr uint32_t kThreads = 1024;          /* the worker: one workgroup of 16 waves */
constexpr uint64_t kIdleTicks = 1000000ull;  /* 10 ms without a batch: the worker leaves */
constexpr uint64_t kLifeTicks = 200000000ull; /* 2 s: no worker outlives this (relaunched on demand) */
constexpr uint32_t kMaxKeys = 4095;          /* per batch: offsets in LDS */
constexpr uint64_t kMaxKeyBytes = 32768;     /* per batch: key bytes in LDS */
constexpr uint32_t kLanes = 2;               /* workers per ring (a power of two) */

/* the control block, host-written and device-written words on their own
 * 128-byte lines */
struct RingCtl {
    uint32_t head; /* host: the lane's batches submitted (for the host's own checks) */
    uint32_t stop; /* host: 1 = the worker returns at its next poll */
    uint32_t pad0[30];
    uint32_t exiting;   /* device: 1 from the moment a worker decides to leave */
    uint32_t processed; /* device: batches finished, in order */
    uint32_t pad1[30];
};

/* a slot's descriptor, written by the host in ONE 64-bit store: batch
 * sequence number + 1 (0 = never used) over mode (4 bits), keys (12 bits) and
 * key bytes (16 bits: up to kMaxKeyBytes) */
__host__ __device__ inline uint64_t desc_pack(uint32_t seq, uint32_t mode, uint32_t nkeys, uint32_t nbytes)
{
    return ((uint64_t)(seq + 1u) << 32) | (uint64_t)(mode & 15u) | ((uint64_t)(nkeys & 0xfffu) << 4) |
           ((uint64_t)(nbytes & 0xffffu) << 16);
}
static_assert(kMaxKeys <= 0xfffu && kMaxKeyBytes <= 0xffffu, "descriptor fields");

__device__ __forceinline__ uint32_t ld_sys(const uint32_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void st_sys(uint32_t *p, uint32_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint64_t ld_sys64(const uint64_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint64_t ticks() { return wall_clock64(); } /* s_memrealtime, 100 MHz */

/* the worker of one lane: its batches are seq = lseq * nlanes + lane for
 * lseq = start, start + 1, ... (ctl is the lane's control block) */
__global__ __launch_bounds__(kThreads) void nc_ring_worker(RingCtl *ctl, const uint64_t *desc, uint32_t *done,
                                                          const uint32_t *offs, const uint8_t *keys, uint32_t *outs,
                                                          uint32_t nslots, uint32_t max_keys, uint64_t kstride,
                                                          uint32_t lseq, uint32_t lane, uint32_t nlanes)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    __shared__ uint32_t crc16t[256], crc32t[256];
    __shared__ uint32_t cmd[2]; /* go, the descriptor's low word */
    const uint32_t t = threadIdx.x;
    uint32_t *loff = reinterpret_cast<uint32_t *>(dyn);
    uint8_t *lkeys = dyn + ((4u * (max_keys + 1u) + 15u) & ~15u);
    for (uint32_t i = t; i < 256u; i += kThreads) {
        crc16t[i] = nc_crc16_entry(i);
        crc32t[i] = nc_crc32_entry(i);
    }
    const uint64_t born = ticks();
    uint64_t last = born;
    for (;;) {
        const uint32_t seq = lseq * nlanes + lane, s = seq % nslots;
        if (t == 0u) {
            uint32_t go = 0, lo = 0;
            for (;;) {
                if (ld_sys(&ctl->stop) != 0u) break;
                const uint64_t d = ld_sys64(desc + s);
                if ((uint32_t)(d >> 32) == seq + 1u) { /* published: the shape came with it */
                    go = 1;
                    lo = (uint32_t)d;
                    break;
                }
                const uint64_t now = ticks();
                if (now - last > kIdleTicks || now - born > kLifeTicks) {
                    st_sys(&ctl->exiting, 1u);
                    __threadfence_system();
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); /* MI355X_MICROARCH.md: the fence's own wait may be dropped */
                    if ((uint32_t)(ld_sys64(desc + s) >> 32) == seq + 1u && now - born <= kLifeTicks) {
                        st_sys(&ctl->exiting, 0u); /* a batch arrived meanwhile: stay */
                        last = now;
                        continue;
                    }
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            cmd[0] = go;
            cmd[1] = lo;
        }
        __syncthreads();
        if (cmd[0] == 0u) break;
        const uint32_t mode = cmd[1] & 15u, nk = (cmd[1] >> 4) & 0xfffu, nb = cmd[1] >> 16;
        /* the slot's key spans and image into LDS: coalesced reads across
         * PCIe that bypass the caches (the host rewrote them), every load of
         * a thread issued before its first LDS write, so the workgroup pays
         * one PCIe round trip */
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const uint32_t *so = offs + (uint64_t)s * max_keys;
        const u32x4 *sk = reinterpret_cast<const u32x4 *>(keys + (uint64_t)s * kstride);
        const uint32_t nq = (nb + 15u) / 16u;
        uint32_t ov[(kMaxKeys + kThreads - 1u) / kThreads];
        u32x4 kv[(kMaxKeyBytes / 16u + kThreads - 1u) / kThreads];
#pragma unroll
        for (uint32_t j = 0; j < sizeof(ov) / sizeof(ov[0]); j++)
            if (t + j * kThreads < nk) ov[j] = __builtin_nontemporal_load(so + t + j * kThreads);
#pragma unroll
        for (uint32_t j = 0; j < sizeof(kv) / sizeof(kv[0]); j++)
            if (t + j * kThreads < nq) kv[j] = __builtin_nontemporal_load(sk + t + j * kThreads);
#pragma unroll
        for (uint32_t j = 0; j < sizeof(ov) / sizeof(ov[0]); j++)
            if (t + j * kThreads < nk) loff[t + j * kThreads] = ov[j];
#pragma unroll
        for (uint32_t j = 0; j < sizeof(kv) / sizeof(kv[0]); j++)
            if (t + j * kThreads < nq) reinterpret_cast<u32x4 *>(lkeys)[t + j * kThreads] = kv[j];
        __syncthreads();
        uint32_t *so_out = outs + (uint64_t)s * max_keys;
        for (uint32_t i = t; i < nk; i += kThreads) {
            const uint32_t sp = loff[i]; /* start | end << 16 in the image */
            so_out[i] = nc_key_hash((int)mode, lkeys + (sp & 0xffffu), (sp >> 16) - (sp & 0xffffu), crc16t, crc32t);
        }
        __builtin_amdgcn_s_waitcnt(0); /* this thread's hash stores acknowledged ... */
        __syncthreads();                /* ... in every wave ... */
        if (t == 0u) { /* ... then one system-scope release for the workgroup before the slot reads as done */
            __threadfence_system();
            /* hipcc (ROCm 7.2, gfx950) drops the fence's vmcnt(0) after its
             * L2 write-back when the scoreboard looks empty, as it does after
             * the s_waitcnt above (MI355X_MICROARCH.md): wait explicitly */
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            st_sys(&ctl->processed, lseq + 1u);
            st_sys(&done[s], seq + 1u);
        }
        last = ticks();
        lseq++;
    }
}

enum { SLOT_FREE = 0, SLOT_RUNNING = 1 };

} // namespace

struct nc_gpuhash_ring {
    int device;
    uint32_t nslots, max_keys;
    uint64_t max_key_bytes, kstride;
    uint8_t *host; /* one mapped, coherent allocation: ctl[kLanes], desc, done, offsets, keys, outputs */
    RingCtl *ctl, *d_ctl; /* one per lane */
    uint64_t *desc, *d_desc;
    uint32_t *done, *d_done, *offs, *d_offs, *outs, *d_outs;
    uint8_t *keys, *d_keys;
    uint32_t nlanes;
    hipStream_t stream[kLanes];
    hipEvent_t ev[kLanes];
    int launched[kLanes];
    uint32_t lseq[kLanes]; /* per lane: batches submitted */
    uint32_t seq;          /* next batch's sequence number */
    uint32_t *slot_state, *slot_ticket, *slot_nkeys;
    uint32_t **slot_out;
    uint64_t launches;
    pthread_mutex_t lock;
};

static rstatus_t ring_fail(hipError_t e)
{
    errno = (e == hipErrorNoDevice || e == hipErrorInvalidDevice) ? ENODEV : (e == hipErrorOutOfMemory ? ENOMEM : EIO);
    return errno == ENOMEM ? NC_ENOMEM : NC_ERROR;
}

static size_t ring_lds(const nc_gpuhash_ring_t *r)
{
    return ((4u * (r->max_keys + 1u) + 15u) & ~(size_t)15u) + r->kstride;
}

/* the key spans of a slot: start | end << 16, bytes in the staged image */
static inline uint32_t span_word(uint64_t a, uint64_t b) { return (uint32_t)a | ((uint32_t)b << 16); }

/* lock held: lane g's worker is running, or one is launched from the lane's
 * `processed` */
static rstatus_t ring_ensure_worker(nc_gpuhash_ring_t *r, uint32_t g)
{
    RingCtl *c = r->ctl + g;
    if (r->launched[g]) {
        if (__atomic_load_n(&c->exiting, __ATOMIC_ACQUIRE) == 0u) return NC_OK; /* alive: it sees the descriptor */
        const hipError_t q = hipEventQuery(r->ev[g]);
        if (q == hipErrorNotReady) return NC_OK; /* still leaving: relaunch on a later poll */
        if (q != hipSuccess) return ring_fail(q);
    }
    const uint32_t start = __atomic_load_n(&c->processed, __ATOMIC_ACQUIRE);
    if (start == r->lseq[g] && r->launched[g]) return NC_OK; /* nothing to do */
    __atomic_store_n(&c->exiting, 0u, __ATOMIC_SEQ_CST);
    hipError_t e = hipSetDevice(r->device);
    if (e != hipSuccess) return ring_fail(e);
    (void)hipGetLastError();
    hipLaunchKernelGGL(nc_ring_worker, dim3(1), dim3(kThreads), ring_lds(r), r->stream[g], r->d_ctl + g, r->d_desc,
                       r->d_done, r->d_offs, r->d_keys, r->d_outs, r->nslots, r->max_keys, r->kstride, start, g,
                       r->nlanes);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipEventRecord(r->ev[g], r->stream[g]);
    if (e != hipSuccess) return ring_fail(e);
    r->launched[g] = 1;
    r->launches++;
    return NC_OK;
}

extern "C" void nc_gpuhash_ring_destroy(nc_gpuhash_ring_t *r)
{
    if (r == NULL) return;
    for (uint32_t g = 0; g < kLanes && r->ctl != NULL; g++) __atomic_store_n(&r->ctl[g].stop, 1u, __ATOMIC_SEQ_CST);
    (void)hipSetDevice(r->device);
    for (uint32_t g = 0; g < kLanes; g++) {
        if (r->launched[g]) (void)hipEventSynchronize(r->ev[g]); /* the worker returns at its next poll */
        if (r->ev[g]) (void)hipEventDestroy(r->ev[g]);
        if (r->stream[g]) (void)hipStreamDestroy(r->stream[g]);
    }
    if (r->host) (void)hipHostFree(r->host);
    free(r->slot_state);
    free(r->slot_ticket);
    free(r->slot_nkeys);
    free(r->slot_out);
    pthread_mutex_destroy(&r->lock);
    free(r);
}

extern "C" nc_gpuhash_ring_t *nc_gpuhash_ring_create(int device, uint32_t nslots, uint32_t max_keys,
                                                     uint64_t max_key_bytes)
{
    if (nslots == 0 || nslots > 1024 || max_keys == 0 || max_keys > kMaxKeys || max_key_bytes == 0 ||
        max_key_bytes > kMaxKeyBytes) {
        errno = EINVAL;
        return NULL;
    }
    if (device < 0 || device >= nc_gpuhash_device_count()) {
        errno = ENODEV;
        return NULL;
    }
    nc_gpuhash_ring_t *r = (nc_gpuhash_ring_t *)calloc(1, sizeof(*r));
    if (r == NULL) {
        errno = ENOMEM;
        return NULL;
    }
    pthread_mutex_init(&r->lock, NULL);
    r->device = device;
    r->nslots = nslots;
    r->nlanes = nslots < kLanes ? 1u : kLanes;
    r->max_keys = max_keys;
    r->max_key_bytes = max_key_bytes;
    r->kstride = (max_key_bytes + NC_GPUHASH_PAD + 15u) & ~15ull;
    r->slot_state = (uint32_t *)calloc(nslots, sizeof(uint32_t));
    r->slot_ticket = (uint32_t *)calloc(nslots, sizeof(uint32_t));
    r->slot_nkeys = (uint32_t *)calloc(nslots, sizeof(uint32_t));
    r->slot_out = (uint32_t **)calloc(nslots, sizeof(uint32_t *));
    const size_t o_ctl = 0, o_desc = sizeof(RingCtl) * kLanes, o_done = o_desc + 8u * nslots,
                 o_offs = (o_done + 4u * nslots + 127u) & ~(size_t)127u,
                 o_keys = (o_offs + 4ull * max_keys * nslots + 127u) & ~(size_t)127u,
                 o_outs = o_keys + r->kstride * nslots, total = o_outs + 4ull * max_keys * nslots;
    hipError_t e = r->slot_state && r->slot_ticket && r->slot_nkeys && r->slot_out ? hipSetDevice(device)
                                                                                    : hipErrorOutOfMemory;
    if (e == hipSuccess) e = hipHostMalloc((void **)&r->host, total, hipHostMallocMapped | hipHostMallocCoherent);
    uint8_t *dev = NULL;
    if (e == hipSuccess) e = hipHostGetDevicePointer((void **)&dev, r->host, 0);
    for (uint32_t g = 0; g < r->nlanes; g++) {
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&r->stream[g], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&r->ev[g], hipEventDisableTiming);
    }
    if (e == hipSuccess && (size_t)(4u * (max_keys + 1u) + r->kstride) > 64u * 1024u) e = hipErrorInvalidValue;
    if (e != hipSuccess) {
        ring_fail(e);
        const int saved = errno;
        nc_gpuhash_ring_destroy(r);
        errno = saved;
        return NULL;
    }
    memset(r->host, 0, total);
    r->ctl = (RingCtl *)(r->host + o_ctl);
    r->desc = (uint64_t *)(r->host + o_desc);
    r->done = (uint32_t *)(r->host + o_done);
    r->offs = (uint32_t *)(r->host + o_offs);
    r->keys = r->host + o_keys;
    r->outs = (uint32_t *)(r->host + o_outs);
    r->d_ctl = (RingCtl *)(dev + o_ctl);
    r->d_desc = (uint64_t *)(dev + o_desc);
    r->d_done = (uint32_t *)(dev + o_done);
    r->d_offs = (uint32_t *)(dev + o_offs);
    r->d_keys = dev + o_keys;
    r->d_outs = (uint32_t *)(dev + o_outs);
    return r;
}

/* lock held: deliver slot s if its batch is done; 1 when the slot is free */
static int ring_reap(nc_gpuhash_ring_t *r, uint32_t s)
{
    if (r->slot_state[s] == SLOT_FREE) return 1;
    if (__atomic_load_n(&r->done[s], __ATOMIC_ACQUIRE) != r->slot_ticket[s] + 1u) return 0;
    memcpy(r->slot_out[s], r->outs + (size_t)s * r->max_keys, (size_t)r->slot_nkeys[s] * sizeof(uint32_t));
    r->slot_state[s] = SLOT_FREE;
    return 1;
}

extern "C" rstatus_t nc_gpuhash_ring_submit_spans(nc_gpuhash_ring_t *r, int mode, const struct nc_keyspan *spans,
                                                  uint32_t nkeys, uint32_t *out, int *ticket)
{
    if (r == NULL || (spans == NULL && nkeys) || out == NULL || ticket == NULL || mode < 0 ||
        mode >= NC_GPUHASH_NMODES) {
        errno = EINVAL;
        return NC_ERROR;
    }
    if (nkeys > r->max_keys) {
        errno = ENOMEM;
        return NC_ENOMEM;
    }
    pthread_mutex_lock(&r->lock);
    const uint32_t seq = r->seq, s = seq % r->nslots, g = seq % r->nlanes;
    if (!ring_reap(r, s)) {
        pthread_mutex_unlock(&r->lock);
        errno = EAGAIN;
        return NC_EAGAIN;
    }
    /* the spans' bytes into the slot's mapped staging (the mbufs may be
     * recycled as soon as this returns, src/nc_mbuf.c:118-128): the region
     * they cover in one memcpy when it fits (keys of one read sit in one
     * mbuf), else key by key */
    uint8_t *kd = r->keys + (size_t)s * r->kstride;
    uint32_t *od = r->offs + (size_t)s * r->max_keys;
    const uint8_t *lo = nkeys ? spans[0].start : NULL, *hi = lo;
    uint64_t klen = 0;
    for (uint32_t i = 0; i < nkeys; i++) {
        if (spans[i].start < lo) lo = spans[i].start;
        if (spans[i].end > hi) hi = spans[i].end;
        klen += (uint64_t)(spans[i].end - spans[i].start);
    }
    if (klen > r->max_key_bytes) {
        pthread_mutex_unlock(&r->lock);
        errno = ENOMEM;
        return NC_ENOMEM;
    }
    uint64_t pos;
    if ((uint64_t)(hi - lo) <= r->max_key_bytes) {
        pos = (uint64_t)(hi - lo);
        if (pos) memcpy(kd, lo, pos);
        for (uint32_t i = 0; i < nkeys; i++) od[i] = span_word(spans[i].start - lo, spans[i].end - lo);
    } else {
        pos = 0;
        for (uint32_t i = 0; i < nkeys; i++) {
            const size_t n = (size_t)(spans[i].end - spans[i].start);
            memcpy(kd + pos, spans[i].start, n);
            od[i] = span_word(pos, pos + n);
            pos += n;
        }
    }
    r->slot_state[s] = SLOT_RUNNING;
    r->slot_ticket[s] = seq;
    r->slot_nkeys[s] = nkeys;
    r->slot_out[s] = out;
    r->seq = seq + 1u;
    r->lseq[g]++;
    /* every staging write before the descriptor; then `exiting`
     * (ring_ensure_worker) after it: the host's half of the leave protocol */
    __atomic_store_n(&r->desc[s], desc_pack(seq, (uint32_t)mode, nkeys, (uint32_t)pos), __ATOMIC_SEQ_CST);
    __atomic_store_n(&r->ctl[g].head, r->lseq[g], __ATOMIC_RELAXED);
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    const rstatus_t rc = ring_ensure_worker(r, g);
    if (rc == NC_OK) *ticket = (int)(seq & 0x7fffffffu);
    pthread_mutex_unlock(&r->lock);
    return rc;
}

extern "C" rstatus_t nc_gpuhash_ring_poll(nc_gpuhash_ring_t *r, int ticket)
{
    if (r == NULL || ticket < 0) {
        errno = EINVAL;
        return NC_ERROR;
    }
    pthread_mutex_lock(&r->lock);
    const uint32_t s = (uint32_t)ticket % r->nslots;
    rstatus_t rc = NC_OK;
    if (r->slot_state[s] == SLOT_RUNNING && r->slot_ticket[s] == (uint32_t)ticket && !ring_reap(r, s)) {
        rc = ring_ensure_worker(r, (uint32_t)ticket % r->nlanes); /* a worker that left while this batch came in is relaunched */
        if (rc == NC_OK) {
            errno = EAGAIN;
            rc = NC_EAGAIN;
        }
    }
    pthread_mutex_unlock(&r->lock);
    return rc;
}

extern "C" rstatus_t nc_gpuhash_ring_wait(nc_gpuhash_ring_t *r, int ticket)
{
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (uint32_t spins = 0;; spins++) {
        const rstatus_t rc = nc_gpuhash_ring_poll(r, ticket);
        if (rc != NC_EAGAIN) return rc;
        if ((spins & 1023u) == 1023u) {
            clock_gettime(CLOCK_MONOTONIC, &t1);
            if (t1.tv_sec - t0.tv_sec > 10) { /* a worker ends within 2 s; this is a dead device */
                errno = EIO;
                return NC_ERROR;
            }
            sched_yield();
        }
    }
}

extern "C" uint64_t nc_gpuhash_ring_launches(const nc_gpuhash_ring_t *r) { return r ? r->launches : 0; }
