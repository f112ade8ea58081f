/*
 * Small batches without a HIP call per batch (the C5 shape:
 * one mbuf's ~600 keys).
 *
 * The context path (nc_gpuhash_submit_spans) spends ~5 µs of host time per
 * batch in hipLaunchKernel and hipEventRecord, and the device idles between
 * batches. Here the batch ring lives in mapped, coherent
 * host memory and ONE resident launch serves it, one workgroup per lane:
 *
 *   lanes: batch `seq` belongs to lane seq % nlanes (up to kMaxLanes), and
 *     each lane's workgroup takes its batches in order, so the lanes' PCIe
 *     round trips (find the batch, fetch it, store the hashes) overlap; every
 *     lane walks the same slots. One launch on one stream (not a stream per
 *     lane): streams share the process's few hardware queues, and a resident
 *     kernel blocks whatever queues behind it.
 *   host submit: copy the bytes under the spans into the slot's staging —
 *     the mbuf region they cover in ONE memcpy when it fits (the keys of a
 *     read are contiguous in their mbuf, src/nc_mbuf.h:25-40), else key by
 *     key — with one u32 per key (its start and end in the staged image, 16
 *     bits each), then publish the slot with ONE 64-bit store of its
 *     descriptor: the batch's tag in the high word, mode / key count / key
 *     bytes packed in the low word. No HIP call while the workers run.
 *   tags: tag(seq) = 2^31 | (seq mod 2^31), never 0 (a slot never used), and
 *     two batches of one slot within 2^31 of each other never share one. The
 *     host numbers batches with a 64-bit seq; a worker carries its next
 *     slot and tag forward by nlanes (no 32-bit product that could wrap), and
 *     its 64-bit `processed` count places a relaunch.
 *   worker: thread 0 polls its next slot's descriptor together with `stop`
 *     and the launch's `closing` word (relaxed loads, one round trip per
 *     poll; the acquire fence only once the descriptor matches); the load
 *     that finds the slot published also carries the batch's shape. The
 *     workgroup stages the slot's spans and key bytes into LDS with
 *     coalesced 16-byte reads (across PCIe, or from HBM with device
 *     staging), all in flight at once, every thread hashes keys from LDS
 *     with the batch kernels' realigning word readers (nc_lds_hash.h:
 *     aligned dwords + v_alignbyte, reads a step ahead, all 12 modes;
 *     byte-at-a-time LDS reads would put one LDS latency on every key
 *     byte) and leaves each hash in LDS; the hashes go to the slot's mapped
 *     output as 16-byte write-through stores (sc0 sc1), every storing wave
 *     drains them, and after a barrier thread 0 stores the slot's done word
 *     — no system-scope release (NC_GPUHASH_RING_WT=0: plain stores and the
 *     release, the A/B).
 *   host poll: one load of that word; the hashes are copied to the caller.
 *
 * Staging in device memory: where the host can store into the device's HBM
 * through the PCIe BAR (a large-BAR device, hipDeviceAttributeIsLargeBar),
 * the host-written, device-read words — descriptors, key spans, key images
 * and the `stop` word — live in ONE uncached device allocation instead: the
 * host's copy crosses PCIe as posted writes (write-combined: 0.41-0.58 us for
 * a C5 mbuf's 15.4 KB by AVX stores, 0.58-0.8 by memcpy,
 * tools/probes/bar_probe.hip), and the worker's poll and
 * fetch read HBM instead of crossing PCIe and back (the round trip of a flag
 * 1.75-2.1 us against 2.5-2.6 us in host memory, the same probe). Uncached:
 * the host rewrites a slot between batches behind L2's back, so no read of
 * that memory may hit a line L2 kept. The device-written words (done,
 * outputs, `exiting`, `processed`) stay in mapped host memory, where the
 * host's poll is a local load. NC_GPUHASH_RING_STAGING=host keeps everything
 * in host memory (the A/B, and devices without a large BAR). By default only
 * rings of 1 or 2 lanes stage in device memory: the host's stores through the
 * BAR cost it ~0.5 us more per C5 batch than a memcpy into host memory,
 * which is what bounds a ring of 4 and more lanes.
 *
 * The launch always ends: on `stop`; and once any lane finds the whole ring
 * idle for kIdleTicks, or the launch older than kLifeTicks (checked when
 * idle and after every batch, and honoured before the next batch is taken,
 * so under load too), it sets the launch's `closing` word and every lane
 * leaves, serving at most one more batch. Leaving is race-free per lane: the worker publishes its
 * lane's `exiting`, fences, then looks at its next slot's descriptor again
 * (and serves it if published); the host publishes a descriptor, fences,
 * then looks at that lane's `exiting`. At least one of them sees the other,
 * so a batch is either served by the leaving worker or the host knows to
 * relaunch — only once the previous launch has completed (its event), never
 * two workers on one lane. A relaunch starts each lane at its `processed`.
 * A batch published while its lane is leaving is therefore served on the
 * next submit or poll that finds the launch finished: poll (or wait) every
 * ticket.
 */
#include <hip/hip_runtime.h>

#include <errno.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <immintrin.h>

#include "nc_gpuhash.h"
#include "nc_gpuhash_probe.h"
#include "nc_hash_algo.h"
#include "nc_lds_hash.h"

namespace {

constexpr uint64_t kIdleTicks = 1000000ull;   /* 10 ms without a batch on any lane: the launch ends */
constexpr uint64_t kLifeTicks = 200000000ull; /* 2 s: no launch outlives this (relaunched on demand) */
constexpr uint32_t kMaxKeys = 4095;           /* per batch: offsets in LDS */
constexpr uint64_t kMaxKeyBytes = 32768;      /* per batch: key bytes in LDS */
constexpr uint32_t kMaxLanes = 8;             /* workgroups per launch */
constexpr uint32_t kTagBit = 0x80000000u, kTagMask = 0x7fffffffu;
static_assert(kMaxLanes == NC_GPUHASH_RING_MAX_LANES, "header limit");

/* a lane's control block in mapped host memory: host-written and
 * device-written words on their own 128-byte lines */
struct RingCtl {
    uint32_t stop; /* host: 1 = the worker returns at its next poll (host staging) */
    uint32_t pad0[31];
    uint32_t exiting;   /* device: 1 from the moment the lane's worker decides to leave */
    uint32_t pad1;
    uint64_t processed; /* device: the lane's batches finished, in order (a 64-bit lane-local count) */
    uint32_t pad2[28];
};
static_assert(sizeof(RingCtl) == 256, "two lines per lane");

/* the launch's shared state, in device memory (workgroups of one launch) */
struct RingDev {
    uint64_t last; /* s_memrealtime of the latest finished batch on any lane */
    uint32_t closing; /* = the launch's epoch once the launch is ending */
    uint32_t pad;
};

__host__ __device__ inline uint32_t ring_tag(uint64_t seq) { return kTagBit | (uint32_t)(seq & kTagMask); }

/* a slot's descriptor, written by the host in ONE 64-bit store: the batch's
 * tag over mode (4 bits), keys (12 bits) and key bytes (16 bits: up to
 * kMaxKeyBytes) */
__host__ __device__ inline uint64_t desc_pack(uint32_t tag, uint32_t mode, uint32_t nkeys, uint32_t nbytes)
{
    return ((uint64_t)tag << 32) | (uint64_t)(mode & 15u) | ((uint64_t)(nkeys & 0xfffu) << 4) |
           ((uint64_t)(nbytes & 0xffffu) << 16);
}
static_assert(kMaxKeys <= 0xfffu && kMaxKeyBytes <= 0xffffu, "descriptor fields");

__device__ __forceinline__ uint32_t ld_rlx(const uint32_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint64_t ld_rlx64(const uint64_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void st_sys(uint32_t *p, uint32_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void st_sys64(uint64_t *p, uint64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

/* a system-scope release whose write-back is waited for: hipcc (ROCm 7.2,
 * gfx950) drops the fence's vmcnt(0) after its L2 write-back when the
 * scoreboard looks empty (MI355X_MICROARCH.md), so wait explicitly */
__device__ __forceinline__ void release_sys()
{
    __threadfence_system();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ uint64_t ticks() { return wall_clock64(); } /* s_memrealtime, 100 MHz */

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

/* 16 hash bytes into the slot's mapped output, write-through (sc0 sc1: the
 * system-scope store form), so that the storing wave's vmcnt(0) wait alone
 * orders them before the done word — no L2 write-back (MI355X_MICROARCH.md,
 * hand-off forms: sc0 sc1 stores, every storing wave drained, a barrier, one
 * lane's flag). One fabric write per 16 bytes, not per 4 (a C5 batch: 147
 * PCIe writes instead of 585). */
__device__ __forceinline__ void st_out4(__amdgpu_buffer_rsrc_t rsrc, uint32_t q, u32x4 v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, q * 16u, 0, 17 /* sc0 sc1 */);
}

/* the batch's keys, thread t taking keys t, t + T, ...: each read from the
 * LDS image by the realigning reader (which may read up to 22 bytes past a
 * key: the image's NC_GPUHASH_PAD tail). Each hash goes to the mapped output
 * (plain stores, published by the release before the done word), or with
 * `wt` in place of its span word in LDS, for one write-through pass out. */
template <int MODE, uint32_t T>
__device__ __forceinline__ void serve(const LdsSrc &src, uint32_t *loff, uint32_t nk, const uint32_t *tab,
                                      uint32_t *so_out, bool wt)
{
    for (uint32_t i = threadIdx.x; i < nk; i += T) {
        const uint32_t sp = loff[i]; /* start | end << 16 in the image */
        const uint32_t h = hash_key<MODE, 0>(src, sp & 0xffffu, (sp >> 16) - (sp & 0xffffu), tab);
        if (wt) loff[i] = h;
        else so_out[i] = h;
    }
}

/* one poll of a lane's next slot: three relaxed loads issued together */
struct Poll {
    uint64_t d;
    uint32_t stop, closing;
    __device__ __forceinline__ void issue(const uint32_t *stopw, const uint64_t *dp, RingDev *dv)
    {
        stop = ld_rlx(stopw);
        d = ld_rlx64(dp);
        closing = __hip_atomic_load(&dv->closing, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
};

/* thread 0: a poll's outcome. 1: stop (go = 0) or the batch is published (go
 * = 1, lo = the descriptor's low word) or, once leaving, nothing came (go =
 * 0); -1: the launch is ending and `exiting` was just published (poll once
 * more); 0: keep polling. The idle and life limits as in the file comment:
 * `closing` (another lane ended the launch) and `expired` (this lane's last
 * batch finished past kLifeTicks, tested after each batch, off the batch's
 * critical path) are honoured BEFORE a published batch is taken, so a lane
 * that always finds its next batch waiting still leaves. Once leaving, the
 * lane serves at most the one batch its post-`exiting` re-read found; every
 * later one is the relaunch's (its `processed` says where to start). */
__device__ __forceinline__ int poll_check(const Poll &p, uint32_t tag, uint32_t epoch, bool expired, uint64_t &last,
                                          bool &leaving, bool &last_taken, RingCtl *c, RingDev *dv, uint32_t &go,
                                          uint32_t &lo)
{
    if (p.stop != 0u) return 1;
    const bool pub = (uint32_t)(p.d >> 32) == tag; /* published: the shape came with it */
    if (leaving) { /* the descriptor was re-read after `exiting`: serve what it found, once; else the host relaunches */
        if (pub && !last_taken) {
            go = 1;
            lo = (uint32_t)p.d;
            last_taken = true;
        }
        return 1;
    }
    bool close = expired || p.closing == epoch;
    if (pub && !close) {
        go = 1;
        lo = (uint32_t)p.d;
        return 1;
    }
    if (!close && !pub) {
        const uint64_t now = ticks();
        if (now - last > kIdleTicks) {
            const uint64_t any = __hip_atomic_load(&dv->last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            close = now > any && now - any > kIdleTicks;
            if (!close) last = any;
        }
    }
    if (!close) return 0;
    __hip_atomic_store(&dv->closing, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    st_sys(&c->exiting, 1u);
    release_sys();
    leaving = true;
    return -1;
}

/* one launch, one workgroup per lane (lane = blockIdx.x): lane g's batches
 * are seq = k * nlanes + g for k = processed, processed + 1, ... */
template <uint32_t T>
__global__ __launch_bounds__(T) void nc_ring_worker(RingCtl *ctl, RingDev *dv, const uint32_t *stopw,
                                                    uint32_t stop_stride, const uint64_t *desc, uint32_t *done,
                                                    const uint32_t *offs, const uint8_t *keys, uint32_t *outs,
                                                    uint32_t nslots, uint32_t max_keys, uint64_t kstride,
                                                    uint32_t nlanes, uint32_t epoch, uint32_t flags, uint64_t *tl)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    __shared__ uint32_t crc16t[256], crc32t[256];
    __shared__ uint32_t cmd[2]; /* go, the descriptor's low word */
    const uint32_t t = threadIdx.x, lane = blockIdx.x;
    RingCtl *c = ctl + lane;
    const uint32_t *stop_lane = stopw + (uint64_t)lane * stop_stride; /* the lane's `stop`, or the ring's one word */
    uint32_t *loff = reinterpret_cast<uint32_t *>(dyn);
    uint8_t *lkeys = dyn + ((4u * (max_keys + 1u) + 15u) & ~15u);
    const bool wt = (flags & 1u) != 0u;
    const uint32_t ostride = (max_keys + 3u) & ~3u; /* outputs: 16-byte aligned slots */
    for (uint32_t i = t; i < 256u; i += T) {
        crc16t[i] = nc_crc16_entry(i);
        crc32t[i] = nc_crc32_entry(i);
    }
    /* where this lane resumes: its next batch's slot and tag, carried forward
     * by nlanes per batch (mod nslots, mod 2^31) */
    uint64_t done_count = __hip_atomic_load(&c->processed, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t seq0 = done_count * nlanes + lane;
    uint32_t s = (uint32_t)(seq0 % nslots), tag = ring_tag(seq0);
    const uint64_t born = ticks();
    uint64_t last = born;
    bool leaving = false;    /* thread 0: `exiting` published and fenced */
    bool last_taken = false; /* thread 0: the one batch a leaving lane serves was taken */
    bool expired = false;    /* thread 0: a batch finished past kLifeTicks */
    uint64_t t_found = 0, t_staged = 0, t_issued = 0; /* thread 0: the diagnostic timeline (tl) */
    uint64_t c_staged = 0, c_issued = 0; /* thread 0: shader-clock cycles (s_memtime) at the same two points */
    for (;;) {
        if (t == 0u) {
            uint32_t go = 0, lo = 0;
            /* one poll at a time: the acquire fence after a match waits for
             * every load in flight, so a second poll in flight (issued half a
             * round trip later) costs the batch more than it saves
             * (measured: depth 1 7.3-7.9 -> 8.1-8.7 us) */
            for (;;) {
                Poll p;
                p.issue(stop_lane, desc + s, dv);
                const int r = poll_check(p, tag, epoch, expired, last, leaving, last_taken, c, dv, go, lo);
                if (r > 0) break;
                if (r == 0) __builtin_amdgcn_s_sleep(2);
            }
            if (go) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); /* system scope: the staging's bytes after the descriptor */
                t_found = ticks();
            }
            cmd[0] = go;
            cmd[1] = lo;
        }
        __syncthreads();
        if (cmd[0] == 0u) break;
        const uint32_t mode = cmd[1] & 15u, nk = (cmd[1] >> 4) & 0xfffu, nb = cmd[1] >> 16;
        /* the slot's key spans and image into LDS: coalesced reads (across
         * PCIe, or from uncached HBM with device staging) that bypass the
         * caches (the host rewrote them), every load of a thread issued
         * before its first LDS write, so the workgroup pays one round trip */
        const uint32_t *so = offs + (uint64_t)s * max_keys;
        const u32x4 *sk = reinterpret_cast<const u32x4 *>(keys + (uint64_t)s * kstride);
        const uint32_t nq = (nb + 15u) / 16u;
        uint32_t ov[(kMaxKeys + T - 1u) / T];
        u32x4 kv[(kMaxKeyBytes / 16u + T - 1u) / T];
#pragma unroll
        for (uint32_t j = 0; j < sizeof(ov) / sizeof(ov[0]); j++)
            if (t + j * T < nk) ov[j] = __builtin_nontemporal_load(so + t + j * T);
#pragma unroll
        for (uint32_t j = 0; j < sizeof(kv) / sizeof(kv[0]); j++)
            if (t + j * T < nq) kv[j] = __builtin_nontemporal_load(sk + t + j * T);
#pragma unroll
        for (uint32_t j = 0; j < sizeof(ov) / sizeof(ov[0]); j++)
            if (t + j * T < nk) loff[t + j * T] = ov[j];
#pragma unroll
        for (uint32_t j = 0; j < sizeof(kv) / sizeof(kv[0]); j++)
            if (t + j * T < nq) reinterpret_cast<u32x4 *>(lkeys)[t + j * T] = kv[j];
        __syncthreads();
        if (tl != nullptr && t == 0u) {
            t_staged = ticks();
            c_staged = __builtin_readcyclecounter();
        }
        uint32_t *so_out = outs + (uint64_t)s * ostride;
        const LdsSrc src{reinterpret_cast<const uint32_t *>(lkeys)};
        switch (mode) {
        case NC_GPUHASH_ONE_AT_A_TIME: serve<NC_GPUHASH_ONE_AT_A_TIME, T>(src, loff, nk, crc32t, so_out, wt); break;
        case NC_GPUHASH_MD5: serve<NC_GPUHASH_MD5, T>(src, loff, nk, crc32t, so_out, wt); break;
        case NC_GPUHASH_CRC16: serve<NC_GPUHASH_CRC16, T>(src, loff, nk, crc16t, so_out, wt); break;
        case NC_GPUHASH_CRC32: serve<NC_GPUHASH_CRC32, T>(src, loff, nk, crc32t, so_out, wt); break;
        case NC_GPUHASH_CRC32A: serve<NC_GPUHASH_CRC32A, T>(src, loff, nk, crc32t, so_out, wt); break;
        case NC_GPUHASH_FNV1_64: serve<NC_GPUHASH_FNV1_64, T>(src, loff, nk, crc32t, so_out, wt); break;
        case NC_GPUHASH_FNV1A_64: serve<NC_GPUHASH_FNV1A_64, T>(src, loff, nk, crc32t, so_out, wt); break;
        case NC_GPUHASH_FNV1_32: serve<NC_GPUHASH_FNV1_32, T>(src, loff, nk, crc32t, so_out, wt); break;
        case NC_GPUHASH_FNV1A_32: serve<NC_GPUHASH_FNV1A_32, T>(src, loff, nk, crc32t, so_out, wt); break;
        case NC_GPUHASH_HSIEH: serve<NC_GPUHASH_HSIEH, T>(src, loff, nk, crc32t, so_out, wt); break;
        case NC_GPUHASH_MURMUR: serve<NC_GPUHASH_MURMUR, T>(src, loff, nk, crc32t, so_out, wt); break;
        default: serve<NC_GPUHASH_JENKINS, T>(src, loff, nk, crc32t, so_out, wt); break;
        }
        uint64_t t_own = 0; /* thread 0: its own wave's keys hashed (before waiting for the others) */
        if (tl != nullptr && t == 0u) t_own = ticks();
        if (wt) { /* the hashes, in LDS, out 16 bytes a lane (up to 3 words past nk: within the slot's ostride) */
            __syncthreads();
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(so_out, 0, 4u * ostride, 0x00020000);
            for (uint32_t q = t; q < (nk + 3u) / 4u; q += T) st_out4(rs, q, reinterpret_cast<const u32x4 *>(loff)[q]);
        }
        if (tl != nullptr) { /* diagnostics: every thread's hashes issued (stores not yet acknowledged) */
            __syncthreads();
            if (t == 0u) {
                t_issued = ticks();
                c_issued = __builtin_readcyclecounter();
            }
        }
        __builtin_amdgcn_s_waitcnt(0); /* this thread's hash stores acknowledged ... */
        __syncthreads();                /* ... in every wave ... */
        done_count++;
        if (t == 0u) { /* ... then one system-scope release for the workgroup before the slot reads as done */
            if (tl != nullptr) { /* found, staged, issued, stored: ordered by the release (or drain) below */
                __hip_atomic_store(&tl[8 * s + 0], (uint64_t)(t_found), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&tl[8 * s + 1], (uint64_t)(t_staged), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&tl[8 * s + 2], (uint64_t)(t_issued), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&tl[8 * s + 3], (uint64_t)(ticks()), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&tl[8 * s + 7], t_own, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                /* [6]: the shader clock over the hash phase, MHz (cycles per 10 ns tick x 100) */
                __hip_atomic_store(&tl[8 * s + 6], t_issued > t_staged ? (c_issued - c_staged) * 100u / (t_issued - t_staged) : 0u,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            if (wt) asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); /* the hashes went through: acknowledged above */
            else release_sys();
            if (tl != nullptr) { /* released (or drained); these two may land just after the done word */
                __hip_atomic_store(&tl[8 * s + 4], ticks(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&tl[8 * s + 5], done_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            /* relaxed stores after the fence: a release store would wait for
             * the write-back again. `processed` is read by the host only
             * once the launch has ended */
            __hip_atomic_store(&done[s], tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&c->processed, done_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            last = ticks();
            expired = last - born > kLifeTicks;
            __hip_atomic_fetch_max(&dv->last, last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        tag = kTagBit | ((tag + nlanes) & kTagMask);
        s += nlanes;
        if (s >= nslots) s -= nslots; /* nlanes <= nslots */
    }
}

typedef void (*worker_fn)(RingCtl *, RingDev *, const uint32_t *, uint32_t, const uint64_t *, uint32_t *,
                          const uint32_t *, const uint8_t *, uint32_t *, uint32_t, uint32_t, uint64_t, uint32_t, uint32_t,
                          uint32_t, uint64_t *);

enum { SLOT_FREE = 0, SLOT_RUNNING = 1 };

} // namespace

/* the staging copy. Into write-combined BAR memory (device staging) whole
 * 64-byte (AVX-512) or 32-byte (AVX2) stores fill the write-combining lines
 * directly: a C5 mbuf's 15.4 KB takes 0.41 us with 32-byte stores against
 * 0.58 us by glibc's memcpy (tools/probes/bar_probe.hip, bar_copy). Into host
 * memory memcpy is as fast (0.08-0.09 us). */
typedef void (*stage_copy_fn)(uint8_t *, const uint8_t *, size_t);

__attribute__((target("avx512f"))) static void copy_wc64(uint8_t *d, const uint8_t *s, size_t n)
{
    size_t i = 0;
    for (; i + 64 <= n; i += 64) _mm512_storeu_si512((void *)(d + i), _mm512_loadu_si512((const void *)(s + i)));
    if (i < n) memcpy(d + i, s + i, n - i);
}

__attribute__((target("avx2"))) static void copy_wc32(uint8_t *d, const uint8_t *s, size_t n)
{
    size_t i = 0;
    for (; i + 32 <= n; i += 32)
        _mm256_storeu_si256((__m256i *)(d + i), _mm256_loadu_si256((const __m256i *)(s + i)));
    if (i < n) memcpy(d + i, s + i, n - i);
}

static void copy_plain(uint8_t *d, const uint8_t *s, size_t n) { memcpy(d, s, n); }

struct nc_gpuhash_ring {
    int device;
    uint32_t nslots, max_keys, nlanes, threads;
    uint64_t max_key_bytes, kstride;
    uint8_t *host; /* one mapped, coherent allocation: ctl[kMaxLanes], done, outputs (+ desc, offsets, keys) */
    uint8_t *stage; /* device staging (large BAR): the stop word, desc, offsets, keys; NULL = all in host */
    uint32_t *stopw, *d_stopw; /* the words the workers poll for `stop` */
    uint32_t stop_stride;      /* in words, between lanes' stop words (0: one word for all) */
    uint32_t flags;            /* the worker's: bit 0 = write-through hashes (st_out4), no release before done */
    stage_copy_fn copy;        /* key bytes into the staging */
    RingCtl *ctl, *d_ctl; /* one per lane */
    uint64_t *desc, *d_desc;
    uint32_t *done, *d_done, *offs, *d_offs, *outs, *d_outs;
    uint8_t *keys, *d_keys;
    RingDev *dv; /* device memory */
    hipStream_t stream;
    hipEvent_t ev;
    int launched;
    int hold; /* diagnostics: no launch while set */
    uint32_t epoch;
    uint64_t seq;  /* next batch's sequence number */
    uint64_t seq0; /* the first one this ring numbered */
    uint64_t *tl, *d_tl; /* diagnostics: 8 words of device timeline per slot */
    int timeline;
    uint32_t *slot_state, *slot_nkeys;
    uint64_t *slot_seq;
    uint32_t **slot_out;
    uint64_t launches;
    pthread_mutex_t lock;
};

static rstatus_t ring_fail(hipError_t e)
{
    errno = (e == hipErrorNoDevice || e == hipErrorInvalidDevice) ? ENODEV : (e == hipErrorOutOfMemory ? ENOMEM : EIO);
    return errno == ENOMEM ? NC_ENOMEM : NC_ERROR;
}

/* the LDS of a lane: span words (then the hashes), the key image, and 96
 * bytes for the realigning reader's look-ahead (md5's final block reads up to
 * 86 bytes past its start, nc_lds_hash.h) */
static size_t ring_lds(const nc_gpuhash_ring_t *r)
{
    return ((4u * (r->max_keys + 1u) + 15u) & ~(size_t)15u) + r->kstride + 96u;
}

static worker_fn ring_kernel(uint32_t threads)
{
    switch (threads) {
    case 256: return nc_ring_worker<256>;
    case 512: return nc_ring_worker<512>;
    default: return nc_ring_worker<1024>;
    }
}

/* lane g's batches numbered below r->seq (its lane-local submit count) */
static inline uint64_t lane_submitted(const nc_gpuhash_ring_t *r, uint32_t g)
{
    return (r->seq + r->nlanes - 1u - g) / r->nlanes;
}

/* the key spans of a slot: start | end << 16, bytes in the staged image */
static inline uint32_t span_word(uint64_t a, uint64_t b) { return (uint32_t)a | ((uint32_t)b << 16); }

/* lock held: lane g's worker is running and will see its published batches,
 * or the launch has ended and a new one starts every lane at its
 * `processed` */
static rstatus_t ring_ensure_worker(nc_gpuhash_ring_t *r, uint32_t g)
{
    if (r->launched) {
        if (__atomic_load_n(&r->ctl[g].exiting, __ATOMIC_ACQUIRE) == 0u) return NC_OK; /* alive: it sees the descriptor */
        const hipError_t q = hipEventQuery(r->ev);
        if (q == hipErrorNotReady) return NC_OK; /* still leaving: relaunch on a later poll */
        if (q != hipSuccess) return ring_fail(q);
        r->launched = 0;
    }
    int pending = 0;
    for (uint32_t h = 0; h < r->nlanes; h++)
        pending |= __atomic_load_n(&r->ctl[h].processed, __ATOMIC_ACQUIRE) != lane_submitted(r, h);
    if (!pending || r->hold) return NC_OK;
    for (uint32_t h = 0; h < r->nlanes; h++) __atomic_store_n(&r->ctl[h].exiting, 0u, __ATOMIC_SEQ_CST);
    hipError_t e = hipSetDevice(r->device);
    if (e != hipSuccess) return ring_fail(e);
    (void)hipGetLastError();
    r->epoch++;
    hipLaunchKernelGGL(ring_kernel(r->threads), dim3(r->nlanes), dim3(r->threads), ring_lds(r), r->stream, r->d_ctl,
                       r->dv, r->d_stopw, r->stop_stride, r->d_desc, r->d_done, r->d_offs, r->d_keys, r->d_outs,
                       r->nslots, r->max_keys, r->kstride, r->nlanes, r->epoch, r->flags,
                       r->timeline ? r->d_tl : nullptr);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipEventRecord(r->ev, r->stream);
    if (e != hipSuccess) return ring_fail(e);
    r->launched = 1;
    r->launches++;
    return NC_OK;
}

extern "C" void nc_gpuhash_ring_destroy(nc_gpuhash_ring_t *r)
{
    if (r == NULL) return;
    for (uint32_t g = 0; g < kMaxLanes && r->ctl != NULL; g++) __atomic_store_n(&r->ctl[g].stop, 1u, __ATOMIC_SEQ_CST);
    if (r->stage != NULL && r->stopw != NULL) { /* through the BAR: a plain store, then a fence that drains it */
        __atomic_store_n(r->stopw, 1u, __ATOMIC_RELEASE);
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
    }
    (void)hipSetDevice(r->device);
    if (r->launched) (void)hipEventSynchronize(r->ev); /* every lane returns at its next poll */
    if (r->ev) (void)hipEventDestroy(r->ev);
    if (r->stream) (void)hipStreamDestroy(r->stream);
    if (r->dv) (void)hipFree(r->dv);
    if (r->host) (void)hipHostFree(r->host);
    if (r->stage) (void)hipFree(r->stage);
    free(r->slot_state);
    free(r->slot_seq);
    free(r->slot_nkeys);
    free(r->slot_out);
    pthread_mutex_destroy(&r->lock);
    free(r);
}

extern "C" nc_gpuhash_ring_t *nc_gpuhash_ring_create_ex(int device, uint32_t nslots, uint32_t max_keys,
                                                        uint64_t max_key_bytes, uint32_t nlanes, uint32_t threads)
{
    if (nslots == 0 || nslots > 1024 || max_keys == 0 || max_keys > kMaxKeys || max_key_bytes == 0 ||
        max_key_bytes > kMaxKeyBytes || nlanes > kMaxLanes ||
        (threads != 0 && threads != 256 && threads != 512 && threads != 1024)) {
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
    if (nlanes == 0) nlanes = NC_GPUHASH_RING_DEFAULT_LANES;
    r->nlanes = nlanes < nslots ? nlanes : nslots;
    r->threads = threads ? threads : NC_GPUHASH_RING_DEFAULT_THREADS;
    r->max_keys = max_keys;
    r->max_key_bytes = max_key_bytes;
    r->kstride = (max_key_bytes + NC_GPUHASH_PAD + 15u) & ~15ull;
    r->slot_state = (uint32_t *)calloc(nslots, sizeof(uint32_t));
    r->slot_seq = (uint64_t *)calloc(nslots, sizeof(uint64_t));
    r->slot_nkeys = (uint32_t *)calloc(nslots, sizeof(uint32_t));
    r->slot_out = (uint32_t **)calloc(nslots, sizeof(uint32_t *));
    /* host-written words (stop, desc, offsets, keys) from o_stop to o_done,
     * device-written ones (ctl's device half, done, outputs, timeline) around
     * them; with device staging the host-written block is the stage */
    const size_t o_ctl = 0, o_stop = sizeof(RingCtl) * kMaxLanes, o_desc = o_stop + 128u,
                 o_offs = (o_desc + 8u * nslots + 127u) & ~(size_t)127u,
                 o_keys = (o_offs + 4ull * max_keys * nslots + 127u) & ~(size_t)127u,
                 o_done = o_keys + r->kstride * nslots, o_outs = (o_done + 4u * nslots + 127u) & ~(size_t)127u,
                 o_tl = (o_outs + 4ull * ((max_keys + 3u) & ~3u) * nslots + 127u) & ~(size_t)127u,
                 total = o_tl + 64ull * nslots;
    hipError_t e = r->slot_state && r->slot_seq && r->slot_nkeys && r->slot_out ? hipSetDevice(device)
                                                                                : hipErrorOutOfMemory;
    int large_bar = 0;
    const char *sv = getenv("NC_GPUHASH_RING_STAGING"), *wv = getenv("NC_GPUHASH_RING_WT");
    r->flags = (wv != NULL && strcmp(wv, "0") == 0) ? 0u : 1u; /* A/B: NC_GPUHASH_RING_WT=0, plain stores + release */
    const int want_dev = sv != NULL ? strcmp(sv, "device") == 0 : r->nlanes <= 2u;
    if (e == hipSuccess) e = hipHostMalloc((void **)&r->host, total, hipHostMallocMapped | hipHostMallocCoherent);
    uint8_t *dev = NULL;
    if (e == hipSuccess) e = hipHostGetDevicePointer((void **)&dev, r->host, 0);
    if (e == hipSuccess) e = hipMalloc((void **)&r->dv, sizeof(RingDev));
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&r->ev, hipEventDisableTiming);
    /* zeroed on the ring's own stream: a device-wide synchronize would wait
     * for another ring's resident worker */
    if (e == hipSuccess) e = hipMemsetAsync(r->dv, 0, sizeof(RingDev), r->stream);
    if (e == hipSuccess && want_dev &&
        hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, device) == hipSuccess && large_bar) {
        /* the host stores into it through the BAR; if it cannot be had, host staging */
        if (hipExtMallocWithFlags((void **)&r->stage, o_done - o_stop, hipDeviceMallocUncached) != hipSuccess) {
            (void)hipGetLastError();
            r->stage = NULL;
        } else {
            e = hipMemsetAsync(r->stage, 0, o_done - o_stop, r->stream);
        }
    }
    if (e == hipSuccess) e = hipStreamSynchronize(r->stream);
    /* NC_GPUHASH_RING_COPY=memcpy|avx2|avx512: the A/B of the staging copy */
    const char *cv = getenv("NC_GPUHASH_RING_COPY");
#if !defined(__HIP_DEVICE_COMPILE__)
    __builtin_cpu_init();
    const bool has512 = __builtin_cpu_supports("avx512f"), has256 = __builtin_cpu_supports("avx2");
#else
    const bool has512 = false, has256 = false;
#endif
    r->copy = copy_plain;
    if (r->stage != NULL && !(cv != NULL && strcmp(cv, "memcpy") == 0)) {
        if (has512 && !(cv != NULL && strcmp(cv, "avx2") == 0)) r->copy = copy_wc64;
        else if (has256) r->copy = copy_wc32;
    }
    if (e == hipSuccess && ring_lds(r) > 64u * 1024u) e = hipErrorInvalidValue;
    if (e != hipSuccess) {
        ring_fail(e);
        const int saved = errno;
        nc_gpuhash_ring_destroy(r);
        errno = saved;
        return NULL;
    }
    memset(r->host, 0, total);
    r->ctl = (RingCtl *)(r->host + o_ctl);
    r->done = (uint32_t *)(r->host + o_done);
    r->outs = (uint32_t *)(r->host + o_outs);
    r->tl = (uint64_t *)(r->host + o_tl);
    r->d_tl = (uint64_t *)(dev + o_tl);
    r->d_ctl = (RingCtl *)(dev + o_ctl);
    r->d_done = (uint32_t *)(dev + o_done);
    r->d_outs = (uint32_t *)(dev + o_outs);
    /* the host-written block: the stage (one address for host and device,
     * the BAR mapping) or the host allocation's own */
    uint8_t *hw = r->stage ? r->stage - o_stop : r->host, *dw = r->stage ? r->stage - o_stop : dev;
    r->desc = (uint64_t *)(hw + o_desc);
    r->offs = (uint32_t *)(hw + o_offs);
    r->keys = hw + o_keys;
    r->d_desc = (uint64_t *)(dw + o_desc);
    r->d_offs = (uint32_t *)(dw + o_offs);
    r->d_keys = dw + o_keys;
    if (r->stage) { /* one stop word for every lane */
        r->stopw = (uint32_t *)r->stage;
        r->d_stopw = (uint32_t *)r->stage;
        r->stop_stride = 0;
    } else {
        r->stopw = &r->ctl[0].stop;
        r->d_stopw = &r->d_ctl[0].stop;
        r->stop_stride = sizeof(RingCtl) / sizeof(uint32_t);
    }
    return r;
}

extern "C" nc_gpuhash_ring_t *nc_gpuhash_ring_create(int device, uint32_t nslots, uint32_t max_keys,
                                                     uint64_t max_key_bytes)
{
    return nc_gpuhash_ring_create_ex(device, nslots, max_keys, max_key_bytes, 0, 0);
}

/* lock held: deliver slot s if its batch is done; 1 when the slot is free */
static int ring_reap(nc_gpuhash_ring_t *r, uint32_t s)
{
    if (r->slot_state[s] == SLOT_FREE) return 1;
    if (__atomic_load_n(&r->done[s], __ATOMIC_ACQUIRE) != ring_tag(r->slot_seq[s])) return 0;
    if (r->slot_out[s] != NULL) /* NULL: the ticket was forgotten (its owner is gone) */
        memcpy(r->slot_out[s], r->outs + (size_t)s * ((r->max_keys + 3u) & ~3u), (size_t)r->slot_nkeys[s] * sizeof(uint32_t));
    r->slot_state[s] = SLOT_FREE;
    return 1;
}

extern "C" rstatus_t nc_gpuhash_ring_submit_spans(nc_gpuhash_ring_t *r, int mode, const struct nc_keyspan *spans,
                                                  uint32_t nkeys, uint32_t *out, int *ticket)
{
    if (r == NULL || (spans == NULL && nkeys) || (out == NULL && nkeys) || ticket == NULL || mode < 0 ||
        mode >= NC_GPUHASH_NMODES) {
        errno = EINVAL;
        return NC_ERROR;
    }
    if (nkeys > r->max_keys) {
        errno = ENOMEM;
        return NC_ENOMEM;
    }
    /* the spans first, before any state changes: an inverted or NULL span is
     * the caller's error */
    const uint8_t *lo = nkeys ? spans[0].start : NULL, *hi = lo;
    uint64_t klen = 0;
    for (uint32_t i = 0; i < nkeys; i++) {
        if (spans[i].start == NULL || spans[i].end < spans[i].start) {
            errno = EINVAL;
            return NC_ERROR;
        }
        if (spans[i].start < lo) lo = spans[i].start;
        if (spans[i].end > hi) hi = spans[i].end;
        klen += (uint64_t)(spans[i].end - spans[i].start);
    }
    if (klen > r->max_key_bytes) {
        errno = ENOMEM;
        return NC_ENOMEM;
    }
    pthread_mutex_lock(&r->lock);
    const uint64_t seq = r->seq;
    const uint32_t s = (uint32_t)(seq % r->nslots), g = (uint32_t)(seq % r->nlanes);
    if (!ring_reap(r, s)) {
        /* the slot's batch still runs — or waits for a worker: its lane may
         * have left with nobody polling the ticket (forgotten), so relaunch
         * here as a poll would */
        const rstatus_t rc = ring_ensure_worker(r, (uint32_t)(r->slot_seq[s] % r->nlanes));
        pthread_mutex_unlock(&r->lock);
        if (rc != NC_OK) return rc;
        errno = EAGAIN;
        return NC_EAGAIN;
    }
    /* the spans' bytes into the slot's mapped staging (the mbufs may be
     * recycled as soon as this returns, src/nc_mbuf.c:118-128): the region
     * they cover in one memcpy when it fits (keys of one read sit in one
     * mbuf), else key by key */
    uint8_t *kd = r->keys + (size_t)s * r->kstride;
    uint32_t *od = r->offs + (size_t)s * r->max_keys;
    uint64_t pos;
    if ((uint64_t)(hi - lo) <= r->max_key_bytes) {
        pos = (uint64_t)(hi - lo);
        if (pos) r->copy(kd, lo, pos);
        for (uint32_t i = 0; i < nkeys; i++) od[i] = span_word(spans[i].start - lo, spans[i].end - lo);
    } else {
        pos = 0;
        for (uint32_t i = 0; i < nkeys; i++) {
            const size_t n = (size_t)(spans[i].end - spans[i].start);
            r->copy(kd + pos, spans[i].start, n);
            od[i] = span_word(pos, pos + n);
            pos += n;
        }
    }
    r->slot_state[s] = SLOT_RUNNING;
    r->slot_seq[s] = seq;
    r->slot_nkeys[s] = nkeys;
    r->slot_out[s] = out;
    r->seq = seq + 1u;
    /* every staging write before the descriptor, then `exiting`
     * (ring_ensure_worker) after it: the host's half of the leave protocol.
     * Two full fences around a plain 64-bit store, no locked instruction:
     * with device staging the stores are write-combined through the BAR (a
     * locked read-modify-write has no business on PCIe), and the fences drain
     * the write-combining buffers in order */
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    __atomic_store_n(&r->desc[s], desc_pack(ring_tag(seq), (uint32_t)mode, nkeys, (uint32_t)pos), __ATOMIC_RELEASE);
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    const rstatus_t rc = ring_ensure_worker(r, g);
    if (rc == NC_OK) *ticket = (int)(seq & kTagMask);
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
    /* the ticket's batch: the latest seq below r->seq with these 31 bits */
    const uint64_t back = (r->seq - (uint64_t)ticket) & kTagMask;
    rstatus_t rc = NC_OK;
    if (back == 0 || back > r->seq - r->seq0) { /* never issued */
        errno = EINVAL;
        rc = NC_ERROR;
    } else if (back <= r->nslots) { /* one of the last nslots batches: its slot holds it or delivered it */
        const uint64_t seq = r->seq - back;
        const uint32_t s = (uint32_t)(seq % r->nslots);
        if (r->slot_seq[s] == seq && r->slot_state[s] == SLOT_RUNNING && !ring_reap(r, s)) {
            /* a lane whose worker left while this batch came in is relaunched */
            rc = ring_ensure_worker(r, (uint32_t)(seq % r->nlanes));
            if (rc == NC_OK) {
                errno = EAGAIN;
                rc = NC_EAGAIN;
            }
        }
    } /* older: its slot was reused, which delivered it first (ring_reap) */
    pthread_mutex_unlock(&r->lock);
    return rc;
}

extern "C" rstatus_t nc_gpuhash_ring_forget(nc_gpuhash_ring_t *r, int ticket)
{
    if (r == NULL || ticket < 0) {
        errno = EINVAL;
        return NC_ERROR;
    }
    pthread_mutex_lock(&r->lock);
    const uint64_t back = (r->seq - (uint64_t)ticket) & kTagMask;
    rstatus_t rc = NC_OK;
    if (back == 0 || back > r->seq - r->seq0) {
        errno = EINVAL;
        rc = NC_ERROR;
    } else if (back <= r->nslots) {
        const uint64_t seq = r->seq - back;
        const uint32_t s = (uint32_t)(seq % r->nslots);
        /* the batch still runs and its slot is reaped as usual; only the copy
         * into the caller's `out` is dropped */
        if (r->slot_seq[s] == seq && r->slot_state[s] == SLOT_RUNNING) r->slot_out[s] = NULL;
    } /* older: already delivered */
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
            if (t1.tv_sec - t0.tv_sec > 10) { /* a launch ends within 2 s; this is a dead device */
                errno = EIO;
                return NC_ERROR;
            }
            sched_yield();
        }
    }
}

extern "C" uint64_t nc_gpuhash_ring_launches(const nc_gpuhash_ring_t *r) { return r ? r->launches : 0; }

extern "C" rstatus_t nc_gpuhash_ring_debug_start_seq(nc_gpuhash_ring_t *r, uint64_t seq)
{
    if (r == NULL) {
        errno = EINVAL;
        return NC_ERROR;
    }
    pthread_mutex_lock(&r->lock);
    const int fresh = r->launches == 0 && r->seq == r->seq0;
    if (fresh) {
        r->seq = r->seq0 = seq;
        for (uint32_t g = 0; g < r->nlanes; g++) __atomic_store_n(&r->ctl[g].processed, lane_submitted(r, g), __ATOMIC_SEQ_CST);
    }
    pthread_mutex_unlock(&r->lock);
    if (!fresh) {
        errno = EBUSY;
        return NC_ERROR;
    }
    return NC_OK;
}

extern "C" rstatus_t nc_gpuhash_ring_debug_hold(nc_gpuhash_ring_t *r, int hold)
{
    if (r == NULL) {
        errno = EINVAL;
        return NC_ERROR;
    }
    pthread_mutex_lock(&r->lock);
    r->hold = hold != 0;
    pthread_mutex_unlock(&r->lock);
    return NC_OK;
}

extern "C" uint32_t nc_gpuhash_ring_lanes(const nc_gpuhash_ring_t *r) { return r ? r->nlanes : 0; }

extern "C" int nc_gpuhash_ring_debug_staging(const nc_gpuhash_ring_t *r) { return r ? (r->stage != NULL) : -1; }

extern "C" rstatus_t nc_gpuhash_ring_limits(const nc_gpuhash_ring_t *r, uint32_t *max_keys, uint64_t *max_key_bytes,
                                            uint32_t *nslots)
{
    if (r == NULL) {
        errno = EINVAL;
        return NC_ERROR;
    }
    if (max_keys) *max_keys = r->max_keys;
    if (max_key_bytes) *max_key_bytes = r->max_key_bytes;
    if (nslots) *nslots = r->nslots;
    return NC_OK;
}

extern "C" rstatus_t nc_gpuhash_ring_debug_timeline(nc_gpuhash_ring_t *r, int on, uint32_t slot, uint64_t out[8])
{
    if (r == NULL || (out != NULL && slot >= r->nslots)) {
        errno = EINVAL;
        return NC_ERROR;
    }
    pthread_mutex_lock(&r->lock);
    const int ok = on < 0 || r->launches == 0 || r->timeline == (on != 0);
    if (on >= 0 && ok) r->timeline = on != 0;
    if (out != NULL)
        for (int i = 0; i < 8; i++) out[i] = __atomic_load_n(&r->tl[8 * slot + i], __ATOMIC_ACQUIRE);
    pthread_mutex_unlock(&r->lock);
    if (!ok) {
        errno = EBUSY;
        return NC_ERROR;
    }
    return NC_OK;
}
