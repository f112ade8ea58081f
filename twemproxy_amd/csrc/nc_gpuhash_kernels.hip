/*
 * gfx950 (MI355X / CDNA4) batched key-hash kernels for the 12 twemproxy
 * hashkit modes, and the device-resident C-ABI launch layer.
 *
 * Data layout in HBM: a packed key byte stream plus a u64
 * offset CSR (key i = keys[off[i] .. off[i+1])) and a u32 output per key.
 *
 * Kernel structure (one template instance per mode, 256-thread workgroups):
 *   - a workgroup owns a TILE of 256 consecutive keys (one per lane) and walks
 *     tiles grid-stride;
 *   - the tile's key SLAB [off[k0], off[k0+256]) is staged HBM -> LDS with
 *     coalesced 16-byte loads (global_load_dwordx4 -> ds_write_b128), so HBM
 *     is read once, in 1 KiB wave-instructions, whatever the key lengths;
 *   - optionally the 256 keys are reordered inside the tile by length class
 *     (wave-ballot multisplit + LDS scan), so the four waves each hash keys of
 *     similar length: a wave runs as long as its longest key (Zipf lengths);
 *   - each lane then hashes its key serially from LDS through a realigning
 *     reader: 8-byte ds_read_b64 at 8-aligned addresses + v_alignbyte funnel
 *     shifts yield the key's little-endian words at any byte alignment;
 *   - tiles whose slab does not fit the LDS budget (very long keys) read the
 *     same realigned words straight from global memory instead.
 * No MFMA: there is no contraction here; the path is HBM- or VALU-bound.
 *
 * Reference semantics: /root/reference/src/hashkit (per-mode file:line in
 * nc_hash_algo.h).
 */
#include <hip/hip_runtime.h>

#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "nc_out_policy.h"
#include "nc_gpuhash.h"
#include "nc_gpuhash_probe.h"
#include "nc_hash_algo.h"
#include "nc_md5_steps.h"
#include "nc_lds_hash.h"

namespace {

constexpr int kBlock = 256;                  /* threads per workgroup = keys per tile */
constexpr int kTile = kBlock;
constexpr int kBuckets = 64;
constexpr uint32_t kLdsBudget = 20480;        /* 8 workgroups per CU (160 KiB LDS) */
constexpr uint32_t kRing = 8;                /* slab-bounds ring slots (tiles t .. t+5 in use) */
constexpr uint32_t kDumpBytes = 256;          /* landing area of the L2-prefetch DMA (never read) */
constexpr uint32_t kSmall = 4 * kTile + 2 * kTile + 8 * kBuckets + 16 + 4 * 256 + 16 * kRing + kDumpBytes;
constexpr uint32_t kSlabCap = ((kLdsBudget - kSmall) / 2) & ~15u; /* per slab buffer (double buffered) */
constexpr int kStageIters = (kSlabCap / 16 + kBlock - 1) / kBlock;

/* LDS carve (one __shared__ array, all offsets 16-byte aligned) */
constexpr uint32_t kOffSlab0 = 0;
constexpr uint32_t kOffSlab1 = kSlabCap;
constexpr uint32_t kOffKey = 2 * kSlabCap;                     /* u32[kTile] key start | length << 16 */
constexpr uint32_t kOffPerm = kOffKey + 4 * kTile;             /* u16[kTile] sorted -> tile index */
constexpr uint32_t kOffHist = kOffPerm + 2 * kTile;            /* u32[2][kBuckets] */
constexpr uint32_t kOffFlag = kOffHist + 8 * kBuckets;         /* u32[2] (+pad) */
constexpr uint32_t kOffTab = kOffFlag + 16;                    /* u32[256] crc table */
constexpr uint32_t kOffRing = kOffTab + 4 * 256;               /* u64[kRing][2] slab bounds {S, E} */
constexpr uint32_t kOffDump = kOffRing + 16 * kRing;           /* prefetch landing area */
constexpr uint32_t kSmemBytes = kOffDump + kDumpBytes;

static_assert(kSmemBytes <= kLdsBudget, "LDS budget");
static_assert(kSlabCap >= 8192 + 48, "a 256 x 32 B tile must fit one slab buffer");
static_assert(kSlabCap < 65536, "sorted key positions are packed in 16 bits");
static_assert(kOffTab % 16 == 0, "LDS carve must stay 16-byte aligned");

/* Length class used to group keys of similar cost into one wave. */
__device__ __forceinline__ uint32_t len_bucket(uint32_t len)
{
    return len < (uint32_t)(kBuckets - 1) ? len : (uint32_t)(kBuckets - 2);
}

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

/* LDS-only workgroup barrier: waits for this wave's LDS traffic, not for its
 * vector-memory (LDS-DMA) loads, so the next tile's slab stays in flight. */
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0) only (gfx9 encoding: vmcnt/expcnt fields saturated) */
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

/* vmcnt(0) + lgkmcnt(0) + barrier, through the builtin so the compiler's
 * waitcnt pass knows every earlier load has completed (an inline-asm wait is
 * opaque to it and it would add its own vmcnt(0) later, e.g. behind a store). */
__device__ __forceinline__ void full_barrier()
{
    __builtin_amdgcn_s_waitcnt(0x0070); /* vmcnt(0) expcnt(7) lgkmcnt(0) */
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

constexpr int kDistNone = -1, kDistKetama = 0, kDistModula = 1, kDistPre = 3, kDistKetamaLut = 4, kDistKetamaLds = 5,
              kDistKetamaLdsPacked = 6;

/* server_pool_idx parameters of one launch (ignored for kDistNone) */
struct WrDist {
    const uint32_t *cont; /* struct continuum {index, value} pairs (src/nc_server.h:64-67) */
    uint32_t ncont;
    uint32_t tag;         /* hash_tag c0 | c1 << 8 | 1 << 16, or 0 for none */
    const uint32_t *lut;  /* ketama lookup table by the hash's top 32 - lut_shift bits (kDistKetamaLut), or null */
    uint32_t lut_shift;   /* 20 (4096 entries, L1-resident) or 16 (65536) */
};

/* ketama_dispatch through a table over the hash's top bits
 * (nc_ketama_lut_kernel; 4096 entries = 16 KiB by default, which stays in
 * the CU's vector L1 beside the continuum): an entry without bit 31 is the
 * server of every hash in its range (no point falls inside the range), else
 * it names the first point >= the range start and the answer is the first
 * point >= h from there (src/hashkit/nc_ketama.c:222-246: the first value >=
 * hash, wrapping to the first point). For an 8 x 160-point pool ~73 % of keys
 * resolve with that one read, the rest read ~1.2 {index, value} pairs (one
 * 8-byte load each) — instead of a binary search of ~4 dependent reads. */
__device__ __forceinline__ uint32_t ketama_find_lut(const uint32_t *c, const uint32_t *lut, uint32_t shift,
                                                    uint32_t n, uint32_t h)
{
    const uint32_t e = lut[h >> shift];
    if ((e >> 31) == 0u) return e;
    uint32_t p = e & 0x7fffffffu;
    for (;;) {
        if (p >= n) return c[0]; /* past the last point: wrap */
        const uint2 iv = reinterpret_cast<const uint2 *>(c)[p];
        if (iv.y >= h) return iv.x;
        p++;
    }
}

/* hash_tag trimming of server_pool_idx (src/nc_server.c:665-677): the first
 * c0, then the first c1 after it; with at least one byte between them the
 * key becomes the bytes in between. Four bytes at a time: a byte equal to c
 * is a zero byte of w ^ c*0x01010101, found with the exact zero-byte test
 * ~(((x & 0x7f7f7f7f) + 0x7f7f7f7f) | x) & 0x80808080 (no carry leaves a
 * byte, so EVERY set bit is a zero byte), then v_ffbl. The cheaper
 * (x - 0x01010101) & ~x test is exact only in its lowest set bit: a borrow
 * out of a true zero flags a 0x01 byte above it, and c1 is searched after
 * masking off the bytes up to c0, where that lowest bit may be gone (tag
 * "::" on key ":;ab:"). */
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x)
{
    return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
}

template <class Src>
__device__ __forceinline__ void tag_trim(const Src &src, typename Src::pos_t &p, uint32_t &len, uint32_t c0,
                                         uint32_t c1)
{
    QStream<Src> st;
    st.init(src, p);
    const uint32_t p0 = c0 * 0x01010101u, p1 = c1 * 0x01010101u;
    uint32_t s = 0xffffffffu, e = 0xffffffffu;
    for (uint32_t i = 0; i < len; i += 8u) {
        const uint2 w2 = st.next8();
#pragma unroll
        for (uint32_t h = 0; h < 2u; h++) {
            const uint32_t w = h ? w2.y : w2.x;
            const uint32_t base = i + 4u * h;
            const uint32_t lim = len > base ? len - base : 0u; /* key bytes in this word */
            const uint32_t valid = lim >= 4u ? 0x80808080u : ((1u << (8u * lim)) - 1u) & 0x80808080u;
            const uint32_t m0 = zero_bytes(w ^ p0) & valid;
            uint32_t m1 = zero_bytes(w ^ p1) & valid;
            if (s == 0xffffffffu) {
                if (m0 != 0u) {
                    const uint32_t b0 = __builtin_ctz(m0); /* bit 7 of the first c0 byte */
                    s = base + (b0 >> 3);
                    m1 &= ~((2u << b0) - 1u); /* c1 strictly after it */
                } else {
                    m1 = 0u;
                }
            }
            if (e == 0xffffffffu && m1 != 0u) e = base + (__builtin_ctz(m1) >> 3);
        }
    }
    if (s != 0xffffffffu && e != 0xffffffffu && e - s > 1u) {
        p += s + 1u;
        len = e - s - 1u;
    }
}

/* ketama_dispatch (src/hashkit/nc_ketama.c:222-246): the first point whose
 * value is >= hash, wrapping to the first point; c = {index, value} pairs */
__device__ __forceinline__ uint32_t ketama_find(const uint32_t *c, uint32_t n, uint32_t h)
{
    uint32_t lo = 0, len = n;
    while (len > 0u) {
        const uint32_t half = len >> 1;
        if (c[2u * (lo + half) + 1u] < h) {
            lo += half + 1u;
            len -= half + 1u;
        } else {
            len = half;
        }
    }
    return c[2u * (lo == n ? 0u : lo)];
}

/* ketama_find narrowed by a 256-bucket index over the top hash byte:
 * bkt[b] = first point with value >= b << 24 (bkt[256] = n), so the answer
 * for h lies in [bkt[h >> 24], bkt[(h >> 24) + 1]] and the search takes
 * ~log2(n / 256) + 1 steps instead of log2(n) */
/* [lo, lo + cnt) of bucket b, both ends clamped to n: a bucket index built
 * over an unsorted continuum (a caller error) can hold a start past n or an
 * end below its start, and the search must still stay inside the continuum
 * and end (tests/test_gpu_zz_robustness.py) */
__device__ __forceinline__ uint32_t bucket_span(const uint32_t *bkt, uint32_t b, uint32_t n, uint32_t &lo)
{
    lo = min(bkt[b], n);
    const uint32_t end = b == 255u ? n : min(bkt[b + 1u], n);
    return end > lo ? end - lo : 0u;
}

__device__ __forceinline__ uint32_t ketama_find_bkt(const uint32_t *c, const uint32_t *bkt, uint32_t n, uint32_t h)
{
    const uint32_t b = h >> 24;
    uint32_t lo;
    uint32_t len = bucket_span(bkt, b, n, lo);
    while (len > 0u) {
        const uint32_t half = len >> 1;
        if (c[2u * (lo + half) + 1u] < h) {
            lo += half + 1u;
            len -= half + 1u;
        } else {
            len = half;
        }
    }
    return c[2u * (lo == n ? 0u : lo)];
}

/* ketama_dispatch over a continuum staged in LDS (the grouped pipeline):
 * vals[i] = point i's value, idx[i] = its server (nserver <= 256), bkt the
 * 256-entry bucket index; every read is an LDS read, where the global form
 * pays ~4 dependent L2 round trips behind the streaming key traffic */
__device__ __forceinline__ uint32_t ketama_find_lds(const uint32_t *vals, const uint8_t *idx, const uint32_t *bkt,
                                                    uint32_t n, uint32_t h)
{
    uint32_t lo;
    uint32_t cnt = bucket_span(bkt, h >> 24, n, lo);
    while (cnt > 0u) {
        const uint32_t half = cnt >> 1;
        if (vals[lo + half] < h) {
            lo += half + 1u;
            cnt -= half + 1u;
        } else {
            cnt = half;
        }
    }
    return idx[lo == n ? 0u : lo];
}

/* ketama_dispatch over a PACKED LDS continuum, one word per point: the
 * value's top 24 bits over the server index (w = v & ~255 | server, pools of
 * <= 256 servers), followed by eight sentinels 0xffffff00 | point 0's server
 * (never below a hash's top 24 bits, so a search stops at them without bounds
 * checks, and a lane that stops on one reads the wrap's answer from it). 4
 * bytes a point keep a 1280-point pool inside the grouped pipeline's four
 * workgroups per CU. A 512-entry u16 bucket index over the hash's top 9 bits
 * (~2.5 points a bucket) gives the start; from it rounded down to a multiple
 * of four, the aligned quad (one ds_read_b128) holds the first word >= hb =
 * h & ~255 unless its last word is below hb, and then the next quads do (the
 * words before the bucket start are below hb: they are below the bucket's
 * first value). Within the quad two compares on the sorted words (pair, word)
 * pick it. The search is bound by LDS bank conflicts, not by ALU: the
 * four-word scan from the unaligned bucket start (rounds 3-4: two
 * ds_read2_b32 a round, two rounds in most waves) cost C2 0.509-0.512 ms,
 * eight words in two ds_read_b128 0.470-0.475, the quad first 0.467-0.468
 * (profiles/r05_sidx_s8_ab.jsonl, r05_sidx_quad_ab.jsonl). Only when the
 * found word shares h's top 24 bits is the answer ambiguous (about one key in
 * 13000 for 1280 points, or h >= 0xffffff00 against a sentinel): that lane
 * finds the word's index and walks the run of such points comparing full
 * values from the continuum in global memory (cont: {server, value} pairs);
 * past the last point the answer wraps to point 0 (w0). */
__device__ __forceinline__ uint32_t ketama_find_lds_packed(const uint32_t *w, const uint16_t *bkt16,
                                                           const uint32_t *cont, uint32_t n, uint32_t w0, uint32_t h)
{
    using u32x4 = uint32_t __attribute__((ext_vector_type(4)));
    const uint32_t hb = h & ~0xffu; /* w >> 8 < h >> 8  <=>  w < hb */
    const u32x4 *q = reinterpret_cast<const u32x4 *>(__builtin_assume_aligned(w, 16));
    /* clamped: an unsorted continuum (a caller error) could leave a bucket
     * unwritten; from at most n the search still ends at the sentinels (it
     * goes on only while a quad's last word is below hb, so it never reads
     * past word n + 3) */
    uint32_t lo = min((uint32_t)bkt16[h >> 23], n) & ~3u;
    u32x4 a = q[lo >> 2];
    if (a.w < hb) { /* the quad's four words all below h: the next ones */
        do {
            lo += 4u;
            a = q[lo >> 2];
        } while (a.w < hb);
    }
    const bool p2 = a.y < hb;
    const uint32_t e0 = p2 ? a.z : a.x, e1 = p2 ? a.w : a.y;
    uint32_t cand = e0 < hb ? e1 : e0;
    if ((cand ^ hb) < 0x100u) { /* rare, the same top 24 bits: full values decide */
        /* from the bucket start again (re-read: keeping lo live past the
         * search loop makes hipcc carry derived addresses through it) */
        uint32_t pos = min((uint32_t)bkt16[h >> 23], n) & ~3u;
        while (w[pos] < hb) pos++;
        while (pos < n && (w[pos] ^ hb) < 0x100u && cont[2u * pos + 1u] < h) pos++;
        cand = pos < n ? w[pos] : w0;
    }
    return cand & 0xffu;
}

/* lower bound of v over the continuum values (no wrap) */
__device__ __forceinline__ uint32_t cont_lower_bound(const uint32_t *c, uint32_t n, uint32_t v)
{
    uint32_t lo = 0, len = n;
    while (len > 0u) {
        const uint32_t half = len >> 1;
        if (c[2u * (lo + half) + 1u] < v) {
            lo += half + 1u;
            len -= half + 1u;
        } else {
            len = half;
        }
    }
    return lo;
}

/* server_pool_idx on the workgroup pipeline (VAR bits 12-13: 1 ketama, 2
 * modula): hash_tag trim, hash 0 for an empty key (src/nc_server.c:639-641),
 * then the dispatch over the continuum in global memory (L2-resident: 8 B
 * per point); ketama narrows its binary search with the 256-entry bucket
 * index bkt (LDS): the answer for h lies in [bkt[h >> 24], bkt[(h >> 24) + 1]]
 * (bkt[256] = n is implicit). */
template <int VAR>
constexpr int wg_dist()
{
    return ((VAR >> 12) & 7) == 1   ? kDistKetama
           : ((VAR >> 12) & 7) == 2 ? kDistModula
           : ((VAR >> 12) & 7) == 3 ? kDistKetamaLut
           : ((VAR >> 12) & 7) == 4 ? kDistKetamaLds
           : ((VAR >> 12) & 7) == 5 ? kDistKetamaLdsPacked
                                    : kDistNone;
}

template <int MODE, int VAR, class Src>
__device__ __forceinline__ uint32_t wg_value(const Src &src, typename Src::pos_t p, uint32_t len,
                                             const uint32_t *tab, const uint32_t *bkt, const WrDist &dist)
{
    constexpr int D = wg_dist<VAR>();
    if constexpr (D == kDistNone) {
        return hash_key<MODE, VAR>(src, p, len, tab);
    } else {
        if constexpr ((VAR & 256) == 0) { /* VAR bit 8: DIAGNOSTIC, no hash_tag code */
            if (dist.tag != 0u) tag_trim(src, p, len, dist.tag & 0xffu, (dist.tag >> 8) & 0xffu);
        }
        uint32_t h = 0u;
        if (len != 0u) h = hash_key<MODE, VAR>(src, p, len, tab);
        const uint32_t *c = dist.cont;
        const uint32_t n = dist.ncont;
        if constexpr (D == kDistKetamaLds || D == kDistKetamaLdsPacked) {
            return h; /* the caller searches its LDS continuum (ketama_find_lds[_packed]) */
        } else if constexpr (D == kDistModula) {
            return c[2u * (h % n)]; /* nc_modula.c:153 */
        } else if constexpr (D == kDistKetamaLut) {
            return ketama_find_lut(c, dist.lut, dist.lut_shift, n, h);
        } else { /* ketama_dispatch, nc_ketama.c:222-246 */
            uint32_t lo;
            uint32_t cnt = bucket_span(bkt, h >> 24, n, lo);
            while (cnt > 0u) {
                const uint32_t half = cnt >> 1;
                if (c[2u * (lo + half) + 1u] < h) {
                    lo += half + 1u;
                    cnt -= half + 1u;
                } else {
                    cnt = half;
                }
            }
            return c[2u * (lo == n ? 0u : lo)];
        }
    }
}

/* This lane's key [s, e) of a tile, loaded one tile ahead of its use: only
 * the LOW dwords of the u64 offsets, since every use is 32-bit (the length,
 * and the start relative to a slab base < 4 GiB away). Loads are clamped so
 * every lane issues them (a fixed per-wave instruction count). */
struct TileOffs {
    uint32_t s, e;
};

template <bool NT = false>
__device__ __forceinline__ TileOffs load_offs(const uint64_t *__restrict__ off, uint64_t tile, uint64_t nkeys,
                                              uint32_t t)
{
    uint64_t k = tile * (uint64_t)kTile + t;
    uint64_t k1 = k + 1;
    if (k > nkeys) k = nkeys;
    if (k1 > nkeys) k1 = nkeys;
    const uint32_t *o32 = reinterpret_cast<const uint32_t *>(off); /* little-endian: low dword first */
    TileOffs o;
    if constexpr (NT) { /* read-once stream: non-temporal */
        o.s = __builtin_nontemporal_load(o32 + 2 * k);
        o.e = __builtin_nontemporal_load(o32 + 2 * k1);
    } else {
        o.s = o32[2 * k];
        o.e = o32[2 * k1];
    }
    return o;
}

__device__ __forceinline__ uint32_t tile_count(uint64_t tile, uint64_t nkeys)
{
    const uint64_t left = nkeys - tile * (uint64_t)kTile;
    return left < (uint64_t)kTile ? (uint32_t)left : (uint32_t)kTile;
}

/* Slab bounds {off[k0], off[k0 + cnt]} of a tile, DMA'd into a ring slot by
 * lanes 0-3 of every wave (four dwords; identical values from every wave).
 * LDS-DMA keeps them out of VGPRs and out of lgkmcnt: nothing in the hash
 * loop ever waits for them. Exactly one VMEM instruction per wave. */
template <int AUX = 0>
__device__ __forceinline__ void issue_bounds(const uint64_t *__restrict__ off, uint64_t tile, uint64_t nkeys,
                                             uint8_t *slot, uint32_t lane)
{
    const uint64_t k0 = tile * (uint64_t)kTile;
    const uint64_t k = k0 + (lane >= 2u ? tile_count(tile, nkeys) : 0u);
    if (lane < 4u) {
        __builtin_amdgcn_global_load_lds((gbl_void_t *)(reinterpret_cast<const uint32_t *>(off + k) + (lane & 1u)),
                                         (lds_void_t *)slot, 4, 0, AUX);
    }
}

/* staged bytes = span rounded up to 16 + 2 look-ahead pieces (the reader
 * touches up to 18 bytes past a key) */
__device__ __forceinline__ bool fits_lds(uint64_t span) { return span + 48u <= (uint64_t)kSlabCap; }

/* Issue the LDS-DMA copy of a slab: 16-byte pieces, one 1 KiB wave-instruction
 * per 64 pieces, landing contiguously at buf (wave-uniform base + lane*16). */
/* AUX: cache-policy bits of the DMA (2 = nt, for the read-once key stream) */
template <int AUX = 0>
__device__ __forceinline__ void issue_slab(const uint8_t *keys_base, uint64_t S16, uint64_t span, uint8_t *buf,
                                           uint32_t t)
{
    const uint32_t nch = (uint32_t)((span + 15u) >> 4) + 2u; /* +2 pieces: reader look-ahead */
    const uint32_t wbase = t & ~63u;
#pragma unroll
    for (int i = 0; i < kStageIters; i++) {
        const uint32_t c = t + (uint32_t)i * kBlock;
        if (wbase + (uint32_t)i * kBlock < nch && c < nch) {
            __builtin_amdgcn_global_load_lds((gbl_void_t *)(keys_base + S16 + 16u * c),
                                             (lds_void_t *)(buf + 16u * (wbase + (uint32_t)i * kBlock)), 16, 0, AUX);
        }
    }
}

/* L2 prefetch of a tile PD tiles ahead (PD = 2..4): one dword per 64-byte
 * sector, DMA'd into a dump area nobody reads. Lanes 0..223 touch the slab
 * (14 KiB), lanes 224..255 the tile's 2 KiB of offsets. It moves that tile's
 * HBM latency off the critical path without spending LDS or VGPRs on
 * buffering: the real staging DMA and offset loads later hit L2. Exactly one
 * VMEM instruction per wave; addresses clamped into the slab / offsets. */
constexpr uint32_t kPfSlabLanes = 224;

__device__ __forceinline__ void issue_prefetch(const uint8_t *keys_base, uint64_t S16, uint64_t span,
                                               const uint64_t *off, uint64_t tile, uint64_t nkeys, uint8_t *dump,
                                               uint32_t t)
{
    const uint8_t *p;
    if (t < kPfSlabLanes) {
        uint64_t o = 64u * (uint64_t)t;
        if (o >= span) o = span > 4u ? ((span - 4u) & ~(uint64_t)3) : 0u;
        p = keys_base + S16 + o;
    } else {
        uint64_t k = tile * (uint64_t)kTile + 8u * (t - kPfSlabLanes); /* 8 offsets per 64-byte sector */
        if (k > nkeys) k = nkeys;
        p = reinterpret_cast<const uint8_t *>(off + k);
    }
    __builtin_amdgcn_global_load_lds((gbl_void_t *)p, (lds_void_t *)dump, 4, 0, 0);
}

__device__ __forceinline__ void read_bounds(const uint8_t *slot, uint64_t delta, uint64_t &S16, uint64_t &span)
{
    const uint64_t *b = reinterpret_cast<const uint64_t *>(slot);
    const uint64_t S = b[0] + delta, E = b[1] + delta;
    S16 = S & ~(uint64_t)15;
    span = E - S16;
}

/*
 * Persistent workgroups walk 256-key tiles grid-stride (tile t below means
 * this workgroup's t-th tile). Iteration t:
 *   top   : counted s_waitcnt + barrier — slab(t), offsets(t) and the bounds
 *           ring are in; only the previous iteration's L2 prefetch (PF) may
 *           still be in flight;
 *   issue : store of tile t-1's hashes (late, so it drains under this tile),
 *           bounds(t+3) -> ring, LDS-DMA of slab(t+1) into the other buffer,
 *           offsets(t+1), L2 prefetch of slab(t+2) (PF);
 *   work  : optional length sort, hash every key from LDS (or from global
 *           memory when the slab exceeds the LDS budget).
 * keys_base is 16-byte aligned; key i is keys_base[off[i]+delta, off[i+1]+delta)
 * and keys_base stays readable NC_GPUHASH_PAD bytes past the last key.
 */
/* minimum waves per SIMD (1: no register cap). Capping md5 at 64 VGPRs for
 * eight waves per SIMD spilled to scratch and ran 8 % slower on C3. */
template <int MODE>
constexpr int kMinWaves()
{
    return 1;
}

template <int MODE, bool SORT, int VAR>
__global__ __launch_bounds__(kBlock, kMinWaves<MODE>()) void nc_hash_kernel(const uint8_t *__restrict__ keys_base,
                                                         const uint64_t *__restrict__ off, uint64_t delta,
                                                         uint64_t nkeys, uint32_t *__restrict__ out,
                                                         uint64_t ntiles, WrDist dist)
{
    /* VAR bits 1-2: L2-prefetch distance code (0 off, 1..3 -> 2..4 tiles ahead) */
    constexpr uint32_t PD = ((VAR >> 1) & 3) ? (uint32_t)((VAR >> 1) & 3) + 1u : 0u;
    constexpr bool PF = PD != 0;
    constexpr bool kNT = (VAR & 64) == 0;      /* read-once streams are non-temporal; variant bit 6
                                                  selects the default cache policy (A/B only) */
    constexpr int kAux = kNT ? 2 : 0;          /* global_load_lds cache-policy bits: 2 = nt */
    /* bounds are DMA'd DB tiles ahead: slab issue needs t+1, prefetch t+PD,
     * and both must be older than the previous iteration's prefetch */
    constexpr uint32_t DB = PD + 1u > 3u ? PD + 1u : 3u;
    static_assert(DB + 1u <= kRing, "bounds ring too small");
    __shared__ __attribute__((aligned(16))) uint8_t smem[kSmemBytes];
    uint32_t *kpos = reinterpret_cast<uint32_t *>(smem + kOffKey);
    uint16_t *perm = reinterpret_cast<uint16_t *>(smem + kOffPerm);
    uint32_t *hist2 = reinterpret_cast<uint32_t *>(smem + kOffHist); /* [2][kBuckets], by iteration parity */
    uint32_t *flag2 = reinterpret_cast<uint32_t *>(smem + kOffFlag); /* [2] */
    uint32_t *tab = reinterpret_cast<uint32_t *>(smem + kOffTab);
    uint8_t *ring = smem + kOffRing;
    uint8_t *dump = smem + kOffDump;

    const uint32_t t = threadIdx.x;
    const uint32_t lane = t & 63u;
    const uint64_t stride = gridDim.x;
    uint64_t tile = blockIdx.x;
    if (tile >= ntiles) return;
    auto tile_at = [&](uint64_t j) -> uint64_t { /* j-th tile of this workgroup, clamped */
        const uint64_t x = tile + j * stride;
        return x < ntiles ? x : tile;
    };

    if constexpr (uses_crc_table<MODE>()) {
        static_assert(!uses_crc_table<MODE>() || wg_dist<VAR>() == kDistNone, "crc modes dispatch on the wave ring");
        tab[t] = (MODE == NC_GPUHASH_CRC16) ? nc_crc16_entry(t) : nc_crc32_entry(t);
    }
    if constexpr (wg_dist<VAR>() == kDistKetama) { /* the bucket index, in the crc table's place */
        tab[t] = cont_lower_bound(dist.cont, dist.ncont, t << 24);
    }
    if constexpr (SORT) {
        if (t < 2u * kBuckets) hist2[t] = 0;
        if (t < 2u) flag2[t] = 0;
    }

    /* prologue: bounds of tiles 0..DB-1 into ring slots 0..DB-1 */
#pragma unroll
    for (uint32_t j = 0; j < DB; j++) issue_bounds<kAux>(off, tile_at(j), nkeys, ring + j * 16, lane);
    full_barrier();
    uint64_t S16, span;
    read_bounds(ring, delta, S16, span);
    uint32_t cnt = tile_count(tile, nkeys);
    if (fits_lds(span)) issue_slab<kAux>(keys_base, S16, span, smem + kOffSlab0, t);
    asm volatile("" ::: "memory");
    TileOffs cur = load_offs<kNT>(off, tile, nkeys, t);
    if constexpr (PF) {
#pragma unroll
        for (uint32_t j = 1; j < PD; j++) {
            uint64_t pS, pspan;
            read_bounds(ring + j * 16, delta, pS, pspan);
            issue_prefetch(keys_base, pS, pspan, off, tile_at(j), nkeys, dump, t);
        }
    }
    uint64_t pend_idx = ~0ull;
    uint32_t pend_h = 0;

    /* one tile; `cur` holds its offsets, `nn` receives the next tile's */
    auto step = [&](TileOffs &cur, TileOffs &nn, uint32_t it) __attribute__((always_inline)) {
        uint8_t *slab = smem + ((it & 1u) ? kOffSlab1 : kOffSlab0);
        uint8_t *slab_next = smem + ((it & 1u) ? kOffSlab0 : kOffSlab1);
        const bool in_lds = fits_lds(span);
        const uint64_t myS16 = S16;
        const uint32_t mycnt = cnt;
        const uint64_t k0 = tile * (uint64_t)kTile;

        /* Everything but the youngest VMEM instruction of the previous
         * iteration (its L2 prefetch) must have landed. */
        if constexpr (PF) {
            __builtin_amdgcn_s_waitcnt(0x0071); /* vmcnt(1) expcnt(7) lgkmcnt(0) */
            asm volatile("" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        } else {
            full_barrier();
        }
        if (pend_idx != ~0ull) {
            if constexpr (kNT) out_st32(out + pend_idx, pend_h);
            else out[pend_idx] = pend_h;
        }
        pend_idx = ~0ull;
        asm volatile("" ::: "memory");

        const uint64_t t1 = tile + stride;
        issue_bounds<kAux>(off, tile_at(DB), nkeys, ring + ((it + DB) % kRing) * 16, lane);
        asm volatile("" ::: "memory");
        if (t1 < ntiles) {
            read_bounds(ring + ((it + 1u) % kRing) * 16, delta, S16, span);
            cnt = tile_count(t1, nkeys);
            if (fits_lds(span)) issue_slab<kAux>(keys_base, S16, span, slab_next, t);
        }
        asm volatile("" ::: "memory");
        if constexpr ((VAR & 16) != 0) {
            /* DIAGNOSTIC ONLY: C3's arithmetic layout (32-byte keys) instead of
             * loading offsets -- isolates the cost of the offsets path */
            const uint64_t kk = (t1 < ntiles ? t1 : tile) * (uint64_t)kTile + t;
            nn.s = (uint32_t)(kk * 32u);
            nn.e = (uint32_t)(kk * 32u + 32u);
        } else {
            nn = load_offs<kNT>(off, t1 < ntiles ? t1 : tile, nkeys, t);
        }
        if constexpr (PF) {
            asm volatile("" ::: "memory");
            uint64_t pS, pspan;
            read_bounds(ring + ((it + PD) % kRing) * 16, delta, pS, pspan);
            issue_prefetch(keys_base, pS, pspan, off, tile_at(PD), nkeys, dump, t);
        }

        const bool valid = t < mycnt;
        const uint32_t len = valid ? cur.e - cur.s : 0u;
        const uint32_t rel = cur.s + (uint32_t)delta - (uint32_t)myS16;

        uint32_t my = t;
        bool sorted = false;
        if constexpr (SORT) {
            /* Group the tile's keys by length so each wave hashes keys of one
             * cost: skipped (one extra barrier) when no wave mixes lengths,
             * and for tiles too long for LDS (start and length must fit 16 bits). */
            uint32_t *hist = hist2 + (it & 1u) * kBuckets;
            const uint32_t bucket = valid ? len_bucket(len) : (uint32_t)(kBuckets - 1);
            const uint32_t b0 = __shfl(bucket, 0);
            if (in_lds && __ballot(bucket != b0) != 0ull && lane == 0) flag2[it & 1u] = 1u;
            /* the other parity's state was last read before this tile's top
             * barrier: clear it for the next tile */
            if (t < (uint32_t)kBuckets) hist2[((it + 1u) & 1u) * kBuckets + t] = 0;
            if (t == 0) flag2[(it + 1u) & 1u] = 0;
            lds_barrier();
            if (flag2[it & 1u] != 0u) {
                sorted = true;
                kpos[t] = rel | (len << 16);
                const uint32_t rank = atomicAdd(&hist[bucket], 1u);
                lds_barrier();
                if (t < 64u) {
                    const uint32_t c = hist[t];
                    uint32_t x = c;
#pragma unroll
                    for (int d = 1; d < 64; d <<= 1) {
                        const uint32_t y = __shfl_up(x, d);
                        if (lane >= (uint32_t)d) x += y;
                    }
                    hist[t] = x - c;
                }
                lds_barrier();
                perm[hist[bucket] + rank] = (uint16_t)t;
                lds_barrier();
                my = perm[t];
            }
        }

        if (my < mycnt) {
            uint32_t klen_my = len;
            uint32_t pos = rel;
            if (sorted) {
                const uint32_t kp = kpos[my];
                pos = kp & 0xffffu;
                klen_my = kp >> 16;
            }
            uint32_t h;
            if constexpr ((VAR & 8) != 0) {
                /* DIAGNOSTIC ONLY (never the default): staging, offsets and
                 * stores as usual, no key reads and no hashing -- the
                 * memory-pipeline ceiling of this kernel structure */
                h = pos ^ klen_my;
            } else if (in_lds) {
                LdsSrc src{reinterpret_cast<const uint32_t *>(slab)};
                h = wg_value<MODE, VAR>(src, pos, klen_my, tab, tab, dist);
            } else {
                GlobalSrc src{reinterpret_cast<const uint32_t *>(keys_base)};
                h = wg_value<MODE, VAR>(src, myS16 + pos, klen_my, tab, tab, dist);
                /* retire the reader's look-ahead load here, so no register
                 * write is left pending where the two paths merge (the
                 * compiler would otherwise wait vmcnt(0) after the merge,
                 * i.e. on the L2 prefetch too) */
                __builtin_amdgcn_s_waitcnt(0x0070);
            }
            pend_idx = k0 + my;
            pend_h = h;
        }
    };
    /* Unrolled by two with the offset registers swapping roles, so a loaded
     * register is never copied at the back-edge (a copy would make the
     * compiler wait vmcnt(0) there — on the L2 prefetch as well). */
    TileOffs other;
    for (uint32_t it = 0;;) {
        if (tile >= ntiles) break;
        step(cur, other, it++);
        tile += stride;
        if (tile >= ntiles) break;
        step(other, cur, it++);
        tile += stride;
    }
    if (pend_idx != ~0ull) out[pend_idx] = pend_h;
}

typedef __attribute__((address_space(3))) const void lds_cvoid_t;

__device__ __forceinline__ uint32_t lds_addr(const void *p)
{
    return (uint32_t)(uintptr_t)(lds_cvoid_t *)p;
}

/* ---------------- grouped workgroup pipeline (variant bit 25) ----------------
 *
 * The workgroup pipeline's tiles (TK keys, TK/64 waves, LDS-DMA slabs, one
 * barrier per tile), with each WAVE hashing one length group of the tile
 * (its 64 keys of one rank range) instead of 64 neighbouring keys: a wave
 * runs as long as its longest key, so under Zipf 8-64 B unsorted waves cost
 * ~61 byte steps each, length-grouped ones ~110 per 256 keys in all (TK =
 * 256, four quartiles) or ~92 (TK = 512, eight octiles). The grouping costs
 * no barrier: a tile's offsets arrive by LDS-DMA D tiles ahead (the whole
 * workgroup sees them after a top barrier), and wave 0 — which hashes the
 * shortest group — counting-sorts tile t+1 while the others hash tile t,
 * leaving the permutation in LDS for the next iteration. Offsets are read
 * from HBM once, the low dword of each (lengths and slab positions are
 * 32-bit; the tile bounds' high dwords come separately).
 *
 * D = 2: slab(t+1) in flight while tile t hashes (the top barrier waits for
 * everything). D = 3: slabs t+1 and t+2 in flight: every wave issues exactly
 * kSlabIters slab DMAs per tile (dummies where a slab needs fewer), so the
 * top barrier waits with a counted vmcnt that leaves the youngest slab in
 * flight. Every LDS access hipcc could hold behind an in-flight LDS-DMA (a
 * write, or a read it cannot prove disjoint) is inline asm. CS: a tile's
 * hashes go to LDS by key index and out as 16-byte-per-lane stores.
 *
 * Iteration t (after the top barrier: slab(t), offsets(t+1 .. t+D-1) and
 * perm(t) in LDS): pending stores of tile t-1; DMA offsets(t+D) and
 * slab(t+D-1); wave 0 sorts tile t+1; every wave hashes its group of tile t. */
template <int D, bool CS, int TK, int RSV = 0>
struct GsLds {
    static_assert(D == 2 || D == 3, "two or three slab buffers");
    static_assert(TK == 256 || TK == 512, "four or eight waves");
    static constexpr uint32_t kOffSlot = 4u * TK + 16u; /* u32 lo[TK], then end lo / hi and start hi */
    static constexpr uint32_t kNOff = D + 1;             /* offsets of tiles t .. t+D */
    static constexpr uint32_t kPermBytes = 2u * 2u * TK; /* u16[2][TK]: sorted position -> key index */
    static constexpr uint32_t kResBytes = CS ? 2u * 4u * TK : 0u; /* u32[2][TK]: hashes by key index */
    static constexpr uint32_t kFixed = kNOff * kOffSlot + kPermBytes + 4 * 64 + 4 * 256 + 16 + kResBytes;
    /* 8 / 7 workgroups of four waves per CU; 4 of eight (1024-key tiles of
     * sixteen waves, two per CU, measured 40 % slower) */
    /* RSV: bytes left to dynamic LDS (a packed ketama continuum) within the
     * same per-workgroup budget */
    static constexpr uint32_t kBudget = (TK == 512 ? 40960 : (D == 2 ? 20480 : 23392)) - RSV;
    static constexpr uint32_t kCap = ((kBudget - kFixed) / D) & ~15u;
    static constexpr uint32_t kOffs = D * kCap;
    static constexpr uint32_t kPerm = kOffs + kNOff * kOffSlot;
    static constexpr uint32_t kHist = kPerm + kPermBytes;       /* u32[64], the sorter's counters */
    static constexpr uint32_t kTab = kHist + 4 * 64;            /* u32[256]: crc table / ketama bucket index */
    static constexpr uint32_t kDump = kTab + 4 * 256;           /* landing area of dummy DMAs */
    static constexpr uint32_t kRes = kDump + 16;
    static constexpr uint32_t kBytes = kRes + kResBytes;
    static constexpr int kSlabIters = (int)((kCap / 16 + TK - 1) / TK);
    static_assert(kBytes <= kBudget, "LDS budget");
    static_assert(kOffs % 16 == 0 && kTab % 16 == 0 && kCap % 16 == 0 && kRes % 16 == 0,
                  "LDS carve must stay 16-byte aligned");
};

template <int TK>
__device__ __forceinline__ uint32_t gs_tile_count(uint64_t tile, uint64_t nkeys)
{
    const uint64_t left = nkeys - tile * (uint64_t)TK;
    return left < (uint64_t)TK ? (uint32_t)left : (uint32_t)TK;
}

/* low dwords of off[k0 .. k0+TK-1] (clamped at nkeys) into slot, one 4-byte
 * DMA per lane; wave 0 adds the end bound off[k0+cnt] (low, high) and the
 * start's high dword at [TK .. TK+2] */
template <int AUX, int TK>
__device__ __forceinline__ void gs_issue_offs(const uint64_t *__restrict__ off, uint64_t tile, uint64_t nkeys,
                                              uint8_t *slot, uint32_t t)
{
    const uint64_t k0 = tile * (uint64_t)TK;
    uint64_t k = k0 + t;
    if (k > nkeys) k = nkeys;
    const uint32_t *o32 = reinterpret_cast<const uint32_t *>(off);
    __builtin_amdgcn_global_load_lds((gbl_void_t *)(o32 + 2u * k), (lds_void_t *)(slot + 4u * (t & ~63u)), 4, 0, AUX);
    if (t < 3u) {
        const uint64_t e = k0 + gs_tile_count<TK>(tile, nkeys);
        const uint32_t *src = t == 0u ? o32 + 2u * e : t == 1u ? o32 + 2u * e + 1u : o32 + 2u * k0 + 1u;
        __builtin_amdgcn_global_load_lds((gbl_void_t *)src, (lds_void_t *)(slot + 4u * TK), 4, 0, AUX);
    }
}

typedef unsigned int gs_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t gs_lo(const uint8_t *slot, uint32_t i)
{
    return reinterpret_cast<const uint32_t *>(slot)[i];
}

/* LDS ops of the sorter as inline asm: hipcc would wait vmcnt(0) before an
 * LDS write while an LDS-DMA is in flight; a wave's LDS operations complete
 * in order, and results are tied to an explicit lgkmcnt wait */
__device__ __forceinline__ void gs_ds_write_b32(uint32_t a, uint32_t v)
{
    asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void gs_ds_write_b16(uint32_t a, uint32_t v)
{
    asm volatile("ds_write_b16 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ uint32_t gs_ds_add_rtn(uint32_t a, uint32_t v)
{
    uint32_t r;
    asm volatile("ds_add_rtn_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(v) : "memory");
    return r;
}
__device__ __forceinline__ uint32_t gs_ds_read_b32(uint32_t a)
{
    uint32_t r;
    asm volatile("ds_read_b32 %0, %1" : "=v"(r) : "v"(a) : "memory");
    return r;
}

/* counting sort of the tile in `slot` by length class (one wave, KPL = TK/64
 * keys per lane): perm[pos] = key index (u16), ascending classes; absent
 * keys (>= cnt) last (class 63; valid keys clamp to 62). hist / perm are
 * LDS byte addresses. */
template <int TK>
__device__ __forceinline__ void gs_sort(const uint8_t *slot, uint32_t cnt, uint32_t hist, uint32_t perm, uint32_t lane)
{
    constexpr int KPL = TK / 64;
    gs_ds_write_b32(hist + 4u * lane, 0u);
    const uint32_t sa = lds_addr(slot) + 4u * KPL * lane;
    uint32_t st[KPL + 1];
#pragma unroll
    for (int q = 0; q <= KPL; q++) st[q] = gs_ds_read_b32(sa + 4u * (uint32_t)q); /* [TK] is lane 63's end bound */
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int q = 0; q <= KPL; q++) asm volatile("" : "+v"(st[q]));
    uint32_t cls[KPL], rk[KPL];
#pragma unroll
    for (int q = 0; q < KPL; q++) {
        const uint32_t i = (uint32_t)KPL * lane + (uint32_t)q;
        const uint32_t len = st[q + 1] - st[q];
        cls[q] = i < cnt ? (len < 62u ? len : 62u) : 63u;
        rk[q] = gs_ds_add_rtn(hist + 4u * cls[q], 1u);
    }
    uint32_t c = gs_ds_read_b32(hist + 4u * lane);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int q = 0; q < KPL; q++) asm volatile("" : "+v"(rk[q]));
    asm volatile("" : "+v"(c));
    uint32_t incl = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t v = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += v;
    }
    gs_ds_write_b32(hist + 4u * lane, incl - c);
    uint32_t b[KPL];
#pragma unroll
    for (int q = 0; q < KPL; q++) b[q] = gs_ds_read_b32(hist + 4u * cls[q]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int q = 0; q < KPL; q++) asm volatile("" : "+v"(b[q]));
#pragma unroll
    for (int q = 0; q < KPL; q++) gs_ds_write_b16(perm + 2u * (b[q] + rk[q]), (uint32_t)KPL * lane + (uint32_t)q);
}

template <int MODE, int VAR, int D, bool CS, int TK, int RSV>
__device__ __forceinline__ void gs_body(const uint8_t *__restrict__ keys_base, const uint64_t *__restrict__ off,
                                        uint64_t delta, uint64_t nkeys, uint32_t *__restrict__ out, uint64_t ntiles,
                                        const WrDist &dist)
{
    using G = GsLds<D, CS, TK, RSV>;
    constexpr int kAux = 2; /* nt: read-once streams */
    __shared__ __attribute__((aligned(16))) uint8_t smem[G::kBytes];
    /* kDistKetamaLds: the continuum's values (u32[ncont]) then servers
     * (u8[ncont]), in dynamic LDS after smem */
    extern __shared__ __attribute__((aligned(16))) uint32_t gs_cont[];
    const uint16_t *perm2 = reinterpret_cast<const uint16_t *>(smem + G::kPerm);
    uint32_t *tab = reinterpret_cast<uint32_t *>(smem + G::kTab);
    const uint32_t lds_base = lds_addr(smem);

    const uint32_t t = threadIdx.x;
    const uint32_t lane = t & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(t >> 6);
    const uint64_t stride = gridDim.x;
    uint64_t tile = blockIdx.x;
    if (tile >= ntiles) return;
    auto tile_at = [&](uint64_t j) -> uint64_t { /* j-th tile from here, clamped */
        const uint64_t x = tile + j * stride;
        return x < ntiles ? x : tile;
    };
    auto offs_slot = [&](uint32_t it) __attribute__((always_inline)) {
        return smem + G::kOffs + (it % G::kNOff) * G::kOffSlot;
    };
    auto slab_buf = [&](uint32_t it) __attribute__((always_inline)) { return smem + (it % (uint32_t)D) * G::kCap; };
    /* the slab of the tile whose offsets are in `slot`: its 16-aligned start
     * and span (inline-asm reads: hipcc would hold a plain LDS read of a slot
     * behind the slab DMA in flight, vmcnt(0), not knowing the two are
     * disjoint) */
    auto bounds = [&](const uint8_t *slot, uint64_t &S16, uint64_t &span) __attribute__((always_inline)) {
        const uint32_t a = lds_addr(slot);
        uint32_t s_lo = gs_ds_read_b32(a), e_lo = gs_ds_read_b32(a + 4u * TK);
        uint32_t e_hi = gs_ds_read_b32(a + 4u * TK + 4u), s_hi = gs_ds_read_b32(a + 4u * TK + 8u);
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(s_lo), "+v"(e_lo), "+v"(e_hi), "+v"(s_hi)::"memory");
        const uint64_t S = (((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(s_hi) << 32) |
                            (uint32_t)__builtin_amdgcn_readfirstlane(s_lo)) + delta;
        const uint64_t E = (((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(e_hi) << 32) |
                            (uint32_t)__builtin_amdgcn_readfirstlane(e_lo)) + delta;
        S16 = S & ~(uint64_t)15;
        span = E - S16;
    };
    auto fits = [&](uint64_t span) __attribute__((always_inline)) { return span + 48u <= (uint64_t)G::kCap; };
    /* slab DMA of one tile: D = 2 as many instructions as its span needs;
     * D = 3 exactly kSlabIters per wave (dummies past the span) */
    auto slab_dma = [&](bool in, uint64_t S16, uint64_t span, uint8_t *buf) __attribute__((always_inline)) {
        const uint32_t nch = in ? (uint32_t)((span + 15u) >> 4) + 2u : 0u; /* +2 pieces: reader look-ahead */
        const uint32_t wbase = t & ~63u;
#pragma unroll
        for (int i = 0; i < G::kSlabIters; i++) {
            const uint32_t c = t + (uint32_t)i * TK;
            if (wbase + (uint32_t)i * TK < nch) {
                if (c < nch)
                    __builtin_amdgcn_global_load_lds((gbl_void_t *)(keys_base + S16 + 16u * c),
                                                     (lds_void_t *)(buf + 16u * (wbase + (uint32_t)i * TK)), 16, 0,
                                                     kAux);
            } else if (D == 3 && lane == 0u) {
                __builtin_amdgcn_global_load_lds((gbl_void_t *)(off + nkeys), (lds_void_t *)(smem + G::kDump), 4, 0,
                                                 0);
            }
        }
    };
    auto top_barrier = [&]() __attribute__((always_inline)) {
        if constexpr (D == 2) {
            full_barrier();
        } else {
            /* everything but the youngest slab's kSlabIters DMAs */
            static_assert(G::kSlabIters <= 15, "vmcnt field");
            __builtin_amdgcn_s_waitcnt(0x0070 | G::kSlabIters); /* vmcnt(kSlabIters) expcnt(7) lgkmcnt(0) */
            asm volatile("" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
    };

    uint32_t pad_src = 0u; /* md5: the padding perms' constant in a VGPR (a uniform selector takes the SGPR slot) */
    if constexpr (MODE == NC_GPUHASH_MD5) asm volatile("v_mov_b32 %0, %1" : "=v"(pad_src) : "i"(nc_md5s::kPadSrc));
    uint32_t pw0 = 0u; /* the packed continuum's first word */
    if (t < 256u) {
        if constexpr (uses_crc_table<MODE>())
            tab[t] = (MODE == NC_GPUHASH_CRC16) ? nc_crc16_entry(t) : nc_crc32_entry(t);
        if constexpr (wg_dist<VAR>() == kDistKetama) tab[t] = cont_lower_bound(dist.cont, dist.ncont, t << 24);
    }
    if constexpr (wg_dist<VAR>() == kDistKetamaLds) {
        uint8_t *ci = reinterpret_cast<uint8_t *>(gs_cont + dist.ncont);
        for (uint32_t i = t; i < dist.ncont; i += TK) {
            gs_cont[i] = dist.cont[2u * i + 1u];
            ci[i] = (uint8_t)dist.cont[2u * i];
        }
        /* the 256 bucket starts from the staged values (as the packed form's
         * below), not by 256 binary searches over global memory */
        __syncthreads();
        const uint32_t n = dist.ncont;
        for (uint32_t i = t; i < n; i += TK) {
            const uint32_t cb = gs_cont[i] >> 24;
            for (uint32_t bb = i == 0u ? 0u : (gs_cont[i - 1u] >> 24) + 1u; bb <= cb; bb++) tab[bb] = i;
            if (i == n - 1u)
                for (uint32_t bb = cb + 1u; bb < 256u; bb++) tab[bb] = n;
        }
    } else if constexpr (wg_dist<VAR>() == kDistKetamaLdsPacked && (VAR & 512) == 0) { /* bit 9: DIAGNOSTIC */
        pw0 = (dist.cont[1] & ~0xffu) | (dist.cont[0] & 0xffu); /* point 0, the wrap's answer */
        /* + eight sentinels: never below a hash's top 24 bits, point 0's
         * server in the low byte (ketama_find_lds_packed) */
        for (uint32_t i = t; i < dist.ncont + 8u; i += TK)
            gs_cont[i] = i < dist.ncont ? (dist.cont[2u * i + 1u] & ~0xffu) | (dist.cont[2u * i] & 0xffu)
                                        : 0xffffff00u | (pw0 & 0xffu);
        /* the u16[512] bucket starts (in the table's 1 KiB) from the staged
         * words, not by 512 binary searches over global memory (eleven
         * dependent L2 round trips in every workgroup's prologue): point i
         * starts the buckets after its predecessor's up to its own, the last
         * point ends the rest at n */
        __syncthreads();
        uint16_t *bkt16 = reinterpret_cast<uint16_t *>(tab);
        const uint32_t n = dist.ncont;
        for (uint32_t i = t; i < n; i += TK) {
            const uint32_t cb = gs_cont[i] >> 23;
            for (uint32_t bb = i == 0u ? 0u : (gs_cont[i - 1u] >> 23) + 1u; bb <= cb; bb++) bkt16[bb] = (uint16_t)i;
            if (i == n - 1u)
                for (uint32_t bb = cb + 1u; bb < 512u; bb++) bkt16[bb] = (uint16_t)n;
        }
    }

    /* prologue: offsets of tiles 0 .. D-1; perm(0); slabs 0 .. D-2 */
#pragma unroll
    for (uint32_t j = 0; j < (uint32_t)D; j++) gs_issue_offs<kAux, TK>(off, tile_at(j), nkeys, offs_slot(j), t);
    full_barrier();
    uint32_t cnt = gs_tile_count<TK>(tile, nkeys);
    if (wave == 0u) gs_sort<TK>(offs_slot(0), cnt, lds_base + G::kHist, lds_base + G::kPerm, lane);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    uint64_t S16, span;
    bounds(offs_slot(0), S16, span);
    slab_dma(fits(span), S16, span, slab_buf(0));
    if constexpr (D == 3) {
        uint64_t s1, p1;
        bounds(offs_slot(1), s1, p1);
        slab_dma(tile_at(1) != tile && fits(p1), s1, p1, slab_buf(1));
    }

    uint64_t pend_idx = ~0ull;
    uint32_t pend_h = 0;
    /* CS: the previous tile's hashes, left in LDS by key index, go out as
     * 16-byte-per-lane stores, one wave per 256 keys (a partial or misaligned
     * tile: one dword per thread) */
    uint64_t pend_tile = ~0ull;
    uint32_t pend_cnt = 0, pend_par = 0;
    const bool out16 = (reinterpret_cast<uintptr_t>(out) & 15u) == 0u;
    auto store_tile = [&]() __attribute__((always_inline)) {
        const uint32_t ra = lds_base + G::kRes + pend_par * 4u * TK;
        uint32_t *dst = out + pend_tile * (uint64_t)TK;
        if (pend_cnt == (uint32_t)TK && out16) {
            if (wave >= 1u && wave <= (uint32_t)TK / 256u) {
                const uint32_t q = 64u * (wave - 1u) + lane; /* 16-byte piece */
                gs_u32x4 v;
                asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(ra + 16u * q) : "memory");
                if constexpr (NC_OUT_POLICY == 0) __builtin_nontemporal_store(v, reinterpret_cast<gs_u32x4 *>(dst) + q);
                else __builtin_amdgcn_raw_buffer_store_b128(
                    v, __builtin_amdgcn_make_buffer_rsrc(dst, 0, 4 * TK, 0x00020000), (int)(16u * q), 0, kAuxOut);
            }
        } else if (t < pend_cnt) {
            uint32_t v;
            asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(ra + 4u * t) : "memory");
            out_st32(dst + t, v);
        }
    };
    for (uint32_t it = 0;; it++) {
        top_barrier(); /* slab(it), offsets(it+1 .. it+D-1), perm(it) in LDS; reads of reused buffers done */
        /* VAR bit 6 (D = 2): the DMAs go out first — no second read of the
         * same bounds, the previous tile's coalesced store after them */
        constexpr bool kIssueFirst = (VAR & 64) != 0 && D == 2 && CS;
        if constexpr (CS && !kIssueFirst) {
            if (pend_tile != ~0ull) store_tile();
        } else if constexpr (!CS) {
            if (pend_idx != ~0ull) out_st32(out + pend_idx, pend_h);
            pend_idx = ~0ull;
        }
        asm volatile("" ::: "memory");
        const uint64_t t1 = tile + stride;
        const bool more = t1 < ntiles;
        const uint32_t cnt1 = more ? gs_tile_count<TK>(t1, nkeys) : 0u;
        /* every LDS read of the offsets slots comes before this iteration's
         * DMAs */
        uint64_t S16n = 0, spann = 0, sn = 0, pn = 0;
        if (more) bounds(offs_slot(it + 1u), S16n, spann);
        if constexpr (kIssueFirst) { /* slab(t + 1): the bounds just read */
            sn = S16n;
            pn = spann;
        } else {
            bounds(offs_slot(it + (uint32_t)D - 1u), sn, pn); /* slab(t + D - 1) */
        }
        const bool dn = tile + (uint64_t)(D - 1) * stride < ntiles && fits(pn);
        gs_issue_offs<kAux, TK>(off, tile_at(D), nkeys, offs_slot(it + (uint32_t)D), t);
        slab_dma(dn, sn, pn, slab_buf(it + (uint32_t)D - 1u));
        asm volatile("" ::: "memory");
        if constexpr (kIssueFirst) {
            if (pend_tile != ~0ull) store_tile();
            asm volatile("" ::: "memory");
        }
        /* wave 0 sorts tile t+1 with its DMAs already out (every LDS access
         * of the sort is inline asm, which hipcc does not hold behind them) */
        if (more && wave == 0u)
            gs_sort<TK>(offs_slot(it + 1u), cnt1, lds_base + G::kHist, lds_base + G::kPerm + ((it + 1u) & 1u) * 2u * TK,
                        lane);
        asm volatile("" ::: "memory");

        /* this wave's length group of tile `tile` */
        const uint8_t *slot = offs_slot(it);
        const uint32_t j = 64u * wave + lane;
        if (j < cnt) {
            const uint32_t i = perm2[(it & 1u) * TK + j];
            const uint32_t s = gs_lo(slot, i);
            /* the DMA clamps at nkeys, so [cnt] holds the end of a partial
             * tile's last key; a full tile's ends at the end bound, [TK] */
            const uint32_t len = gs_lo(slot, i + 1u) - s;
            const uint32_t pos = s + (uint32_t)delta - (uint32_t)S16;
            uint32_t h;
            if constexpr ((VAR & 8) != 0) {
                h = pos ^ len; /* DIAGNOSTIC ONLY: the memory pipeline without hashing */
            } else if (fits(span)) {
                if constexpr (MODE == NC_GPUHASH_MD5 && wg_dist<VAR>() == kDistNone) {
                    h = nc_md5s::md5_slab_key(reinterpret_cast<const uint32_t *>(slab_buf(it)), pos, len, pad_src);
                } else {
                    LdsSrc src{reinterpret_cast<const uint32_t *>(slab_buf(it))};
                    h = wg_value<MODE, VAR>(src, pos, len, tab, tab, dist);
                }
            } else {
                GlobalSrc src{reinterpret_cast<const uint32_t *>(keys_base)};
                h = wg_value<MODE, VAR>(src, S16 + pos, len, tab, tab, dist);
                __builtin_amdgcn_s_waitcnt(0x0070); /* retire the reader's loads before the paths merge */
            }
            if constexpr (wg_dist<VAR>() == kDistKetamaLds)
                h = ketama_find_lds(gs_cont, reinterpret_cast<const uint8_t *>(gs_cont + dist.ncont), tab, dist.ncont,
                                    h);
            else if constexpr (wg_dist<VAR>() == kDistKetamaLdsPacked && (VAR & 128) == 0) /* bit 7: DIAGNOSTIC */
                h = ketama_find_lds_packed(gs_cont, reinterpret_cast<const uint16_t *>(tab), dist.cont, dist.ncont,
                                           pw0, h);

            if constexpr (CS) {
                gs_ds_write_b32(lds_base + G::kRes + (it & 1u) * 4u * TK + 4u * i, h);
            } else {
                pend_idx = tile * (uint64_t)TK + i;
                pend_h = h;
            }
        }
        pend_tile = tile;
        pend_cnt = cnt;
        pend_par = it & 1u;
        if (!more) break;
        tile = t1;
        cnt = cnt1;
        S16 = S16n;
        span = spann;
    }
    if constexpr (CS) {
        full_barrier(); /* every wave's hashes of the last tile are in LDS */
        store_tile();
    } else {
        if (pend_idx != ~0ull) out[pend_idx] = pend_h;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); /* no LDS-DMA may outlive the workgroup */
}

template <int MODE, int VAR, int D, bool CS, int TK, int RSV = 0>
__global__ __launch_bounds__(TK) void nc_hash_kernel_gs(const uint8_t *__restrict__ keys_base,
                                                        const uint64_t *__restrict__ off, uint64_t delta,
                                                        uint64_t nkeys, uint32_t *__restrict__ out, uint64_t ntiles,
                                                        WrDist dist)
{
    gs_body<MODE, VAR, D, CS, TK, RSV>(keys_base, off, delta, nkeys, out, ntiles, dist);
}

/* The same with a dynamic-LDS reserve (the packed ketama continuum): its
 * budget is set for four 512-key workgroups per CU, so the waves must fit
 * eight per SIMD (<= 64 VGPRs; unconstrained, the dispatch's registers take
 * it to 71 and three workgroups) */
template <int MODE, int VAR, int D, bool CS, int TK, int RSV>
__global__ __launch_bounds__(TK, 8) void nc_hash_kernel_gs_rsv(const uint8_t *__restrict__ keys_base,
                                                             const uint64_t *__restrict__ off, uint64_t delta,
                                                             uint64_t nkeys, uint32_t *__restrict__ out,
                                                             uint64_t ntiles, WrDist dist)
{
    static_assert(TK == 512 && RSV > 0, "the reserve form is for 512-key tiles");
    gs_body<MODE, VAR, D, CS, TK, RSV>(keys_base, off, delta, nkeys, out, ntiles, dist);
}

/* ---------------- register-staged pipeline (variant bit 5) ----------------
 *
 * Same tiles, same hashing, different staging: every lane keeps the NEXT-BUT-
 * ONE tile's slab pieces in VGPRs (kRsK x 16 bytes, ordinary coalesced
 * global_load_dwordx4 = 1 KiB per wave-instruction) while the next tile's
 * pieces are still landing, and copies a tile into the single LDS slab
 * buffer just before hashing it. Two slabs per workgroup are in flight
 * without a second LDS buffer, so twice the bytes per CU are outstanding
 * (Little's law: that is what this HBM-latency-bound loop needs). Every load
 * targets VGPRs, so hipcc's own waitcnt pass orders everything; register sets
 * alternate by tile parity (loop unrolled by two) so no loaded register is
 * ever copied.
 */
/* A tile's slab bounds by ONE vector load per wave (lane 0: off[k0],
 * lane 1: off[k0 + cnt]), read back with v_readlane. A scalar load would
 * count in lgkmcnt and stall the hashing loop's first LDS wait. */
__device__ __forceinline__ uint64_t load_bounds(const uint64_t *__restrict__ off, uint64_t tile, uint64_t nkeys,
                                                uint32_t lane)
{
    const uint64_t k0 = tile * (uint64_t)kTile;
    return off[k0 + (lane == 1u ? tile_count(tile, nkeys) : 0u)];
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l)
{
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

constexpr int kRsK = 3;                                      /* 16-byte pieces per lane per tile */
constexpr uint32_t kRsCap = (uint32_t)kRsK * kBlock * 16u;    /* 12 KiB slab */
constexpr uint32_t kRsOffKey = kRsCap;
constexpr uint32_t kRsOffPerm = kRsOffKey + 4 * kTile;
constexpr uint32_t kRsOffHist = kRsOffPerm + 2 * kTile;
constexpr uint32_t kRsOffFlag = kRsOffHist + 8 * kBuckets;
constexpr uint32_t kRsOffTab = kRsOffFlag + 16;
constexpr uint32_t kRsSmem = kRsOffTab + 4 * 256;
static_assert(kRsOffTab % 16 == 0, "LDS carve must stay 16-byte aligned");
static_assert(kRsCap < 65536, "sorted key positions are packed in 16 bits");

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

/* Named members, not an array: an array member passed by reference through
 * a lambda was left in scratch memory by hipcc. */
struct RsSlab {
    u32x4_t a, b, c;
};
static_assert(kRsK == 3, "RsSlab holds three pieces per lane");

/* Per-lane sink for the output stores of lanes without a key, so that every
 * wave issues exactly one store per tile (the hand counts below rely on it). */
__device__ uint32_t g_rs_sink[kBlock];

/* ---- hand-counted VMEM (inline asm: invisible to hipcc's waitcnt pass) ----
 * Every load and store of the pipeline is issued here, unconditionally, so
 * each wave issues exactly 7 VMEM instructions per tile in a fixed order:
 *   O(j+1): 2 x global_load_dword      (this lane's key start / end, low dwords)
 *   B(j+3): 1 x global_load_dwordx2    (slab bounds, lanes 0/1)
 *   R(j+2): 3 x global_load_dwordx4    (slab pieces)
 *   S(j)  : 1 x global_store_dword     (this lane's hash, or the sink)
 * and waits with counted vmcnt(N) whose asm rewrites the guarded registers,
 * so no use of a loaded value can be scheduled above its wait. */
template <bool NT = false>
__device__ __forceinline__ uint32_t asm_ld32(const void *p)
{
    uint32_t v;
    if constexpr (NT) asm volatile("global_load_dword %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
    else asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ uint64_t asm_ld64(const void *p)
{
    u32x2_t v;
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    return ((uint64_t)v.y << 32) | v.x;
}
template <bool NT = false>
__device__ __forceinline__ u32x4_t asm_ld128(const void *p)
{
    u32x4_t v;
    if constexpr (NT) asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
    else asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    return v;
}
template <bool NT = false>
__device__ __forceinline__ void asm_st32(void *p, uint32_t v)
{
    if constexpr (NT) out_asm_st32(p, v); /* the hash outputs' policy (nc_out_policy.h) */
    else asm volatile("global_store_dword %0, %1, off" : : "v"(p), "v"(v) : "memory");
}

/* Uniform per-tile staging facts, derived from the tile's bounds. */
struct RsMeta {
    uint64_t S16;   /* 16-byte aligned slab start (keys_base-relative) */
    uint32_t nch;   /* 16-byte pieces covering the slab */
    uint32_t cnt;   /* keys in the tile */
    bool in_lds;    /* slab fits the LDS buffer */
};

__device__ __forceinline__ RsMeta rs_meta(uint64_t bnd, uint64_t tile, uint64_t nkeys, uint64_t delta)
{
    RsMeta m;
    const uint64_t S = readlane64(bnd, 0) + delta;
    const uint64_t E = readlane64(bnd, 1) + delta;
    m.S16 = S & ~(uint64_t)15;
    const uint64_t span = E - m.S16;
    m.in_lds = span <= (uint64_t)kRsCap;
    m.nch = m.in_lds ? (uint32_t)((span + 15u) >> 4) : 0u;
    m.cnt = tile_count(tile, nkeys);
    return m;
}

template <bool NT>
__device__ __forceinline__ RsSlab rs_load(const uint8_t *keys_base, const RsMeta &m, uint32_t t)
{
    const u32x4_t *g = reinterpret_cast<const u32x4_t *>(keys_base + m.S16);
    const uint32_t last = m.nch ? m.nch - 1u : 0u;
    const uint32_t c0 = t, c1 = t + kBlock, c2 = t + 2u * kBlock;
    RsSlab r;
    r.a = asm_ld128<NT>(g + (c0 < last ? c0 : last));
    r.b = asm_ld128<NT>(g + (c1 < last ? c1 : last));
    r.c = asm_ld128<NT>(g + (c2 < last ? c2 : last));
    return r;
}

__device__ __forceinline__ void rs_store_lds(uint8_t *slab, const RsMeta &m, uint32_t t, const RsSlab &r)
{
    u32x4_t *l = reinterpret_cast<u32x4_t *>(slab);
    if (t < m.nch) l[t] = r.a;
    if (t + kBlock < m.nch) l[t + kBlock] = r.b;
    if (t + 2u * kBlock < m.nch) l[t + 2u * kBlock] = r.c;
}

template <bool NT>
__device__ __forceinline__ TileOffs rs_offs(const uint64_t *__restrict__ off, uint64_t tile, uint64_t nkeys,
                                            uint32_t t)
{
    uint64_t k = tile * (uint64_t)kTile + t;
    uint64_t k1 = k + 1;
    if (k > nkeys) k = nkeys;
    if (k1 > nkeys) k1 = nkeys;
    TileOffs o;
    o.s = asm_ld32<NT>(off + k);  /* low dword (little-endian) */
    o.e = asm_ld32<NT>(off + k1);
    return o;
}

__device__ __forceinline__ uint64_t rs_bounds(const uint64_t *__restrict__ off, uint64_t tile, uint64_t nkeys,
                                              uint32_t lane)
{
    const uint64_t k0 = tile * (uint64_t)kTile;
    return asm_ld64(off + k0 + (lane == 1u ? tile_count(tile, nkeys) : 0u));
}

template <int MODE, bool SORT, int VAR>
__global__ __launch_bounds__(kBlock) void nc_hash_kernel_rs(const uint8_t *__restrict__ keys_base,
                                                            const uint64_t *__restrict__ off, uint64_t delta,
                                                            uint64_t nkeys, uint32_t *__restrict__ out,
                                                            uint64_t ntiles, WrDist)
{
    __shared__ __attribute__((aligned(16))) uint8_t smem[kRsSmem];
    uint8_t *slab = smem;
    uint32_t *kpos = reinterpret_cast<uint32_t *>(smem + kRsOffKey);
    uint16_t *perm = reinterpret_cast<uint16_t *>(smem + kRsOffPerm);
    uint32_t *hist2 = reinterpret_cast<uint32_t *>(smem + kRsOffHist);
    uint32_t *flag2 = reinterpret_cast<uint32_t *>(smem + kRsOffFlag);
    uint32_t *tab = reinterpret_cast<uint32_t *>(smem + kRsOffTab);

    const uint32_t t = threadIdx.x;
    const uint32_t lane = t & 63u;
    const uint64_t stride = gridDim.x;
    const uint64_t tile0 = blockIdx.x;
    if (tile0 >= ntiles) return;
    auto tile_at = [&](uint64_t j) -> uint64_t {
        const uint64_t x = tile0 + j * stride;
        return x < ntiles ? x : tile0;
    };
    uint32_t *sink = g_rs_sink + t;
    constexpr bool kNT = (VAR & 64) == 0; /* nt streams unless variant bit 6 (default policy) */

    if constexpr (uses_crc_table<MODE>()) {
        tab[t] = (MODE == NC_GPUHASH_CRC16) ? nc_crc16_entry(t) : nc_crc32_entry(t);
    }
    if constexpr (SORT) {
        if (t < 2u * kBuckets) hist2[t] = 0;
        if (t < 2u) flag2[t] = 0;
    }

    /* Prologue: bounds of the first two tiles (waited), then the steady-state
     * order as if steps -2 and -1 had run: R(0) S O(0) B(2) R(1) S */
    uint64_t b0 = rs_bounds(off, tile_at(0), nkeys, lane);
    uint64_t b1 = rs_bounds(off, tile_at(1), nkeys, lane);
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(b0), "+v"(b1) : : "memory");
    RsMeta m0 = rs_meta(b0, tile_at(0), nkeys, delta);
    RsMeta m1 = rs_meta(b1, tile_at(1), nkeys, delta);
    RsSlab ra = rs_load<kNT>(keys_base, m0, t);
    asm_st32(sink, 0u);
    TileOffs oa = rs_offs<kNT>(off, tile_at(0), nkeys, t), ob;
    uint64_t bq = rs_bounds(off, tile_at(2), nkeys, lane);
    RsSlab rb = rs_load<kNT>(keys_base, m1, t);
    asm_st32(sink, 0u);

    /* tile j: slab in `r`, offsets in `oc`, next offsets into `on`, meta in
     * `mc` (which receives tile j+D's meta at the end). */
    auto step = [&](uint64_t j, RsSlab &r, TileOffs &oc, TileOffs &on, RsMeta &mc)
        __attribute__((always_inline)) {
        const uint64_t tile = tile0 + j * stride;
        const uint64_t k0 = tile * (uint64_t)kTile;
        lds_barrier(); /* everyone is done with the previous tile's LDS */
        /* R(j): younger are S(j-2) and the 7 ops of step j-1 */
        asm volatile("s_waitcnt vmcnt(8)" : "+v"(r.a), "+v"(r.b), "+v"(r.c) : : "memory");
        if (mc.in_lds) rs_store_lds(slab, mc, t, r);
        on = rs_offs<kNT>(off, tile_at(j + 1), nkeys, t);
        /* B(j+2): younger are R(j+1) x3, S(j-1), O(j+1) x2 */
        asm volatile("s_waitcnt vmcnt(6)" : "+v"(bq) : : "memory");
        const RsMeta mD = rs_meta(bq, tile_at(j + 2u), nkeys, delta);
        bq = rs_bounds(off, tile_at(j + 3u), nkeys, lane);
        r = rs_load<kNT>(keys_base, mD, t);
        lds_barrier(); /* the slab is in LDS */
        /* O(j): younger are B, R x3, S of step j-1 and O x2, B, R x3 of step j */
        asm volatile("s_waitcnt vmcnt(11)" : "+v"(oc.s), "+v"(oc.e) : : "memory");

        const bool valid = t < mc.cnt;
        const uint32_t len = valid ? oc.e - oc.s : 0u;
        const uint32_t rel = oc.s + (uint32_t)delta - (uint32_t)mc.S16;
        uint32_t my = t;
        bool sorted = false;
        if constexpr (SORT) {
            uint32_t *hist = hist2 + (uint32_t)(j & 1u) * kBuckets;
            const uint32_t bucket = valid ? len_bucket(len) : (uint32_t)(kBuckets - 1);
            const uint32_t bb = __shfl(bucket, 0);
            if (mc.in_lds && __ballot(bucket != bb) != 0ull && lane == 0) flag2[j & 1u] = 1u;
            if (t < (uint32_t)kBuckets) hist2[(uint32_t)((j + 1u) & 1u) * kBuckets + t] = 0;
            if (t == 0) flag2[(j + 1u) & 1u] = 0;
            lds_barrier();
            if (flag2[j & 1u] != 0u) {
                sorted = true;
                kpos[t] = rel | (len << 16);
                const uint32_t rank = atomicAdd(&hist[bucket], 1u);
                lds_barrier();
                if (t < 64u) {
                    const uint32_t c = hist[t];
                    uint32_t x = c;
#pragma unroll
                    for (int d = 1; d < 64; d <<= 1) {
                        const uint32_t y = __shfl_up(x, d);
                        if (lane >= (uint32_t)d) x += y;
                    }
                    hist[t] = x - c;
                }
                lds_barrier();
                perm[hist[bucket] + rank] = (uint16_t)t;
                lds_barrier();
                my = perm[t];
            }
        }
        uint32_t h = 0;
        if (my < mc.cnt) {
            uint32_t klen_my = len, pos = rel;
            if (sorted) {
                const uint32_t kp = kpos[my];
                pos = kp & 0xffffu;
                klen_my = kp >> 16;
            }
            if (mc.in_lds) {
                LdsSrc src{reinterpret_cast<const uint32_t *>(slab)};
                h = hash_key<MODE, VAR>(src, pos, klen_my, tab);
            } else {
                /* long-key path: hipcc's own loads; it waits vmcnt(0) for
                 * them, which is only an over-wait for the hand counts */
                GlobalSrc src{reinterpret_cast<const uint32_t *>(keys_base)};
                h = hash_key<MODE, VAR>(src, mc.S16 + pos, klen_my, tab);
                __builtin_amdgcn_s_waitcnt(0x0070);
            }
        }
        asm_st32<kNT>(my < mc.cnt ? (void *)(out + k0 + my) : (void *)sink, h);
        mc = mD;
    };

    for (uint64_t j = 0;;) {
        if (tile0 + j * stride >= ntiles) break;
        step(j, ra, oa, ob, m0);
        j++;
        if (tile0 + j * stride >= ntiles) break;
        step(j, rb, ob, oa, m1);
        j++;
    }
    asm volatile("s_waitcnt vmcnt(0)" : : : "memory");
}

/* ---------------- wave-ring pipeline (variant bit 7; fused dispatch) ----------------
 *
 * Every wave runs its own pipeline over its own part of LDS: there is no
 * barrier in the loop, so waves drift apart and the memory system sees a
 * smooth request stream instead of lock-stepped bursts.
 *
 * A wave tile is 128 consecutive keys (lane l hashes keys k0+l and k0+64+l).
 * Its offsets off[k0 .. k0+128] and its key slab come HBM -> LDS by LDS-DMA
 * only, issued as inline asm so that hipcc's waitcnt pass never sees them
 * (it would wait for a pending DMA before LDS reads). Iteration j issues
 * exactly P + 4 VMEM instructions, in this order:
 *   OFF(j+DO) : global_load_lds_dwordx4 (off[k0 .. k0+128), two per lane)
 *               + global_load_lds_dword on lanes 0-1 (off[k0 + cnt])
 *   SLAB(j+DS): P x global_load_lds_dwordx4 (1 KiB each; pieces the slab
 *               does not need become one-lane dword DMAs into a dump word)
 *   ST(j)     : 2 x global_store_dword (lanes without a key store to a sink)
 * so both waits are constant vmcnt(N):
 *   OFF(j+DS) landed, before SLAB(j+DS) is issued : N = (DO - DS)(P + 4)
 *   SLAB(j) landed, before tile j is hashed        : N = DS (P + 4)
 * The counter retires in order, so the first wait also retires every slab
 * older than OFF(j+DS); DO >= 2 DS - 1 keeps SLAB(j+1) out of it. Extra VMEM
 * instructions (the global-memory reader of a tile too long for its slab
 * slot) only make the waits conservative; an instruction is never skipped,
 * which is what would make them unsafe.
 *
 * DIST selects what is stored per key: the hash (kDistNone, the hashkit
 * function), or server_pool_idx (src/nc_server.c:647-700): hash_tag trimming,
 * hash 0 for an empty key, then ketama_dispatch / modula_dispatch over a
 * continuum staged in LDS (kDistKetama / kDistModula), or the hash before
 * dispatch (kDistPre, for continua too large for LDS). WPW waves per
 * workgroup share the crc table and the continuum; each owns its ring.
 */
constexpr int kWrTile = 128; /* keys per wave tile (64: one key per lane, the short-key shape) */
/* TK = 256 (four keys per lane) sorts the tile's keys by length inside the
 * wave and hashes them in four rounds of 64 similar lengths: a round runs as
 * long as its longest key, so Zipf lengths cost ~the sum of the four quartile
 * maxima instead of four times the tile maximum. */
template <int P, int DS, int DO, int TK = kWrTile, bool SR = (TK == 256)>
struct WrRing {
    static_assert(DO > DS && DS >= 1 && DO >= 2 * DS - 1, "offsets must run far enough ahead of slabs");
    static_assert(TK == 64 || TK == 128 || TK == 256, "a wave tile is one, two or four keys per lane");
    static constexpr uint32_t kOffSlot = 8u * TK + 16u;  /* off[k0 .. k0+TK) + end bound, 16-aligned */
    static constexpr int NST = TK / 64;                  /* output stores per tile */
    static constexpr int NOFF = TK == 256 ? 2 : 1;       /* 16-B offset DMAs per lane per tile */
    static constexpr int kIter = P + NOFF + 1 + NST;     /* VMEM instructions per iteration, fixed */
    static constexpr uint32_t NS = DS + 1;            /* slab slots: tiles j .. j+DS */
    static constexpr uint32_t NO = DO + 1;            /* offset slots: tiles j .. j+DO */
    static constexpr uint32_t kSlot = (uint32_t)P * 1024u;
    static constexpr uint32_t kOffOffs = NS * kSlot;  /* slab over-reads land in the next slot / the offsets */
    static constexpr uint32_t kOffDump = kOffOffs + NO * kOffSlot;
    static constexpr uint32_t kSortOffs = kOffDump + 16u; /* sorted rounds: u32 hist[64] + u32 order[TK] */
    static constexpr uint32_t kBytes = kSortOffs + (SR ? 4u * (64u + (uint32_t)TK) : 0u);
    static constexpr int kWaitOff = (DO - DS) * kIter;
    static constexpr int kWaitSlab = DS * kIter;
    static_assert(kWaitSlab <= 63 && kWaitOff <= 63, "vmcnt is 6 bits");
};


/* LDS-DMA through M0 (saved and restored: M0 is compiler-reserved) */
template <bool NT>
__device__ __forceinline__ void glds16(const void *g, uint32_t lds)
{
    uint32_t keep;
    if constexpr (NT)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\t"
                     "s_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
                     "s_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}
__device__ __forceinline__ void glds4(const void *g, uint32_t lds)
{
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm()
{
    static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int TK>
__device__ __forceinline__ uint32_t wr_count(uint64_t tile, uint64_t nkeys)
{
    const uint64_t left = nkeys - tile * (uint64_t)TK;
    return left < (uint64_t)TK ? (uint32_t)left : (uint32_t)TK;
}

/* {off[k0], off[k0+cnt]} + delta of the tile whose offsets are at ob, wave-uniform */
template <int TK>
__device__ __forceinline__ void wr_bounds(const uint32_t *ob, uint64_t delta, uint64_t &S, uint64_t &E)
{
    /* readfirstlane returns int: through uint32_t, or a low dword >= 2^31
     * sign-extends over the high one (key buffers past 2 GiB) */
    const uint32_t s_lo = (uint32_t)__builtin_amdgcn_readfirstlane(ob[0]);
    const uint32_t s_hi = (uint32_t)__builtin_amdgcn_readfirstlane(ob[1]);
    const uint32_t e_lo = (uint32_t)__builtin_amdgcn_readfirstlane(ob[2 * TK]);
    const uint32_t e_hi = (uint32_t)__builtin_amdgcn_readfirstlane(ob[2 * TK + 1]);
    S = (((uint64_t)s_hi << 32) | s_lo) + delta;
    E = (((uint64_t)e_hi << 32) | e_lo) + delta;
}

constexpr uint32_t kBktBytes = 4u * 260u; /* u32[257] bucket index after an LDS-staged ketama continuum */

template <int MODE, int VAR, int DIST, class Src>
__device__ __forceinline__ uint32_t key_value(const Src &src, typename Src::pos_t p, uint32_t len,
                                              const uint32_t *tab, const WrDist &dist, const uint32_t *cont)
{
    if constexpr (DIST == kDistNone && (VAR & 8) != 0) {
        return (uint32_t)p ^ len; /* DIAGNOSTIC ONLY: the memory pipeline without hashing */
    } else if constexpr (DIST == kDistNone) {
        return hash_key<MODE, VAR>(src, p, len, tab);
    } else {
        if (dist.tag != 0u) tag_trim(src, p, len, dist.tag & 0xffu, (dist.tag >> 8) & 0xffu);
        uint32_t h = 0u; /* server_pool_hash: keylen 0 hashes to 0 (src/nc_server.c:639-641) */
        if (len != 0u) h = hash_key<MODE, VAR>(src, p, len, tab);
        if constexpr (DIST == kDistKetama) return ketama_find_bkt(cont, cont + 2u * dist.ncont, dist.ncont, h);
        else if constexpr (DIST == kDistModula) return cont[2u * (h % dist.ncont)]; /* nc_modula.c:153 */
        else return h;
    }
}

/* VAR bit 2 on the wave ring: hash the tile in length-sorted rounds (always
 * for 256-key tiles) */
template <int VAR, int TK>
constexpr bool wr_sorted()
{
    return TK == 256 || (VAR & 4) != 0;
}

template <int MODE, int DIST, int P, int DS, int DO, int WPW, int TK = kWrTile, int VAR = 0>
constexpr uint32_t wr_lds_fixed()
{
    return (uint32_t)WPW * WrRing<P, DS, DO, TK, wr_sorted<VAR, TK>()>::kBytes +
           (uses_crc_table<MODE>() ? ((VAR & kHkCrcSliced) != 0 ? 1024u * kSliceTables : 1024u) : 0u);
}

template <int MODE, int VAR, int P, int DS, int DO, int DIST, int WPW, int TK = kWrTile>
__global__ __launch_bounds__(64 * WPW) void nc_hash_kernel_wr(const uint8_t *__restrict__ keys_base,
                                                              const uint64_t *__restrict__ off, uint64_t delta,
                                                              uint64_t nkeys, uint32_t *__restrict__ out,
                                                              uint64_t ntiles, WrDist dist)
{
    constexpr bool kSortRounds = wr_sorted<VAR, TK>();
    using R = WrRing<P, DS, DO, TK, kSortRounds>;
    constexpr uint32_t NS = R::NS, NO = R::NO;
    constexpr uint32_t kWrOffSlot = R::kOffSlot;
    constexpr bool kNT = (VAR & 64) == 0;
    constexpr uint32_t kTabOffs = (uint32_t)WPW * R::kBytes;
    constexpr uint32_t kContOffs = wr_lds_fixed<MODE, DIST, P, DS, DO, WPW, TK, VAR>();
    extern __shared__ __attribute__((aligned(16))) uint8_t wr_lds[];

    const uint32_t t = threadIdx.x;
    const uint32_t lane = t & 63u;
    const uint32_t wave = WPW == 1 ? 0u : (uint32_t)__builtin_amdgcn_readfirstlane(t >> 6);
    uint8_t *smem = wr_lds + wave * R::kBytes;
    uint32_t *tab = reinterpret_cast<uint32_t *>(wr_lds + kTabOffs);
    uint32_t *cont = reinterpret_cast<uint32_t *>(wr_lds + kContOffs);

    /* shared set-up, before any DMA is in flight */
    if constexpr (uses_crc_table<MODE>() && (VAR & kHkCrcSliced) != 0) {
        for (uint32_t i = t; i < 256u * kSliceTables; i += 64u * WPW) tab[i] = nc_slice::entry<MODE>(i >> 8, i & 255u);
    } else if constexpr (uses_crc_table<MODE>()) {
        for (uint32_t i = t; i < 256u; i += 64u * WPW)
            tab[i] = (MODE == NC_GPUHASH_CRC16) ? nc_crc16_entry(i) : nc_crc32_entry(i);
    }
    if constexpr (DIST == kDistKetama || DIST == kDistModula) {
        for (uint32_t i = t; i < 2u * dist.ncont; i += 64u * WPW) cont[i] = dist.cont[i];
    }
    if constexpr (DIST == kDistKetama) {
        __syncthreads();
        uint32_t *bkt = cont + 2u * dist.ncont;
        for (uint32_t j = t; j <= 256u; j += 64u * WPW)
            bkt[j] = j == 256u ? dist.ncont : cont_lower_bound(cont, dist.ncont, j << 24);
    }
    if constexpr (WPW > 1 || DIST == kDistKetama) __syncthreads();

    const uint64_t W = (uint64_t)gridDim.x * WPW;
    const uint64_t tile0 = (uint64_t)blockIdx.x * WPW + wave;
    if (tile0 >= ntiles) return;
    uint32_t *sink = g_rs_sink + lane;
    const uint32_t smem_lds = lds_addr(smem);

    /* a VMEM instruction that moves one word nobody reads: keeps the
     * per-iteration count fixed. `src` is a word the wave touches anyway
     * (its own slab or offsets), so the dummies of all waves do not pile
     * onto one L2 line. */
    auto dummy = [&](const void *src) __attribute__((always_inline)) {
        if (lane == 0u) glds4(src, smem_lds + R::kOffDump);
    };
    /* OFF(tile) into offset slot `oslot`: 2 instructions */
    auto issue_off = [&](uint64_t tile, uint32_t oslot) __attribute__((always_inline)) {
        if (tile >= ntiles) {
#pragma unroll
            for (int h = 0; h <= R::NOFF; h++) dummy(off + nkeys);
            return;
        }
        const uint64_t k0 = tile * (uint64_t)TK;
        const uint64_t last_pair = (nkeys - 1u) & ~(uint64_t)1; /* pairs (p, p+1) stay <= nkeys */
        const uint32_t dst = smem_lds + R::kOffOffs + oslot * kWrOffSlot;
#pragma unroll
        for (int h = 0; h < R::NOFF; h++) {
            uint64_t p = k0 + 128u * (uint32_t)h + 2u * lane;
            if (p > last_pair) p = last_pair;
            if (TK >= 128 || lane < (uint32_t)TK / 2u) glds16<kNT>(off + p, dst + 1024u * (uint32_t)h);
        }
        if (lane < 2u) {
            const uint64_t e = k0 + wr_count<TK>(tile, nkeys);
            glds4(reinterpret_cast<const uint32_t *>(off + e) + lane, dst + 8u * TK);
        }
    };
    /* SLAB(tile) into slab slot `sslot`: P instructions; OFF(tile) has landed */
    auto issue_slab = [&](uint64_t tile, uint32_t oslot, uint32_t sslot) __attribute__((always_inline)) {
        uint32_t nins = 0, nch = 0;
        uint64_t S16 = 0;
        if (tile < ntiles) {
            uint64_t S, E;
            wr_bounds<TK>(reinterpret_cast<const uint32_t *>(smem + R::kOffOffs + oslot * kWrOffSlot), delta, S, E);
            S16 = S & ~(uint64_t)15;
            const uint64_t span = E - S16;
            if (span <= (uint64_t)R::kSlot) {
                nch = (uint32_t)((span + 15u) >> 4);
                nins = (nch + 63u) >> 6;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); /* earlier reads of the slot have retired */
        const uint32_t dst = smem_lds + sslot * R::kSlot;
#pragma unroll
        for (int i = 0; i < P; i++) {
            if ((uint32_t)i < nins) {
                uint32_t c = 64u * (uint32_t)i + lane;
                if (c >= nch) c = nch - 1u; /* stay inside the key buffer (+ NC_GPUHASH_PAD) */
                glds16<kNT>(keys_base + S16 + 16u * c, dst + 1024u * (uint32_t)i);
            } else if (tile < ntiles) {
                dummy(keys_base + S16); /* the tile's first 16-byte block: readable */
            } else {
                /* past the last tile S16 is 0, and keys_base itself need not be
                 * readable (a batch's offsets may start anywhere: a chunk of a
                 * larger CSR hands in keys - offsets[0]) */
                dummy(off + nkeys);
            }
        }
    };

    /* prologue: the steady-state queue, as if iterations -DO .. -1 had run */
#pragma unroll
    for (int jj = -DO; jj < 0; jj++) {
        issue_off(tile0 + (uint64_t)(jj + DO) * W, (uint32_t)(jj + DO) % NO);
        if (jj + DS >= 0) {
            wait_vm<R::kWaitOff>();
            issue_slab(tile0 + (uint64_t)(jj + DS) * W, (uint32_t)(jj + DS) % NO, (uint32_t)(jj + DS) % NS);
        } else {
#pragma unroll
            for (int i = 0; i < P; i++) dummy(off + nkeys);
        }
#pragma unroll
        for (int i = 0; i < R::NST; i++) dummy(off + nkeys);
    }

    for (uint32_t j = 0;; j++) {
        const uint64_t tile = tile0 + (uint64_t)j * W;
        if (tile >= ntiles) break;
        issue_off(tile + (uint64_t)DO * W, (j + DO) % NO);
        wait_vm<R::kWaitOff>();
        issue_slab(tile + (uint64_t)DS * W, (j + DS) % NO, (j + DS) % NS);
        wait_vm<R::kWaitSlab>();

        const uint32_t *ob = reinterpret_cast<const uint32_t *>(smem + R::kOffOffs + (j % NO) * kWrOffSlot);
        const uint8_t *slab = smem + (j % NS) * R::kSlot;
        const uint32_t cnt = wr_count<TK>(tile, nkeys);
        uint64_t S, E;
        wr_bounds<TK>(ob, delta, S, E);
        const uint64_t S16 = S & ~(uint64_t)15;
        const bool in_lds = E - S16 <= (uint64_t)R::kSlot;
        const uint64_t k0 = tile * (uint64_t)TK;

        uint32_t h[R::NST];
        uint32_t key_of[R::NST]; /* tile index of the key each round hashes */
#pragma unroll
        for (int q = 0; q < R::NST; q++) key_of[q] = lane + 64u * (uint32_t)q;
        constexpr bool kPair = TK == 128 && (VAR & 512) != 0 && DIST == kDistNone && MODE != NC_GPUHASH_HSIEH &&
                               MODE != NC_GPUHASH_MURMUR && MODE != NC_GPUHASH_JENKINS;
        if constexpr (kPair) {
            if (in_lds) {
                uint32_t len2[2], pos2[2];
#pragma unroll
                for (int q = 0; q < 2; q++) {
                    const uint32_t i = lane + 64u * (uint32_t)q;
                    const uint32_t ie = i + 1u >= cnt ? (uint32_t)TK : i + 1u;
                    const uint32_t s = ob[2u * i];
                    len2[q] = i < cnt ? ob[2u * ie] - s : 0u;
                    pos2[q] = i < cnt ? s + (uint32_t)delta - (uint32_t)S16 : 0u;
                }
                LdsSrc src{reinterpret_cast<const uint32_t *>(slab)};
                if constexpr (MODE == NC_GPUHASH_MD5)
                    hash_md5_pair(src, pos2[0], len2[0], pos2[1], len2[1], h[0], h[1]);
                else
                    hash_bytes_pair<MODE, VAR>(src, pos2[0], len2[0], pos2[1], len2[1], tab, h[0], h[1]);
                goto stores;
            }
        }
        if constexpr (kSortRounds) {
            /* counting sort of the tile's keys by length class, in LDS: one
             * wave, so its LDS operations retire in order */
            uint32_t *hist = reinterpret_cast<uint32_t *>(smem + R::kSortOffs);
            uint32_t *order = hist + 64;
            uint32_t bk[R::NST], rk[R::NST];
            hist[lane] = 0u;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int q = 0; q < R::NST; q++) {
                const uint32_t i = key_of[q];
                const uint32_t ie = i + 1u >= cnt ? (uint32_t)TK : i + 1u;
                const uint32_t len = i < cnt ? ob[2u * ie] - ob[2u * i] : 0u;
                bk[q] = i < cnt ? (len < 62u ? len : 62u) : 63u; /* absent keys last */
                rk[q] = __hip_atomic_fetch_add(hist + bk[q], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const uint32_t c = hist[lane];
            uint32_t incl = c;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t v = __shfl_up(incl, d, 64);
                if (lane >= (uint32_t)d) incl += v;
            }
            hist[lane] = incl - c; /* first rank of length class `lane` */
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int q = 0; q < R::NST; q++) order[hist[bk[q]] + rk[q]] = key_of[q];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int q = 0; q < R::NST; q++) key_of[q] = order[64u * (uint32_t)q + lane];
        }
#pragma unroll
        for (int q = 0; q < R::NST; q++) {
            const uint32_t i = key_of[q];
            const bool valid = i < cnt;
            const uint32_t ie = i + 1u >= cnt ? (uint32_t)TK : i + 1u; /* key cnt-1 ends at the end bound */
            const uint32_t s = ob[2u * i];
            const uint32_t e = ob[2u * ie];
            const uint32_t len = valid ? e - s : 0u;
            const uint32_t pos = valid ? s + (uint32_t)delta - (uint32_t)S16 : 0u;
            if (in_lds) {
                LdsSrc src{reinterpret_cast<const uint32_t *>(slab)};
                h[q] = key_value<MODE, VAR, DIST>(src, pos, len, tab, dist, cont);
            } else {
                GlobalSrc src{reinterpret_cast<const uint32_t *>(keys_base)};
                h[q] = key_value<MODE, VAR, DIST>(src, S16 + pos, len, tab, dist, cont);
                /* retire the global reader's own loads before the paths
                 * merge: a load still pending there makes hipcc wait
                 * vmcnt(0) at the merge, draining the DMA ring */
                __builtin_amdgcn_s_waitcnt(0x0070);
            }
        }
    stores:
#pragma unroll
        for (int q = 0; q < R::NST; q++) {
            const uint32_t i = key_of[q];
            asm_st32<kNT>(i < cnt ? (void *)(out + k0 + i) : (void *)sink, h[q]);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); /* no LDS-DMA may outlive the workgroup */
}

/* the ketama lookup table (ketama_find_lut): one thread per range of 2^shift
 * hash values */
__global__ __launch_bounds__(256) void nc_ketama_lut_kernel(const uint32_t *__restrict__ cont, uint32_t n,
                                                            uint32_t *__restrict__ lut, uint32_t shift)
{
    const uint32_t b = blockIdx.x * 256u + threadIdx.x;
    if (b >= (1u << (32u - shift))) return;
    const uint32_t lo = b << shift, hi = lo | ((1u << shift) - 1u);
    const uint32_t p = cont_lower_bound(cont, n, lo);
    if (p == n) lut[b] = cont[0];                             /* every hash here wraps to the first point */
    else if (cont[2u * p + 1u] > hi) lut[b] = cont[2u * p];   /* no point inside: one server for the range */
    else lut[b] = 0x80000000u | p;
}

/* ketama / modula over pre-dispatch hashes, in place (continua too large
 * for the fused kernel's LDS); the continuum is read through L2 */
template <int DIST>
__global__ __launch_bounds__(256) void nc_dispatch_kernel(const uint32_t *__restrict__ cont, uint32_t ncont,
                                                          uint32_t *__restrict__ io, uint64_t n)
{
    /* ketama: the 257-entry bucket index of the continuum (ketama_find_bkt),
     * built once per workgroup in LDS; each lookup then searches ~log2(n/256)
     * points of the L2-resident continuum */
    __shared__ uint32_t bkt[DIST == kDistKetama ? 260 : 1];
    if constexpr (DIST == kDistKetama) {
        for (uint32_t j = threadIdx.x; j <= 256u; j += 256u)
            bkt[j] = j == 256u ? ncont : cont_lower_bound(cont, ncont, j << 24);
        __syncthreads();
    }
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u) {
        const uint32_t h = io[i];
        io[i] = DIST == kDistKetama ? ketama_find_bkt(cont, bkt, ncont, h) : cont[2u * (h % ncont)];
    }
}

} // namespace

/* ---------------- launch layer ----------------
 *
 * This file is compiled once per hash mode (-DNC_TU_MODE=<mode id>: that
 * mode's kernels and its nc_tu::entry<MODE>) and once without NC_TU_MODE (the
 * C ABI, the policy and the process-wide tuning state), so the 12 code
 * objects build in parallel. */
namespace nc_tu {
extern int g_grid_cap; /* 0 = persistent: every resident workgroup slot once */
extern int g_sort;     /* 1 on, 0 off */
extern int g_variant;  /* variant bits, include/nc_gpuhash_probe.h (nc_gpuhash_set_tuning) */
/* the tuning globals are read and written with __atomic builtins (any thread) */
extern int g_num_cus[64];

/* one launch of mode MODE: the wave ring when var bit 7 is set (offsets
 * 16-byte aligned), else the workgroup pipeline */
template <int MODE>
hipError_t entry(const uint8_t *base, const uint64_t *off, uint64_t delta, uint64_t nkeys, uint32_t *out,
                 hipStream_t stream, bool sort, int var);

/* server_pool_idx of one launch: continuum {index, value} pairs in device
 * memory, hash_tag (c0 | c1 << 8 | 1 << 16, or 0), kind 0 ketama / 1 modula */
struct DistArgs {
    const uint32_t *cont;
    uint32_t ncont;
    uint32_t tag;
    int kind;
    bool wide; /* 5 KiB slab slots two tiles ahead (keys of 20+ B) instead of 3 KiB one ahead */
    bool wg;   /* the workgroup pipeline (continuum in L2, bucket index in LDS) instead of the wave ring */
    bool gs;   /* the grouped workgroup pipeline (one length quartile per wave), continuum as for wg */
    int gs_var; /* its launch options (variant bits 21-22: resident sets) */
    const uint32_t *lut; /* ketama lookup table (ketama_find_lut) for the workgroup pipelines, or null */
    uint32_t lut_shift;
    bool lds_cont; /* ketama on the grouped pipeline with the continuum staged in LDS (ketama_find_lds) */
};
/* fused hash -> dispatch of mode MODE on the wave ring (offsets 16-byte aligned) */
template <int MODE>
hipError_t entry_dist(const uint8_t *base, const uint64_t *off, uint64_t delta, uint64_t nkeys, uint32_t *out,
                      hipStream_t stream, const DistArgs &d);
} // namespace nc_tu

namespace nc_md5 {
/* md5 on the direct per-lane block pipeline (nc_md5_kernels.hip); keys is any
 * byte address, nkeys < 2^32 */
hipError_t launch(const uint8_t *d_keys, const uint64_t *d_off, uint64_t nkeys, uint32_t *d_out, hipStream_t stream,
                  int var, uint32_t fl, uint32_t max_len);
} // namespace nc_md5

namespace nc_bytes {
/* the byte-serial modes on the direct pipeline (nc_bytes_kernels.hip) */
bool supports(int mode);
/* hsieh, murmur, jenkins on its short-key kernel only */
bool supports_short_words(int mode);
hipError_t launch(int mode, const uint8_t *d_keys, const uint64_t *d_off, uint64_t nkeys, uint32_t *d_out,
                  hipStream_t stream, int var, uint32_t max_len);
} // namespace nc_bytes

namespace nc_wsort {
/* fnv x4 and one_at_a_time on the wave-sorted pipeline (nc_wsort_kernels.hip):
 * 256-key tiles per wave, length-sorted rounds */
bool supports(int mode);
hipError_t launch(int mode, const uint8_t *d_keys, const uint64_t *d_off, uint64_t nkeys, uint32_t *d_out,
                  hipStream_t stream, int var);
} // namespace nc_wsort

namespace {
using nc_tu::g_grid_cap;
using nc_tu::g_num_cus;
using nc_tu::g_sort;
using nc_tu::g_variant;

/* Auto-policy choices (variant bits): the workgroup pipeline (bit 16 only
 * marks an explicit choice; it is stripped before launch), the register-staged
 * workgroup pipeline, and the wave ring with 5 KiB / 4 KiB slab slots. */
[[maybe_unused]] constexpr int kVarWorkgroup = 1 << 16;
[[maybe_unused]] constexpr int kVarRegStaged = 32;
[[maybe_unused]] constexpr int kVarRingP5 = 128 | (3 << 8);
[[maybe_unused]] constexpr int kVarRingP4 = 128;
[[maybe_unused]] constexpr int kVarSorted = 1 << 17; /* group the tile's keys by length (the SORT pipeline) */
constexpr int kVarOver = 1 << 18; /* workgroup pipelines: three resident sets of workgroups per launch */
constexpr int kVarMd5Direct = 1 << 19; /* the direct per-lane block pipeline: md5 (nc_md5_kernels.hip) and
                                          the byte-serial modes (nc_bytes_kernels.hip); options in bits 20-23 */
[[maybe_unused]] constexpr int kVarDirect = kVarMd5Direct;
constexpr int kVarDirectLds = 4 << 20; /* its LDS-DMA block image (long keys) */
constexpr int kVarDirectIl32 = (8 | 2) << 20; /* a wave's tiles interleaved over the grid, 32 per wave (nc_direct.h
                                                 wave_tiles) */
constexpr int kVarWsort = 1 << 24; /* the wave-sorted pipeline (nc_wsort_kernels.hip); options in bits 20-23 */
constexpr int kVarNoFixedLen = 1 << 26; /* md5: no fixed-length specialisation (A/B) */
constexpr int kVarGsort = 1 << 25; /* the grouped workgroup pipeline (nc_hash_kernel_gs); options in bits 20-23 */
constexpr int kVarGsortCs = 1 << 27; /* its hashes stored once per tile, 16 bytes per lane */
constexpr int kVarGsort512 = 1 << 26; /* with kVarGsortCs: 512-key tiles, eight waves (length octiles) */
constexpr int kVarGsortIssue = 1 << 28; /* A/B: the grouped tile's DMAs issued before the previous tile's store */
constexpr uint32_t kLdsContMax = 4800; /* ketama points the grouped pipeline stages in LDS (5 B each) */
constexpr uint32_t kLdsPackedMax = 1280; /* ... packed, 4 B each (+ 8 sentinels), beside four 512-key
                                            workgroups per CU */
constexpr int kVarNoPacked = 1 << 27; /* server_idx A/B: the 5-byte LDS continuum even where the packed one fits */
/* direct byte kernels' options beyond bits 20-23, in bits only the ring
 * pipeline reads otherwise (bit 19 selects the direct pipeline first) */
constexpr int kVarDirect8 = 1 << 12;     /* line image: eight-wave workgroups, one per CU */
constexpr int kVarDirectS8 = 1 << 13;    /* crcs: slicing-by-8 tables */
constexpr int kVarDirectNoHash = 1 << 14; /* DIAGNOSTIC (fnv1a_64, crc32): xor of words, not a hash */
constexpr int kVarMd5PadTab = 1 << 15;    /* md5: padding selectors from an LDS table */
constexpr int kVarMd5FullLines = 1 << 12; /* md5 (shares kVarDirect8's bit): whole-line output stores; A/B:
                                             bit 13 (the crcs' S8) the line kernel's offsets non-temporal,
                                             bit 14 (NoHash) no S64 form for shapes of keys <= 64 B */
constexpr int kVarDirectShort = 1 << 11;  /* byte modes, keys <= 32 B: eight waves per CU, tiles in flight */
constexpr int kVarDirectPairs = 1 << 10;  /* with kVarDirect8: the line image in rounds of two lines */
constexpr int kVarDirectOffDefault = 1 << 9; /* A/B (crc32, fnv1a_64): the offsets with the default cache policy
                                                (bits 8-9 are ring options, unread on the direct path) */
static_assert(((kVarDirect8 | kVarDirectS8 | kVarDirectNoHash | kVarMd5PadTab | kVarDirectShort | kVarDirectPairs) &
               (kVarMd5Direct | (15 << 20) | kVarNoFixedLen | kVarWsort | kVarGsort | kVarNoPacked | (3 << 29))) == 0,
              "direct-pipeline options overlap the pipeline choice, its nibble or the server_idx bits");

int load_i(const int *p) { return __atomic_load_n(p, __ATOMIC_RELAXED); }
void store_i(int *p, int v) { __atomic_store_n(p, v, __ATOMIC_RELAXED); }

/* Occupancy of one kernel instantiation at one dynamic LDS size, cached as
 * ONE word (lds << 32 | blocks per CU) so threads launching with different
 * LDS sizes (different continuum sizes) never read a torn pair; a miss just
 * asks HIP again. */
template <class K>
int cached_occupancy(uint64_t *cache, K kern, int block, size_t lds, int dflt)
{
    const uint64_t v = __atomic_load_n(cache, __ATOMIC_RELAXED);
    if ((uint32_t)v != 0u && (v >> 32) == (uint64_t)lds) return (int)(uint32_t)v;
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kern, block, lds) != hipSuccess || b <= 0) b = dflt;
    __atomic_store_n(cache, ((uint64_t)lds << 32) | (uint32_t)b, __ATOMIC_RELAXED);
    return b;
}

int grid_cap()
{
    int v = load_i(&g_grid_cap);
    if (v < 0) {
        const char *e = getenv("NC_GPUHASH_GRID");
        v = e ? atoi(e) : 0;
        if (v < 0) v = 0;
        int unset = -1; /* an explicit nc_gpuhash_set_tuning wins over the environment */
        if (!__atomic_compare_exchange_n(&g_grid_cap, &unset, v, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) v = unset;
    }
    return v;
}

bool sort_enabled()
{
    int v = load_i(&g_sort);
    if (v < 0) {
        const char *e = getenv("NC_GPUHASH_SORT");
        v = e ? (atoi(e) ? 1 : 0) : 0;
        int unset = -1;
        if (!__atomic_compare_exchange_n(&g_sort, &unset, v, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) v = unset;
    }
    return v == 1;
}

int num_cus()
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    int n = load_i(&g_num_cus[dev]);
    if (n == 0) {
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        store_i(&g_num_cus[dev], n); /* every thread stores the same value */
    }
    return n;
}

template <int MODE, bool SORT, int VAR>
hipError_t launch_kernel(const uint8_t *base, const uint64_t *off, uint64_t delta, uint64_t nkeys, uint32_t *out,
                         hipStream_t stream, int var, const WrDist &dist = WrDist{nullptr, 0u, 0u, nullptr})
{
    /* persistent grid: every resident workgroup slot once (occupancy query
     * cached per instantiation), unless a cap is set */
    void (*kern)(const uint8_t *, const uint64_t *, uint64_t, uint64_t, uint32_t *, uint64_t, WrDist);
    if constexpr ((VAR & 32) != 0) kern = nc_hash_kernel_rs<MODE, SORT, VAR>;
    else kern = nc_hash_kernel<MODE, SORT, VAR>;
    static uint64_t occ = 0;
    const int per_cu = cached_occupancy(&occ, kern, kBlock, 0, 4);
    const uint64_t ntiles = (nkeys + kTile - 1) / kTile;
    const int cap = grid_cap();
    /* kVarOver: three resident sets of workgroups instead of one. The grid
     * stride still walks every tile, but workgroups whose keys ran short
     * finish early and new ones fill their slots: with varying key lengths
     * (Zipf) this balances the CUs (C2 fnv1a_64: 0.49 -> 0.45 ms). The
     * plain hashing workgroup pipeline takes six sets (C2 fnv1a_64 0.450 ->
     * 0.443 ms, hsieh 0.451 -> 0.443, crc32 0.649 -> 0.627 in a same-process
     * grid sweep, profiles/r02_c2_grid_sweep.jsonl; four and eight sets are
     * slower than three); the sorted, register-staged and dispatch forms keep
     * three (fused ketama server_idx on C2: 0.637 ms at three sets, 0.643 at
     * six, profiles/r02f_sidx_grid_sweep.jsonl). */
    constexpr uint64_t kOverSets = (!SORT && (VAR & 32) == 0 && wg_dist<VAR>() == kDistNone) ? 6u : 3u;
    const uint64_t over = (var & kVarOver) ? kOverSets : 1u;
    uint64_t grid = cap > 0 ? (uint64_t)cap : (uint64_t)num_cus() * (uint64_t)per_cu * over;
    if (grid > ntiles) grid = ntiles;
    (void)hipGetLastError(); /* a stale error from another library's call must not be reported as ours */
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kBlock), 0, stream, base, off, delta, nkeys, out, ntiles,
                       dist);
    return hipGetLastError();
}

constexpr bool has_mul_variant(int mode) { return mode == NC_GPUHASH_FNV1A_64 || mode == NC_GPUHASH_FNV1_64; }

template <int MODE, bool SORT>
hipError_t launch_sorted(const uint8_t *base, const uint64_t *off, uint64_t delta, uint64_t nkeys, uint32_t *out,
                         hipStream_t stream, int var)
{
    /* variant bit 0: shift-add FNV multiply (FNV-64 modes); bit 3: no-hash
     * diagnostic (fnv1a_64 unsorted). The L2-prefetch distance (bits 1-2) is
     * only built into the bit-3 diagnostic: it made the pipeline slower at
     * every distance. */
    if constexpr (MODE == NC_GPUHASH_FNV1A_64 && !SORT) {
        if (var & 8) {
            switch (var & 6) {
            case 2: return launch_kernel<MODE, SORT, 10>(base, off, delta, nkeys, out, stream, var);
            case 4: return launch_kernel<MODE, SORT, 12>(base, off, delta, nkeys, out, stream, var);
            case 6: return launch_kernel<MODE, SORT, 14>(base, off, delta, nkeys, out, stream, var);
            default: return launch_kernel<MODE, SORT, 8>(base, off, delta, nkeys, out, stream, var);
            }
        }
        if (var & 16) return launch_kernel<MODE, SORT, 16>(base, off, delta, nkeys, out, stream, var);
    }
    if constexpr (MODE == NC_GPUHASH_FNV1A_64 || MODE == NC_GPUHASH_MD5) {
        if (var & 64) return (var & 32) ? launch_kernel<MODE, SORT, 32 | 64>(base, off, delta, nkeys, out, stream, var)
                                        : launch_kernel<MODE, SORT, 64>(base, off, delta, nkeys, out, stream, var);
    }
    if (var & 32) {
        if constexpr (has_mul_variant(MODE)) {
            if (var & 1) return launch_kernel<MODE, SORT, 33>(base, off, delta, nkeys, out, stream, var);
        }
        return launch_kernel<MODE, SORT, 32>(base, off, delta, nkeys, out, stream, var);
    }
    if constexpr (has_mul_variant(MODE)) {
        if (var & 1) return launch_kernel<MODE, SORT, 1>(base, off, delta, nkeys, out, stream, var);
    }
    return launch_kernel<MODE, SORT, 0>(base, off, delta, nkeys, out, stream, var);
}

template <int MODE>
hipError_t launch_mode(const uint8_t *base, const uint64_t *off, uint64_t delta, uint64_t nkeys, uint32_t *out,
                       hipStream_t stream, bool sort, int var)
{
    return sort ? launch_sorted<MODE, true>(base, off, delta, nkeys, out, stream, var)
                : launch_sorted<MODE, false>(base, off, delta, nkeys, out, stream, var);
}

/* One grouped-workgroup launch (variant bit 25): a persistent grid of
 * `sets` resident sets of workgroups (bits 21-22: 6, 1, 3, 8), so
 * workgroups whose tiles ran short hand their slots to new ones. */
template <int MODE, int VAR, int D, bool CS = false, int TK = 256, int RSV = 0>
hipError_t launch_gs(const uint8_t *base, const uint64_t *off, uint64_t delta, uint64_t nkeys, uint32_t *out,
                     hipStream_t stream, int var, const WrDist &dist = WrDist{nullptr, 0u, 0u, nullptr},
                     size_t dyn_lds = 0)
{
    void (*kern)(const uint8_t *, const uint64_t *, uint64_t, uint64_t, uint32_t *, uint64_t, WrDist);
    if constexpr (RSV > 0) kern = nc_hash_kernel_gs_rsv<MODE, VAR, D, CS, TK, RSV>;
    else kern = nc_hash_kernel_gs<MODE, VAR, D, CS, TK, RSV>;
    /* occupancy per instantiation and dynamic LDS size (the LDS continuum's) */
    static uint64_t occ = 0;
    const int per_cu = cached_occupancy(&occ, kern, TK, dyn_lds, 4);
    static const uint64_t kSets[4] = {6, 1, 3, 8};
    const uint64_t ntiles = (nkeys + TK - 1) / TK;
    const int cap = grid_cap();
    uint64_t grid = cap > 0 ? (uint64_t)cap : (uint64_t)num_cus() * (uint64_t)per_cu * kSets[(var >> 21) & 3];
    if (grid > ntiles) grid = ntiles;
    (void)hipGetLastError();
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(TK), dyn_lds, stream, base, off, delta, nkeys, out, ntiles,
                       dist);
    return hipGetLastError();
}

/* bit 20: DIAGNOSTIC no-hash build (fnv1a_64 only; outputs are not hashes);
 * bit 23: three slab buffers (two slabs in flight) */
template <int MODE>
hipError_t launch_gs_mode(const uint8_t *base, const uint64_t *off, uint64_t delta, uint64_t nkeys, uint32_t *out,
                          hipStream_t stream, int var)
{
    const bool d3 = (var & (1 << 23)) != 0;
    if constexpr (MODE == NC_GPUHASH_FNV1A_64) {
        if (var & (1 << 20)) {
            if ((var & kVarGsortCs) && (var & kVarGsort512))
                return launch_gs<MODE, 8, 2, true, 512>(base, off, delta, nkeys, out, stream, var);
            if (var & kVarGsortCs) return launch_gs<MODE, 8, 2, true>(base, off, delta, nkeys, out, stream, var);
            return d3 ? launch_gs<MODE, 8, 3>(base, off, delta, nkeys, out, stream, var)
                      : launch_gs<MODE, 8, 2>(base, off, delta, nkeys, out, stream, var);
        }
    }
    if (var & kVarGsortCs) { /* the previous tile's hashes as one coalesced store */
        if ((var & kVarGsortIssue) != 0 && (var & kVarGsort512) != 0) /* A/B: DMAs before the store */
            return launch_gs<MODE, 64, 2, true, 512>(base, off, delta, nkeys, out, stream, var);
        if constexpr (MODE == NC_GPUHASH_FNV1A_64) { /* DIAGNOSTIC A/B (bits 29-30): occupancy vs slab size */
            if ((var & kVarGsort512) != 0 && (var & (3 << 29)) == (3 << 29)) /* both: the 5 KiB as dynamic LDS */
                return launch_gs<MODE, 0, 2, true, 512, 5136>(base, off, delta, nkeys, out, stream, var,
                                                              WrDist{nullptr, 0u, 0u, nullptr}, 5136);
            if ((var & kVarGsort512) != 0 && (var & (1 << 29)) != 0) /* 6400 B of unused dynamic LDS */
                return launch_gs<MODE, 0, 2, true, 512>(base, off, delta, nkeys, out, stream, var,
                                                        WrDist{nullptr, 0u, 0u, nullptr}, 6400);
            if ((var & kVarGsort512) != 0 && (var & (1 << 30)) != 0) /* a 5 KiB smaller slab budget */
                return launch_gs<MODE, 0, 2, true, 512, 5120>(base, off, delta, nkeys, out, stream, var);
        }
        if (var & kVarGsort512) /* 512-key tiles, eight waves, length octiles */
            return launch_gs<MODE, 0, 2, true, 512>(base, off, delta, nkeys, out, stream, var);
        return d3 ? launch_gs<MODE, 0, 3, true>(base, off, delta, nkeys, out, stream, var)
                  : launch_gs<MODE, 0, 2, true>(base, off, delta, nkeys, out, stream, var);
    }
    return d3 ? launch_gs<MODE, 0, 3>(base, off, delta, nkeys, out, stream, var)
              : launch_gs<MODE, 0, 2>(base, off, delta, nkeys, out, stream, var);
}

/* One wave-ring launch: a persistent grid of every resident workgroup slot
 * (occupancy cached per instantiation and LDS size) unless capped. */
template <int MODE, int VAR, int P, int DS, int DO, int DIST, int WPW, int TK = kWrTile>
hipError_t launch_wr(const uint8_t *base, const uint64_t *off, uint64_t delta, uint64_t nkeys, uint32_t *out,
                     hipStream_t stream, const WrDist &dist, size_t lds)
{
    void (*kern)(const uint8_t *, const uint64_t *, uint64_t, uint64_t, uint32_t *, uint64_t, WrDist) =
        nc_hash_kernel_wr<MODE, VAR, P, DS, DO, DIST, WPW, TK>;
    if (lds > 65536u) (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    static uint64_t occ = 0;
    const int per_cu = cached_occupancy(&occ, kern, 64 * WPW, lds, 1);
    const uint64_t ntiles = (nkeys + TK - 1) / TK;
    const uint64_t max_grid = (ntiles + WPW - 1) / WPW;
    const int cap = grid_cap();
    uint64_t grid = cap > 0 ? (uint64_t)cap : (uint64_t)num_cus() * (uint64_t)per_cu;
    if (grid > max_grid) grid = max_grid;
    (void)hipGetLastError(); /* a stale error from another library's call must not be reported as ours */
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * WPW), lds, stream, base, off, delta, nkeys, out, ntiles,
                       dist);
    return hipGetLastError();
}

template <int MODE, int VAR, int P, int DS, int DO, int WPW = 1, int TK = kWrTile>
hipError_t launch_wr_plain(const uint8_t *base, const uint64_t *off, uint64_t delta, uint64_t nkeys, uint32_t *out,
                           hipStream_t stream)
{
    const WrDist none{nullptr, 0u, 0u, nullptr};
    return launch_wr<MODE, VAR, P, DS, DO, kDistNone, WPW, TK>(base, off, delta, nkeys, out, stream, none,
                                                               wr_lds_fixed<MODE, kDistNone, P, DS, DO, WPW, TK, VAR>());
}

/* Wave-ring options, built for fnv1a_64 and md5 only: bit 11 = four waves per
 * workgroup (one per SIMD), bit 12 = pair-interleaved hashing, bit 13 =
 * 64-key tiles, bit 14 = 256-key tiles hashed in length-sorted rounds (the
 * shape policy's md5 choice for short varying keys), bit 15 = 128-key tiles
 * in two sorted rounds; bits 8-10 the shape */
template <int MODE, int VAR>
hipError_t launch_wr_x(const uint8_t *base, const uint64_t *off, uint64_t delta, uint64_t nkeys, uint32_t *out,
                       hipStream_t stream, int var)
{
    const bool w4 = (var & 2048) != 0;
    if (var & 32768) /* 128-key tiles in two length-sorted rounds, 3 KiB slots (ties the workgroup x3 on C2) */
        return w4 ? launch_wr_plain<MODE, VAR | 4, 3, 1, 2, 4>(base, off, delta, nkeys, out, stream)
                  : launch_wr_plain<MODE, VAR | 4, 3, 1, 2, 1>(base, off, delta, nkeys, out, stream);
    if (var & 16384) { /* 256-key tiles sorted by length, four rounds per wave */
        switch ((var >> 8) & 7) {
        case 1: return w4 ? launch_wr_plain<MODE, VAR, 8, 1, 2, 4, 256>(base, off, delta, nkeys, out, stream)
                          : launch_wr_plain<MODE, VAR, 8, 1, 2, 1, 256>(base, off, delta, nkeys, out, stream);
        case 3: return w4 ? launch_wr_plain<MODE, VAR, 6, 2, 3, 4, 256>(base, off, delta, nkeys, out, stream)
                          : launch_wr_plain<MODE, VAR, 6, 2, 3, 1, 256>(base, off, delta, nkeys, out, stream);
        case 7: return w4 ? launch_wr_plain<MODE, VAR, 5, 1, 2, 4, 256>(base, off, delta, nkeys, out, stream)
                          : launch_wr_plain<MODE, VAR, 5, 1, 2, 1, 256>(base, off, delta, nkeys, out, stream);
        default: return w4 ? launch_wr_plain<MODE, VAR, 6, 1, 2, 4, 256>(base, off, delta, nkeys, out, stream)
                           : launch_wr_plain<MODE, VAR, 6, 1, 2, 1, 256>(base, off, delta, nkeys, out, stream);
        }
    }
    if (var & 8192) { /* 64-key tiles, one key per lane */
        switch ((var >> 8) & 7) {
        case 1: return w4 ? launch_wr_plain<MODE, VAR, 2, 1, 2, 4, 64>(base, off, delta, nkeys, out, stream)
                          : launch_wr_plain<MODE, VAR, 2, 1, 2, 1, 64>(base, off, delta, nkeys, out, stream);
        case 3: return w4 ? launch_wr_plain<MODE, VAR, 3, 2, 3, 4, 64>(base, off, delta, nkeys, out, stream)
                          : launch_wr_plain<MODE, VAR, 3, 2, 3, 1, 64>(base, off, delta, nkeys, out, stream);
        case 7: return w4 ? launch_wr_plain<MODE, VAR, 2, 3, 5, 4, 64>(base, off, delta, nkeys, out, stream)
                          : launch_wr_plain<MODE, VAR, 2, 3, 5, 1, 64>(base, off, delta, nkeys, out, stream);
        default: return w4 ? launch_wr_plain<MODE, VAR, 2, 2, 3, 4, 64>(base, off, delta, nkeys, out, stream)
                           : launch_wr_plain<MODE, VAR, 2, 2, 3, 1, 64>(base, off, delta, nkeys, out, stream);
        }
    }
    switch ((var >> 8) & 7) {
    case 1: return w4 ? launch_wr_plain<MODE, VAR, 4, 1, 2, 4>(base, off, delta, nkeys, out, stream)
                      : launch_wr_plain<MODE, VAR, 4, 1, 2, 1>(base, off, delta, nkeys, out, stream);
    case 3: return w4 ? launch_wr_plain<MODE, VAR, 5, 2, 3, 4>(base, off, delta, nkeys, out, stream)
                      : launch_wr_plain<MODE, VAR, 5, 2, 3, 1>(base, off, delta, nkeys, out, stream);
    case 7: return w4 ? launch_wr_plain<MODE, VAR, 3, 1, 2, 4>(base, off, delta, nkeys, out, stream)
                      : launch_wr_plain<MODE, VAR, 3, 1, 2, 1>(base, off, delta, nkeys, out, stream);
    default: return w4 ? launch_wr_plain<MODE, VAR, 4, 2, 3, 4>(base, off, delta, nkeys, out, stream)
                       : launch_wr_plain<MODE, VAR, 4, 2, 3, 1>(base, off, delta, nkeys, out, stream);
    }
}

/* plain hashing on the wave ring; variant bits 8-10 pick the ring shape
 * (P KiB slab slots, slabs DS and offsets DO tiles ahead) */
template <int MODE, int VAR>
hipError_t launch_wr_hash(const uint8_t *base, const uint64_t *off, uint64_t delta, uint64_t nkeys, uint32_t *out,
                          hipStream_t stream, int var)
{
    switch ((var >> 8) & 7) {
    case 1: return launch_wr_plain<MODE, VAR, 4, 1, 2>(base, off, delta, nkeys, out, stream);
    case 2: return launch_wr_plain<MODE, VAR, 4, 3, 5>(base, off, delta, nkeys, out, stream);
    case 3: return launch_wr_plain<MODE, VAR, 5, 2, 3>(base, off, delta, nkeys, out, stream);
    case 4: return launch_wr_plain<MODE, VAR, 6, 2, 3>(base, off, delta, nkeys, out, stream);
    case 5: return launch_wr_plain<MODE, VAR, 5, 1, 2>(base, off, delta, nkeys, out, stream);
    case 6: return launch_wr_plain<MODE, VAR, 3, 2, 3>(base, off, delta, nkeys, out, stream);
    case 7: return launch_wr_plain<MODE, VAR, 3, 1, 2>(base, off, delta, nkeys, out, stream);
    default: return launch_wr_plain<MODE, VAR, 4, 2, 3>(base, off, delta, nkeys, out, stream);
    }
}

template <int MODE>
hipError_t launch_wr_mode(const uint8_t *base, const uint64_t *off, uint64_t delta, uint64_t nkeys, uint32_t *out,
                          hipStream_t stream, int var)
{
    if constexpr (MODE == NC_GPUHASH_FNV1A_64 || MODE == NC_GPUHASH_MD5) {
        if (var & (2048 | 4096 | 8192 | 16384 | 32768)) {
            if ((var & 4096) && !(var & 16384)) return launch_wr_x<MODE, 512>(base, off, delta, nkeys, out, stream, var);
            return launch_wr_x<MODE, 0>(base, off, delta, nkeys, out, stream, var);
        }
        if (var & 8) { /* DIAGNOSTIC no-hash build: default and P5 ring shapes only */
            if (((var >> 8) & 7) == 3) return launch_wr_plain<MODE, 8, 5, 2, 3>(base, off, delta, nkeys, out, stream);
            if (((var >> 8) & 7) == 7) return launch_wr_plain<MODE, 8, 3, 1, 2>(base, off, delta, nkeys, out, stream);
            return launch_wr_plain<MODE, 8, 4, 2, 3>(base, off, delta, nkeys, out, stream);
        }
    }
    if constexpr (has_mul_variant(MODE)) { /* shift-add multiply: default ring shape only */
        if (var & 1) return launch_wr_plain<MODE, 1, 4, 2, 3>(base, off, delta, nkeys, out, stream);
    }
    if constexpr (uses_crc_table<MODE>()) {
        /* bit 11: slicing-by-16 tables (16 KiB) shared by the workgroup's
         * waves; bits 12-13 the ring: P5 x 7 waves, P5 x 6, P5 x 4, P4 x 8 */
        if (var & 2048) {
            constexpr int V = kHkCrcSliced;
            switch ((var >> 12) & 3) {
            case 0: return launch_wr_plain<MODE, V, 5, 2, 3, 7>(base, off, delta, nkeys, out, stream);
            case 1: return launch_wr_plain<MODE, V, 5, 2, 3, 6>(base, off, delta, nkeys, out, stream);
            case 2: return launch_wr_plain<MODE, V, 5, 2, 3, 4>(base, off, delta, nkeys, out, stream);
            default: return launch_wr_plain<MODE, V, 4, 2, 3, 8>(base, off, delta, nkeys, out, stream);
            }
        }
    }
    return launch_wr_hash<MODE, 0>(base, off, delta, nkeys, out, stream, var);
}

} // namespace

#ifdef NC_TU_MODE
template <int MODE>
hipError_t nc_tu::entry(const uint8_t *base, const uint64_t *off, uint64_t delta, uint64_t nkeys, uint32_t *out,
                        hipStream_t stream, bool sort, int var)
{
    if ((var & kVarGsort) != 0) return launch_gs_mode<MODE>(base, off, delta, nkeys, out, stream, var);
    if ((var & 128) != 0) return launch_wr_mode<MODE>(base, off, delta, nkeys, out, stream, var);
    return launch_mode<MODE>(base, off, delta, nkeys, out, stream, sort, var);
}
template hipError_t nc_tu::entry<NC_TU_MODE>(const uint8_t *, const uint64_t *, uint64_t, uint64_t, uint32_t *,
                                             hipStream_t, bool, int);

/* The continuum is staged in LDS next to four waves' rings when it fits
 * (ketama: 160 points per server, src/hashkit/nc_ketama.c:26-27, so up to
 * ~100 servers); a larger one takes the hash-then-dispatch pair of launches,
 * the second reading the continuum through L2. */
namespace {
/* ketama / modula over the pre-dispatch hashes in out, in place */
hipError_t dispatch_launch(const nc_tu::DistArgs &d, uint32_t *out, uint64_t nkeys, hipStream_t stream)
{
    uint64_t grid = (nkeys + 255u) / 256u;
    const uint64_t cap = (uint64_t)num_cus() * 8u;
    if (grid > cap) grid = cap;
    (void)hipGetLastError();
    if (d.kind == 0)
        hipLaunchKernelGGL(nc_dispatch_kernel<kDistKetama>, dim3((unsigned)grid), dim3(256), 0, stream, d.cont, d.ncont,
                           out, nkeys);
    else
        hipLaunchKernelGGL(nc_dispatch_kernel<kDistModula>, dim3((unsigned)grid), dim3(256), 0, stream, d.cont, d.ncont,
                           out, nkeys);
    return hipGetLastError();
}

/* server_pool_idx on ring shape <P, DS, DO>, four waves per workgroup */
template <int MODE, int P, int DS, int DO>
hipError_t dist_launch(const uint8_t *base, const uint64_t *off, uint64_t delta, uint64_t nkeys, uint32_t *out,
                       hipStream_t stream, const nc_tu::DistArgs &d)
{
    constexpr int WPW = 4;
    constexpr size_t kMaxLds = 160u * 1024u;
    const WrDist wd{d.cont, d.ncont, d.tag, d.lut, d.lut_shift};
    const size_t fixed = wr_lds_fixed<MODE, kDistKetama, P, DS, DO, WPW>();
    const size_t lds = fixed + 8u * (size_t)d.ncont + (d.kind == 0 ? kBktBytes : 0u);
    if (lds <= kMaxLds) {
        return d.kind == 0 ? launch_wr<MODE, 0, P, DS, DO, kDistKetama, WPW>(base, off, delta, nkeys, out, stream, wd, lds)
                           : launch_wr<MODE, 0, P, DS, DO, kDistModula, WPW>(base, off, delta, nkeys, out, stream, wd, lds);
    }
    hipError_t e = launch_wr<MODE, 0, P, DS, DO, kDistPre, WPW>(base, off, delta, nkeys, out, stream, wd, fixed);
    if (e != hipSuccess) return e;
    return dispatch_launch(d, out, nkeys, stream);
}
} // namespace

template <int MODE>
hipError_t nc_tu::entry_dist(const uint8_t *base, const uint64_t *off, uint64_t delta, uint64_t nkeys,
                             uint32_t *out, hipStream_t stream, const DistArgs &d)
{
    if constexpr (!uses_crc_table<MODE>()) { /* the crc modes need the workgroup's LDS table slot */
        if (d.gs) {
            const WrDist wd{d.cont, d.ncont, d.tag, d.lut, d.lut_shift};
            if constexpr (MODE != NC_GPUHASH_MD5) { /* md5's registers do not fit eight waves per SIMD */
                if (d.kind == 0 && d.lds_cont && d.ncont <= kLdsPackedMax && (d.gs_var & kVarNoPacked) == 0) {
                    /* packed words within a 5 KiB reserve of the 512-key
                     * tiles' budget: four workgroups per CU, as without a
                     * dispatch */
                    const int sets = (d.gs_var & (3 << 21)) != 0 ? d.gs_var : (d.gs_var | (2 << 21));
                    constexpr int kR = (kLdsPackedMax + 8) * 4;
                    const size_t dyn = ((size_t)d.ncont + 8u) * 4u;
                    if constexpr (MODE == NC_GPUHASH_FNV1A_64) { /* DIAGNOSTIC (tuning bits 19 / 20): what the
                                                                    dispatch costs — no hash_tag code / no search */
                        switch ((d.gs_var >> 19) & 3) {
                        case 1: return launch_gs<MODE, (5 << 12) | 256, 2, true, 512, kR>(base, off, delta, nkeys, out,
                                                                                            stream, sets, wd, dyn);
                        case 2: return launch_gs<MODE, (5 << 12) | 128, 2, true, 512, kR>(base, off, delta, nkeys, out,
                                                                                            stream, sets, wd, dyn);
                        case 3:
                            if (d.gs_var & (1 << 26)) /* ... and no continuum staging in the prologue */
                                return launch_gs<MODE, (5 << 12) | 896, 2, true, 512, kR>(base, off, delta, nkeys, out,
                                                                                            stream, sets, wd, dyn);
                            return launch_gs<MODE, (5 << 12) | 384, 2, true, 512, kR>(base, off, delta, nkeys, out,
                                                                                            stream, sets, wd, dyn);
                        default: break;
                        }
                    }
                    return launch_gs<MODE, 5 << 12, 2, true, 512, kR>(base, off, delta, nkeys, out, stream, sets, wd,
                                                                       dyn);
                }
            }
            if (d.kind == 0 && d.lds_cont) { /* values + u8 servers in dynamic LDS */
                const size_t vb = (size_t)d.ncont * 4u + (((size_t)d.ncont + 15u) & ~(size_t)15u);
                if (d.gs_var & kVarGsort512) /* A/B: 512-key tiles (slower: three workgroups per CU) */
                    return launch_gs<MODE, 4 << 12, 2, true, 512>(base, off, delta, nkeys, out, stream, d.gs_var, wd,
                                                                   vb);
                return launch_gs<MODE, 4 << 12, 2, true>(base, off, delta, nkeys, out, stream, d.gs_var, wd, vb);
            }
            if (d.kind == 0 && d.lut != nullptr)
                return launch_gs<MODE, 3 << 12, 2, true>(base, off, delta, nkeys, out, stream, d.gs_var, wd);
            return d.kind == 0 ? launch_gs<MODE, 1 << 12, 2, true>(base, off, delta, nkeys, out, stream, d.gs_var, wd)
                               : launch_gs<MODE, 2 << 12, 2, true>(base, off, delta, nkeys, out, stream, d.gs_var, wd);
        }
        if (d.wg) {
            const WrDist wd{d.cont, d.ncont, d.tag, d.lut, d.lut_shift};
            if (d.kind == 0 && d.lut != nullptr)
                return launch_kernel<MODE, false, 3 << 12>(base, off, delta, nkeys, out, stream, kVarOver, wd);
            return d.kind == 0 ? launch_kernel<MODE, false, 1 << 12>(base, off, delta, nkeys, out, stream, kVarOver, wd)
                               : launch_kernel<MODE, false, 2 << 12>(base, off, delta, nkeys, out, stream, kVarOver, wd);
        }
    }
    return d.wide ? dist_launch<MODE, 5, 2, 3>(base, off, delta, nkeys, out, stream, d)
                  : dist_launch<MODE, 3, 1, 2>(base, off, delta, nkeys, out, stream, d);
}
template hipError_t nc_tu::entry_dist<NC_TU_MODE>(const uint8_t *, const uint64_t *, uint64_t, uint64_t, uint32_t *,
                                                  hipStream_t, const DistArgs &);
#else /* the C ABI */

int nc_tu::g_grid_cap = -1;
int nc_tu::g_sort = -1;
int nc_tu::g_variant = 0;
int nc_tu::g_num_cus[64];

namespace {

/* Kernel choice of the auto policy (g_variant == 0) from the batch shape,
 * measured on MI355X over fixed 8-256 B, Zipf 8-64 B and uniform 8-64 B key
 * sets (profiles/r01_policy_sweep.txt). Every choice gives
 * identical outputs. */
int pick_variant(int mode, uint64_t nkeys, const nc_gpuhash_shape *sh)
{
    if (mode == NC_GPUHASH_MD5) {
        /* the direct per-lane block pipeline for every shape; keys of 64+ bytes
         * on average take its LDS-DMA variant (option bit 2 = variant bit 22),
         * whose 64-byte pieces spare the texture addresser (C4 shard 3.1 ->
         * 2.1 ms, 128-byte keys 0.80 -> 0.62 ms; short keys are faster direct) */
        const bool lds = sh != nullptr && nkeys != 0 && sh->key_bytes / nkeys >= 64u;
        /* ... with a wave's tiles interleaved over the grid (option bit 3):
         * C4 shard 1.822-1.857 -> 1.803-1.830 ms in two same-box A/Bs
         * (profiles/r04_lines_chunk_ab.jsonl, r04_crc_bytetable_ab.jsonl) */
        /* ... and the per-lane padding selectors from the 512-byte LDS table
         * (pad_block_tab): C2 SQ_INSTS_VALU 443 M -> 408 M per launch,
         * 0.7319 -> 0.7259 and 0.7345 -> 0.7278 ms on two boxes
         * (profiles/r05_md5_padtab_ab.jsonl, pmc_r05_md5pt.json); and
         * whole-line output stores (the tail keys store a placeholder first,
         * nc_md5_kernels.hip FS): C2 0.7333 -> 0.7048 ms, same box, same
         * process (profiles/r06f_md5_fullline_ab.jsonl); with a shape whose
         * keys are <= 64 B, the S64 form (no chaining state): C2
         * SQ_INSTS_VALU 400.7 M -> 383.4 M, 0.7184 -> 0.7123 ms
         * (profiles/r06s_md5_s64_ab.jsonl, pmc_r06s_md5_s64_valu.json) */
        return kVarMd5Direct | (lds ? (12 << 20) : kVarMd5PadTab | kVarMd5FullLines);
    }
    if (sh == nullptr || nkeys == 0 || sh->key_bytes == 0) return kVarRegStaged;
    const uint64_t mean = sh->key_bytes / nkeys;
    const bool fixed = sh->max_len >= sh->min_len && sh->max_len - sh->min_len <= 4u;
    const bool crc = mode == NC_GPUHASH_CRC16 || mode == NC_GPUHASH_CRC32 || mode == NC_GPUHASH_CRC32A;
    const bool fnv_like = mode == NC_GPUHASH_FNV1_64 || mode == NC_GPUHASH_FNV1A_64 || mode == NC_GPUHASH_FNV1_32 ||
                          mode == NC_GPUHASH_FNV1A_32 || mode == NC_GPUHASH_HSIEH || mode == NC_GPUHASH_MURMUR;
    /* the byte-serial modes of the direct pipeline (nc_bytes_kernels.hip) */
    const bool direct_bytes = crc || mode == NC_GPUHASH_ONE_AT_A_TIME || mode == NC_GPUHASH_FNV1_64 ||
                              mode == NC_GPUHASH_FNV1A_64 || mode == NC_GPUHASH_FNV1_32 || mode == NC_GPUHASH_FNV1A_32;
    if (mean >= 80u) {
        /* long keys: the direct pipeline's LDS-DMA block image (C4 shard
         * crc32 3.56 -> 2.24 ms, fnv1a_64 3.06 -> 2.15, one_at_a_time 3.22 ->
         * 2.48; 128-byte keys 0.79 -> 0.62 ms); the word modes keep the wave
         * ring, deeper or wider slab slots */
        /* interleaved: C4 shard 1.92 -> 1.84 ms (crc32), 1.75 -> 1.66 (fnv1a_64);
         * the fnvs at half the resident waves, 1.55 -> 1.52 (their streams
         * contend for HBM; crc32's table lookups need the waves: 1.83 -> 2.22,
         * profiles/r04_lines_occupancy_ab.jsonl) */
        /* ... and, from 160-byte keys on average, the fnvs' rounds take two
         * lines of every key (twice the bytes in flight per wave): C4 shard
         * fnv1a_64 1.622 -> 1.542 ms, fnv1_32 1.625 -> 1.542, uniform
         * 80-400 B 1.241 -> 1.129; fixed 128 B keys lose (0.429 -> 0.491: half
         * of each round's image idle) (profiles/r05_c4_pairs_ab.jsonl,
         * r05_c4_pairs_crc_ab.jsonl) */
        const bool fnv = mode == NC_GPUHASH_FNV1_64 || mode == NC_GPUHASH_FNV1A_64 || mode == NC_GPUHASH_FNV1_32 ||
                         mode == NC_GPUHASH_FNV1A_32;
        if (direct_bytes)
            return kVarDirect | kVarDirectLds | kVarDirectIl32 |
                   (fnv ? kVarDirect8 | (mean >= 160u ? kVarDirectPairs : 0) : 0);
        if (mode == NC_GPUHASH_HSIEH) return kVarRingP5;
        return kVarRingP4;
    }
    /* fixed-length keys of 20-32 bytes (C3): the direct pipeline's short-key
     * kernel (eight waves per CU, persistent, three tiles in flight per wave)
     * for crc32 / crc32a (slicing-by-8 tables) and one_at_a_time: C3 crc32
     * 0.578 -> 0.541 ms, crc32a 0.580 -> 0.541, one_at_a_time 0.581 -> 0.525
     * (profiles/r05_c3_short8_ab2.jsonl); crc16 0.580 -> 0.603 keeps the
     * 32-wave kernel, the fnvs tie the wave ring (0.522-0.529) and keep it */
    if (fixed && mean >= 20u && sh->max_len <= 32u &&
        (mode == NC_GPUHASH_CRC32 || mode == NC_GPUHASH_CRC32A || mode == NC_GPUHASH_ONE_AT_A_TIME))
        return kVarDirect | kVarDirectShort | (2 << 20) | (mode == NC_GPUHASH_ONE_AT_A_TIME ? 0 : (1 << 22));
    /* ... and murmur, one tile in flight: 0.541 -> 0.517 ms (hsieh keeps the
     * ring, 0.509 vs 0.521; jenkins the register-staged pipeline, 0.601 vs
     * 0.648: its mix chain needs more than two waves per SIMD;
     * profiles/r05_c3_short_words_ab.jsonl) */
    if (fixed && mean >= 20u && sh->max_len <= 32u && mode == NC_GPUHASH_MURMUR)
        return kVarDirect | kVarDirectShort | (1 << 20);
    /* crc16 at SIXTEEN waves per CU on the same kernel (its chain needs the
     * waves; slicing-by-4, two tiles in flight): 0.575-0.577 -> 0.549-0.550 ms
     * (profiles/r05_c3_short16_ab.jsonl, r05_c3_crc16_fl32_ab.jsonl; crc32
     * ties, one_at_a_time loses 7 %, jenkins ties the register-staged
     * pipeline at 1.056 x the algorithmic bytes instead of 1.028,
     * r05b_modes_c3.json, and keeps it) */
    if (fixed && mean >= 20u && sh->max_len <= 32u && mode == NC_GPUHASH_CRC16)
        return kVarDirect | kVarDirectShort | kVarDirect8;
    /* ... and jenkins (round 6): 0.5974 -> 0.5858 ms against its
     * register-staged pipeline, same process; one to three tiles in flight
     * within 0.4 % (profiles/r06j_c3_jenkins_short16_ab.jsonl) */
    if (fixed && mean >= 20u && sh->max_len <= 32u && mode == NC_GPUHASH_JENKINS)
        return kVarDirect | kVarDirectShort | kVarDirect8;
    /* fixed-length short keys: the crcs' slicing-by-4 tables on the direct
     * pipeline (C3: 0.70 -> 0.61 ms); varying lengths keep the length-grouped
     * workgroup pipelines (a direct wave runs to its longest key) */
    if (crc && fixed && mean <= 64u) return kVarDirect | kVarDirectIl32; /* interleaved: C3 crc32 0.62 -> 0.575 ms */
    if (fixed) {
        if (mean >= 20u && mean <= 40u) { /* C3 */
            if (fnv_like) return kVarRingP5;
            return kVarRegStaged;
        }
        if (mean < 20u) return kVarWorkgroup;
        return kVarRegStaged;
    }
    /* varying lengths: a wave runs as long as its longest key; length-grouped
     * tiles and oversubscribed grids rebalance that */
    if (mean < 22u) { /* C2 */
        /* the grouped workgroup pipeline (each wave hashes one length
         * quartile of the tile; its 6.5 KiB slab holds a 256-key tile up to
         * ~25 B per key) with one coalesced store per tile: C2 fnv x4
         * 0.449-0.454 -> 0.429-0.431 ms, hsieh 0.447 -> 0.433, murmur 0.435
         * -> 0.425, jenkins 0.526 -> 0.445, crc16 0.690 -> 0.645, and the
         * coalesced store a further 3.5 % on fnv1a_64 (0.452 -> 0.436 on
         * one box); one_at_a_time 0.504 (wave-sorted) -> 0.476 at three
         * resident sets (profiles/r03_c2_gsort.jsonl); crc32 / crc32a tie the
         * workgroup x6 and keep it */
        if (mode == NC_GPUHASH_CRC32 || mode == NC_GPUHASH_CRC32A) return kVarWorkgroup | kVarOver;
        /* 512-key tiles of eight waves, length octiles: fnv1a_64 0.431 ->
         * 0.409 ms, murmur 0.436 -> 0.403 at three resident sets,
         * one_at_a_time 0.473 -> 0.465 at six; crc16 (its 1 KiB table),
         * hsieh and jenkins keep 256-key tiles (0.662 vs 0.812, 0.414 vs
         * 0.417, 0.450 vs 0.459; profiles/r03_c2_gsort.jsonl) */
        if (mode == NC_GPUHASH_CRC16 || mode == NC_GPUHASH_HSIEH || mode == NC_GPUHASH_JENKINS)
            return kVarGsort | kVarGsortCs;
        /* one_at_a_time (the most VALU per byte) issues a tile's DMAs before
         * the previous tile's store: 0.464 -> 0.453 ms; fnv x4 / murmur lose
         * ~1 % that way (profiles/r03_c2_gs_ab.jsonl) */
        if (mode == NC_GPUHASH_ONE_AT_A_TIME) return kVarGsort | kVarGsortCs | kVarGsort512 | kVarGsortIssue;
        /* the fnvs at six resident sets, murmur at three: fnv1a_64 0.4186 ->
         * 0.4119-0.4145 ms on one box, 0.4131 -> 0.4118 on another, fnv1_32
         * 0.4129 -> 0.4111, murmur 0.4077 -> 0.4095
         * (profiles/r04_c2_gs_sets_ab.jsonl) */
        if (mode == NC_GPUHASH_MURMUR) return kVarGsort | kVarGsortCs | kVarGsort512 | (2 << 21);
        return kVarGsort | kVarGsortCs | kVarGsort512;
    }
    if (crc || mode == NC_GPUHASH_ONE_AT_A_TIME) return kVarRegStaged | kVarOver;
    return kVarRegStaged;
}

hipError_t launch(int mode, const uint8_t *d_keys, const uint64_t *d_off, uint64_t nkeys, uint32_t *d_out,
                  hipStream_t stream, const nc_gpuhash_shape *shape)
{
    const uintptr_t kp = reinterpret_cast<uintptr_t>(d_keys);
    const uint8_t *base = reinterpret_cast<const uint8_t *>(kp & ~(uintptr_t)15);
    const uint64_t delta = (uint64_t)(kp & 15u);
    const int tuned = load_i(&g_variant);
    int var = tuned != 0 ? tuned : pick_variant(mode, nkeys, shape);
    if ((var & kVarDirect) != 0 && nkeys < (1ull << 32)) { /* bits 20-23: options */
        if (mode == NC_GPUHASH_MD5) {
            /* fixed-length keys (the caller's shape; bit 26 turns it off for A/B) */
            const uint32_t fl = shape != nullptr && nkeys != 0 && shape->min_len == shape->max_len &&
                                        (var & kVarNoFixedLen) == 0
                                    ? (uint32_t)shape->min_len
                                    : 0u;
            return nc_md5::launch(d_keys, d_off, nkeys, d_out, stream,
                                  ((var >> 20) & 15) | ((var & kVarMd5PadTab) != 0 ? 16 : 0) |
                                      ((var & kVarMd5FullLines) != 0 ? 32 : 0) |
                                      ((var & kVarDirectS8) != 0 ? 64 : 0) | ((var & kVarDirectNoHash) != 0 ? 128 : 0),
                                  fl,
                                  shape != nullptr && nkeys != 0 && shape->max_len <= 0xffffffffull
                                      ? (uint32_t)shape->max_len
                                      : 0xffffffffu);
        }
        const bool short_words = (var & kVarDirectShort) != 0 && nc_bytes::supports_short_words(mode) &&
                                 shape != nullptr && nkeys != 0 && shape->max_len <= 32u;
        if (nc_bytes::supports(mode) || short_words)
            return nc_bytes::launch(mode, d_keys, d_off, nkeys, d_out, stream,
                                    ((var >> 20) & 15) | ((var & kVarDirect8) != 0 ? 16 : 0) |
                                        ((var & kVarDirectS8) != 0 ? 32 : 0) | ((var & kVarDirectNoHash) != 0 ? 64 : 0) |
                                        ((var & kVarDirectShort) != 0 ? 128 : 0) | ((var & kVarDirectPairs) != 0 ? 256 : 0) |
                                        ((var & kVarDirectOffDefault) != 0 ? 512 : 0),
                                    shape != nullptr && nkeys != 0 ? (uint32_t)shape->max_len : 0xffffffffu);
    }
    if ((var & kVarWsort) != 0 && nkeys < (1ull << 32) && nc_wsort::supports(mode))
        return nc_wsort::launch(mode, d_keys, d_off, nkeys, d_out, stream, (var >> 20) & 15);
    if ((var & kVarGsort) != 0) {
        switch (mode) {
#define NC_CASE(M) \
    case M: return nc_tu::entry<M>(base, d_off, delta, nkeys, d_out, stream, false, var);
            NC_CASE(NC_GPUHASH_ONE_AT_A_TIME)
            NC_CASE(NC_GPUHASH_MD5)
            NC_CASE(NC_GPUHASH_CRC16)
            NC_CASE(NC_GPUHASH_CRC32)
            NC_CASE(NC_GPUHASH_CRC32A)
            NC_CASE(NC_GPUHASH_FNV1_64)
            NC_CASE(NC_GPUHASH_FNV1A_64)
            NC_CASE(NC_GPUHASH_FNV1_32)
            NC_CASE(NC_GPUHASH_FNV1A_32)
            NC_CASE(NC_GPUHASH_HSIEH)
            NC_CASE(NC_GPUHASH_MURMUR)
            NC_CASE(NC_GPUHASH_JENKINS)
#undef NC_CASE
        default:
            return hipErrorInvalidValue;
        }
    }
    var &= ~(kVarDirect | kVarWsort | kVarNoFixedLen | (15 << 20));
    const bool sort = sort_enabled() || (var & kVarSorted) != 0;
    var &= ~(kVarWorkgroup | kVarSorted); /* kVarOver rides along to launch_kernel */
    /* the wave ring DMAs offsets 16 bytes per lane: it needs 16-byte aligned
     * offsets (any other alignment takes the workgroup pipeline) */
    if ((var & 128) != 0 && (reinterpret_cast<uintptr_t>(d_off) & 15u) != 0) var = tuned != 0 ? 0 : 32;
    switch (mode) {
#define NC_CASE(M) \
    case M: return nc_tu::entry<M>(base, d_off, delta, nkeys, d_out, stream, sort, var);
        NC_CASE(NC_GPUHASH_ONE_AT_A_TIME)
        NC_CASE(NC_GPUHASH_MD5)
        NC_CASE(NC_GPUHASH_CRC16)
        NC_CASE(NC_GPUHASH_CRC32)
        NC_CASE(NC_GPUHASH_CRC32A)
        NC_CASE(NC_GPUHASH_FNV1_64)
        NC_CASE(NC_GPUHASH_FNV1A_64)
        NC_CASE(NC_GPUHASH_FNV1_32)
        NC_CASE(NC_GPUHASH_FNV1A_32)
        NC_CASE(NC_GPUHASH_HSIEH)
        NC_CASE(NC_GPUHASH_MURMUR)
        NC_CASE(NC_GPUHASH_JENKINS)
#undef NC_CASE
    default:
        return hipErrorInvalidValue;
    }
}

rstatus_t fail(int err)
{
    errno = err;
    return NC_ERROR;
}

/* a launch error, named on stderr when NC_GPUHASH_DEBUG is set */
rstatus_t fail_launch(hipError_t e, const char *what)
{
    if (getenv("NC_GPUHASH_DEBUG") != nullptr) fprintf(stderr, "nc_gpuhash: %s: %s\n", what, hipGetErrorString(e));
    return fail(e == hipErrorNoDevice ? ENODEV : EIO);
}

} // namespace

extern "C" rstatus_t nc_gpuhash_batch_device_shaped(int mode, const uint8_t *d_keys, const uint64_t *d_offsets,
                                                    uint64_t nkeys, uint32_t *d_out,
                                                    const struct nc_gpuhash_shape *shape, void *stream)
{
    if (mode < 0 || mode >= NC_GPUHASH_NMODES) return fail(EINVAL);
    if (nkeys == 0) return NC_OK;
    if (d_keys == nullptr || d_offsets == nullptr || d_out == nullptr) return fail(EINVAL);
    hipError_t err = launch(mode, d_keys, d_offsets, nkeys, d_out, reinterpret_cast<hipStream_t>(stream), shape);
    if (err != hipSuccess) return fail_launch(err, "nc_gpuhash_batch_device_shaped");
    return NC_OK;
}

extern "C" rstatus_t nc_gpuhash_batch_device(int mode, const uint8_t *d_keys, const uint64_t *d_offsets,
                                             uint64_t nkeys, uint32_t *d_out, void *stream)
{
    return nc_gpuhash_batch_device_shaped(mode, d_keys, d_offsets, nkeys, d_out, nullptr, stream);
}

extern "C" rstatus_t nc_gpuhash_server_idx_device(int mode, int dist, const uint8_t *d_keys,
                                                  const uint64_t *d_offsets, uint64_t nkeys,
                                                  const struct nc_gpuhash_continuum *d_continuum,
                                                  uint32_t ncontinuum, uint32_t nserver, const char *hash_tag,
                                                  const struct nc_gpuhash_shape *shape, uint32_t *d_out,
                                                  void *stream)
{
    if (mode < 0 || mode >= NC_GPUHASH_NMODES) return fail(EINVAL);
    if (dist != NC_GPUHASH_DIST_KETAMA && dist != NC_GPUHASH_DIST_MODULA) return fail(EINVAL);
    if (nserver == 0) return fail(EINVAL);
    if (nkeys == 0) return NC_OK;
    if (d_keys == nullptr || d_offsets == nullptr || d_out == nullptr) return fail(EINVAL);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (nserver == 1) { /* src/nc_server.c:655-658: no hashing, no dispatch */
        const hipError_t e = hipMemsetAsync(d_out, 0, (size_t)nkeys * sizeof(uint32_t), st);
        return e == hipSuccess ? NC_OK : fail(e == hipErrorNoDevice ? ENODEV : EIO);
    }
    if (d_continuum == nullptr || ncontinuum == 0) return fail(EINVAL);
    if ((reinterpret_cast<uintptr_t>(d_offsets) & 15u) != 0) return fail(EINVAL);
    const uintptr_t kp = reinterpret_cast<uintptr_t>(d_keys);
    const uint8_t *base = reinterpret_cast<const uint8_t *>(kp & ~(uintptr_t)15);
    const uint64_t delta = (uint64_t)(kp & 15u);
    const bool wide = shape != nullptr && shape->key_bytes > 20u * nkeys;
    /* pipeline: the workgroup pipeline (continuum in L2, bucket index in LDS)
     * for ketama pools and for any hash_tag: its eight waves per SIMD hide the
     * search's and the tag scan's latency (C3 ketama 1.22 -> 0.71 ms, C2 with
     * "{}" 1.56 -> 1.26, C2 ketama 0.69 -> 0.66), and for short keys (C2
     * modula 0.56 -> 0.53); modula without a tag on 20+ B keys keeps the wave
     * ring (one continuum read per key, ring 4-11 % ahead on C3).
     * The crc modes always take the ring (their table has the LDS slot).
     * Variant bit 29 forces the workgroup pipeline, bit 28 the ring, bit 30
     * the grouped pipeline (A/B). */
    const int tuned = load_i(&g_variant);
    bool wg = dist == NC_GPUHASH_DIST_KETAMA || hash_tag != nullptr || !wide;
    /* keys of varying length under ~22 B (C2) with a hash_tag or modula: the
     * grouped pipeline, whose waves hash one length quartile each (C2 ketama
     * with "{}" 1.307 -> 0.897 ms, modula 0.524 -> 0.496; ketama without a
     * tag ties the workgroup pipeline and keeps it, profiles/r03_sidx.jsonl) */
    const bool crc = mode == NC_GPUHASH_CRC16 || mode == NC_GPUHASH_CRC32 || mode == NC_GPUHASH_CRC32A;
    /* ketama pools whose continuum fits LDS beside the grouped pipeline's
     * tiles (values + u8 servers, up to 24 KiB: ~30 servers of 160 points)
     * take it on C2-like shapes too, the whole search in LDS */
    const bool lds_cont = dist == NC_GPUHASH_DIST_KETAMA && nserver <= 256u && ncontinuum <= kLdsContMax &&
                          (tuned & (7 << 23)) == 0;
    bool gs = !crc && shape != nullptr && shape->key_bytes != 0u && shape->key_bytes < 22u * nkeys &&
              shape->min_len != shape->max_len && (hash_tag != nullptr || dist == NC_GPUHASH_DIST_MODULA || lds_cont);
    if (tuned & (1 << 30)) gs = true;
    if (tuned & (3 << 28)) gs = false;
    if (tuned & (1 << 29)) wg = true;
    if (tuned & (1 << 28)) wg = false;
    nc_tu::DistArgs d{reinterpret_cast<const uint32_t *>(d_continuum), ncontinuum, 0u, dist, wide, wg, gs,
                      tuned & ((3 << 19) | (3 << 21) | (1 << 26) | kVarNoPacked), nullptr, 20u, gs && lds_cont};
    if (hash_tag != nullptr)
        d.tag = (uint32_t)(uint8_t)hash_tag[0] | ((uint32_t)(uint8_t)hash_tag[1] << 8) | (1u << 16);
    /* A/B only: ketama on the workgroup pipelines through a lookup table
     * over the hash's top bits, built on the stream (a few us) in
     * stream-ordered scratch, so most keys resolve with one read
     * (ketama_find_lut). Variant bit 24: 65536 entries; bit 23: 4096 (16 KiB).
     * Both lose to the bucket index's binary search without a hash tag (C2
     * 0.717 / 0.668-0.688 vs 0.659-0.661 ms, profiles/r03_sidx.jsonl): under
     * the streaming key traffic a table read is an L2 round trip whatever
     * its size. Bit 25: the bucket index without the LDS continuum. */
    uint32_t *lut = nullptr;
    if (tuned & (1 << 24)) d.lut_shift = 16u;
    const size_t lut_n = (size_t)1 << (32u - d.lut_shift);
    if ((gs || wg) && dist == NC_GPUHASH_DIST_KETAMA && nkeys >= 65536u && (tuned & (3 << 23)) != 0 && !crc &&
        ncontinuum < 0x80000000u && hipMallocAsync((void **)&lut, lut_n * sizeof(uint32_t), st) == hipSuccess) {
        (void)hipGetLastError();
        hipLaunchKernelGGL(nc_ketama_lut_kernel, dim3((unsigned)((lut_n + 255u) / 256u)), dim3(256), 0, st, d.cont,
                           ncontinuum, lut, d.lut_shift);
        if (hipGetLastError() == hipSuccess) {
            d.lut = lut;
        } else {
            (void)hipFreeAsync(lut, st);
            lut = nullptr;
        }
    }
    hipError_t e;
    switch (mode) {
#define NC_DCASE(M) \
    case M: e = nc_tu::entry_dist<M>(base, d_offsets, delta, nkeys, d_out, st, d); break;
        NC_DCASE(NC_GPUHASH_ONE_AT_A_TIME)
        NC_DCASE(NC_GPUHASH_MD5)
        NC_DCASE(NC_GPUHASH_CRC16)
        NC_DCASE(NC_GPUHASH_CRC32)
        NC_DCASE(NC_GPUHASH_CRC32A)
        NC_DCASE(NC_GPUHASH_FNV1_64)
        NC_DCASE(NC_GPUHASH_FNV1A_64)
        NC_DCASE(NC_GPUHASH_FNV1_32)
        NC_DCASE(NC_GPUHASH_FNV1A_32)
        NC_DCASE(NC_GPUHASH_HSIEH)
        NC_DCASE(NC_GPUHASH_MURMUR)
        NC_DCASE(NC_GPUHASH_JENKINS)
#undef NC_DCASE
    default:
        e = hipErrorInvalidValue;
    }
    if (lut != nullptr) (void)hipFreeAsync(lut, st); /* after the launch that reads it, in stream order */
    if (e == hipErrorInvalidValue && (mode < 0 || mode >= NC_GPUHASH_NMODES)) return fail(EINVAL);
    if (e != hipSuccess) return fail_launch(e, "nc_gpuhash_server_idx_device");
    return NC_OK;
}

extern "C" int nc_gpuhash_pick_variant(int mode, uint64_t nkeys, const struct nc_gpuhash_shape *shape)
{
    if (mode < 0 || mode >= NC_GPUHASH_NMODES) {
        errno = EINVAL;
        return -1;
    }
    return pick_variant(mode, nkeys, shape);
}

extern "C" rstatus_t nc_gpuhash_set_tuning(int grid_cap_, int sort, int variant)
{
    if (grid_cap_ >= 0) store_i(&g_grid_cap, grid_cap_);
    if (sort >= 0) store_i(&g_sort, sort ? 1 : 0);
    if (variant >= 0) store_i(&g_variant, variant);
    return NC_OK;
}

extern "C" rstatus_t nc_gpuhash_time_device(int mode, const uint8_t *d_keys, const uint64_t *d_offsets,
                                            uint64_t nkeys, uint32_t *d_out, void *stream, int iters,
                                            float *avg_ms)
{
    return nc_gpuhash_time_device_shaped(mode, d_keys, d_offsets, nkeys, d_out, nullptr, stream, iters, avg_ms);
}

extern "C" rstatus_t nc_gpuhash_time_device_shaped(int mode, const uint8_t *d_keys, const uint64_t *d_offsets,
                                                   uint64_t nkeys, uint32_t *d_out,
                                                   const struct nc_gpuhash_shape *shape, void *stream, int iters,
                                                   float *avg_ms)
{
    if (mode < 0 || mode >= NC_GPUHASH_NMODES || iters <= 0 || avg_ms == nullptr) return fail(EINVAL);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess) return fail(ENODEV);
    if (hipEventCreate(&b) != hipSuccess) {
        (void)hipEventDestroy(a);
        return fail(ENODEV);
    }
    rstatus_t rc = NC_OK;
    (void)hipEventRecord(a, st);
    for (int i = 0; i < iters && rc == NC_OK; i++) {
        rc = nc_gpuhash_batch_device_shaped(mode, d_keys, d_offsets, nkeys, d_out, shape, stream);
    }
    (void)hipEventRecord(b, st);
    if (hipEventSynchronize(b) != hipSuccess) rc = fail(EIO);
    float ms = 0.f;
    if (rc == NC_OK && hipEventElapsedTime(&ms, a, b) != hipSuccess) rc = fail(EIO);
    if (rc == NC_OK) *avg_ms = ms / (float)iters;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return rc;
}

#endif /* NC_TU_MODE */
