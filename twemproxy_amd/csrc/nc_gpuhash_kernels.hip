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
#include <stdlib.h>

#include "nc_gpuhash.h"
#include "nc_hash_algo.h"

namespace {

constexpr int kBlock = 256;                  /* threads per workgroup = keys per tile */
constexpr int kTile = kBlock;
constexpr uint32_t kSlabCap = 16384 + 208;    /* staged key bytes per tile: 8 workgroups fit one CU (160 KiB) */
constexpr int kStageIters = (kSlabCap / 16 + kBlock - 1) / kBlock;
constexpr int kBuckets = 64;

/* LDS carve (one __shared__ array, all offsets 16-byte aligned) */
constexpr uint32_t kOffSlab = 0;
constexpr uint32_t kOffStart = kOffSlab + kSlabCap;            /* u32[kTile] key start in slab */
constexpr uint32_t kOffLen = kOffStart + 4 * kTile;            /* u32[kTile] key length */
constexpr uint32_t kOffPerm = kOffLen + 4 * kTile;             /* u16[kTile] sorted -> tile index */
constexpr uint32_t kOffHist = kOffPerm + 2 * kTile;            /* u32[kBuckets] */
constexpr uint32_t kOffFlag = kOffHist + 4 * kBuckets;         /* u32[4] */
constexpr uint32_t kOffTab = kOffFlag + 16;                    /* u32[256] crc table */
constexpr uint32_t kSmemBytes = kOffTab + 4 * 256;

static_assert(kOffTab % 16 == 0, "LDS carve must stay 16-byte aligned");

/* ---------------- realigning readers ---------------- */

struct LdsSrc {
    typedef uint32_t pos_t;
    const uint8_t *base;
    __device__ __forceinline__ uint2 q(uint32_t i) const { return reinterpret_cast<const uint2 *>(base)[i]; }
};

struct GlobalSrc {
    typedef uint64_t pos_t;
    const uint8_t *base;
    __device__ __forceinline__ uint2 q(uint64_t i) const { return reinterpret_cast<const uint2 *>(base)[i]; }
};

/* Sequential little-endian words of a byte string starting at any byte
 * position p: two aligned 8-byte reads are funnel-shifted with v_alignbyte. */
template <class Src>
struct QStream {
    Src src;
    typename Src::pos_t qi;
    uint32_t sel;   /* (p & 7) >= 4 */
    uint32_t sh;    /* p & 3 */
    uint2 cur;

    __device__ __forceinline__ void init(const Src &s, typename Src::pos_t p)
    {
        src = s;
        qi = p >> 3;
        sel = ((uint32_t)p >> 2) & 1u;
        sh = (uint32_t)p & 3u;
        cur = src.q(qi);
    }
    /* next 8 bytes as two words */
    __device__ __forceinline__ uint2 next8()
    {
        uint2 nx = src.q(++qi);
        uint32_t a = sel ? cur.y : cur.x;
        uint32_t b = sel ? nx.x : cur.y;
        uint32_t c = sel ? nx.y : nx.x;
        uint2 r;
        r.x = __builtin_amdgcn_alignbyte(b, a, sh);
        r.y = __builtin_amdgcn_alignbyte(c, b, sh);
        cur = nx;
        return r;
    }
};

/* One word at a time on top of QStream (word-granular modes). */
template <class Src>
struct WStream {
    QStream<Src> q;
    uint32_t pend;
    bool has;
    __device__ __forceinline__ void init(const Src &s, typename Src::pos_t p)
    {
        q.init(s, p);
        has = false;
        pend = 0;
    }
    __device__ __forceinline__ uint32_t next()
    {
        if (has) {
            has = false;
            return pend;
        }
        uint2 r = q.next8();
        pend = r.y;
        has = true;
        return r.x;
    }
};

__device__ __forceinline__ uint32_t keep_bytes(uint32_t w, uint32_t nb)
{
    return nb >= 4u ? w : (nb == 0u ? 0u : (w & (0xffffffffu >> (32u - 8u * nb))));
}

/* ---------------- byte-serial modes ---------------- */

template <int MODE>
__device__ __forceinline__ uint32_t byte_init()
{
    if constexpr (MODE == NC_GPUHASH_FNV1_64 || MODE == NC_GPUHASH_FNV1A_64) return NC_FNV64_INIT32;
    if constexpr (MODE == NC_GPUHASH_FNV1_32 || MODE == NC_GPUHASH_FNV1A_32) return NC_FNV32_INIT;
    if constexpr (MODE == NC_GPUHASH_CRC32 || MODE == NC_GPUHASH_CRC32A) return 0xffffffffu;
    return 0u; /* one_at_a_time, crc16 */
}

template <int MODE>
__device__ __forceinline__ uint32_t byte_step(uint32_t h, uint32_t b, const uint32_t *tab)
{
    if constexpr (MODE == NC_GPUHASH_FNV1A_64) return nc_fnv1a_64_step(h, b);
    if constexpr (MODE == NC_GPUHASH_FNV1_64) return nc_fnv1_64_step(h, b);
    if constexpr (MODE == NC_GPUHASH_FNV1_32) return nc_fnv1_32_step(h, b);
    if constexpr (MODE == NC_GPUHASH_FNV1A_32) return nc_fnv1a_32_step(h, b);
    if constexpr (MODE == NC_GPUHASH_ONE_AT_A_TIME) return nc_oaat_step(h, b);
    if constexpr (MODE == NC_GPUHASH_CRC16) return NC_CRC16_NEXT(h, tab[NC_CRC16_IDX(h, b)]);
    if constexpr (MODE == NC_GPUHASH_CRC32 || MODE == NC_GPUHASH_CRC32A) return NC_CRC32_NEXT(h, tab[NC_CRC32_IDX(h, b)]);
    return h;
}

template <int MODE>
__device__ __forceinline__ uint32_t byte_final(uint32_t h)
{
    if constexpr (MODE == NC_GPUHASH_ONE_AT_A_TIME) return nc_oaat_final(h);
    if constexpr (MODE == NC_GPUHASH_CRC32) return nc_crc32_final(h);
    if constexpr (MODE == NC_GPUHASH_CRC32A) return nc_crc32a_final(h);
    return h;
}

template <int MODE>
__device__ __forceinline__ uint32_t word_bytes(uint32_t h, uint32_t w, const uint32_t *tab)
{
    h = byte_step<MODE>(h, w & 0xffu, tab);
    h = byte_step<MODE>(h, (w >> 8) & 0xffu, tab);
    h = byte_step<MODE>(h, (w >> 16) & 0xffu, tab);
    h = byte_step<MODE>(h, w >> 24, tab);
    return h;
}

template <int MODE, class Src>
__device__ __forceinline__ uint32_t hash_bytes(const Src &src, typename Src::pos_t p, uint32_t len,
                                               const uint32_t *tab)
{
    QStream<Src> st;
    st.init(src, p);
    uint32_t h = byte_init<MODE>();
    const uint32_t n8 = len >> 3;
    for (uint32_t i = 0; i < n8; i++) {
        uint2 w = st.next8();
        h = word_bytes<MODE>(h, w.x, tab);
        h = word_bytes<MODE>(h, w.y, tab);
    }
    const uint32_t rem = len & 7u;
    if (rem) {
        uint2 w = st.next8();
        if (rem >= 4) {
            h = word_bytes<MODE>(h, w.x, tab);
            w.x = w.y;
        }
        for (uint32_t k = 0; k < (rem & 3u); k++) {
            h = byte_step<MODE>(h, (w.x >> (8u * k)) & 0xffu, tab);
        }
    }
    return byte_final<MODE>(h);
}

/* ---------------- word-granular modes ---------------- */

template <class Src>
__device__ __forceinline__ uint32_t hash_hsieh_dev(const Src &src, typename Src::pos_t p, uint32_t len)
{
    if (len == 0) return 0; /* nc_hsieh.c:44 */
    QStream<Src> st;
    st.init(src, p);
    uint32_t h = 0;
    const uint32_t nw = len >> 2;
    for (uint32_t i = 0; i < (nw >> 1); i++) {
        uint2 w = st.next8();
        h = nc_hsieh_word(h, w.x);
        h = nc_hsieh_word(h, w.y);
    }
    const uint32_t rem = len & 3u;
    if ((nw & 1u) || rem) {
        uint2 w = st.next8();
        uint32_t tail = w.x;
        if (nw & 1u) {
            h = nc_hsieh_word(h, w.x);
            tail = w.y;
        }
        h = nc_hsieh_tail(h, tail, rem);
    }
    return nc_hsieh_final(h);
}

template <class Src>
__device__ __forceinline__ uint32_t hash_murmur_dev(const Src &src, typename Src::pos_t p, uint32_t len)
{
    QStream<Src> st;
    st.init(src, p);
    uint32_t h = nc_murmur_init(len);
    const uint32_t nw = len >> 2;
    for (uint32_t i = 0; i < (nw >> 1); i++) {
        uint2 w = st.next8();
        h = nc_murmur_word(h, w.x);
        h = nc_murmur_word(h, w.y);
    }
    const uint32_t rem = len & 3u;
    if ((nw & 1u) || rem) {
        uint2 w = st.next8();
        uint32_t tail = w.x;
        if (nw & 1u) {
            h = nc_murmur_word(h, w.x);
            tail = w.y;
        }
        h = nc_murmur_tail(h, tail, rem);
    }
    return nc_murmur_final(h);
}

template <class Src>
__device__ __forceinline__ uint32_t hash_jenkins_dev(const Src &src, typename Src::pos_t p, uint32_t len)
{
    uint32_t a, b, c;
    a = b = c = nc_jenkins_init(len);
    if (len == 0) return c; /* nc_jenkins.c:121 */
    WStream<Src> ws;
    ws.init(src, p);
    uint32_t n = len;
    while (n > 12) {
        a += ws.next();
        b += ws.next();
        c += ws.next();
        NC_JENKINS_MIX(a, b, c);
        n -= 12;
    }
    /* last 1..12 bytes, zero-extended */
    a += keep_bytes(ws.next(), n);
    if (n > 4) b += keep_bytes(ws.next(), n - 4);
    if (n > 8) c += keep_bytes(ws.next(), n - 8);
    NC_JENKINS_FINAL(a, b, c);
    return c;
}

template <class Src>
__device__ __forceinline__ uint32_t hash_md5_dev(const Src &src, typename Src::pos_t p, uint32_t len)
{
    QStream<Src> st;
    st.init(src, p);
    uint32_t s[4] = {NC_MD5_A0, NC_MD5_B0, NC_MD5_C0, NC_MD5_D0};
    uint32_t w[16];
    const uint32_t nfull = len >> 6;
    for (uint32_t blk = 0; blk < nfull; blk++) {
#pragma unroll
        for (int t = 0; t < 8; t++) {
            uint2 r = st.next8();
            w[2 * t] = r.x;
            w[2 * t + 1] = r.y;
        }
        nc_md5_block(s, w);
    }
    /* final block(s): remaining rem bytes, 0x80, zeros, 64-bit bit length */
    const uint32_t rem = len & 63u;
#pragma unroll
    for (int t = 0; t < 8; t++) {
        uint2 r = make_uint2(0u, 0u);
        if (8u * t < rem) r = st.next8();
        w[2 * t] = nc_md5_pad_word(r.x, 2 * t, rem);
        w[2 * t + 1] = nc_md5_pad_word(r.y, 2 * t + 1, rem);
    }
    const uint64_t bits = (uint64_t)len << 3;
    if (rem >= 56) {
        nc_md5_block(s, w);
#pragma unroll
        for (int t = 0; t < 16; t++) w[t] = 0;
    }
    w[14] = (uint32_t)bits;
    w[15] = (uint32_t)(bits >> 32);
    nc_md5_block(s, w);
    return s[0]; /* digest bytes 0..3 little-endian (nc_md5.c:317-320) */
}

template <int MODE, class Src>
__device__ __forceinline__ uint32_t hash_key(const Src &src, typename Src::pos_t p, uint32_t len,
                                             const uint32_t *tab)
{
    if constexpr (MODE == NC_GPUHASH_MD5) return hash_md5_dev(src, p, len);
    else if constexpr (MODE == NC_GPUHASH_HSIEH) return hash_hsieh_dev(src, p, len);
    else if constexpr (MODE == NC_GPUHASH_MURMUR) return hash_murmur_dev(src, p, len);
    else if constexpr (MODE == NC_GPUHASH_JENKINS) return hash_jenkins_dev(src, p, len);
    else return hash_bytes<MODE>(src, p, len, tab);
}

template <int MODE>
constexpr bool uses_crc_table()
{
    return MODE == NC_GPUHASH_CRC16 || MODE == NC_GPUHASH_CRC32 || MODE == NC_GPUHASH_CRC32A;
}

/* Length class used to group keys of similar cost into one wave. */
__device__ __forceinline__ uint32_t len_bucket(uint32_t len)
{
    uint32_t b = (len + 3u) >> 2;
    return b < (uint32_t)(kBuckets - 1) ? b : (uint32_t)(kBuckets - 1);
}

/*
 * keys_base is 16-byte aligned; key i occupies keys_base[off[i] + delta ..
 * off[i+1] + delta) and keys_base stays readable NC_GPUHASH_PAD bytes past
 * the last key.
 */
template <int MODE, bool SORT>
__global__ __launch_bounds__(kBlock) void nc_hash_kernel(const uint8_t *__restrict__ keys_base,
                                                         const uint64_t *__restrict__ off, uint64_t delta,
                                                         uint64_t nkeys, uint32_t *__restrict__ out,
                                                         uint64_t ntiles)
{
    __shared__ __attribute__((aligned(16))) uint8_t smem[kSmemBytes];
    uint8_t *slab = smem + kOffSlab;
    uint32_t *kstart = reinterpret_cast<uint32_t *>(smem + kOffStart);
    uint32_t *klen = reinterpret_cast<uint32_t *>(smem + kOffLen);
    uint16_t *perm = reinterpret_cast<uint16_t *>(smem + kOffPerm);
    uint32_t *hist = reinterpret_cast<uint32_t *>(smem + kOffHist);
    uint32_t *flag = reinterpret_cast<uint32_t *>(smem + kOffFlag);
    uint32_t *tab = reinterpret_cast<uint32_t *>(smem + kOffTab);

    const uint32_t t = threadIdx.x;
    const uint32_t lane = t & 63u;

    if constexpr (uses_crc_table<MODE>()) {
        tab[t] = (MODE == NC_GPUHASH_CRC16) ? nc_crc16_entry(t) : nc_crc32_entry(t);
        __syncthreads();
    }

    for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t k0 = tile * (uint64_t)kTile;
        const uint64_t left = nkeys - k0;
        const uint32_t cnt = left < (uint64_t)kTile ? (uint32_t)left : (uint32_t)kTile;
        const bool valid = t < cnt;

        uint64_t s = 0, e = 0;
        if (valid) {
            s = off[k0 + t];
            e = off[k0 + t + 1];
        }
        const uint64_t S = off[k0] + delta;
        const uint64_t E = off[k0 + cnt] + delta;
        const uint64_t S16 = S & ~(uint64_t)15;
        const uint64_t span = E - S16;
        const bool in_lds = span + 16u <= (uint64_t)kSlabCap;
        const uint32_t len = (uint32_t)(e - s);

        if (in_lds) {
            /* coalesced 16-byte staging of [S16, roundup16(E) + 16) */
            const uint32_t nch = (uint32_t)((span + 15u) >> 4) + 1u;
            const uint4 *g = reinterpret_cast<const uint4 *>(keys_base + S16);
            uint4 *l = reinterpret_cast<uint4 *>(slab);
            uint4 v[kStageIters];
#pragma unroll
            for (int i = 0; i < kStageIters; i++) {
                const uint32_t c = t + (uint32_t)i * kBlock;
                if (c < nch) v[i] = g[c];
            }
#pragma unroll
            for (int i = 0; i < kStageIters; i++) {
                const uint32_t c = t + (uint32_t)i * kBlock;
                if (c < nch) l[c] = v[i];
            }
        }

        uint32_t my = t;
        if constexpr (SORT) {
            /* Group keys by length class: wave-ballot multisplit, one LDS
             * atomic per (wave, class), then an exclusive scan over classes. */
            const uint32_t bucket = valid ? len_bucket(len) : (uint32_t)(kBuckets - 1);
            if (t < (uint32_t)kBuckets) hist[t] = 0;
            if (t == 0) flag[0] = 0;
            kstart[t] = in_lds ? (uint32_t)(s + delta - S16) : 0u;
            klen[t] = len;
            __syncthreads();
            const uint32_t b0 = __shfl(bucket, 0);
            if (__ballot(bucket != b0) != 0ull && lane == 0) flag[0] = 1u;
            /* flag only grows: any lane writing 1 makes the tile sortable */
            __syncthreads();
            if (flag[0] != 0u) {
                const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64u - lane));
                uint32_t rank = 0;
                bool done = false;
                while (true) {
                    const uint64_t act = __ballot(!done);
                    if (act == 0ull) break;
                    const uint32_t lead = (uint32_t)__ffsll((unsigned long long)act) - 1u;
                    const uint32_t bl = __shfl(bucket, (int)lead);
                    const bool mine = !done && bucket == bl;
                    const uint64_t m = __ballot(mine);
                    uint32_t base = 0;
                    if (lane == lead) base = atomicAdd(&hist[bl], (uint32_t)__popcll(m));
                    base = __shfl(base, (int)lead);
                    if (mine) {
                        rank = base + (uint32_t)__popcll(m & lt);
                        done = true;
                    }
                }
                __syncthreads();
                if (t < 64u) {
                    /* exclusive scan of the 64 class counts by wave 0 */
                    const uint32_t c = hist[t];
                    uint32_t x = c;
#pragma unroll
                    for (int d = 1; d < 64; d <<= 1) {
                        const uint32_t y = __shfl_up(x, d);
                        if (lane >= (uint32_t)d) x += y;
                    }
                    hist[t] = x - c;
                }
                __syncthreads();
                perm[hist[bucket] + rank] = (uint16_t)t;
                __syncthreads();
                my = perm[t];
            }
        }

        if (my < cnt) {
            uint32_t h;
            uint32_t klen_my = len;
            if constexpr (SORT) klen_my = klen[my];
            if (in_lds) {
                uint32_t pos = (uint32_t)(s + delta - S16);
                if constexpr (SORT) pos = kstart[my];
                LdsSrc src{slab};
                h = hash_key<MODE>(src, pos, klen_my, tab);
            } else {
                uint64_t pos = s + delta;
                if constexpr (SORT) {
                    if (my != t) pos = off[k0 + my] + delta;
                }
                GlobalSrc src{keys_base};
                h = hash_key<MODE>(src, pos, klen_my, tab);
            }
            out[k0 + my] = h;
        }
        __syncthreads(); /* the next tile restages the LDS */
    }
}

/* ---------------- launch layer ---------------- */

int g_grid_cap = -1; /* 0 = one workgroup per tile */
int g_sort = -1;     /* 1 on, 0 off */

int grid_cap()
{
    if (g_grid_cap < 0) {
        const char *e = getenv("NC_GPUHASH_GRID");
        g_grid_cap = e ? atoi(e) : 0;
        if (g_grid_cap < 0) g_grid_cap = 0;
    }
    return g_grid_cap;
}

bool sort_enabled()
{
    if (g_sort < 0) {
        const char *e = getenv("NC_GPUHASH_SORT");
        g_sort = e ? (atoi(e) ? 1 : 0) : 1;
    }
    return g_sort == 1;
}

template <int MODE>
hipError_t launch_mode(const uint8_t *base, const uint64_t *off, uint64_t delta, uint64_t nkeys,
                       uint32_t *out, hipStream_t stream, bool sort)
{
    const uint64_t ntiles = (nkeys + kTile - 1) / kTile;
    uint64_t grid = ntiles;
    const int cap = grid_cap();
    if (cap > 0 && grid > (uint64_t)cap) grid = (uint64_t)cap;
    if (grid > 0x7fffffffull) grid = 0x7fffffffull;
    if (sort) {
        hipLaunchKernelGGL((nc_hash_kernel<MODE, true>), dim3((unsigned)grid), dim3(kBlock), 0, stream, base, off,
                           delta, nkeys, out, ntiles);
    } else {
        hipLaunchKernelGGL((nc_hash_kernel<MODE, false>), dim3((unsigned)grid), dim3(kBlock), 0, stream, base,
                           off, delta, nkeys, out, ntiles);
    }
    return hipGetLastError();
}

hipError_t launch(int mode, const uint8_t *d_keys, const uint64_t *d_off, uint64_t nkeys, uint32_t *d_out,
                  hipStream_t stream)
{
    const uintptr_t kp = reinterpret_cast<uintptr_t>(d_keys);
    const uint8_t *base = reinterpret_cast<const uint8_t *>(kp & ~(uintptr_t)15);
    const uint64_t delta = (uint64_t)(kp & 15u);
    const bool sort = sort_enabled();
    switch (mode) {
#define NC_CASE(M) \
    case M: return launch_mode<M>(base, d_off, delta, nkeys, d_out, stream, sort);
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

} // namespace

extern "C" rstatus_t nc_gpuhash_batch_device(int mode, const uint8_t *d_keys, const uint64_t *d_offsets,
                                             uint64_t nkeys, uint32_t *d_out, void *stream)
{
    if (mode < 0 || mode >= NC_GPUHASH_NMODES) return fail(EINVAL);
    if (nkeys == 0) return NC_OK;
    if (d_keys == nullptr || d_offsets == nullptr || d_out == nullptr) return fail(EINVAL);
    hipError_t err = launch(mode, d_keys, d_offsets, nkeys, d_out, reinterpret_cast<hipStream_t>(stream));
    if (err != hipSuccess) return fail(err == hipErrorNoDevice ? ENODEV : EIO);
    return NC_OK;
}

extern "C" rstatus_t nc_gpuhash_set_tuning(int grid_cap_, int sort)
{
    if (grid_cap_ >= 0) g_grid_cap = grid_cap_;
    if (sort >= 0) g_sort = sort ? 1 : 0;
    return NC_OK;
}

extern "C" rstatus_t nc_gpuhash_time_device(int mode, const uint8_t *d_keys, const uint64_t *d_offsets,
                                            uint64_t nkeys, uint32_t *d_out, void *stream, int iters,
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
        rc = nc_gpuhash_batch_device(mode, d_keys, d_offsets, nkeys, d_out, stream);
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
