/*
 * Per-lane hashing of one key from LDS (or global memory) for the gfx950
 * kernels: the realigning word readers (aligned dwords funnel-shifted with
 * v_alignbyte, reads issued a step ahead) and the per-mode hash of a key at
 * a byte position, for all 12 hashkit modes. Shared by the batch kernels
 * (nc_gpuhash_kernels.hip) and the batch ring's workers (nc_ring.hip), which
 * hash keys staged in LDS. Step functions and constants are nc_hash_algo.h's
 * (reference citations there).
 */
#ifndef NC_LDS_HASH_H
#define NC_LDS_HASH_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nc_crc_slice.h"
#include "nc_gpuhash.h"
#include "nc_hash_algo.h"

namespace {

/* hash_key VAR bit: crc16 / crc32 / crc32a by slicing-by-16 over 16 tables
 * (tab[k * 256 + e] = nc_slice::entry<MODE>(k, e), 16 KiB) instead of the
 * byte table: a 32-byte key is two dependent steps of sixteen independent
 * lookups instead of 32 chained ones */
constexpr int kHkCrcSliced = 1 << 16;
constexpr uint32_t kSliceTables = 16;

/* ---------------- realigning readers ---------------- */

struct LdsSrc {
    typedef uint32_t pos_t;
    static constexpr bool kOverread = true; /* reads past a key stay inside LDS */
    const uint32_t *base; /* 16-byte aligned LDS slab, read as dwords */
    /* dwords i, i+1 (4-byte aligned): one ds_read2_b32 */
    __device__ __forceinline__ uint2 d2(uint32_t i) const { return make_uint2(base[i], base[i + 1]); }
    __device__ __forceinline__ uint32_t d1(uint32_t i) const { return base[i]; }
};

struct GlobalSrc {
    typedef uint64_t pos_t;
    static constexpr bool kOverread = false; /* at most NC_GPUHASH_PAD past the last key */
    const uint32_t *base; /* 16-byte aligned key buffer */
    __device__ __forceinline__ uint2 d2(uint64_t i) const { return make_uint2(base[i], base[i + 1]); }
    __device__ __forceinline__ uint32_t d1(uint64_t i) const { return base[i]; }
};

/* Sequential little-endian words of a byte string starting at any byte
 * position p: aligned dwords funnel-shifted by (p & 3) bytes with
 * v_alignbyte_b32; one ds_read2_b32 per 8 bytes, no selects. Reads at most
 * 14 bytes past the end of the string (covered by the staged look-ahead
 * piece / NC_GPUHASH_PAD). */
template <class Src, bool kDeep = false>
struct QStream {
    /* kDeep (LDS only): reads run two steps ahead, so a step never waits for
     * the read the previous step issued */
    static constexpr bool D2 = kDeep && Src::kOverread;
    Src src;
    typename Src::pos_t di;
    uint32_t sh;
    uint32_t prev;
    uint2 ahead;  /* dwords di+1, di+2, read one step early */
    uint2 ahead2; /* dwords di+3, di+4 (D2 only) */

    __device__ __forceinline__ void init(const Src &s, typename Src::pos_t p)
    {
        src = s;
        di = p >> 2;
        sh = (uint32_t)p & 3u;
        prev = src.d1(di);
        ahead = src.d2(di + 1);
        if constexpr (D2) ahead2 = src.d2(di + 3);
    }
    /* next 8 bytes as two words; the read for the following 8 is issued now
     * (it may touch up to 22 bytes past the string: inside the staged
     * look-ahead piece / NC_GPUHASH_PAD) */
    __device__ __forceinline__ uint2 next8()
    {
        const uint2 d = ahead;
        di += 2;
        if constexpr (D2) {
            ahead = ahead2;
            ahead2 = src.d2(di + 3);
            asm volatile("" ::: "memory"); /* keep the read here, not at its use */
        } else {
            ahead = src.d2(di + 1);
        }
        uint2 r;
        r.x = __builtin_amdgcn_alignbyte(d.x, prev, sh);
        r.y = __builtin_amdgcn_alignbyte(d.y, d.x, sh);
        prev = d.y;
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

/* Shift counts the compiler cannot see through: with them, (h << s1) + h
 * stays three full-rate v_lshl_add_u32 (3h, 27h, 435h = h * 0x1b3) instead of
 * being folded back into the multi-pass v_mul_lo_u32, and — unlike inline asm
 * — the instructions stay visible to the scheduler and hazard recognizer. */
struct ShiftK {
    uint32_t s1, s3, s4;
};
__device__ __forceinline__ ShiftK opaque_shifts()
{
    ShiftK k;
    asm volatile("s_mov_b32 %0, 1" : "=s"(k.s1));
    asm volatile("s_mov_b32 %0, 3" : "=s"(k.s3));
    asm volatile("s_mov_b32 %0, 4" : "=s"(k.s4));
    return k;
}
__device__ __forceinline__ uint32_t mul_0x1b3(uint32_t h, const ShiftK &k)
{
    const uint32_t t3 = (h << k.s1) + h;
    const uint32_t t27 = (t3 << k.s3) + t3;
    return (t27 << k.s4) + t3;
}

/* VAR bit 0: FNV-64-truncated multiply by shift-adds. */
template <int MODE, int VAR = 0>
__device__ __forceinline__ uint32_t byte_step(uint32_t h, uint32_t b, const uint32_t *tab, const ShiftK &k)
{
    if constexpr (MODE == NC_GPUHASH_FNV1A_64 && (VAR & 1)) return mul_0x1b3(h ^ nc_sx8(b), k);
    if constexpr (MODE == NC_GPUHASH_FNV1_64 && (VAR & 1)) return mul_0x1b3(h, k) ^ nc_sx8(b);
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

template <int MODE, int VAR>
__device__ __forceinline__ uint32_t word_bytes(uint32_t h, uint32_t w, const uint32_t *tab, const ShiftK &k)
{
    h = byte_step<MODE, VAR>(h, w & 0xffu, tab, k);
    h = byte_step<MODE, VAR>(h, (w >> 8) & 0xffu, tab, k);
    h = byte_step<MODE, VAR>(h, (w >> 16) & 0xffu, tab, k);
    h = byte_step<MODE, VAR>(h, w >> 24, tab, k);
    return h;
}

template <int MODE, int VAR, class Src>
__device__ __forceinline__ uint32_t hash_bytes(const Src &src, typename Src::pos_t p, uint32_t len,
                                               const uint32_t *tab)
{
    ShiftK k{0u, 0u, 0u};
    if constexpr ((VAR & 1) != 0) k = opaque_shifts();
    QStream<Src, (VAR & 1024) != 0> st;
    st.init(src, p);
    uint32_t h = byte_init<MODE>();
    const uint32_t n8 = len >> 3;
#pragma unroll 2
    for (uint32_t i = 0; i < n8; i++) {
        uint2 w = st.next8();
        h = word_bytes<MODE, VAR>(h, w.x, tab, k);
        h = word_bytes<MODE, VAR>(h, w.y, tab, k);
    }
    const uint32_t rem = len & 7u;
    if (rem) {
        uint2 w = st.next8();
        if (rem >= 4) {
            h = word_bytes<MODE, VAR>(h, w.x, tab, k);
            w.x = w.y;
        }
        for (uint32_t j = 0; j < (rem & 3u); j++) {
            h = byte_step<MODE, VAR>(h, (w.x >> (8u * j)) & 0xffu, tab, k);
        }
    }
    return byte_final<MODE>(h);
}

/* Two keys of one lane hashed in one loop, so the two dependent chains
 * interleave (ILP for the latency-bound byte recurrences). LDS only: the
 * shorter key's stream reads on past its end (garbage bytes, never used). */
template <int MODE, int VAR>
__device__ __forceinline__ void hash_bytes_pair(const LdsSrc &src, uint32_t pa, uint32_t la, uint32_t pb,
                                                uint32_t lb, const uint32_t *tab, uint32_t &ra, uint32_t &rb)
{
    ShiftK k{0u, 0u, 0u};
    if constexpr ((VAR & 1) != 0) k = opaque_shifts();
    QStream<LdsSrc, (VAR & 1024) != 0> sa, sb;
    sa.init(src, pa);
    sb.init(src, pb);
    uint32_t ha = byte_init<MODE>(), hb = ha;
    const uint32_t na = la >> 3, nb = lb >> 3;
    const uint32_t nmax = na > nb ? na : nb;
    for (uint32_t i = 0; i < nmax; i++) {
        const uint2 wa = sa.next8(), wb = sb.next8();
        uint32_t xa = ha, xb = hb;
        /* byte-granular alternation: in-order issue overlaps the two chains
         * only if their steps alternate in the instruction stream */
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const uint32_t va = ((b < 4 ? wa.x : wa.y) >> (8 * (b & 3))) & 0xffu;
            const uint32_t vb = ((b < 4 ? wb.x : wb.y) >> (8 * (b & 3))) & 0xffu;
            xa = byte_step<MODE, VAR>(xa, va, tab, k);
            xb = byte_step<MODE, VAR>(xb, vb, tab, k);
        }
        if (i < na) ha = xa;
        if (i < nb) hb = xb;
    }
    /* tails: each key's stream is re-anchored on its tail */
    auto tail = [&](uint32_t h, uint32_t p, uint32_t len) __attribute__((always_inline)) {
        const uint32_t rem = len & 7u;
        if (rem) {
            QStream<LdsSrc> st;
            st.init(src, p + (len & ~7u));
            uint2 w = st.next8();
            if (rem >= 4) {
                h = word_bytes<MODE, VAR>(h, w.x, tab, k);
                w.x = w.y;
            }
            for (uint32_t j = 0; j < (rem & 3u); j++) h = byte_step<MODE, VAR>(h, (w.x >> (8u * j)) & 0xffu, tab, k);
        }
        return byte_final<MODE>(h);
    };
    ra = tail(ha, pa, la);
    rb = tail(hb, pb, lb);
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
    /* final block(s): remaining rem bytes, 0x80, zeros, 64-bit bit length.
     * Word t is raw for t < q, the partial word | 0x80 pad for t == q, and 0
     * after it (q = rem / 4). From LDS all 8 reads are unconditional (no
     * per-lane branches; over-read bytes are masked off here). */
    const uint32_t rem = len & 63u;
    const uint32_t q = rem >> 2;
    const uint32_t sh = (rem & 3u) << 3;
    const uint32_t keep = (1u << sh) - 1u; /* low rem%4 bytes of the partial word */
    const uint32_t pad = 0x80u << sh;
#pragma unroll
    for (int t = 0; t < 8; t++) {
        uint2 r = make_uint2(0u, 0u);
        if constexpr (Src::kOverread) r = st.next8();
        else if (8u * t < rem) r = st.next8();
        const uint32_t t0 = 2u * t, t1 = 2u * t + 1u;
        w[t0] = t0 < q ? r.x : (t0 == q ? ((r.x & keep) | pad) : 0u);
        w[t1] = t1 < q ? r.y : (t1 == q ? ((r.y & keep) | pad) : 0u);
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

/* Message words of block `blk` of a key of `len` bytes read from `st`: the
 * key's bytes, then 0x80, zeros and, in its last block, the bit length
 * (src/hashkit/nc_md5.c:245-274). LDS only: the reads run past the key. */
__device__ __forceinline__ void md5_words(QStream<LdsSrc> &st, uint32_t w[16], uint32_t len, uint32_t blk)
{
    const int32_t rem = (int32_t)len - 64 * (int32_t)blk; /* message bytes from the block start */
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const uint2 r = st.next8();
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const uint32_t v = h ? r.y : r.x;
            const int32_t nb = rem - (8 * t + 4 * h); /* message bytes in this word */
            const uint32_t part = nb <= 0 ? 0u : (v & (0xffffffffu >> (32u - 8u * (uint32_t)nb)));
            const uint32_t pad = (nb >= 0 && nb < 4) ? (0x80u << (8u * (uint32_t)nb)) : 0u;
            w[2 * t + h] = nb >= 4 ? v : (part | pad);
        }
    }
    if (blk == (len + 8u) / 64u) { /* the last block */
        w[14] = len << 3;
        w[15] = len >> 29;
    }
}

/* md5 of a lane's two keys with their blocks interleaved step by step
 * (nc_md5_block2): two independent chains per lane instead of one. */
__device__ __forceinline__ void hash_md5_pair(const LdsSrc &src, uint32_t pa, uint32_t la, uint32_t pb,
                                              uint32_t lb, uint32_t &ra, uint32_t &rb)
{
    QStream<LdsSrc> sa, sb;
    sa.init(src, pa);
    sb.init(src, pb);
    uint32_t A[4] = {NC_MD5_A0, NC_MD5_B0, NC_MD5_C0, NC_MD5_D0};
    uint32_t B[4] = {NC_MD5_A0, NC_MD5_B0, NC_MD5_C0, NC_MD5_D0};
    const uint32_t na = (la + 8u) / 64u + 1u, nb = (lb + 8u) / 64u + 1u;
    const uint32_t n = na > nb ? na : nb;
    for (uint32_t blk = 0; blk < n; blk++) {
        uint32_t wa[16], wb[16];
        md5_words(sa, wa, la, blk);
        md5_words(sb, wb, lb, blk);
        uint32_t ta[4] = {A[0], A[1], A[2], A[3]}, tb[4] = {B[0], B[1], B[2], B[3]};
        nc_md5_block2(ta, wa, tb, wb);
        if (blk < na) {
            A[0] = ta[0];
            A[1] = ta[1];
            A[2] = ta[2];
            A[3] = ta[3];
        }
        if (blk < nb) {
            B[0] = tb[0];
            B[1] = tb[1];
            B[2] = tb[2];
            B[3] = tb[3];
        }
    }
    ra = A[0]; /* digest bytes 0..3 little-endian (nc_md5.c:317-320) */
    rb = B[0];
}

/* sixteen bytes w[0..3] into crc state h: byte i through table 15 - i, the
 * state folded into the first four (nc_crc_slice.h word() / word2(), one
 * copy of each table) */
template <int MODE>
__device__ __forceinline__ uint32_t crc_slice16(uint32_t h, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3,
                                                const uint32_t *tab)
{
    using nc_slice::look;
    if constexpr (MODE == NC_GPUHASH_CRC16) {
        const uint32_t v = ((h & 0xffffu) << 16) ^ __builtin_bswap32(w0);
        const uint32_t a = __builtin_bswap32(w1), b = __builtin_bswap32(w2), c = __builtin_bswap32(w3);
        return (look<1>(tab, v >> 24, 0, 15) ^ look<1>(tab, (v >> 16) & 0xffu, 0, 14) ^
                look<1>(tab, (v >> 8) & 0xffu, 0, 13) ^ look<1>(tab, v & 0xffu, 0, 12)) ^
               (look<1>(tab, a >> 24, 0, 11) ^ look<1>(tab, (a >> 16) & 0xffu, 0, 10) ^
                look<1>(tab, (a >> 8) & 0xffu, 0, 9) ^ look<1>(tab, a & 0xffu, 0, 8)) ^
               (look<1>(tab, b >> 24, 0, 7) ^ look<1>(tab, (b >> 16) & 0xffu, 0, 6) ^
                look<1>(tab, (b >> 8) & 0xffu, 0, 5) ^ look<1>(tab, b & 0xffu, 0, 4)) ^
               (look<1>(tab, c >> 24, 0, 3) ^ look<1>(tab, (c >> 16) & 0xffu, 0, 2) ^
                look<1>(tab, (c >> 8) & 0xffu, 0, 1) ^ look<1>(tab, c & 0xffu, 0, 0));
    } else {
        const uint32_t x = h ^ w0;
        return (look<1>(tab, x & 0xffu, 0, 15) ^ look<1>(tab, (x >> 8) & 0xffu, 0, 14) ^
                look<1>(tab, (x >> 16) & 0xffu, 0, 13) ^ look<1>(tab, x >> 24, 0, 12)) ^
               (look<1>(tab, w1 & 0xffu, 0, 11) ^ look<1>(tab, (w1 >> 8) & 0xffu, 0, 10) ^
                look<1>(tab, (w1 >> 16) & 0xffu, 0, 9) ^ look<1>(tab, w1 >> 24, 0, 8)) ^
               (look<1>(tab, w2 & 0xffu, 0, 7) ^ look<1>(tab, (w2 >> 8) & 0xffu, 0, 6) ^
                look<1>(tab, (w2 >> 16) & 0xffu, 0, 5) ^ look<1>(tab, w2 >> 24, 0, 4)) ^
               (look<1>(tab, w3 & 0xffu, 0, 3) ^ look<1>(tab, (w3 >> 8) & 0xffu, 0, 2) ^
                look<1>(tab, (w3 >> 16) & 0xffu, 0, 1) ^ look<1>(tab, w3 >> 24, 0, 0));
    }
}

/* crc16 / crc32 / crc32a of a key by slicing-by-16 (kHkCrcSliced): whole
 * 16-byte pieces, then one 8-byte and one 4-byte piece when they fit, then
 * single bytes through table 0. crc16 leaves its last 2+ bytes to the byte
 * steps, which rebuild the unmasked state's history bits (nc_crc_slice.h). */
template <int MODE, class Src>
__device__ __forceinline__ uint32_t hash_crc_sliced(const Src &src, typename Src::pos_t p, uint32_t len,
                                                    const uint32_t *tab)
{
    constexpr int32_t kKeep = MODE == NC_GPUHASH_CRC16 ? 2 : 0; /* bytes left to the byte steps */
    QStream<Src> st;
    st.init(src, p);
    uint32_t h = MODE == NC_GPUHASH_CRC16 ? 0u : 0xffffffffu;
    int32_t n = (int32_t)len;
    while (n >= 16 + kKeep) {
        const uint2 a = st.next8(), b = st.next8();
        h = crc_slice16<MODE>(h, a.x, a.y, b.x, b.y, tab);
        n -= 16;
    }
    /* n < 16 + kKeep bytes left: up to 20 of them in r[0..4] */
    uint32_t r[6] = {0u, 0u, 0u, 0u, 0u, 0u};
#pragma unroll
    for (int q = 0; q < 3; q++) {
        if (Src::kOverread || n > 8 * q) {
            const uint2 a = st.next8();
            r[2 * q] = a.x;
            r[2 * q + 1] = a.y;
        }
    }
    uint32_t k = 0; /* words of r consumed */
    if (n >= 8 + kKeep) {
        h = nc_slice::word2<MODE, 1>(h, r[0], r[1], tab, 0u);
        n -= 8;
        k = 2;
    }
    if (n >= 4 + kKeep) {
        h = nc_slice::word<MODE, 1>(h, k ? r[2] : r[0], tab, 0u);
        n -= 4;
        k += 1;
    }
    /* n <= 3 + kKeep bytes from word k on */
    const uint32_t lo = k == 0 ? r[0] : (k == 1 ? r[1] : (k == 2 ? r[2] : r[3]));
    const uint32_t hi = k == 0 ? r[1] : (k == 1 ? r[2] : (k == 2 ? r[3] : r[4]));
#pragma unroll
    for (int j = 0; j < 4 + kKeep; j++) {
        if (j < n) {
            const uint32_t w = j < 4 ? lo : hi;
            h = nc_slice::byte<MODE, 1>(h, (w >> (8 * (j & 3))) & 0xffu, tab, 0u);
        }
    }
    if constexpr (MODE == NC_GPUHASH_CRC32) return nc_crc32_final(h);
    else if constexpr (MODE == NC_GPUHASH_CRC32A) return nc_crc32a_final(h);
    else return h;
}

template <int MODE, int VAR, class Src>
__device__ __forceinline__ uint32_t hash_key(const Src &src, typename Src::pos_t p, uint32_t len,
                                             const uint32_t *tab)
{
    if constexpr ((VAR & kHkCrcSliced) != 0 && (MODE == NC_GPUHASH_CRC16 || MODE == NC_GPUHASH_CRC32 ||
                                                 MODE == NC_GPUHASH_CRC32A))
        return hash_crc_sliced<MODE>(src, p, len, tab);
    else if constexpr (MODE == NC_GPUHASH_MD5) return hash_md5_dev(src, p, len);
    else if constexpr (MODE == NC_GPUHASH_HSIEH) return hash_hsieh_dev(src, p, len);
    else if constexpr (MODE == NC_GPUHASH_MURMUR) return hash_murmur_dev(src, p, len);
    else if constexpr (MODE == NC_GPUHASH_JENKINS) return hash_jenkins_dev(src, p, len);
    else return hash_bytes<MODE, VAR>(src, p, len, tab);
}

template <int MODE>
constexpr bool uses_crc_table()
{
    return MODE == NC_GPUHASH_CRC16 || MODE == NC_GPUHASH_CRC32 || MODE == NC_GPUHASH_CRC32A;
}

} // namespace

#endif
