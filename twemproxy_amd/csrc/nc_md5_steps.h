/*
 * The 64 md5 steps for gfx950 kernels (RFC 1321; src/hashkit/nc_md5.c:89-194),
 * unrolled at compile time: step I updates one of the four state words
 * (a, d, c, b in turn). Shared by nc_md5_kernels.hip and the VALU probes.
 */
#ifndef NC_MD5_STEPS_H
#define NC_MD5_STEPS_H

#include <stdint.h>

#include <utility>

#include "nc_hash_algo.h"

namespace nc_md5s {

/* the 64 steps' constants, message word and shift, from NC_MD5_ROUNDS
 * (RFC 1321; src/hashkit/nc_md5.c:89-194) */
#define NC_MD5_KT(f, a, b, c, d, k, t, s) t,
#define NC_MD5_KM(f, a, b, c, d, k, t, s) k,
#define NC_MD5_KS(f, a, b, c, d, k, t, s) s,
constexpr uint32_t kT[64] = {NC_MD5_ROUNDS(NC_MD5_KT)};
constexpr int kM[64] = {NC_MD5_ROUNDS(NC_MD5_KM)};
constexpr int kS[64] = {NC_MD5_ROUNDS(NC_MD5_KS)};

/* The round function of step I. H (b ^ c ^ d) is one v_bitop3_b32 (truth
 * table 0x96), where hipcc's own choice is two dependent v_xor_b32: 16 VALU
 * per block fewer. F, G and I already compile to one v_bitop3 each. */
template <int I>
__device__ __forceinline__ uint32_t md5_f(uint32_t b, uint32_t c, uint32_t d)
{
    if constexpr (I < 16) return NC_MD5_F(b, c, d);
    else if constexpr (I < 32) return NC_MD5_G(b, c, d);
    else if constexpr (I < 48) return __builtin_amdgcn_bitop3_b32(b, c, d, 0x96);
    else return NC_MD5_I(b, c, d);
}

/* Step I updates one of the four state words: a, d, c, b in turn. */
template <int I>
__device__ __forceinline__ void md5_step(uint32_t (&v)[4], const uint32_t (&w)[16])
{
    constexpr int u = (4 - (I & 3)) & 3;
    const uint32_t b = v[(u + 1) & 3], c = v[(u + 2) & 3], d = v[(u + 3) & 3];
    const uint32_t f = md5_f<I>(b, c, d);
    /* w + T by a VOP2 literal add off the step's dependency chain, then
     * a + (w + T) + f by one v_add3_u32: five VALU instructions per step, no
     * scalar s_mov of T, and a four-op chain f -> add3 -> rotate -> add
     * (tools/probes/md5_rate.hip form 3: 13 % faster than a + w + f, + T at 4
     * waves per SIMD, 1 % at 8; hipcc's default form, a + w, s_mov T, v_add3,
     * is slower than both) */
    uint32_t wt = w[kM[I]] + kT[I];
    asm("" : "+v"(wt)); /* keeps T out of the sum: hipcc would reassociate it into an s_mov + v_add3 */
    v[u] = nc_rotl(v[u] + wt + f, kS[I]) + b;
}

template <int... I>
__device__ __forceinline__ void md5_steps(uint32_t (&v)[4], const uint32_t (&w)[16], std::integer_sequence<int, I...>)
{
    (md5_step<I>(v, w), ...);
}

/* steps OFF, OFF + 1, ... */
template <int OFF, int... I>
__device__ __forceinline__ void md5_steps_at(uint32_t (&v)[4], const uint32_t (&w)[16], std::integer_sequence<int, I...>)
{
    (md5_step<OFF + I>(v, w), ...);
}

/* Steps 0..3 of a key's FIRST block, whose state word v[u] is still the
 * initial constant (RFC 1321 A0..D0): v[u] + T folds into one constant (an
 * SGPR operand of v_add3), and step 0's round function is a constant too —
 * four VALU per step, three for step 0. Past step 3 every state word is data. */
template <int I>
__device__ __forceinline__ void md5_step_first(uint32_t (&v)[4], const uint32_t (&w)[16])
{
    static_assert(I < 4, "the initial state is constant only through step 3");
    constexpr uint32_t kInit[4] = {NC_MD5_A0, NC_MD5_B0, NC_MD5_C0, NC_MD5_D0};
    constexpr int u = (4 - (I & 3)) & 3;
    const uint32_t b = v[(u + 1) & 3], c = v[(u + 2) & 3], d = v[(u + 3) & 3];
    const uint32_t f = md5_f<I>(b, c, d);
    v[u] = nc_rotl(w[kM[I]] + f + (kInit[u] + kT[I]), kS[I]) + b;
}

/* steps 0..60 of a key's first block from the initial state (v holds it) */
__device__ __forceinline__ void md5_steps_first61(uint32_t (&v)[4], const uint32_t (&w)[16])
{
    md5_step_first<0>(v, w);
    md5_step_first<1>(v, w);
    md5_step_first<2>(v, w);
    md5_step_first<3>(v, w);
    md5_steps_at<4>(v, w, std::make_integer_sequence<int, 57>{});
}

template <int... I>
__device__ __forceinline__ void md5_steps_from61(uint32_t (&v)[4], const uint32_t (&w)[16],
                                                 std::integer_sequence<int, I...>)
{
    (md5_step<61 + I>(v, w), ...);
}

/* ---- fixed-length keys of FL bytes (1..55): one block, and every message
 * word past the key's data is a compile-time constant: zeros, the 0x80 pad
 * when it starts a word, the bit length FL * 8 in word 14
 * (src/hashkit/nc_md5.c:249-274). Such a word's w + T folds into one
 * constant (an SGPR operand of the v_add3): four VALU per step instead of
 * five. */
template <int FL>
constexpr bool fl_const(int k)
{
    return k > FL / 4 || (k == FL / 4 && FL % 4 == 0);
}

template <int FL>
constexpr uint32_t fl_word(int k)
{
    return k == 14 ? (uint32_t)FL * 8u : ((k == FL / 4 && FL % 4 == 0) ? 0x80u : 0u);
}

template <int I, int FL>
__device__ __forceinline__ void md5_step_fl(uint32_t (&v)[4], const uint32_t (&w)[16])
{
    static_assert(FL >= 1 && FL <= 55, "one block with the length behind the pad");
    constexpr int k = kM[I];
    if constexpr (fl_const<FL>(k)) {
        constexpr int u = (4 - (I & 3)) & 3;
        const uint32_t b = v[(u + 1) & 3], c = v[(u + 2) & 3], d = v[(u + 3) & 3];
        const uint32_t f = md5_f<I>(b, c, d);
        constexpr uint32_t wt = fl_word<FL>(k) + kT[I];
        v[u] = nc_rotl(v[u] + f + wt, kS[I]) + b;
    } else {
        md5_step<I>(v, w);
    }
}

template <int FL, int... I>
__device__ __forceinline__ void md5_steps_fl(uint32_t (&v)[4], const uint32_t (&w)[16],
                                             std::integer_sequence<int, I...>)
{
    (md5_step_fl<I, FL>(v, w), ...);
}

/* ---- the data-free last block of a key (src/hashkit/nc_md5.c:263-274):
 * words 1..13 are zero, so their steps take w + T as one constant; words 0
 * (0x80 or 0), 14 and 15 (the bit length) stay per lane ---- */
template <int I>
__device__ __forceinline__ void md5_step_tail(uint32_t (&v)[4], const uint32_t (&w)[16])
{
    constexpr int k = kM[I];
    if constexpr (k >= 1 && k <= 13) {
        constexpr int u = (4 - (I & 3)) & 3;
        const uint32_t b = v[(u + 1) & 3], c = v[(u + 2) & 3], d = v[(u + 3) & 3];
        const uint32_t f = md5_f<I>(b, c, d);
        v[u] = nc_rotl(v[u] + f + kT[I], kS[I]) + b;
    } else {
        md5_step<I>(v, w);
    }
}

template <int... I>
__device__ __forceinline__ void md5_steps_tail(uint32_t (&v)[4], const uint32_t (&w)[16],
                                               std::integer_sequence<int, I...>)
{
    (md5_step_tail<I>(v, w), ...);
}

/* A after a data-free last block w (words 1..13 zero) */
__device__ __forceinline__ uint32_t md5_tail_final_a(const uint32_t (&st)[4], const uint32_t (&w)[16])
{
    uint32_t v[4] = {st[0], st[1], st[2], st[3]};
    md5_steps_tail(v, w, std::make_integer_sequence<int, 61>{});
    return st[0] + v[0];
}

/* final block: only A is returned, and A's last update is step 60 */
__device__ __forceinline__ uint32_t md5_block_final_a(const uint32_t (&st)[4], const uint32_t (&w)[16])
{
    uint32_t v[4] = {st[0], st[1], st[2], st[3]};
    md5_steps(v, w, std::make_integer_sequence<int, 61>{});
    return st[0] + v[0];
}

/* ---- message padding by byte permutes ----
 * Word t of a key's last data block, with m = bytes of the key left in the
 * block (1..64): bytes j with 4t + j < m are the key's, byte m is 0x80,
 * the rest are 0. v_perm_b32(d, 0x80000000, sel) picks byte 4+j of d (key
 * byte j), byte 3 of 0x80000000 (the pad) or bytes 0-2 (zero). The selector
 * of word t is clamp(Y0 - t * kStep, 0, kKeep):
 *   kKeep = 0x07060504 (whole word kept), 0 (whole word zero), and for the
 *   word holding byte m (t = m / 4) one of kBoundary[m % 4], which lies
 *   strictly between them; kStep exceeds both gaps, so words before t clamp
 *   to kKeep and words after it to 0. */
constexpr uint32_t kPadSrc = 0x80000000u;
constexpr int32_t kKeep = 0x07060504;
constexpr int32_t kStep = 0x06000000;
constexpr uint32_t kBoundary0 = 0x02020203u; /* [pad, 0, 0, 0] */
constexpr uint32_t kBoundary1 = 0x02020304u; /* [key, pad, 0, 0] */
constexpr uint32_t kBoundary2 = 0x02030504u; /* [key, key, pad, 0] */
constexpr uint32_t kBoundary3 = 0x03060504u; /* [key, key, key, pad] */
static_assert(kStep > kKeep - (int32_t)kBoundary0 && kStep > (int32_t)kBoundary3, "selector ordering");
static_assert(16ll * kStep + (int64_t)kBoundary3 < (1ll << 31), "selector form fits int32");

__device__ __forceinline__ uint32_t pad_word(uint32_t d, int32_t y)
{
    const int32_t sel = y < 0 ? 0 : (y > kKeep ? kKeep : y); /* v_med3_i32 */
    return __builtin_amdgcn_perm(d, kPadSrc, (uint32_t)sel);
}

/* The message words y0 selector of a key of m (0..64) bytes in its last
 * data block, per lane: kBoundary[m % 4] + (m / 4) * kStep, no branches */
__device__ __forceinline__ int32_t pad_y0(uint32_t m)
{
    const uint32_t r = m & 3u;
    const uint64_t pair = (r & 2u) ? ((uint64_t)kBoundary3 << 32 | kBoundary2) : ((uint64_t)kBoundary1 << 32 | kBoundary0);
    const uint32_t bnd = (uint32_t)(pair >> (32u * (r & 1u)));
    return (int32_t)bnd + (int32_t)(m >> 2) * kStep;
}

/* The 16 message words of a block holding m (1..64) of the key's bytes, the
 * pad byte after them and zeros (no bit length: the caller adds it). When m
 * is the same on every active lane (fixed-length keys) the selectors are
 * wave-uniform and computed on the scalar unit; when it is 64 on every lane
 * (a full data block of long keys) the words stay as loaded. */
typedef unsigned int md5_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void msg_words(const md5_u32x4 (&d)[4], int32_t m, uint32_t pad_src, uint32_t (&w)[16])
{
    const int32_t m0 = __builtin_amdgcn_readfirstlane(m);
    if (__ballot(m != m0) == 0ull && m0 >= 64) {
#pragma unroll
        for (int t = 0; t < 16; t++) w[t] = d[t >> 2][t & 3];
    } else if (__ballot(m != m0) == 0ull) {
        const uint32_t r = (uint32_t)m0 & 3u;
        const uint32_t bnd = r == 0u ? kBoundary0 : (r == 1u ? kBoundary1 : (r == 2u ? kBoundary2 : kBoundary3));
        const int32_t y0 = (int32_t)bnd + (m0 >> 2) * kStep;
#pragma unroll
        for (int t = 0; t < 16; t++) {
            /* the clamp on the scalar unit (hipcc would use v_med3) and the
             * selector as the perm's one SGPR operand */
            uint32_t sel;
            asm("s_max_i32 %0, %1, 0\n\ts_min_i32 %0, %0, %2" : "=&s"(sel) : "s"(y0 - t * kStep), "s"(kKeep));
            w[t] = __builtin_amdgcn_perm(d[t >> 2][t & 3], pad_src, sel);
        }
    } else {
        const int32_t y0 = pad_y0((uint32_t)m);
#pragma unroll
        for (int t = 0; t < 16; t++) w[t] = pad_word(d[t >> 2][t & 3], y0 - t * kStep);
    }
}

/* The same, IN PLACE in the block's registers, per lane (the direct kernel,
 * whose steps read the block's own register set): the 16 words are rewritten
 * where they stand, so the register allocator keeps one set of 16 words. (A
 * wave-uniform branch with scalar selectors here made hipcc allocate 16 more
 * VGPRs for it and copy them back: occupancy 8 -> 6 waves per SIMD. Tiles of
 * one fixed length take the kernel's FL form instead.) */
__device__ __forceinline__ void pad_block(md5_u32x4 (&d)[4], int32_t m, uint32_t pad_src)
{
    const int32_t y0 = pad_y0((uint32_t)m);
#pragma unroll
    for (int t = 0; t < 16; t++) d[t >> 2][t & 3] = pad_word(d[t >> 2][t & 3], y0 - t * kStep);
}

/* The selectors as a table (pad_block_tab): the selector of a word with d
 * key bytes left from its start is kKeep for d >= 4, kBoundary[d] for d in
 * 0..3 and 0 (every byte from kPadSrc's zero byte) for d < 0. Entry i holds
 * d = 64 - i, so word t of a block holding m key bytes reads entry
 * 64 - m + 4t: one per-lane base and the word's offset as the LDS read's
 * immediate. 128 entries cover m = 1..64, t = 0..15. Lanes whose m differ by
 * 28 or 32 meet in a bank (~3.5 conflict cycles per read on C2); a second
 * copy 16 banks over for long keys moved the conflicts rather than removing
 * them (57 values of m over 32 banks), profiles/pmc_r05_md5pt.json. */
constexpr uint32_t kPadTabWords = 128;

__device__ __forceinline__ uint32_t pad_tab_entry(uint32_t i)
{
    const int32_t d = 64 - (int32_t)i;
    if (d >= 4) return (uint32_t)kKeep;
    if (d < 0) return 0u;
    return d == 0 ? kBoundary0 : (d == 1 ? kBoundary1 : (d == 2 ? kBoundary2 : kBoundary3));
}

/* pad_block with its selectors read from the LDS table gtab (eight
 * ds_read2_b32 on the LDS pipe) instead of computed: one VALU per word (the
 * perm) instead of three (the form's subtract, the clamp, the perm) */
__device__ __forceinline__ void pad_block_tab(md5_u32x4 (&d)[4], int32_t m, uint32_t pad_src, const uint32_t *gtab)
{
    const uint32_t *g = gtab + (64 - m);
    uint32_t sel[16];
#pragma unroll
    for (int t = 0; t < 16; t++) sel[t] = g[4 * t];
#pragma unroll
    for (int t = 0; t < 16; t++) d[t >> 2][t & 3] = __builtin_amdgcn_perm(d[t >> 2][t & 3], pad_src, sel[t]);
}

/* pad_block with the wave-uniform cases of msg_words (the line kernel, whose
 * blocks come from LDS reads, so no load is in flight into d): a length
 * shared by every lane pads by scalar selectors, a full block (m = 64 on
 * every lane) stays as read — 16 v_perm / v_mov fewer per block of a long
 * key. */
__device__ __forceinline__ void pad_block_u(md5_u32x4 (&d)[4], int32_t m, uint32_t pad_src)
{
    const int32_t m0 = __builtin_amdgcn_readfirstlane(m);
    if (__ballot(m != m0) == 0ull) {
        if (m0 < 64) {
            const uint32_t r = (uint32_t)m0 & 3u;
            const uint32_t bnd = r == 0u ? kBoundary0 : (r == 1u ? kBoundary1 : (r == 2u ? kBoundary2 : kBoundary3));
            const int32_t y0 = (int32_t)bnd + (m0 >> 2) * kStep;
#pragma unroll
            for (int t = 0; t < 16; t++) {
                uint32_t sel;
                asm("s_max_i32 %0, %1, 0\n\ts_min_i32 %0, %0, %2" : "=&s"(sel) : "s"(y0 - t * kStep), "s"(kKeep));
                d[t >> 2][t & 3] = __builtin_amdgcn_perm(d[t >> 2][t & 3], pad_src, sel);
            }
        }
    } else {
        pad_block(d, m, pad_src);
    }
}

/* md5 of a key of len bytes at byte p of a dword-readable slab (LDS, or a
 * 16-byte aligned global buffer): the direct pipeline's blocks (padding by
 * byte permutes, the final block's 61 steps, a data-free tail block when the
 * padding does not fit; src/hashkit/nc_md5.c:245-321), message words
 * realigned from dword reads. Reads up to 68 bytes past each block's start. */
template <class Words>
__device__ __forceinline__ uint32_t md5_slab_key(const Words &slab, uint32_t p, uint32_t len, uint32_t pad_src)
{
    uint32_t st[4] = {NC_MD5_A0, NC_MD5_B0, NC_MD5_C0, NC_MD5_D0};
    const uint32_t sh = p & 3u;
    const uint32_t w0 = p >> 2;
    uint32_t res = 0u;
    const uint32_t nb = (len + 63u) >> 6; /* blocks holding key bytes */
    for (uint32_t b = 0; b < nb; b++) {
        const int32_t rem = (int32_t)len - 64 * (int32_t)b;
        uint32_t a[17];
#pragma unroll
        for (int k = 0; k < 17; k++) a[k] = slab[w0 + 16u * b + (uint32_t)k];
        md5_u32x4 d[4];
#pragma unroll
        for (int k = 0; k < 16; k++) d[k >> 2][k & 3] = __builtin_amdgcn_alignbyte(a[k + 1], a[k], sh);
        uint32_t w[16];
        msg_words(d, rem < 64 ? rem : 64, pad_src, w);
        const bool fin = rem <= 55; /* the bit length fits behind the pad */
        if (fin) {
            w[14] = len << 3;
            w[15] = len >> 29;
        }
        uint32_t v[4] = {st[0], st[1], st[2], st[3]};
        md5_steps(v, w, std::make_integer_sequence<int, 61>{});
        if (fin) {
            res = st[0] + v[0]; /* digest bytes 0..3 (nc_md5.c:317-320): state A */
        } else {
            md5_steps_from61(v, w, std::make_integer_sequence<int, 3>{});
            st[0] += v[0];
            st[1] += v[1];
            st[2] += v[2];
            st[3] += v[3];
        }
    }
    const uint32_t last = len - 64u * (nb ? nb - 1u : 0u); /* key bytes in the last data block */
    if (len == 0u || last >= 56u) {
        uint32_t w[16] = {};
        w[0] = (len & 63u) == 0u ? 0x80u : 0u;
        w[14] = len << 3;
        w[15] = len >> 29;
        res = md5_tail_final_a(st, w);
    }
    return res;
}

} // namespace nc_md5s

#endif
