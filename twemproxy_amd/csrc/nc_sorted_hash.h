/*
 * Byte-serial key hashes over length-sorted rounds, shared by the
 * wave-sorted pipeline (nc_wsort_kernels.hip) and the wave ring's sorted
 * rounds (nc_gpuhash_kernels.hip): fnv1_64, fnv1a_64, fnv1_32, fnv1a_32
 * (src/hashkit/nc_fnv.c:26-82) and one_at_a_time
 * (src/hashkit/nc_one_at_a_time.c:35-51).
 *
 * A round is 64 keys, one per lane, in an LDS slab, sorted by length so the
 * round's shortest (Lmin) and longest (Lmax) key bound its work. Words every
 * key covers run plain; the words between Lmin and Lmax keep, per lane, the
 * state after its key's last byte (selects, no exec-mask branches).
 */
#ifndef NC_SORTED_HASH_H
#define NC_SORTED_HASH_H

#include <hip/hip_runtime.h>

#include <stdint.h>

#include "nc_gpuhash.h"
#include "nc_hash_algo.h"

namespace nc_sh {

template <int MODE>
constexpr bool supports()
{
    return MODE == NC_GPUHASH_ONE_AT_A_TIME || MODE == NC_GPUHASH_FNV1_64 || MODE == NC_GPUHASH_FNV1A_64 ||
           MODE == NC_GPUHASH_FNV1_32 || MODE == NC_GPUHASH_FNV1A_32;
}

template <int MODE>
__device__ __forceinline__ uint32_t init_state()
{
    if constexpr (MODE == NC_GPUHASH_FNV1_64 || MODE == NC_GPUHASH_FNV1A_64) return NC_FNV64_INIT32;
    if constexpr (MODE == NC_GPUHASH_FNV1_32 || MODE == NC_GPUHASH_FNV1A_32) return NC_FNV32_INIT;
    return 0u; /* one_at_a_time */
}

template <int MODE>
__device__ __forceinline__ uint32_t final_state(uint32_t h)
{
    if constexpr (MODE == NC_GPUHASH_ONE_AT_A_TIME) return nc_oaat_final(h);
    return h;
}

template <int MODE>
__device__ __forceinline__ uint32_t byte_step(uint32_t h, uint32_t b)
{
    if constexpr (MODE == NC_GPUHASH_FNV1A_64) return nc_fnv1a_64_step(h, b);
    else if constexpr (MODE == NC_GPUHASH_FNV1_64) return nc_fnv1_64_step(h, b);
    else if constexpr (MODE == NC_GPUHASH_FNV1_32) return nc_fnv1_32_step(h, b);
    else if constexpr (MODE == NC_GPUHASH_FNV1A_32) return nc_fnv1a_32_step(h, b);
    else return nc_oaat_step(h, b);
}

template <int MODE>
__device__ __forceinline__ uint32_t word_step(uint32_t h, uint32_t w)
{
#pragma unroll
    for (int j = 0; j < 4; j++) h = byte_step<MODE>(h, (w >> (8 * j)) & 0xffu);
    return h;
}

/* The four byte states of word x after h; the state after the key's last
 * byte of this word is kept: kb = key bytes left from this word's first
 * (<= 0: none of it). */
template <int MODE>
__device__ __forceinline__ uint32_t ragged_word(uint32_t h, uint32_t x, int32_t kb)
{
    const uint32_t h1 = byte_step<MODE>(h, x & 0xffu);
    const uint32_t h2 = byte_step<MODE>(h1, (x >> 8) & 0xffu);
    const uint32_t h3 = byte_step<MODE>(h2, (x >> 16) & 0xffu);
    const uint32_t h4 = byte_step<MODE>(h3, x >> 24);
    return kb >= 4 ? h4 : kb == 3 ? h3 : kb == 2 ? h2 : kb == 1 ? h1 : h;
}

/* Key of `len` bytes at slab byte p in a round whose keys are Lmin .. Lmax
 * bytes (wave-uniform, the round is sorted). Dwords come aligned from LDS and
 * are realigned with v_alignbyte. Words every lane's key covers run plain;
 * the words between the round's shortest and longest key keep, per lane, the
 * state after its last byte (no exec-mask branches). */
template <int MODE>
__device__ __forceinline__ uint32_t hash_slab(const uint32_t *slab, uint32_t p, uint32_t len, uint32_t Lmin,
                                              uint32_t Lmax)
{
    uint32_t h = init_state<MODE>();
    const uint32_t *sw = slab + (p >> 2);
    const uint32_t sh = p & 3u;
    for (uint32_t g = 0; 64u * g < Lmax; g++) {
        const uint32_t Lg = Lmax - 64u * g;                      /* uniform bytes left in the round */
        const int32_t Ng = (int32_t)Lmin - 64 * (int32_t)g;      /* uniform: bytes every key still has */
        /* dwords in groups of four (uniform conditions), all issued before
         * the first word is hashed */
        const uint32_t *sg = sw + 16u * g;
        const int32_t kb0 = (int32_t)len - 64 * (int32_t)g;
        uint32_t w[17];
#pragma unroll
        for (int t = 0; t < 5; t++) w[t] = sg[t];
#pragma unroll
        for (int grp = 1; grp < 4; grp++) {
            if (Lg > 16u * (uint32_t)grp) {
#pragma unroll
                for (int t = 4 * grp + 1; t < 4 * grp + 5; t++) w[t] = sg[t];
            }
        }
#pragma unroll
        for (int t = 0; t < 16; t++) {
            if (4u * (uint32_t)t >= Lg) break;
            const uint32_t x = __builtin_amdgcn_alignbyte(w[t + 1], w[t], sh);
            if (4 * t + 4 <= Ng) h = word_step<MODE>(h, x);
            else h = ragged_word<MODE>(h, x, kb0 - 4 * t);
        }
    }
    return h;
}

/* exclusive prefix sum over the wave's 64 lanes */
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t lane)
{
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, d);
        if (lane >= (uint32_t)d) x += y;
    }
    return x - v;
}

/* maximum over the wave's 64 lanes (uniform result) */
__device__ __forceinline__ uint32_t wave_max(uint32_t v)
{
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_xor((int)v, d);
        v = v > y ? v : y;
    }
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

/* minimum over the wave's 64 lanes (uniform result) */
__device__ __forceinline__ uint32_t wave_min(uint32_t v)
{
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_xor((int)v, d);
        v = v < y ? v : y;
    }
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

} // namespace nc_sh

#endif
