/*
 * Slicing-by-4 crc16 / crc32 / crc32a (src/hashkit/nc_crc16.c:56-66,
 * nc_crc32.c:99-123) for gfx950 kernels that keep the tables in LDS: the
 * direct pipeline (nc_bytes_kernels.hip).
 *
 * Four tables T0..T3 of 256 entries: T0 is the byte table (generated from the
 * polynomials, nc_hash_algo.h), Tk advances Tk-1 by one more zero byte, so a
 * whole word costs four INDEPENDENT lookups (one LDS latency) instead of four
 * chained ones. Each entry is stored R times, copy c for lanes with
 * (lane & (R-1)) == c: word (k * 256 + e) * R + c. ds_read_b32 serves 32 lanes
 * per LDS cycle over 32 banks (MI355X_MICROARCH.md §LDS); with R = 8 the
 * lanes of one copy class meet only when their entries agree mod 4, which
 * keeps a 64-lane lookup near conflict-free. 4 KiB x R.
 */
#ifndef NC_CRC_SLICE_H
#define NC_CRC_SLICE_H

#include <hip/hip_runtime.h>

#include <stdint.h>

#include "nc_gpuhash.h"
#include "nc_hash_algo.h"

namespace nc_slice {

template <int MODE>
constexpr bool is_crc()
{
    return MODE == NC_GPUHASH_CRC16 || MODE == NC_GPUHASH_CRC32 || MODE == NC_GPUHASH_CRC32A;
}

/* NT tables (4: slicing-by-4; 8: slicing-by-8) of 256 entries, R copies */
template <uint32_t R, uint32_t NT = 4>
constexpr uint32_t table_words()
{
    return NT * 256u * R;
}

/* entry e of table k */
template <int MODE>
__device__ __forceinline__ uint32_t entry(uint32_t k, uint32_t e)
{
    if constexpr (MODE == NC_GPUHASH_CRC16) { /* Tk[e] = e * x^(16 + 8k) mod P, 16 bits */
        uint32_t v = nc_crc16_entry(e);
        for (uint32_t j = 0; j < k; j++) v = ((v << 8) ^ nc_crc16_entry(v >> 8)) & 0xffffu;
        return v;
    } else { /* reflected: Tk[e] = (Tk-1[e] >> 8) ^ T0[Tk-1[e] & 0xff] */
        uint32_t v = nc_crc32_entry(e);
        for (uint32_t j = 0; j < k; j++) v = (v >> 8) ^ nc_crc32_entry(v & 0xffu);
        return v;
    }
}

/* fill the R-copy tables at tab, threads t = first, first + step, ... */
template <int MODE, uint32_t R, uint32_t NT = 4>
__device__ __forceinline__ void fill(uint32_t *tab, uint32_t first, uint32_t step)
{
    for (uint32_t i = first; i < NT * 256u; i += step) {
        const uint32_t v = entry<MODE>(i >> 8, i & 255u);
#pragma unroll
        for (uint32_t c = 0; c < R; c++) tab[i * R + c] = v;
    }
}

/* this lane's copy, as a byte offset: (lane & (R-1)) * 4 */
template <uint32_t R>
__device__ __forceinline__ uint32_t copy_of(uint32_t lane)
{
    return (lane & (R - 1u)) * 4u;
}

/* table k, entry idx (0..255), in the copy at byte offset cb */
template <uint32_t R>
__device__ __forceinline__ uint32_t look(const uint32_t *tab, uint32_t idx, uint32_t cb, uint32_t k = 0)
{
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(tab) + (k << (10 + __builtin_ctz(R))) +
                                               ((idx * R * 4u) | cb));
}

/* byte b into state h, through T0 */
template <int MODE, uint32_t R>
__device__ __forceinline__ uint32_t byte(uint32_t h, uint32_t b, const uint32_t *tab, uint32_t cb)
{
    if constexpr (MODE == NC_GPUHASH_CRC16) return NC_CRC16_NEXT(h, look<R>(tab, NC_CRC16_IDX(h, b), cb));
    else return NC_CRC32_NEXT(h, look<R>(tab, NC_CRC32_IDX(h, b), cb));
}

/* the 4 bytes of word w */
template <int MODE, uint32_t R>
__device__ __forceinline__ uint32_t word(uint32_t h, uint32_t w, const uint32_t *tab, uint32_t cb)
{
    if constexpr (MODE == NC_GPUHASH_CRC16) {
        /* MSB-first slicing-by-4 on the 16-bit crc: V = crc << 16 ^ the word's
         * bytes big-endian; crc' = V * x^16 mod P. The unmasked 32-bit state
         * (nc_crc16.c:59-65) keeps shifted history in bits 16-31; those are
         * rebuilt by the byte steps at the key's end (callers leave the last
         * kWhole - 4 >= 2 bytes to them), so here only the low 16 bits are
         * carried. */
        const uint32_t v = ((h & 0xffffu) << 16) ^ __builtin_bswap32(w);
        return look<R>(tab, v >> 24, cb, 3) ^ look<R>(tab, (v >> 16) & 0xffu, cb, 2) ^
               look<R>(tab, (v >> 8) & 0xffu, cb, 1) ^ look<R>(tab, v & 0xffu, cb, 0);
    } else {
        /* reflected slicing-by-4: the word meets the state's low bytes */
        const uint32_t x = h ^ w;
        return look<R>(tab, x >> 24, cb, 0) ^ look<R>(tab, (x >> 16) & 0xffu, cb, 1) ^
               look<R>(tab, (x >> 8) & 0xffu, cb, 2) ^ look<R>(tab, x & 0xffu, cb, 3);
    }
}

/* the 8 bytes of words w0, w1 (slicing-by-8: eight independent lookups, half
 * the dependent steps of slicing-by-4); tables 0..7 */
template <int MODE, uint32_t R>
__device__ __forceinline__ uint32_t word2(uint32_t h, uint32_t w0, uint32_t w1, const uint32_t *tab, uint32_t cb)
{
    if constexpr (MODE == NC_GPUHASH_CRC16) {
        /* MSB first: the state meets the first two bytes; byte i of the 8
         * goes through table 7 - i (the history bits: as in word()) */
        const uint32_t v = ((h & 0xffffu) << 16) ^ __builtin_bswap32(w0);
        const uint32_t u = __builtin_bswap32(w1);
        return (look<R>(tab, v >> 24, cb, 7) ^ look<R>(tab, (v >> 16) & 0xffu, cb, 6)) ^
               (look<R>(tab, (v >> 8) & 0xffu, cb, 5) ^ look<R>(tab, v & 0xffu, cb, 4)) ^
               (look<R>(tab, u >> 24, cb, 3) ^ look<R>(tab, (u >> 16) & 0xffu, cb, 2)) ^
               (look<R>(tab, (u >> 8) & 0xffu, cb, 1) ^ look<R>(tab, u & 0xffu, cb, 0));
    } else {
        /* reflected: byte i of the 8 (LSB of w0 first) through table 7 - i */
        const uint32_t x = h ^ w0;
        return (look<R>(tab, x & 0xffu, cb, 7) ^ look<R>(tab, (x >> 8) & 0xffu, cb, 6)) ^
               (look<R>(tab, (x >> 16) & 0xffu, cb, 5) ^ look<R>(tab, x >> 24, cb, 4)) ^
               (look<R>(tab, w1 & 0xffu, cb, 3) ^ look<R>(tab, (w1 >> 8) & 0xffu, cb, 2)) ^
               (look<R>(tab, (w1 >> 16) & 0xffu, cb, 1) ^ look<R>(tab, w1 >> 24, cb, 0));
    }
}

/* the 4 * NW bytes of words w[0 .. NW) (slicing-by-4NW: NW = 1, 2, 4 words,
 * one dependent step); byte i of the group through table 4 * NW - 1 - i */
template <int MODE, uint32_t R, int NW>
__device__ __forceinline__ uint32_t words(uint32_t h, const uint32_t *w, const uint32_t *tab, uint32_t cb)
{
    constexpr uint32_t T = 4u * NW - 1u;
    uint32_t acc = 0u;
    if constexpr (MODE == NC_GPUHASH_CRC16) {
#pragma unroll
        for (int i = 0; i < NW; i++) {
            const uint32_t v = (i == 0 ? (h & 0xffffu) << 16 : 0u) ^ __builtin_bswap32(w[i]);
            acc ^= (look<R>(tab, v >> 24, cb, T - 4u * i) ^ look<R>(tab, (v >> 16) & 0xffu, cb, T - 4u * i - 1u)) ^
                   (look<R>(tab, (v >> 8) & 0xffu, cb, T - 4u * i - 2u) ^ look<R>(tab, v & 0xffu, cb, T - 4u * i - 3u));
        }
    } else {
#pragma unroll
        for (int i = 0; i < NW; i++) {
            const uint32_t x = (i == 0 ? h : 0u) ^ w[i];
            acc ^= (look<R>(tab, x & 0xffu, cb, T - 4u * i) ^ look<R>(tab, (x >> 8) & 0xffu, cb, T - 4u * i - 1u)) ^
                   (look<R>(tab, (x >> 16) & 0xffu, cb, T - 4u * i - 2u) ^ look<R>(tab, x >> 24, cb, T - 4u * i - 3u));
        }
    }
    return acc;
}

/* a word is taken whole only when at least kWhole key bytes start at it */
template <int MODE>
constexpr int32_t whole()
{
    return MODE == NC_GPUHASH_CRC16 ? 6 : 4;
}

/* the first nb (per lane, <= 0 for none) bytes of word w, one at a time */
template <int MODE, uint32_t R>
__device__ __forceinline__ uint32_t bytes(uint32_t h, uint32_t w, int32_t nb, const uint32_t *tab, uint32_t cb)
{
#pragma unroll
    for (int j = 0; j < 4; j++)
        if (j < nb) h = byte<MODE, R>(h, (w >> (8 * j)) & 0xffu, tab, cb);
    return h;
}

/* word w of a key with nb (per lane) bytes left from its start */
template <int MODE, uint32_t R>
__device__ __forceinline__ uint32_t step(uint32_t h, uint32_t w, int32_t nb, const uint32_t *tab, uint32_t cb)
{
    if (nb >= whole<MODE>()) return word<MODE, R>(h, w, tab, cb);
    if (nb > 0) return bytes<MODE, R>(h, w, nb, tab, cb);
    return h;
}

} // namespace nc_slice

#endif
