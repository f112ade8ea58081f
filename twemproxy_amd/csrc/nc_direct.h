/*
 * The direct per-lane pipeline shared by nc_md5_kernels.hip and
 * nc_bytes_kernels.hip (gfx950): a wave owns 64-key tiles (lane = key) and
 * reads each key's bytes in 64-byte blocks, one block of every lane's key per
 * ROUND, with the next round's block in flight while a round computes.
 *
 *   - Every load goes through a buffer resource with a wave-uniform base
 *     (SGPRs) and a 32-bit per-lane offset: no 64-bit address arithmetic in
 *     the loop, and loads past the resource end return zeros instead of
 *     faulting (no clamping).
 *   - Offsets: each lane loads the low dwords of its key's start and end (a
 *     64-key tile spans < 4 GiB), the tile's 64-bit base comes by one scalar
 *     load.
 *   - A block reaches the lanes either straight into registers (four
 *     unaligned 16-byte loads per lane, only the chunks that hold key bytes:
 *     gfx9 global memory runs in unaligned mode), or — for long keys, where
 *     64 scattered lanes per instruction saturate the texture addresser — by
 *     LDS-DMA in 64-byte pieces into a per-wave 4 KiB image (key k's block at
 *     k * 64), 16 pieces per instruction.
 */
#ifndef NC_DIRECT_H
#define NC_DIRECT_H

#include <hip/hip_runtime.h>

#include <stdint.h>

#include "nc_gpuhash.h"

namespace nc_direct {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr int kRsrcWord3 = 0x00020000; /* gfx9 raw buffer: DATA_FORMAT 32, no swizzle */
constexpr int kAuxNt = 2;              /* slc: the streaming cache policy (nt) */
constexpr uint32_t kImage = 64u * 64u;      /* one 64-byte block of each of a tile's 64 keys */
constexpr uint32_t kLineImage = 64u * 128u; /* one 128-byte line of each of a tile's 64 keys */

__device__ __forceinline__ rsrc_t make_rsrc(const void *base, uint64_t nbytes)
{
    /* the clamp by the high dword, on the scalar unit: hipcc turns a plain
     * C form back into a 64-bit unsigned compare, which gfx9 can only do on
     * the VALU (the SALU has no 64-bit less-than). nbytes is wave-uniform. */
    uint32_t n;
    asm("s_cmp_lg_u32 %1, 0\n\ts_cselect_b32 %0, -1, %2"
        : "=s"(n)
        : "s"((uint32_t)(nbytes >> 32)), "s"((uint32_t)nbytes)
        : "scc");
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)n, kRsrcWord3);
}

/* A tile's keys as the lanes hold them. */
struct TileKeys {
    uint64_t s0;   /* wave-uniform: off[k0], the tile's first key (the data resource's base) */
    uint32_t srel; /* this lane's key start - s0 */
    uint32_t len;
    bool valid;
    uint32_t nv; /* wave-uniform: the tile's keys below nkeys (valid = lane < nv) */
};

/* Offsets of a tile, as loaded (consumed one round later). */
struct Offs {
    uint32_t s, e; /* low dwords of this lane's key start and end */
    uint64_t s0;
};

/* A wave's tiles: local index j = 0 .. n-1 is global tile base + j * S.
 * Consecutive (IL false, S = 1: `chunk` neighbouring tiles per wave) or
 * interleaved over the grid (IL, S = every wave of the launch), in which case
 * the resident waves read neighbouring tiles at any moment instead of regions
 * `chunk` tiles apart. Either way the grid covers every tile once. Every
 * index is 32-bit: the direct pipeline takes batches of < 2^32 keys (the
 * launcher checks), so tiles, key indices and their compares stay on the
 * scalar unit. */
template <bool IL>
struct Tiles {
    uint32_t base, S, n;
    __device__ __forceinline__ uint32_t at(uint32_t j) const { return IL ? base + j * S : base + j; }
};

template <bool IL>
__device__ __forceinline__ Tiles<IL> wave_tiles(uint64_t ntiles64, uint32_t chunk, uint32_t waves_per_block,
                                                uint32_t wave)
{
    const uint32_t ntiles = (uint32_t)ntiles64; /* < 2^26 */
    const uint32_t w = blockIdx.x * waves_per_block + wave;
    Tiles<IL> t;
    if constexpr (IL) {
        t.base = w;
        t.S = gridDim.x * waves_per_block;
        t.n = w < ntiles ? (ntiles - w + t.S - 1u) / t.S : 0u;
    } else {
        t.base = w * chunk;
        t.S = 1u;
        t.n = t.base < ntiles ? ntiles - t.base : 0u;
    }
    if (t.n > chunk) t.n = chunk;
    return t;
}

template <bool IL>
struct Walker {
    const uint8_t *keys;
    const uint64_t *off;
    uint32_t nkeys;  /* < 2^32 (the launchers check) */
    uint64_t kbytes; /* readable bytes from keys: off[nkeys] + NC_GPUHASH_PAD */
    Tiles<IL> tiles; /* this wave's tiles; local indices below */
    uint32_t tlast;  /* = tiles.n */
    uint32_t lane;

    __device__ __forceinline__ void init(const uint8_t *k, const uint64_t *o, uint64_t n, const Tiles<IL> &tl,
                                         uint32_t ln)
    {
        keys = k;
        off = o;
        nkeys = (uint32_t)n;
        kbytes = off[n] + (uint64_t)NC_GPUHASH_PAD;
        tiles = tl;
        tlast = tl.n;
        lane = ln;
    }

    /* first key of local tile tl */
    __device__ __forceinline__ uint32_t key0(uint32_t tl) const { return tiles.at(tl) * 64u; }

    /* offsets of local tile tl; this wave's last tile again past its range, so
     * that every round issues the same loads (keys past nkeys read as 0).
     * (Measured: taking a key's end from the next lane by DPP, or the tile
     * base by vector load + v_readlane, costs md5 1.5 % each and gains the
     * crcs nothing.) AUX: the loads' cache policy — streaming for the byte
     * kernels, the default for md5 (profiles/r03_cache_policy_ab.md). */
    template <int AUX = kAuxNt>
    __device__ __forceinline__ Offs load_off(uint32_t tl) const
    {
        const uint32_t k0 = key0(tl < tlast ? tl : tlast - 1u);
        const rsrc_t r = make_rsrc(off + k0, ((uint64_t)(nkeys - k0) + 1u) * 8u);
        Offs o;
        o.s = __builtin_amdgcn_raw_buffer_load_b32(r, (int)(lane * 8u), 0, AUX);
        o.e = __builtin_amdgcn_raw_buffer_load_b32(r, (int)(lane * 8u + 8u), 0, AUX);
        o.s0 = off[k0];
        return o;
    }

    __device__ __forceinline__ TileKeys keys_of(uint32_t tl, const Offs &o) const
    {
        TileKeys t;
        t.s0 = o.s0;
        t.srel = o.s - (uint32_t)o.s0;
        t.len = o.e - o.s;
        /* the tile's key count, uniform and 32-bit (lane < it: one VALU compare) */
        const uint32_t k0 = key0(tl);
        /* on the scalar unit: hipcc turns the plain form into a saturating
         * VALU subtract (and the tile selects that follow into v_cndmask) */
        uint32_t nv;
        asm("s_sub_u32 %0, %1, %2\n\ts_cselect_b32 %0, 0, %0" : "=&s"(nv) : "s"(nkeys), "s"(k0) : "scc");
        t.valid = lane < nv;
        t.nv = nv;
        return t;
    }

    /* block b of the lanes' keys into registers: only the 16-byte chunks that
     * hold key bytes (a chunk past the key keeps stale words; callers mask) */
    __device__ __forceinline__ void load_regs(const TileKeys &t, uint32_t b, u32x4 (&d)[4]) const
    {
        const rsrc_t r = make_rsrc(keys + t.s0, kbytes - t.s0);
        const int vo = (int)(t.srel + 64u * b);
        const int32_t rem = (int32_t)t.len - 64 * (int32_t)b;
        if (rem > 0) d[0] = __builtin_amdgcn_raw_buffer_load_b128(r, vo, 0, 0);
        if (rem > 16) d[1] = __builtin_amdgcn_raw_buffer_load_b128(r, vo + 16, 0, 0);
        if (rem > 32) d[2] = __builtin_amdgcn_raw_buffer_load_b128(r, vo + 32, 0, 0);
        if (rem > 48) d[3] = __builtin_amdgcn_raw_buffer_load_b128(r, vo + 48, 0, 0);
    }

    /* block b of the lanes' keys into the wave's LDS image by LDS-DMA:
     * instruction i moves keys 16i .. 16i+15, four lanes per key */
    __device__ __forceinline__ void dma(const TileKeys &t, uint32_t b, uint8_t *img) const
    {
        const rsrc_t r = make_rsrc(keys + t.s0, kbytes - t.s0);
        const uint32_t j = lane & 3u;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int src = 16 * i + (int)(lane >> 2);
            const uint32_t vo = (uint32_t)__shfl((int)t.srel, src);
            const int32_t rem = __shfl((int)t.len, src) - 64 * (int32_t)b;
            if (rem > (int32_t)(16u * j))
                __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)(img + 1024 * i),
                                                          16, vo + 64u * b + 16u * j, 0, 0, 0);
        }
    }

    /* Long keys, whole lines: bytes [128b, 128b + 128) of the lanes' keys
     * into an 8 KiB image (key k's 128 bytes at k * 128) — full 128-byte
     * lines, so a line's two 64-byte halves are not fetched a round apart
     * (the second fetch missed L2 three times in four: 1.74x the HBM bytes on
     * 256-byte keys). Instruction i moves keys 8i .. 8i+7, eight lanes per
     * key. Chunk j of key k lands in slot j ^ ((k >> 1) & 7) of its row, so
     * the readers' ds_read_b128 at a 128-byte lane stride hit distinct banks:
     * a 16-lane group of ds_read_b128 ({0-3,12-15,20-27}, {4-11,16-19,28-31},
     * the same + 32; MI355X_MICROARCH.md §LDS) holds eight even and eight odd
     * lanes, whose rows start on bank 0 and 32, and (k >> 1) & 7 differs
     * across each eight (with k & 7, lanes 0 and 24 met: one conflict cycle
     * per key, SQ_LDS_BANK_CONFLICT = 2^25 on the C4 shard, pmc_r04d.json). */
    __device__ __forceinline__ void dma_lines(const TileKeys &t, uint32_t b, uint8_t *img) const
    {
        const rsrc_t r = make_rsrc(keys + t.s0, kbytes - t.s0);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int key = 8 * i + (int)(lane >> 3);
            const uint32_t j = (lane & 7u) ^ (((uint32_t)key >> 1) & 7u); /* the global chunk for this slot */
            const uint32_t vo = (uint32_t)__shfl((int)t.srel, key);
            const int32_t rem = __shfl((int)t.len, key) - 128 * (int32_t)b;
            if (rem > (int32_t)(16u * j))
                __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)(img + 1024 * i),
                                                          16, vo + 128u * b + 16u * j, 0, 0, 0);
        }
    }

    /* Long keys, two whole lines per round: bytes [256b, 256b + 256) of the
     * lanes' keys into a 16 KiB image (key k's 256 bytes at k * 256), for
     * workgroups few enough to double the bytes in flight per wave (eight
     * waves per CU: 128 KiB). Instruction i moves keys 4i .. 4i+3, sixteen
     * lanes per key; chunk j of key k lands in slot j ^ (k & 15): every row
     * starts on bank 0, so slot s sits on banks 4s .. 4s+3, and the 16 lanes
     * of each ds_read_b128 lane group (MI355X_MICROARCH.md §LDS: k mod 16
     * distinct within a group) read 16 distinct slots. */
    __device__ __forceinline__ void dma_pairs(const TileKeys &t, uint32_t b, uint8_t *img) const
    {
        const rsrc_t r = make_rsrc(keys + t.s0, kbytes - t.s0);
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int key = 4 * i + (int)(lane >> 4);
            const uint32_t j = (lane & 15u) ^ ((uint32_t)key & 15u); /* the global chunk for this slot */
            const uint32_t vo = (uint32_t)__shfl((int)t.srel, key);
            const int32_t rem = __shfl((int)t.len, key) - 256 * (int32_t)b;
            if (rem > (int32_t)(16u * j))
                __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)(img + 1024 * i),
                                                          16, vo + 256u * b + 16u * j, 0, 0, 0);
        }
    }

    /* this lane's 256 bytes from the pair image (see dma_pairs) */
    __device__ __forceinline__ void read_pairs(const uint8_t *img, u32x4 (&d)[16]) const
    {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint8_t *row = img + lane * 256u;
        const uint32_t sw = lane & 15u;
#pragma unroll
        for (int c = 0; c < 16; c++) d[c] = *reinterpret_cast<const u32x4 *>(row + 16u * ((uint32_t)c ^ sw));
    }

    /* this lane's 128 bytes from the line image (see dma_lines) */
    __device__ __forceinline__ void read_lines(const uint8_t *img, u32x4 (&d0)[4], u32x4 (&d1)[4]) const
    {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint8_t *row = img + lane * 128u;
        const uint32_t sw = (lane >> 1) & 7u;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            d0[c] = *reinterpret_cast<const u32x4 *>(row + 16u * ((uint32_t)c ^ sw));
            d1[c] = *reinterpret_cast<const u32x4 *>(row + 16u * ((uint32_t)(c + 4) ^ sw));
        }
    }

    /* this lane's block from the LDS image, DMA'd during the previous round.
     * hipcc does not order these reads after a loop-carried LDS-DMA: wait for
     * every outstanding vector-memory op (the DMA and the offset loads issued
     * right after it) */
    __device__ __forceinline__ void read_img(const uint8_t *img, u32x4 (&d)[4]) const
    {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int c = 0; c < 4; c++) d[c] = *reinterpret_cast<const u32x4 *>(img + lane * 64u + 16u * c);
    }
};

} // namespace nc_direct

#endif
