/*
 * Byte-serial modes on the wave-sorted pipeline (gfx950): fnv1_64, fnv1a_64,
 * fnv1_32, fnv1a_32 (src/hashkit/nc_fnv.c:26-82) and one_at_a_time
 * (src/hashkit/nc_one_at_a_time.c:35-51) for short keys of varying length
 * (Zipf 8-64 B).
 *
 * One lane per key makes a wave run as long as its longest key: under Zipf
 * 8-64 B a 64-key wave pays ~61 byte steps for a 19.3-byte mean. Here a WAVE
 * owns a 256-key tile and, with no workgroup barrier:
 *
 *   1. stages the tile's byte span in its private LDS slab by coalesced
 *      16-byte loads (lane i moves bytes 16(i + 64j) .. +15, j < 6: every
 *      wave instruction reads 1 KiB contiguous), issued one tile ahead into
 *      registers so they are in flight while the previous tile hashes;
 *   2. counting-sorts the 256 keys by length (one LDS atomic per key, a
 *      64-lane scan) into four rounds of 64;
 *   3. hashes the rounds from LDS, each lane one key, realigned dwords
 *      (v_alignbyte), so a round costs its own longest key: ~110 byte steps
 *      per 256 keys instead of ~243 (four unsorted waves).
 *
 * A tile whose span does not fit the slab (long keys) hashes straight from
 * global memory, one key after another per lane.
 */
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "nc_direct.h"
#include "nc_out_policy.h"
#include "nc_gpuhash.h"
#include "nc_hash_algo.h"
#include "nc_sorted_hash.h"

namespace {

using nc_direct::kAuxNt;
using nc_direct::make_rsrc;
using nc_direct::rsrc_t;
using nc_direct::Tiles;
using nc_direct::u32x4;
using nc_direct::wave_tiles;
using nc_sh::byte_step;
using nc_sh::final_state;
using nc_sh::hash_slab;
using nc_sh::init_state;
using nc_sh::wave_excl_scan;
using nc_sh::wave_max;
using nc_sh::wave_min;

constexpr uint32_t kTK = 256;                 /* keys per tile (one wave) */
constexpr uint32_t kJ = 6;                    /* 16-byte slab chunks per lane */
constexpr uint32_t kCap = 64u * 16u * kJ;     /* 6 KiB slab: Zipf 8-64 B tiles average 4.9 KiB */
constexpr uint32_t kClasses = 64;             /* length classes 0..63 (63 = 63+) */
constexpr uint32_t kWaves = 4;                /* waves per workgroup (independent) */

/* A wave's LDS: 7.5 KiB, so five 4-wave workgroups (20 waves) fit a CU. */
struct WaveLds {
    uint32_t slab[kCap / 4];
    uint32_t ent[kTK];  /* sorted position -> slab offset | len << 16 */
    uint32_t cnt[kClasses];
    uint8_t perm[kTK];  /* sorted position -> key index in the tile */
};
static_assert(sizeof(WaveLds) == 7680, "five 4-wave workgroups per CU");

/* A tile as the wave tracks it (uniform, but the per-lane entries). */
struct TileInfo {
    uint64_t k0;        /* first key */
    uint64_t abase;     /* keys + off[k0] rounded down to 16 bytes */
    uint32_t nvalid;    /* keys of the tile below nkeys */
    uint32_t need;      /* bytes from abase to the tile's end if they fit the slab, else 0xffffffff */
    uint32_t ent[4];    /* this lane's keys 4i..4i+3: start - abase | len << 16 (if in the slab) */
};

/* raw offsets of a tile: off[k0 + 4i .. 4i + 4] for lane i, and the two
 * uniform bounds */
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
struct TileOffs {
    u32x4 a, b;
    u32x2 e;
};

/* raw offsets of tile k0: lane i gets off[k0 + 4i .. 4i + 4] (3 loads) */
__device__ __forceinline__ void load_offs(TileOffs &o, const uint64_t *off, uint64_t nkeys, uint64_t k0, uint32_t lane)
{
    const rsrc_t r = make_rsrc(off + k0, (nkeys + 1u - k0) * 8u);
    o.a = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(lane * 32u), 0, kAuxNt);
    o.b = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(lane * 32u + 16u), 0, kAuxNt);
    o.e = __builtin_amdgcn_raw_buffer_load_b64(r, (int)(lane * 32u + 32u), 0, kAuxNt);
}

/* The tile's uniform bounds from its offsets, and this lane's four keys as
 * slab entries (key start - abase | len << 16; meaningful if the tile fits
 * the slab). */
__device__ __forceinline__ TileInfo tile_info(const uint8_t *keys, const uint64_t *off, uint64_t nkeys, uint64_t k0,
                                              const TileOffs &o, uint32_t lane)
{
    TileInfo t;
    t.k0 = k0;
    t.nvalid = (uint32_t)(nkeys - k0 < kTK ? nkeys - k0 : kTK);
    /* every dword of the loads is consumed here (the high ones through the
     * uniform bounds), so none of their registers is reused while in flight */
    asm volatile("" ::"v"(o.a), "v"(o.b), "v"(o.e));
    /* s0 = off[k0] from lane 0; the tile's end off[k0 + nvalid] from the
     * lane and slot that hold it */
    const uint64_t s0 = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)o.a.x) |
                        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)o.a.y) << 32);
    uint64_t e;
    if (t.nvalid == kTK)
        e = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)o.e.x, 63) |
            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)o.e.y, 63) << 32);
    else
        e = off[k0 + t.nvalid]; /* the batch's last, partial tile */
    const uint64_t a = (uint64_t)(uintptr_t)(keys + s0);
    t.abase = a & ~(uint64_t)15u;
    const uint32_t head = (uint32_t)(a & 15u);
    const uint64_t need = head + (e - s0);
    t.need = need <= kCap ? (uint32_t)need : 0xffffffffu;
    /* low dwords suffice in the slab (span < 6 KiB); the fallback re-reads */
    const uint32_t st[5] = {o.a.x, o.a.z, o.b.x, o.b.z, o.e.x};
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const bool valid = 4u * lane + (uint32_t)q < t.nvalid;
        t.ent[q] = valid ? (st[q] - (uint32_t)s0 + head) | ((st[q + 1] - st[q]) << 16) : 0u;
    }
    return t;
}

/* Counting sort of a tile's 256 entries by length class (63 = 63+) into
 * entry set `es` / `ps`: one LDS atomic per key, a 64-lane scan. */
__device__ __forceinline__ void sort_tile(uint32_t *es, uint8_t *ps, uint32_t *cnt, const uint32_t (&ent)[4],
                                          uint32_t lane)
{
    cnt[lane] = 0u;
    __builtin_amdgcn_wave_barrier();
    uint32_t cls[4], rk[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t len = ent[q] >> 16;
        cls[q] = len < kClasses - 1u ? len : kClasses - 1u;
        rk[q] = atomicAdd(&cnt[cls[q]], 1u);
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t c = cnt[lane];
    const uint32_t base = wave_excl_scan(c, lane);
    cnt[lane] = base;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t pos = cnt[cls[q]] + rk[q];
        es[pos] = ent[q];
        ps[pos] = (uint8_t)(4u * lane + (uint32_t)q);
    }
    __builtin_amdgcn_wave_barrier();
}

} // namespace

template <int MODE, bool NOHASH, bool IL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5, 8))) void nc_wsort_kernel(
    const uint8_t *__restrict__ keys, const uint64_t *__restrict__ off, uint64_t nkeys, uint32_t *__restrict__ out,
    uint64_t ntiles, uint32_t chunk)
{
    __shared__ WaveLds lds_all[kWaves];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    WaveLds &L = lds_all[wave];
    /* wave w takes `chunk` tiles: consecutive ones (a grid of many
     * short-lived waves: a new wave's first loads overlap the others'
     * hashing), or (IL) tiles w, w + W, w + 2W, ... of the grid's W waves, so
     * the resident waves stream neighbouring tiles (nc_direct.h wave_tiles) */
    const Tiles<IL> tiles = wave_tiles<IL>(ntiles, chunk, kWaves, wave);
    const uint64_t n = tiles.n;
    if (n == 0) return;
    auto k0_of = [&](uint64_t j) __attribute__((always_inline)) { return tiles.at(j < n ? j : n - 1u) * kTK; };

    /* slab loads of a tile: the 16-byte chunks from abase up to its end
     * (rounded up: a load that crosses the resource's end reads zeros WHOLE;
     * the key buffer is readable NC_GPUHASH_PAD bytes past the last key) */
    u32x4 R[kJ];
    auto load_slab = [&](const TileInfo &ti) __attribute__((always_inline)) {
        const uint32_t nb = ti.need <= kCap ? (ti.need + 15u) & ~15u : 0u;
        const rsrc_t rs = make_rsrc((const void *)(uintptr_t)ti.abase, nb);
#pragma unroll
        for (uint32_t j = 0; j < kJ; j++)
            R[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(16u * (lane + 64u * j)), 0, kAuxNt);
    };

    /* prologue: tile 0's offsets and slab, tile 1's offsets */
    TileOffs o;
    load_offs(o, off, nkeys, k0_of(0), lane);
    TileInfo nxt = tile_info(keys, off, nkeys, k0_of(0), o, lane);
    load_slab(nxt); /* the loop's order: slab, then offsets (hipcc's waits count on it) */
    load_offs(o, off, nkeys, k0_of(1), lane);

    /* a tile's four results per lane are stored during the NEXT tile, right
     * after its successor's offsets are consumed: a store issued before that
     * point would sit in the wave's vmcnt queue ahead of the wait for them */
    uint32_t hq[4] = {0u, 0u, 0u, 0u}, kq = 0u; /* kq: the four key indices, a byte each */
    uint64_t pk0 = 0;
    uint32_t pnv = 0;
    auto store_prev = [&]() __attribute__((always_inline)) {
        /* uniform, re-asserted: hipcc loses track of it through the loop's
         * phis and would waterfall the store resource */
        const uint64_t k0 = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)pk0) |
                            ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(pk0 >> 32)) << 32);
        const uint32_t nv = (uint32_t)__builtin_amdgcn_readfirstlane((int)pnv);
        const rsrc_t rout = make_rsrc(out + k0, (uint64_t)nv * 4u); /* keys past nkeys: dropped */
#pragma unroll
        for (int q = 0; q < 4; q++)
            __builtin_amdgcn_raw_buffer_store_b32(hq[q], rout, (int)(4u * ((kq >> (8 * q)) & 0xffu)), 0, kAuxOut);
    };

    for (uint64_t t = 0; t < n; t++) {
        const TileInfo cur = nxt;
        const bool inslab = cur.need <= kCap;
        /* the slab of tile t into LDS (loaded during the previous tile), its
         * keys sorted */
        if (inslab) {
#pragma unroll
            for (uint32_t j = 0; j < kJ; j++)
                if (1024u * j < cur.need) *reinterpret_cast<u32x4 *>(&L.slab[4u * (lane + 64u * j)]) = R[j];
            sort_tile(L.ent, L.perm, L.cnt, cur.ent, lane);
        }
        /* next tile: consume its offsets, store the previous tile's results,
         * then its slab and its successor's offsets go out */
        if (t + 1u < n) {
            nxt = tile_info(keys, off, nkeys, k0_of(t + 1u), o, lane);
            if (t > 0u) store_prev();
            load_slab(nxt);
            load_offs(o, off, nkeys, k0_of(t + 2u), lane);
        } else if (t > 0u) {
            store_prev();
        }
        pk0 = cur.k0;
        pnv = cur.nvalid;
        if (inslab) {
            kq = 0u;
#pragma unroll
            for (int r = 0; r < 4; r++) kq |= (uint32_t)L.perm[64u * r + lane] << (8 * r);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const uint32_t e = L.ent[64u * r + lane];
                const uint32_t len = e >> 16;
                /* ascending by class within the round: lane 0 the shortest
                 * and lane 63 the longest, unless that lane's key is in the
                 * last class (63+), whose lengths are unordered: then a wave
                 * reduction */
                uint32_t lmin = (uint32_t)__builtin_amdgcn_readlane((int)len, 0);
                uint32_t lmax = (uint32_t)__builtin_amdgcn_readlane((int)len, 63);
                if (lmin >= kClasses - 1u) lmin = wave_min(len);
                if (lmax >= kClasses - 1u) lmax = wave_max(len);
                if constexpr (NOHASH) hq[r] = len;
                else hq[r] = final_state<MODE>(hash_slab<MODE>(L.slab, e & 0xffffu, len, lmin, lmax));
            }
        } else {
            /* span past the slab: each lane walks its four keys from global
             * memory, byte by byte (sign-extending loads), 64-bit offsets
             * re-read (a tile may span more than 4 GiB here) */
            kq = 0x03020100u + 0x04040404u * lane;
#pragma unroll
            for (uint32_t q = 0; q < 4u; q++) {
                const uint32_t k = 4u * lane + q;
                uint32_t h = init_state<MODE>();
                if (k < cur.nvalid) {
                    const uint64_t s0 = off[cur.k0 + k], s1 = off[cur.k0 + k + 1u];
                    const int8_t *p = reinterpret_cast<const int8_t *>(keys) + s0;
                    for (uint64_t i = 0; i < s1 - s0; i++) h = byte_step<MODE>(h, (uint32_t)(int32_t)p[i]);
                }
                hq[q] = final_state<MODE>(h);
            }
        }
    }
    store_prev();
}

namespace nc_wsort {

template <int MODE, bool NH, bool IL>
hipError_t launch_k(const uint8_t *d_keys, const uint64_t *d_off, uint64_t nkeys, uint32_t *d_out, hipStream_t stream,
                    uint32_t chunk)
{
    const uint64_t ntiles = (nkeys + kTK - 1u) / kTK;
    const uint64_t grid = (ntiles + (uint64_t)kWaves * chunk - 1u) / ((uint64_t)kWaves * chunk);
    if (grid == 0) return hipSuccess;
    if (grid > 0x7fffffffu) return hipErrorInvalidValue;
    (void)hipGetLastError();
    hipLaunchKernelGGL((nc_wsort_kernel<MODE, NH, IL>), dim3((unsigned)grid), dim3(64 * kWaves), 0, stream, d_keys, d_off,
                       nkeys, d_out, ntiles, chunk);
    return hipGetLastError();
}

template <int MODE>
hipError_t launch_mode(const uint8_t *d_keys, const uint64_t *d_off, uint64_t nkeys, uint32_t *d_out,
                       hipStream_t stream, int var)
{
    static const uint32_t kChunk[4] = {4, 2, 8, 16};
    const uint32_t chunk = kChunk[var & 3];
    const bool il = (var & 8) != 0;
    if (var & 4) { /* DIAGNOSTIC: no hashing (outputs are key lengths), fnv1a_64 only */
        if (MODE != NC_GPUHASH_FNV1A_64) return hipErrorInvalidValue;
        return il ? launch_k<NC_GPUHASH_FNV1A_64, true, true>(d_keys, d_off, nkeys, d_out, stream, chunk)
                  : launch_k<NC_GPUHASH_FNV1A_64, true, false>(d_keys, d_off, nkeys, d_out, stream, chunk);
    }
    return il ? launch_k<MODE, false, true>(d_keys, d_off, nkeys, d_out, stream, chunk)
              : launch_k<MODE, false, false>(d_keys, d_off, nkeys, d_out, stream, chunk);
}

/* var: bits 0-1 tiles per wave (4, 2, 8, 16), bit 2 DIAGNOSTIC no-hash
 * build (fnv1a_64), bit 3 a wave's tiles interleaved over the grid.
 * nkeys < 2^32. */
bool supports(int mode)
{
    switch (mode) {
    case NC_GPUHASH_ONE_AT_A_TIME:
    case NC_GPUHASH_FNV1_64:
    case NC_GPUHASH_FNV1A_64:
    case NC_GPUHASH_FNV1_32:
    case NC_GPUHASH_FNV1A_32:
        return true;
    default:
        return false;
    }
}

hipError_t launch(int mode, const uint8_t *d_keys, const uint64_t *d_off, uint64_t nkeys, uint32_t *d_out,
                  hipStream_t stream, int var)
{
    switch (mode) {
    case NC_GPUHASH_ONE_AT_A_TIME: return launch_mode<NC_GPUHASH_ONE_AT_A_TIME>(d_keys, d_off, nkeys, d_out, stream, var);
    case NC_GPUHASH_FNV1_64: return launch_mode<NC_GPUHASH_FNV1_64>(d_keys, d_off, nkeys, d_out, stream, var);
    case NC_GPUHASH_FNV1A_64: return launch_mode<NC_GPUHASH_FNV1A_64>(d_keys, d_off, nkeys, d_out, stream, var);
    case NC_GPUHASH_FNV1_32: return launch_mode<NC_GPUHASH_FNV1_32>(d_keys, d_off, nkeys, d_out, stream, var);
    case NC_GPUHASH_FNV1A_32: return launch_mode<NC_GPUHASH_FNV1A_32>(d_keys, d_off, nkeys, d_out, stream, var);
    default: return hipErrorInvalidValue;
    }
}

} // namespace nc_wsort
