/*
 * Byte-serial hashkit modes on the direct per-lane pipeline (nc_direct.h):
 * crc16, crc32, crc32a (src/hashkit/nc_crc16.c:56-66, nc_crc32.c:99-123),
 * fnv1_64, fnv1a_64, fnv1_32, fnv1a_32 (nc_fnv.c:26-82) and one_at_a_time
 * (nc_one_at_a_time.c:35-51). One lane hashes one key, 64 bytes per round,
 * from registers (fixed-length keys: every lane of a wave runs the same byte
 * count) or, for long keys, from the LDS-DMA block image.
 *
 * The crc table lookup is the crc modes' bottleneck on the byte-table
 * pipelines: one 1 KiB table, a random entry per lane (~3.5-way bank
 * conflicts) and a dependent lookup per byte. Here whole words go through
 * slicing-by-4 tables (four independent lookups) replicated over 8 bank
 * groups (nc_crc_slice.h).
 */
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "nc_crc_slice.h"
#include "nc_direct.h"
#include "nc_gpuhash.h"
#include "nc_hash_algo.h"

namespace {

using namespace nc_direct;

constexpr uint32_t kWaves = 16; /* 1024-thread workgroups share one table */

template <int MODE>
constexpr bool has_table()
{
    return MODE == NC_GPUHASH_CRC16 || MODE == NC_GPUHASH_CRC32 || MODE == NC_GPUHASH_CRC32A;
}

template <int MODE>
__device__ __forceinline__ uint32_t init_state()
{
    if constexpr (MODE == NC_GPUHASH_FNV1_64 || MODE == NC_GPUHASH_FNV1A_64) return NC_FNV64_INIT32;
    if constexpr (MODE == NC_GPUHASH_FNV1_32 || MODE == NC_GPUHASH_FNV1A_32) return NC_FNV32_INIT;
    if constexpr (MODE == NC_GPUHASH_CRC32 || MODE == NC_GPUHASH_CRC32A) return 0xffffffffu;
    return 0u; /* one_at_a_time, crc16 */
}

template <int MODE>
__device__ __forceinline__ uint32_t final_state(uint32_t h)
{
    if constexpr (MODE == NC_GPUHASH_ONE_AT_A_TIME) return nc_oaat_final(h);
    if constexpr (MODE == NC_GPUHASH_CRC32) return nc_crc32_final(h);
    if constexpr (MODE == NC_GPUHASH_CRC32A) return nc_crc32a_final(h);
    return h;
}

/* ---- crc tables: slicing-by-4 (nc_crc_slice.h), replicated over 8 bank
 * groups (R = 8, 32 KiB); OPT bit 0: slicing-by-8 (8 tables: R = 8, 64 KiB,
 * or R = 4 beside the line image) ---- */
constexpr uint32_t kCopies = 8;
constexpr uint32_t kTabWords = nc_slice::table_words<kCopies>();
constexpr int kOptS8 = 1;     /* slicing-by-8 crcs */
constexpr int kOptNoHash = 2; /* DIAGNOSTIC: xor of the key's words, not a hash (the pipeline's memory side) */

template <int MODE, bool LDS, int OPT>
struct Tab {
    static constexpr bool S8 = (OPT & kOptS8) != 0 && (MODE == NC_GPUHASH_CRC16 || MODE == NC_GPUHASH_CRC32 ||
                                                        MODE == NC_GPUHASH_CRC32A);
    static constexpr uint32_t R = S8 && LDS ? 4u : kCopies;
    static constexpr uint32_t NT = S8 ? 8u : 4u;
    static constexpr uint32_t kWords = nc_slice::table_words<R, NT>();
};

/* byte j (0..3) of word w into state h (the crcs through T0) */
template <int MODE, uint32_t R = kCopies>
__device__ __forceinline__ uint32_t byte_step(uint32_t h, uint32_t w, int j, const uint32_t *tab, uint32_t lane4)
{
    const uint32_t b = (w >> (8 * j)) & 0xffu;
    if constexpr (has_table<MODE>()) return nc_slice::byte<MODE, R>(h, b, tab, lane4);
    else if constexpr (MODE == NC_GPUHASH_FNV1A_64) return nc_fnv1a_64_step(h, b);
    else if constexpr (MODE == NC_GPUHASH_FNV1_64) return nc_fnv1_64_step(h, b);
    else if constexpr (MODE == NC_GPUHASH_FNV1_32) return nc_fnv1_32_step(h, b);
    else if constexpr (MODE == NC_GPUHASH_FNV1A_32) return nc_fnv1a_32_step(h, b);
    else return nc_oaat_step(h, b);
}

/* the 4 bytes of word w */
template <int MODE, uint32_t R = kCopies>
__device__ __forceinline__ uint32_t word_step(uint32_t h, uint32_t w, const uint32_t *tab, uint32_t lc4)
{
    if constexpr (has_table<MODE>()) {
        return nc_slice::word<MODE, R>(h, w, tab, lc4);
    } else {
#pragma unroll
        for (int j = 0; j < 4; j++) h = byte_step<MODE, R>(h, w, j, tab, lc4);
        return h;
    }
}

/* the first nb (1..4, per lane) bytes of word w, one at a time */
template <int MODE, uint32_t R = kCopies>
__device__ __forceinline__ uint32_t bytes_step(uint32_t h, uint32_t w, int32_t nb, const uint32_t *tab, uint32_t lc4)
{
#pragma unroll
    for (int j = 0; j < 4; j++)
        if (j < nb) h = byte_step<MODE, R>(h, w, j, tab, lc4);
    return h;
}

/* nb (per lane, may exceed 64) key bytes of one block in d */
template <int MODE, bool LDS, int OPT>
__device__ __forceinline__ uint32_t block_step(uint32_t h, const u32x4 (&d)[4], int32_t nb, const uint32_t *tab,
                                               uint32_t lane4)
{
    using TB = Tab<MODE, LDS, OPT>;
    constexpr uint32_t R = TB::R;
    if constexpr ((OPT & kOptNoHash) != 0) {
#pragma unroll
        for (int t = 0; t < 16; t++)
            if (nb > 4 * t) h ^= d[t >> 2][t & 3];
        return h;
    }
    /* crc16 keeps its key's last 2+ bytes for the byte steps, which
     * rebuild the state's history bits (nc_crc_slice.h word) */
    constexpr int32_t kWhole = nc_slice::whole<MODE>();
    if constexpr (TB::S8) {
#pragma unroll
        for (int t = 0; t < 16; t += 2) {
            const int32_t kb = nb - 4 * t;
            const uint32_t w0 = d[t >> 2][t & 3], w1 = d[t >> 2][(t & 3) + 1];
            if (kb >= kWhole + 4) {
                h = nc_slice::word2<MODE, R>(h, w0, w1, tab, lane4);
            } else {
                if (kb >= kWhole) h = word_step<MODE, R>(h, w0, tab, lane4);
                else if (kb > 0) h = bytes_step<MODE, R>(h, w0, kb, tab, lane4);
                if (kb - 4 >= kWhole) h = word_step<MODE, R>(h, w1, tab, lane4);
                else if (kb - 4 > 0) h = bytes_step<MODE, R>(h, w1, kb - 4, tab, lane4);
            }
        }
        return h;
    }
#pragma unroll
    for (int t = 0; t < 16; t++) {
        const int32_t kb = nb - 4 * t;
        const uint32_t w = d[t >> 2][t & 3];
        if (kb >= kWhole) h = word_step<MODE, R>(h, w, tab, lane4);
        else if (kb > 0) h = bytes_step<MODE, R>(h, w, kb, tab, lane4);
    }
    return h;
}

} // namespace

/*
 * One wave = one 64-key tile at a time (lane = key), `chunk` consecutive
 * tiles per wave. Round (tile, b) feeds block b (bytes 64b .. 64b+63) of every
 * key that has one into its state; the next round's block is in flight (the
 * other register set, or the LDS image) while this one computes.
 */
template <int MODE, bool LDS, bool IL, int WAVES = kWaves, int OPT = 0>
__global__ __launch_bounds__(64 * WAVES) void nc_bytes_direct_kernel(const uint8_t *__restrict__ keys,
                                                              const uint64_t *__restrict__ off, uint64_t nkeys,
                                                              uint32_t *__restrict__ out, uint64_t ntiles,
                                                              uint32_t chunk)
{
    /* a round consumes RB bytes of every key: one 64-byte block from
     * registers, or (LDS) one 128-byte line from the image */
    constexpr uint32_t RB = LDS ? 128u : 64u;
    using TB = Tab<MODE, LDS, OPT>;
    constexpr bool kTable = has_table<MODE>() && (OPT & kOptNoHash) == 0;
    __shared__ uint32_t tab[kTable ? TB::kWords : 1];
    __shared__ __attribute__((aligned(16))) uint8_t kbuf[LDS ? WAVES * kLineImage : 16];
    if constexpr (kTable) {
        nc_slice::fill<MODE, TB::R, TB::NT>(tab, threadIdx.x, 64u * WAVES);
        __syncthreads();
    }
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane4 = nc_slice::copy_of<TB::R>(lane); /* this lane's table copy */
    const Tiles<IL> tiles = wave_tiles<IL>(ntiles, chunk, WAVES, wave);
    uint32_t tile = 0; /* local tile index */
    const uint32_t tlast = tiles.n;
    if (tile >= tlast) return;
    Walker<IL> wk;
    wk.init(keys, off, nkeys, tiles, lane);
    uint8_t *const img = kbuf + (LDS ? wave * kLineImage : 0u);

    TileKeys cur_t = wk.keys_of(tile, wk.load_off(tile));
    Offs no = wk.load_off(tile + 1u);
    u32x4 da[4], db[4];
    if constexpr (LDS) wk.dma_lines(cur_t, 0u, img);
    else wk.load_regs(cur_t, 0u, da);
    uint32_t b = 0;
    uint32_t h = init_state<MODE>();

    /* one round on `cur` (and, LDS, `nxt` as the line's second half); the
     * next round's bytes go to `nxt` (registers) or to the LDS image */
    auto round = [&](u32x4 (&cur)[4], u32x4 (&nxt)[4]) __attribute__((always_inline)) {
        const bool more = __ballot(cur_t.valid && cur_t.len > RB * (b + 1u)) != 0ull;
        const TileKeys nxt_t = wk.keys_of(tile + 1u, no);
        if constexpr (LDS) {
            wk.read_lines(img, cur, nxt);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); /* the image's reads are done */
            wk.dma_lines(more ? cur_t : nxt_t, more ? b + 1u : 0u, img);
        } else {
            wk.load_regs(more ? cur_t : nxt_t, more ? b + 1u : 0u, nxt);
        }
        /* offsets two tiles ahead, straight into `no` (it was consumed above);
         * a re-read of the next tile's while this one still has blocks */
        no = wk.load_off(more ? tile + 1u : tile + 2u);

        const int32_t rem = (int32_t)cur_t.len - (int32_t)RB * (int32_t)b;
        if (cur_t.valid && (rem > 0 || (b == 0u && cur_t.len == 0u))) {
            h = block_step<MODE, LDS, OPT>(h, cur, rem, tab, lane4);
            if constexpr (LDS) {
                if (rem > 64) h = block_step<MODE, LDS, OPT>(h, nxt, rem - 64, tab, lane4);
            }
            if (rem <= (int32_t)RB) {
                const rsrc_t rout = make_rsrc(out + wk.key0(tile), 256u);
                __builtin_amdgcn_raw_buffer_store_b32(final_state<MODE>(h), rout, (int)(lane * 4u), 0, kAuxNt);
            }
        }
        if (more) {
            b++;
        } else {
            tile++;
            b = 0;
            cur_t = nxt_t;
            h = init_state<MODE>();
        }
    };
    for (;;) {
        if constexpr (LDS) {
            round(da, db);
        } else {
            round(da, db);
            if (tile >= tlast) break;
            round(db, da);
        }
        if (tile >= tlast) break;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); /* no LDS-DMA may outlive the workgroup */
}

namespace nc_bytes {

template <int MODE, int OPT>
hipError_t launch_opt(const uint8_t *d_keys, const uint64_t *d_off, uint64_t nkeys, uint32_t *d_out,
                      hipStream_t stream, int var)
{
    static const uint32_t kChunk[4] = {16, 8, 32, 64};
    const uint32_t chunk = kChunk[var & 3];
    const uint64_t ntiles = (nkeys + 63u) / 64u;
    const uint64_t grid = (ntiles + (uint64_t)kWaves * chunk - 1u) / ((uint64_t)kWaves * chunk);
    if (grid > 0x7fffffffu) return hipErrorInvalidValue;
    (void)hipGetLastError();
    const bool il = (var & 8) != 0;
    if ((var & 4) && (var & 16) && il) {
        /* var bit 4: eight-wave workgroups, one per CU (unused dynamic LDS
         * keeps a second out): half the concurrent key streams */
        const uint64_t grid8 = (ntiles + 8u * chunk - 1u) / (8u * chunk);
        if (grid8 > 0x7fffffffu) return hipErrorInvalidValue;
        const uint32_t pad = has_table<MODE>() ? 0u : 40960u;
        if (pad)
            (void)hipFuncSetAttribute((const void *)nc_bytes_direct_kernel<MODE, true, true, 8, OPT>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)pad);
        hipLaunchKernelGGL((nc_bytes_direct_kernel<MODE, true, true, 8, OPT>), dim3((unsigned)grid8), dim3(512), pad,
                           stream, d_keys, d_off, nkeys, d_out, ntiles, chunk);
        return hipGetLastError();
    }
    if (var & 4) {
        if (il)
            hipLaunchKernelGGL((nc_bytes_direct_kernel<MODE, true, true, kWaves, OPT>), dim3((unsigned)grid), dim3(1024),
                               0, stream, d_keys, d_off, nkeys, d_out, ntiles, chunk);
        else
            hipLaunchKernelGGL((nc_bytes_direct_kernel<MODE, true, false, kWaves, OPT>), dim3((unsigned)grid), dim3(1024),
                               0, stream, d_keys, d_off, nkeys, d_out, ntiles, chunk);
    } else if (il) {
        hipLaunchKernelGGL((nc_bytes_direct_kernel<MODE, false, true, kWaves, OPT>), dim3((unsigned)grid), dim3(1024), 0,
                           stream, d_keys, d_off, nkeys, d_out, ntiles, chunk);
    } else {
        hipLaunchKernelGGL((nc_bytes_direct_kernel<MODE, false, false, kWaves, OPT>), dim3((unsigned)grid), dim3(1024),
                           0, stream, d_keys, d_off, nkeys, d_out, ntiles, chunk);
    }
    return hipGetLastError();
}

/* var bits 5-6: OPT (bit 5 slicing-by-8 crcs, bit 6 the DIAGNOSTIC no-hash
 * build, fnv1a_64 and crc32 only) */
template <int MODE>
hipError_t launch_mode(const uint8_t *d_keys, const uint64_t *d_off, uint64_t nkeys, uint32_t *d_out,
                       hipStream_t stream, int var)
{
    if constexpr (MODE == NC_GPUHASH_FNV1A_64 || MODE == NC_GPUHASH_CRC32) {
        if (var & 64) return launch_opt<MODE, kOptNoHash>(d_keys, d_off, nkeys, d_out, stream, var);
    }
    if constexpr (has_table<MODE>()) {
        if (var & 32) return launch_opt<MODE, kOptS8>(d_keys, d_off, nkeys, d_out, stream, var);
    }
    return launch_opt<MODE, 0>(d_keys, d_off, nkeys, d_out, stream, var);
}

/* the byte-serial modes on the direct pipeline; var: bits 0-1 tiles per wave
 * (16, 8, 32, 64), bit 2 the LDS-DMA block image (long keys), bit 3 a wave's
 * tiles interleaved over the grid (else consecutive), bit 4 (with 2 and 3)
 * eight-wave workgroups, one per CU. nkeys < 2^32. */
bool supports(int mode)
{
    switch (mode) {
    case NC_GPUHASH_ONE_AT_A_TIME:
    case NC_GPUHASH_CRC16:
    case NC_GPUHASH_CRC32:
    case NC_GPUHASH_CRC32A:
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
    case NC_GPUHASH_CRC16: return launch_mode<NC_GPUHASH_CRC16>(d_keys, d_off, nkeys, d_out, stream, var);
    case NC_GPUHASH_CRC32: return launch_mode<NC_GPUHASH_CRC32>(d_keys, d_off, nkeys, d_out, stream, var);
    case NC_GPUHASH_CRC32A: return launch_mode<NC_GPUHASH_CRC32A>(d_keys, d_off, nkeys, d_out, stream, var);
    case NC_GPUHASH_FNV1_64: return launch_mode<NC_GPUHASH_FNV1_64>(d_keys, d_off, nkeys, d_out, stream, var);
    case NC_GPUHASH_FNV1A_64: return launch_mode<NC_GPUHASH_FNV1A_64>(d_keys, d_off, nkeys, d_out, stream, var);
    case NC_GPUHASH_FNV1_32: return launch_mode<NC_GPUHASH_FNV1_32>(d_keys, d_off, nkeys, d_out, stream, var);
    case NC_GPUHASH_FNV1A_32: return launch_mode<NC_GPUHASH_FNV1A_32>(d_keys, d_off, nkeys, d_out, stream, var);
    default: return hipErrorInvalidValue;
    }
}

} // namespace nc_bytes
