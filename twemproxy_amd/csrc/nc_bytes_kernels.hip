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

#include <atomic>

#include "nc_crc_slice.h"
#include "nc_direct.h"
#include "nc_out_policy.h"
#include "nc_gpuhash.h"
#include "nc_hash_algo.h"
#include "nc_hash_key.h"

/* hipFuncSetAttribute(MaxDynamicSharedMemorySize) holds per device: set it
 * once per kernel and device (the bit of each device already set in `done`)
 * and report its failure instead of launching into it */
static inline hipError_t dyn_lds_once(const void *kern, int bytes, std::atomic<uint64_t> &done)
{
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const uint64_t bit = dev < 64 ? 1ull << dev : 0ull;
    if (bit != 0u && (done.load(std::memory_order_acquire) & bit) != 0u) return hipSuccess;
    e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess && bit != 0u) done.fetch_or(bit, std::memory_order_acq_rel);
    return e;
}

namespace {

using namespace nc_direct;

constexpr uint32_t kWaves = 16; /* 1024-thread workgroups share one table */

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

template <int MODE>
constexpr bool has_table()
{
    return MODE == NC_GPUHASH_CRC16 || MODE == NC_GPUHASH_CRC32 || MODE == NC_GPUHASH_CRC32A;
}

/* the word modes, on the short-key kernel only (src/hashkit/nc_hsieh.c,
 * nc_murmur.c, nc_jenkins.c) */
template <int MODE>
constexpr bool is_word_mode()
{
    return MODE == NC_GPUHASH_HSIEH || MODE == NC_GPUHASH_MURMUR || MODE == NC_GPUHASH_JENKINS;
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
constexpr int kOptPairs = 16; /* the line image's rounds of two lines (256 B per key; eight-wave workgroups) */
constexpr int kOptOffDefault = 32; /* A/B: the offsets with the default cache policy instead of nt */

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
     * registers, (LDS) one 128-byte line from the image, or (PAIRS) two */
    constexpr bool PAIRS = LDS && (OPT & kOptPairs) != 0;
    constexpr uint32_t RB = PAIRS ? 256u : (LDS ? 128u : 64u);
    constexpr uint32_t kImg = PAIRS ? 2u * kLineImage : kLineImage;
    using TB = Tab<MODE, LDS, OPT>;
    constexpr bool kTable = has_table<MODE>() && (OPT & kOptNoHash) == 0;
    __shared__ uint32_t tab[kTable ? TB::kWords : 1];
    __shared__ __attribute__((aligned(16))) uint8_t kbuf[LDS ? WAVES * kImg : 16];
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
    uint8_t *const img = kbuf + (LDS ? wave * kImg : 0u);

    /* the offsets' cache policy: the default for the crcs' line image (a
     * lane's start and end dwords share lines nt can evict between the two
     * loads: C4 shard crc32 1.7965 -> 1.7758 ms, HBM reads 9.32 -> 9.16 GB,
     * profiles/r06k_c4_offsets_policy_ab_crc32.jsonl), nt elsewhere (the
     * fnvs' line kernel ties, 1.5361 vs 1.5391; A/B: kOptOffDefault) */
    constexpr int kOffAux = ((OPT & kOptOffDefault) != 0 || (LDS && has_table<MODE>())) ? 0 : kAuxNt;
    TileKeys cur_t = wk.keys_of(tile, wk.template load_off<kOffAux>(tile));
    Offs no = wk.template load_off<kOffAux>(tile + 1u);
    u32x4 da[4], db[4];
    if constexpr (PAIRS) wk.dma_pairs(cur_t, 0u, img);
    else if constexpr (LDS) wk.dma_lines(cur_t, 0u, img);
    else wk.load_regs(cur_t, 0u, da);
    uint32_t b = 0;
    uint32_t h = init_state<MODE>();

    /* one round on `cur` (and, LDS, `nxt` as the line's second half); the
     * next round's bytes go to `nxt` (registers) or to the LDS image */
    auto round = [&](u32x4 (&cur)[4], u32x4 (&nxt)[4]) __attribute__((always_inline)) {
        const bool more = __ballot(cur_t.valid && cur_t.len > RB * (b + 1u)) != 0ull;
        const TileKeys nxt_t = wk.keys_of(tile + 1u, no);
        u32x4 dp[PAIRS ? 16 : 1];
        if constexpr (PAIRS) {
            wk.read_pairs(img, dp);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); /* the image's reads are done */
            wk.dma_pairs(more ? cur_t : nxt_t, more ? b + 1u : 0u, img);
        } else if constexpr (LDS) {
            wk.read_lines(img, cur, nxt);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); /* the image's reads are done */
            wk.dma_lines(more ? cur_t : nxt_t, more ? b + 1u : 0u, img);
        } else {
            wk.load_regs(more ? cur_t : nxt_t, more ? b + 1u : 0u, nxt);
        }
        /* offsets two tiles ahead, straight into `no` (it was consumed above);
         * a re-read of the next tile's while this one still has blocks */
        no = wk.template load_off<kOffAux>(more ? tile + 1u : tile + 2u);

        const int32_t rem = (int32_t)cur_t.len - (int32_t)RB * (int32_t)b;
        if (cur_t.valid && (rem > 0 || (b == 0u && cur_t.len == 0u))) {
            if constexpr (PAIRS) {
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const u32x4 d4[4] = {dp[4 * q], dp[4 * q + 1], dp[4 * q + 2], dp[4 * q + 3]};
                    if (q == 0 || rem > 64 * q) h = block_step<MODE, LDS, OPT>(h, d4, rem - 64 * q, tab, lane4);
                }
            } else {
                h = block_step<MODE, LDS, OPT>(h, cur, rem, tab, lane4);
                if constexpr (LDS) {
                    if (rem > 64) h = block_step<MODE, LDS, OPT>(h, nxt, rem - 64, tab, lane4);
                }
            }
            if (rem <= (int32_t)RB) {
                const rsrc_t rout = make_rsrc(out + wk.key0(tile), 256u);
                __builtin_amdgcn_raw_buffer_store_b32(final_state<MODE>(h), rout, (int)(lane * 4u), 0, kAuxOut);
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

/* A word mode's hash of a key of len (<= 16 * NC) bytes held from its first
 * byte in d[0 .. NC) (the short-key kernel's unaligned loads put byte 0 of
 * the key in byte 0 of d): hsieh SuperFastHash (src/hashkit/nc_hsieh.c:39-93),
 * MurmurHash2 (nc_murmur.c:38-99), lookup3 hashlittle (nc_jenkins.c:76-230),
 * as nc_lds_hash.h's stream forms but with every word index static (a
 * lane's tail word by selects), so nothing leaves registers. */
template <int MODE, int NC>
__device__ __forceinline__ uint32_t short_words(const u32x4 (&d)[NC], uint32_t len)
{
    constexpr int NW = 4 * NC;
    auto W = [&](int t) __attribute__((always_inline)) { return t < NW ? d[t >> 2][t & 3] : 0u; };
    if constexpr (MODE == NC_GPUHASH_JENKINS) {
        const uint32_t init = nc_jenkins_init(len);
        uint32_t a = init, b = init, c = init;
        constexpr int kMaxBlocks = (16 * NC - 1) / 12; /* 12-byte blocks before the last 1..12 bytes */
        const uint32_t nb = len > 12u ? (len - 1u) / 12u : 0u;
#pragma unroll
        for (int k = 0; k < kMaxBlocks; k++) {
            if ((uint32_t)k < nb) {
                a += W(3 * k);
                b += W(3 * k + 1);
                c += W(3 * k + 2);
                NC_JENKINS_MIX(a, b, c);
            }
        }
        uint32_t wa = W(0), wb = W(1), wc = W(2);
#pragma unroll
        for (int k = 1; k <= kMaxBlocks; k++) {
            if (nb == (uint32_t)k) {
                wa = W(3 * k);
                wb = W(3 * k + 1);
                wc = W(3 * k + 2);
            }
        }
        const uint32_t n = len - 12u * nb; /* 1..12 */
        /* m = 0 (an empty key) keeps nothing; no shift by 32 (undefined) */
        auto keep = [](uint32_t w, uint32_t m) {
            return m >= 4u ? w : (m == 0u ? 0u : (w & (0xffffffffu >> (32u - 8u * m))));
        };
        a += keep(wa, n);
        if (n > 4u) b += keep(wb, n - 4u);
        if (n > 8u) c += keep(wc, n - 8u);
        NC_JENKINS_FINAL(a, b, c);
        return len == 0u ? init : c; /* nc_jenkins.c:121 */
    } else {
        const uint32_t nw = len >> 2, rem = len & 3u;
        uint32_t h = MODE == NC_GPUHASH_MURMUR ? nc_murmur_init(len) : 0u;
        uint32_t tw = W(0);
#pragma unroll
        for (int t = 0; t < NW; t++) {
            if ((uint32_t)t < nw) h = MODE == NC_GPUHASH_MURMUR ? nc_murmur_word(h, W(t)) : nc_hsieh_word(h, W(t));
            if (nw == (uint32_t)t + 1u) tw = W(t + 1);
        }
        if constexpr (MODE == NC_GPUHASH_MURMUR) return nc_murmur_final(nc_murmur_tail(h, tw, rem));
        else return len == 0u ? 0u : nc_hsieh_final(nc_hsieh_tail(h, tw, rem)); /* nc_hsieh.c:44 */
    }
}

/* the first nb (per lane, <= 16 * NC) key bytes of words d[0 .. NC); the crcs
 * take NW words (slicing-by-4NW, tables in R copies) per dependent step where
 * the whole group belongs to the key */
template <int MODE, int NC, int NW, uint32_t R>
__device__ __forceinline__ uint32_t short_step(uint32_t h, const u32x4 (&d)[NC], int32_t nb, const uint32_t *tab,
                                               uint32_t lane4)
{
    constexpr int32_t kWhole = nc_slice::whole<MODE>();
    if constexpr (has_table<MODE>() && NW > 1) {
#pragma unroll
        for (int t = 0; t < 4 * NC; t += NW) {
            const int32_t kb = nb - 4 * t;
            uint32_t w[NW];
#pragma unroll
            for (int i = 0; i < NW; i++) w[i] = d[(t + i) >> 2][(t + i) & 3];
            if (kb >= kWhole + 4 * (NW - 1)) {
                h = nc_slice::words<MODE, R, NW>(h, w, tab, lane4);
            } else {
#pragma unroll
                for (int i = 0; i < NW; i++) {
                    if (kb - 4 * i >= kWhole) h = nc_slice::word<MODE, R>(h, w[i], tab, lane4);
                    else if (kb - 4 * i > 0) h = nc_slice::bytes<MODE, R>(h, w[i], kb - 4 * i, tab, lane4);
                }
            }
        }
        return h;
    }
#pragma unroll
    for (int t = 0; t < 4 * NC; t++) {
        const int32_t kb = nb - 4 * t;
        const uint32_t w = d[t >> 2][t & 3];
        if (kb >= kWhole) h = word_step<MODE, R>(h, w, tab, lane4);
        else if (kb > 0) h = bytes_step<MODE, R>(h, w, kb, tab, lane4);
    }
    return h;
}

/*
 * Short keys (the caller's shape: every key at most 16 * NC bytes, C3's
 * 32-byte keys): the direct pipeline's per-lane tiles at EIGHT waves per CU
 * (one 512-thread workgroup, held alone on its CU by its LDS), a persistent
 * grid of one workgroup per CU whose waves walk tiles interleaved over the
 * whole batch, and DEPTH - 1 tiles of key bytes in flight per wave. The
 * direct kernel's 32 waves per CU read and write HBM in too many concurrent
 * streams: its memory pattern alone (no hash) runs 0.56-0.59 ms on C3, the
 * same pattern at eight waves per CU with two tiles in flight 0.517
 * (tools/probes/direct_depth.hip, profiles/r05_direct_depth.jsonl).
 *
 * Round j of a wave: issue the offsets of tile j + DEPTH, then tile
 * j + DEPTH - 1's NC 16-byte loads per lane (its offsets came during round
 * j - 1), then hash tile j (loaded DEPTH - 1 rounds ago) and store it. Every
 * round issues the same loads (past the wave's last tile the last one is
 * re-read), so hipcc's waitcnt pass counts them exactly and leaves the
 * younger tiles in flight. A tile holding a longer key (the shape was wrong)
 * ends the pipelined loop; that tile and the rest go block by block from
 * global memory: slower, never wrong.
 */
template <int MODE, int NC, int DEPTH, int WAVES, int NW, uint32_t R>
__global__ __launch_bounds__(64 * WAVES) void nc_bytes_short_kernel(const uint8_t *__restrict__ keys,
                                                                   const uint64_t *__restrict__ off, uint64_t nkeys,
                                                                   uint32_t *__restrict__ out, uint64_t ntiles)
{
    static_assert(NC >= 1 && NC <= 2 && DEPTH >= 2 && DEPTH <= 4, "keys of <= 16 or 32 B; 1-3 tiles ahead");
    constexpr uint32_t kTabWords = nc_slice::table_words<R, 4u * NW>();
    __shared__ uint32_t tab[has_table<MODE>() ? kTabWords : 1];
    if constexpr (has_table<MODE>()) {
        nc_slice::fill<MODE, R, 4u * NW>(tab, threadIdx.x, 64u * WAVES);
        __syncthreads();
    }
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane4 = nc_slice::copy_of<R>(lane);
    const Tiles<true> tiles = wave_tiles<true>(ntiles, 0xffffffffu, WAVES, wave);
    const uint32_t n = tiles.n;
    if (n == 0u) return;
    const uint32_t nk32 = (uint32_t)nkeys;
    const uint64_t kbytes = off[nkeys] + (uint64_t)NC_GPUHASH_PAD;

    /* The crcs take a tile's base (off[k0]) from lane 0's vector-loaded
     * start (v_readfirstlane once the loads are waited for): a scalar load of
     * it shares lgkmcnt with the table's LDS reads, so every lookup's wait
     * would also wait for the offsets of a tile DEPTH rounds ahead (measured:
     * crc32 0.65 -> 0.60 ms on C3). The other modes read no LDS and keep the
     * scalar load, whose own counter leaves the vector waits exact (their
     * vector-base build measured 1-6 % slower). */
    constexpr bool kVB = has_table<MODE>();
    struct Offs {
        uint32_t s, s_hi, e;
        uint64_t s0;
    };
    auto key0 = [&](uint32_t j) { return tiles.at(j < n ? j : n - 1u) * 64u; };
    auto load_off = [&](uint32_t j) __attribute__((always_inline)) {
        const uint32_t k0 = key0(j);
        const rsrc_t r = make_rsrc(off + k0, ((uint64_t)(nk32 - k0) + 1u) * 8u);
        Offs o;
        if constexpr (kVB) {
            const u32x2 sv = __builtin_amdgcn_raw_buffer_load_b64(r, (int)(lane * 8u), 0, kAuxNt);
            o.s = sv.x;
            o.s_hi = sv.y;
            o.s0 = 0;
        } else {
            o.s = __builtin_amdgcn_raw_buffer_load_b32(r, (int)(lane * 8u), 0, kAuxNt);
            o.s_hi = 0;
            o.s0 = off[k0];
        }
        o.e = __builtin_amdgcn_raw_buffer_load_b32(r, (int)(lane * 8u + 8u), 0, kAuxNt);
        return o;
    };
    auto base_of = [&](const Offs &o) __attribute__((always_inline)) {
        if constexpr (!kVB) return o.s0;
        return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)o.s) |
               ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)o.s_hi) << 32);
    };
    auto load_data = [&](const Offs &o, u32x4 (&d)[NC]) __attribute__((always_inline)) {
        const uint64_t s0 = base_of(o);
        const rsrc_t r = make_rsrc(keys + s0, kbytes - s0);
        const int vo = (int)(o.s - (uint32_t)s0);
#pragma unroll
        for (int c = 0; c < NC; c++) d[c] = __builtin_amdgcn_raw_buffer_load_b128(r, vo + 16 * c, 0, 0);
    };

    u32x4 dat[DEPTH][NC];
    uint32_t klen[DEPTH]; /* the tiles' key lengths */
    Offs ob[DEPTH];       /* offsets ring: tile j's in ob[j % DEPTH] (period DEPTH, as the unrolled rounds) */
    /* prologue: tiles 0 .. DEPTH - 2 in flight, offsets of tile DEPTH - 1 */
#pragma unroll
    for (int q = 0; q < DEPTH - 1; q++) {
        const Offs o = load_off((uint32_t)q);
        klen[q] = o.e - o.s;
        load_data(o, dat[q]);
    }
    ob[DEPTH - 1] = load_off((uint32_t)(DEPTH - 1));

    uint32_t jbad = n; /* the first tile with a key longer than 16 * NC bytes */
    for (uint32_t j0 = 0; jbad == n && j0 < n; j0 += DEPTH) {
#pragma unroll
        for (int q = 0; q < DEPTH; q++) {
            const uint32_t j = j0 + (uint32_t)q;
            if (j >= n) break;
            const int qa = (q + DEPTH - 1) % DEPTH; /* the data set tile j + DEPTH - 1 goes to */
            ob[q] = load_off(j + (uint32_t)DEPTH);  /* (j + DEPTH) % DEPTH == q */
            klen[qa] = ob[qa].e - ob[qa].s;
            load_data(ob[qa], dat[qa]);
            const uint32_t k0 = tiles.at(j) * 64u;
            const uint32_t nv = nk32 - k0 < 64u ? nk32 - k0 : 64u;
            const uint32_t len = klen[q];
            if (__ballot(lane < nv && len > 16u * NC) != 0ull) { /* the shape was wrong: the slow loop below */
                jbad = j;
                break;
            }
            uint32_t hv;
            if constexpr (is_word_mode<MODE>()) {
                hv = short_words<MODE, NC>(dat[q], len);
            } else {
                hv = final_state<MODE>(short_step<MODE, NC, NW, R>(init_state<MODE>(), dat[q], (int32_t)len, tab, lane4));
            }
            const rsrc_t rout = make_rsrc(out + k0, 4u * nv); /* lanes past the batch: dropped */
            __builtin_amdgcn_raw_buffer_store_b32(hv, rout, (int)(lane * 4u), 0, kAuxOut);
        }
    }
    /* tiles jbad .. n - 1 (only when a key was longer than the shape said),
     * outside the pipelined loop so that its waits stay exact: 64-byte blocks
     * from global memory, one tile at a time */
    for (uint32_t j = jbad; j < n; j++) {
        const Offs o = load_off(j);
        const uint32_t k0 = tiles.at(j) * 64u;
        const uint32_t nv = nk32 - k0 < 64u ? nk32 - k0 : 64u;
        const uint64_t s0 = base_of(o);
        const rsrc_t r = make_rsrc(keys + s0, kbytes - s0);
        const uint32_t vo = o.s - (uint32_t)s0;
        int32_t rem = lane < nv ? (int32_t)(o.e - o.s) : 0;
        if constexpr (is_word_mode<MODE>()) { /* byte loads, one lane per key (nc_hash_key.h) */
            const uint32_t hw = lane < nv ? nc_key_hash(MODE, keys + s0 + vo, (uint64_t)rem, nullptr, nullptr) : 0u;
            const rsrc_t rw = make_rsrc(out + k0, 4u * nv);
            __builtin_amdgcn_raw_buffer_store_b32(hw, rw, (int)(lane * 4u), 0, kAuxOut);
            continue;
        }
        uint32_t h = init_state<MODE>();
        for (uint32_t b = 0; __ballot(rem > 0) != 0ull; b++) {
            u32x4 d4[4];
#pragma unroll
            for (int c = 0; c < 4; c++)
                d4[c] = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(vo + 64u * b + 16u * (uint32_t)c), 0, 0);
            if (rem > 0) {
#pragma unroll
                for (int t = 0; t < 16; t++) {
                    const int32_t kb = rem - 4 * t;
                    const uint32_t w = d4[t >> 2][t & 3];
                    if (kb >= nc_slice::whole<MODE>()) h = word_step<MODE, R>(h, w, tab, lane4);
                    else if (kb > 0) h = bytes_step<MODE, R>(h, w, kb, tab, lane4);
                }
            }
            rem -= 64;
        }
        const rsrc_t rout = make_rsrc(out + k0, 4u * nv);
        __builtin_amdgcn_raw_buffer_store_b32(final_state<MODE>(h), rout, (int)(lane * 4u), 0, kAuxOut);
    }
}

namespace nc_bytes {

static int num_cus()
{
    static int n = 0;
    if (n == 0) {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
            n = v;
        else
            return 256;
    }
    return n;
}

/* the short-key kernel: every key <= 16 * NC bytes; a persistent grid of
 * one eight-wave workgroup per CU (dynamic LDS keeps a second one out);
 * var bits 0-1 the depth (3, 2, 4 tiles: 2, 1, 3 ahead), bits 2-3 the crcs'
 * tables (slicing-by-4 in 8 copies, by-8 in 8 copies, by-16 in 8, by-4 in 32:
 * one copy per lane of a ds_read_b32 lane group, conflict-free) */
template <int MODE, int NC, int DEPTH, int NW, uint32_t R, int kW = 8>
hipError_t launch_short_t(const uint8_t *d_keys, const uint64_t *d_off, uint64_t nkeys, uint32_t *d_out,
                          hipStream_t stream)
{
    const uint64_t ntiles = (nkeys + 63u) / 64u;
    uint64_t grid = (uint64_t)num_cus();
    const uint64_t need = (ntiles + kW - 1u) / kW;
    if (grid > need) grid = need;
    /* more than half the CU's 160 KiB in all: one workgroup per CU */
    constexpr uint32_t kTab = has_table<MODE>() ? nc_slice::table_words<R, 4u * NW>() * 4u : 0u;
    const uint32_t pad = kTab >= 90112u ? 0u : 90112u - kTab;
    auto k = nc_bytes_short_kernel<MODE, NC, DEPTH, kW, NW, R>;
    static std::atomic<uint64_t> attr_done{0}; /* per instantiation: the devices it is set on */
    const hipError_t ea = dyn_lds_once((const void *)k, (int)pad, attr_done);
    if (ea != hipSuccess) return ea;
    (void)hipGetLastError();
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(64 * kW), pad, stream, d_keys, d_off, nkeys, d_out, ntiles);
    return hipGetLastError();
}

template <int MODE, int NC, int DEPTH>
hipError_t launch_short_d(const uint8_t *d_keys, const uint64_t *d_off, uint64_t nkeys, uint32_t *d_out,
                          hipStream_t stream, int var)
{
    if constexpr (has_table<MODE>()) {
        switch ((var >> 2) & 3) {
        case 1:
            if (var & 16) return launch_short_t<MODE, NC, DEPTH, 2, 8, 16>(d_keys, d_off, nkeys, d_out, stream);
            return launch_short_t<MODE, NC, DEPTH, 2, 8>(d_keys, d_off, nkeys, d_out, stream);
        case 2: return launch_short_t<MODE, NC, DEPTH, 4, 8>(d_keys, d_off, nkeys, d_out, stream);
        case 3: return launch_short_t<MODE, NC, DEPTH, 1, 32>(d_keys, d_off, nkeys, d_out, stream);
        default: break;
        }
    }
    /* var bit 4: sixteen waves per CU (one 1024-thread workgroup) */
    if (var & 16) return launch_short_t<MODE, NC, DEPTH, 1, 8, 16>(d_keys, d_off, nkeys, d_out, stream);
    return launch_short_t<MODE, NC, DEPTH, 1, 8>(d_keys, d_off, nkeys, d_out, stream);
}

template <int MODE, int NC>
hipError_t launch_short(const uint8_t *d_keys, const uint64_t *d_off, uint64_t nkeys, uint32_t *d_out,
                        hipStream_t stream, int var)
{
    /* jenkins: one tile ahead only (deeper, hipcc spills its mix state) */
    if constexpr (MODE == NC_GPUHASH_JENKINS) {
        return launch_short_d<MODE, NC, 2>(d_keys, d_off, nkeys, d_out, stream, var);
    } else {
        switch (var & 3) {
        case 1: return launch_short_d<MODE, NC, 2>(d_keys, d_off, nkeys, d_out, stream, var);
        case 2: return launch_short_d<MODE, NC, 4>(d_keys, d_off, nkeys, d_out, stream, var);
        default: return launch_short_d<MODE, NC, 3>(d_keys, d_off, nkeys, d_out, stream, var);
        }
    }
}

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
        if constexpr (!has_table<MODE>() && (OPT & kOptNoHash) == 0) {
            /* two lines per round: 16 KiB images, 128 KiB per workgroup, one per
             * CU (the crcs' table does not fit beside them at 16 waves, and at
             * eight their lookups run 2.08-2.24 ms on the C4 shard against
             * 1.84, profiles/r05_c4_pairs_crc_ab.jsonl) */
            if (var & 256) {
                hipLaunchKernelGGL((nc_bytes_direct_kernel<MODE, true, true, 8, OPT | kOptPairs>), dim3((unsigned)grid8),
                                   dim3(512), 0, stream, d_keys, d_off, nkeys, d_out, ntiles, chunk);
                return hipGetLastError();
            }
        }
        const uint32_t pad = has_table<MODE>() ? 0u : 40960u;
        if (pad) {
            static std::atomic<uint64_t> attr_done{0};
            const hipError_t ea =
                dyn_lds_once((const void *)nc_bytes_direct_kernel<MODE, true, true, 8, OPT>, (int)pad, attr_done);
            if (ea != hipSuccess) return ea;
        }
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
 * build, fnv1a_64 and crc32 only); bit 7: the short-key kernel for keys of at
 * most max_len (<= 32) bytes */
template <int MODE>
hipError_t launch_mode(const uint8_t *d_keys, const uint64_t *d_off, uint64_t nkeys, uint32_t *d_out,
                       hipStream_t stream, int var, uint32_t max_len)
{
    if ((var & 128) && max_len <= 32u) {
        if (max_len <= 16u) return launch_short<MODE, 1>(d_keys, d_off, nkeys, d_out, stream, var);
        return launch_short<MODE, 2>(d_keys, d_off, nkeys, d_out, stream, var);
    }
    if constexpr (is_word_mode<MODE>()) {
        return hipErrorInvalidValue; /* the word modes run on the short-key kernel only */
    } else {
    if constexpr (MODE == NC_GPUHASH_FNV1A_64 || MODE == NC_GPUHASH_CRC32) {
        if (var & 64) return launch_opt<MODE, kOptNoHash>(d_keys, d_off, nkeys, d_out, stream, var);
        if (var & 512) return launch_opt<MODE, kOptOffDefault>(d_keys, d_off, nkeys, d_out, stream, var);
    }
    if constexpr (has_table<MODE>()) {
        if (var & 32) return launch_opt<MODE, kOptS8>(d_keys, d_off, nkeys, d_out, stream, var);
    }
    return launch_opt<MODE, 0>(d_keys, d_off, nkeys, d_out, stream, var);
    }
}

/* the byte-serial modes on the direct pipeline; var: bits 0-1 tiles per wave
 * (16, 8, 32, 64), bit 2 the LDS-DMA block image (long keys), bit 3 a wave's
 * tiles interleaved over the grid (else consecutive), bit 4 (with 2 and 3)
 * eight-wave workgroups, one per CU (bit 8 with them, no crc table: rounds
 * of two lines, dma_pairs), bits 5-7 as launch_mode. max_len: the caller's
 * longest key (its shape; 0xffffffff unknown). nkeys < 2^32. */

/* hsieh, murmur, jenkins: the short-key kernel only (var bit 7, max_len <= 32) */
bool supports_short_words(int mode)
{
    return mode == NC_GPUHASH_HSIEH || mode == NC_GPUHASH_MURMUR || mode == NC_GPUHASH_JENKINS;
}

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
                  hipStream_t stream, int var, uint32_t max_len)
{
    switch (mode) {
    case NC_GPUHASH_ONE_AT_A_TIME: return launch_mode<NC_GPUHASH_ONE_AT_A_TIME>(d_keys, d_off, nkeys, d_out, stream, var, max_len);
    case NC_GPUHASH_CRC16: return launch_mode<NC_GPUHASH_CRC16>(d_keys, d_off, nkeys, d_out, stream, var, max_len);
    case NC_GPUHASH_CRC32: return launch_mode<NC_GPUHASH_CRC32>(d_keys, d_off, nkeys, d_out, stream, var, max_len);
    case NC_GPUHASH_CRC32A: return launch_mode<NC_GPUHASH_CRC32A>(d_keys, d_off, nkeys, d_out, stream, var, max_len);
    case NC_GPUHASH_FNV1_64: return launch_mode<NC_GPUHASH_FNV1_64>(d_keys, d_off, nkeys, d_out, stream, var, max_len);
    case NC_GPUHASH_FNV1A_64: return launch_mode<NC_GPUHASH_FNV1A_64>(d_keys, d_off, nkeys, d_out, stream, var, max_len);
    case NC_GPUHASH_FNV1_32: return launch_mode<NC_GPUHASH_FNV1_32>(d_keys, d_off, nkeys, d_out, stream, var, max_len);
    case NC_GPUHASH_FNV1A_32: return launch_mode<NC_GPUHASH_FNV1A_32>(d_keys, d_off, nkeys, d_out, stream, var, max_len);
    case NC_GPUHASH_HSIEH: return launch_mode<NC_GPUHASH_HSIEH>(d_keys, d_off, nkeys, d_out, stream, var, max_len);
    case NC_GPUHASH_MURMUR: return launch_mode<NC_GPUHASH_MURMUR>(d_keys, d_off, nkeys, d_out, stream, var, max_len);
    case NC_GPUHASH_JENKINS: return launch_mode<NC_GPUHASH_JENKINS>(d_keys, d_off, nkeys, d_out, stream, var, max_len);
    default: return hipErrorInvalidValue;
    }
}

} // namespace nc_bytes
