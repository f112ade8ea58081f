/*
 * hash_md5 (src/hashkit/nc_md5.c:301-321: md5_signature's digest bytes 0..3 as
 * a little-endian u32) on gfx950 — the direct per-lane pipeline.
 *
 * md5 is VALU-bound (64 steps of ~5 dependent integer ops per 64-byte block),
 * so this kernel is built around the block, not around the byte stream:
 *
 *   - a wave owns a tile of 64 consecutive keys, one per lane, and walks its
 *     tiles grid-stride (persistent waves, no workgroup barrier anywhere);
 *   - a ROUND hashes one 64-byte block of every active lane's key. Its
 *     message words come straight from HBM/L2 with four unaligned 16-byte
 *     loads per lane (gfx9 global memory runs in unaligned mode), issued one
 *     round ahead into a second register set, so the loads of round r+1 fly
 *     while round r computes;
 *   - the key's last data block is padded in registers by ONE v_perm_b32 per
 *     word: the selector keeps a message byte, injects the 0x80 pad byte, or
 *     zeroes it (src/hashkit/nc_md5.c:249-262), and comes from one clamp of a
 *     per-lane linear form (v_med3_i32) — three VALU ops per word, no
 *     per-word compares or selects;
 *   - a key whose padding does not fit its last data block (length % 64 in
 *     56..63, a multiple of 64, or empty) needs one more block that holds no
 *     key bytes: 0x80 or 0, zeros, and the bit length (nc_md5.c:263-274).
 *     Such lanes park their state in a per-wave LDS queue and the wave runs
 *     those tail blocks 64 at a time, so a Zipf tile with three 60-byte keys
 *     does not pay a second block for all 64 lanes; a 56-64-byte key parks
 *     after step 60 and its tail round runs steps 61-63 (run_tail), and the
 *     workgroup pools its queues' leftovers at the end (flush_tails);
 *   - the final block of a key stops after step 60: the digest word returned
 *     is state A (nc_md5.c:317-320), and steps 61-63 only update B, C, D.
 *
 * Every round issues the same six vector-memory loads (two offset words,
 * four message chunks; addresses of chunks a lane does not need are clamped
 * into the buffer), so hipcc's waitcnt pass can count them exactly.
 */
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <array>
#include <type_traits>
#include <utility>

#include "nc_gpuhash.h"
#include "nc_hash_algo.h"
#include "nc_md5_steps.h"
#include "nc_direct.h"
#include "nc_out_policy.h"

namespace {

using namespace nc_md5s;

using namespace nc_direct;

/* per-wave LDS queue of keys waiting for their data-free last block */
constexpr uint32_t kQ = 128;        /* entries per wave (>= 64 + 63) */
constexpr uint32_t kQWords = 9;     /* state X0..X3, length, key index, message words 11, 2, 9 */
constexpr uint32_t kWaves = 4;      /* waves per workgroup */
constexpr uint32_t kQBytes = kQ * kQWords * 4u;

struct Queue {
    uint32_t *w; /* SoA: w[f * kQ + slot] */
    uint32_t head, count; /* wave-uniform */
};

/* the lanes where p holds, as a wave mask: the builtin straight from the
 * compare's mask (HIP's __ballot(int) widens the bool to a VGPR 0/1 and
 * compares it again: two VALU per use) */
__device__ __forceinline__ uint64_t ballot(bool p)
{
    return __builtin_amdgcn_ballot_w64(p);
}

__device__ __forceinline__ uint32_t lanemask_lt_popc(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

/* Tail blocks of up to 64 queued keys: message 0x80-or-0, zeros, bit length
 * (src/hashkit/nc_md5.c:263-274); out[index] = A + the block's A. A key of
 * 56..64 bytes (its one data block could not take the length) was queued
 * after step 60 of that block: X is the working state then, and steps 61..63
 * (message words 11, 2, 9) and the state add finish here, 64 lanes at a
 * time, instead of in every round a wave holds such a key. Any other queued
 * key (empty, or longer than 64 bytes) carries its chaining state in X. */
__device__ __forceinline__ void tail_entry(const uint32_t *qw, uint32_t slot, uint32_t *__restrict__ out)
{
    const uint32_t len = qw[4 * kQ + slot], idx = qw[5 * kQ + slot];
    uint32_t st[4] = {qw[0 * kQ + slot], qw[1 * kQ + slot], qw[2 * kQ + slot], qw[3 * kQ + slot]};
    if (len - 56u <= 8u) {
        uint32_t w[16];
        w[11] = qw[6 * kQ + slot];
        w[2] = qw[7 * kQ + slot];
        w[9] = qw[8 * kQ + slot];
        md5_steps_from61(st, w, std::make_integer_sequence<int, 3>{});
        st[0] += NC_MD5_A0;
        st[1] += NC_MD5_B0;
        st[2] += NC_MD5_C0;
        st[3] += NC_MD5_D0;
    }
    uint32_t w[16] = {};
    w[0] = (len & 63u) == 0u ? 0x80u : 0u;
    w[14] = len << 3;
    w[15] = len >> 29;
    /* words 1..13 are zero: folded into the steps' constants */
    out_st32(out + idx, md5_tail_final_a(st, w));
}

__device__ __forceinline__ void run_tail(Queue &q, uint32_t lane, uint32_t *__restrict__ out)
{
    const uint32_t n = q.count < 64u ? q.count : 64u;
    if (lane < n) tail_entry(q.w, (q.head + lane) & (kQ - 1u), out);
    q.head = (q.head + n) & (kQ - 1u);
    q.count -= n;
}

/* The workgroup's leftover queue entries at the end, pooled: batch k of 64
 * from the concatenation of the waves' queues goes to wave k mod kWaves
 * (one partly filled tail round per wave would cost each wave a full round
 * of steps for its last few keys). Every wave of the workgroup calls it. */
__device__ __forceinline__ void flush_tails(uint32_t *qmem, uint32_t (*qmeta)[2], const Queue &q, uint32_t wave,
                                            uint32_t lane, uint32_t *__restrict__ out)
{
    if (lane == 0u) {
        qmeta[wave][0] = q.head;
        qmeta[wave][1] = q.count;
    }
    __syncthreads();
    uint32_t head[kWaves], pre[kWaves + 1];
    pre[0] = 0u;
#pragma unroll
    for (uint32_t i = 0; i < kWaves; i++) {
        head[i] = (uint32_t)__builtin_amdgcn_readfirstlane((int)qmeta[i][0]);
        pre[i + 1] = pre[i] + (uint32_t)__builtin_amdgcn_readfirstlane((int)qmeta[i][1]);
    }
    for (uint32_t e0 = 64u * wave; e0 < pre[kWaves]; e0 += 64u * kWaves) {
        const uint32_t e = e0 + lane;
        if (e < pre[kWaves]) {
            uint32_t sw = 0u;
#pragma unroll
            for (uint32_t i = 1; i < kWaves; i++) sw += e >= pre[i] ? 1u : 0u;
            uint32_t h = head[0], p = pre[0];
#pragma unroll
            for (uint32_t i = 1; i < kWaves; i++) {
                h = sw == i ? head[i] : h;
                p = sw == i ? pre[i] : p;
            }
            tail_entry(qmem + sw * kQWords * kQ, (h + e - p) & (kQ - 1u), out);
        }
    }
}

} // namespace

/*
 * One wave = one 64-key tile at a time (lane = key). Round (tile, b) hashes
 * data block b of every key of the tile that has one; its 16 message words
 * are in `cur`, loaded during the previous round. keys is any byte address;
 * key i = keys[off[i], off[i+1]); keys stays readable NC_GPUHASH_PAD bytes
 * past off[nkeys]. A tile of 64 keys spans less than 4 GiB.
 */
/* S64: the caller's shape says every key has at most 64 bytes (C2): one
 * data block per key, so no round ever continues a key — no chaining state,
 * no block-index bookkeeping, no second gen copy (and their loop-carried
 * register copies). Each round checks its tile (one compare and a ballot);
 * a tile with a longer key (a wrong shape) ends the fast loop, and that
 * tile and the wave's later ones run the generic rounds: slower, never
 * wrong. */
template <bool LDS, bool IL, int FL = 0, bool PT = false, bool FS = false, bool S64 = false>
__global__ __launch_bounds__(256, 8) void nc_md5_direct_kernel(const uint8_t *__restrict__ keys,
                                                           const uint64_t *__restrict__ off, uint64_t nkeys,
                                                           uint32_t *__restrict__ out, uint64_t ntiles, uint32_t chunk)
{
    __shared__ uint32_t qmem[kWaves * kQWords * kQ];
    __shared__ uint32_t qmeta[kWaves][2];
    /* PT: the padding selectors from a 512-byte LDS table (pad_block_tab) */
    __shared__ uint32_t ptab[PT ? kPadTabWords : 1];
    if constexpr (PT) {
        for (uint32_t i = threadIdx.x; i < kPadTabWords; i += 256u) ptab[i] = pad_tab_entry(i);
        __syncthreads();
    }
    /* LDS: the next round's blocks arrive by LDS-DMA into a per-wave 4 KiB
     * image (key k's 64 bytes at k * 64) instead of into registers */
    __shared__ __attribute__((aligned(16))) uint8_t kbuf[LDS ? kWaves * kImage : 16];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    /* a wave owns `chunk` consecutive tiles; the grid covers every tile once
     * and the hardware dispatcher balances the waves (no persistent grid to
     * size from an occupancy estimate) */
    const Tiles<IL> tiles = wave_tiles<IL>(ntiles, chunk, kWaves, wave);
    uint32_t tile = 0; /* local tile index */
    const uint32_t tlast = tiles.n;
    Queue q{qmem + wave * kQWords * kQ, 0u, 0u};
    if (tile < tlast) { /* a wave without tiles still joins the workgroup's tail flush */
    Walker<IL> wk;
    wk.init(keys, off, nkeys, tiles, lane);
    uint8_t *const img = kbuf + (LDS ? wave * kImage : 0u);
    auto load_blk = [&](const TileKeys &t, uint32_t b, u32x4 (&d)[4]) __attribute__((always_inline)) {
        if constexpr (LDS) wk.dma(t, b, img);
        else wk.load_regs(t, b, d);
    };

    /* prologue: offsets of the first tile (waited), of the second (in
     * flight), block 0 of the first tile (in flight). The offsets take the
     * default cache policy here (the byte kernels' nt is 2 % slower for md5:
     * C2 0.787 -> 0.772 ms in an A/B/A/B, profiles/r03_cache_policy_ab.md) */
    TileKeys cur_t = wk.keys_of(tile, wk.template load_off<0>(tile));
    Offs no = wk.template load_off<0>(tile + 1u);
    u32x4 da[4], db[4];
    load_blk(cur_t, 0u, da);
    uint32_t b = 0;
    /* the chaining state of keys with a later block (set by block 0's round;
     * a first block starts from the constants, md5_steps_first61) */
    uint32_t st[4] = {NC_MD5_A0, NC_MD5_B0, NC_MD5_C0, NC_MD5_D0};
    uint32_t pad_src; /* kPadSrc in a VGPR: a uniform selector takes the perm's SGPR slot */
    asm volatile("v_mov_b32 %0, %1" : "=v"(pad_src) : "i"(kPadSrc));

    /* One round: block b of every key of the tile that has one, from `cur`
     * (loaded during the previous round). Its message words are padded out of
     * `cur` first; then the next round's loads (block b+1 of this tile if any
     * key has one, else block 0 of the next tile, whose offsets are in `no`)
     * go to the OTHER register set `nxt` and fly during the 64 steps. Two
     * sets, alternating (the loop below runs rounds in pairs), so that a
     * message word taken as loaded — a fixed-length key's data words, a full
     * block — is read by the steps in place: with one set it had to be copied
     * out before the next round's loads could land there (24 v_mov per round
     * in the fixed-length form). */
    bool bail = false; /* S64: this wave met a key longer than 64 bytes */
    auto round = [&](auto fast_c, u32x4 (&cur)[4], u32x4 (&nxt)[4]) __attribute__((always_inline)) {
        constexpr bool S = decltype(fast_c)::value;
        bool more = false;
        if constexpr (S) {
            if (ballot((lane < cur_t.nv) && cur_t.len > 64u) != 0ull) {
                bail = true; /* nothing of this tile consumed yet */
                return;
            }
        } else {
            more = ballot((lane < cur_t.nv) && cur_t.len > 64u * (b + 1u)) != 0ull;
        }
        const TileKeys nxt_t = wk.keys_of(tile + 1u, no);
        const int32_t rem = (int32_t)cur_t.len - 64 * (int32_t)b; /* key bytes from this block's start */
        const uint32_t len = cur_t.len;
        const bool act = (lane < cur_t.nv) && rem > 0;
        /* keys whose last data block could not take the length (or empty
         * keys) queue their state for a data-free tail block; the mask is
         * taken here, under the full exec mask (inside the steps' divergent
         * region hipcc rebuilds it with a select and a compare) */
        const bool tail = (lane < cur_t.nv) && (S ? (len >= 56u || len == 0u)
                                                  : ((rem <= 64 && rem >= 56) || (b == 0u && len == 0u)));
        const uint64_t tm = ballot(tail);
        if constexpr (LDS) wk.read_img(img, cur); /* this round's block, DMA'd during the previous round */
        /* FL: a tile whose keys all have FL bytes (checked: the shape only
         * picks the instantiation) takes its data words as loaded, the
         * boundary word by one constant perm, and constants for the rest.
         * Every form pads `cur` in place: the steps read it as it stands. */
        bool fl_tile = false;
        if constexpr (FL > 0) fl_tile = ballot((lane < cur_t.nv) && cur_t.len != (uint32_t)FL) == 0ull;
        if (fl_tile) {
            if constexpr (FL > 0 && FL % 4 != 0) {
                constexpr uint32_t bnd = FL % 4 == 1 ? kBoundary1 : (FL % 4 == 2 ? kBoundary2 : kBoundary3);
                cur[(FL / 4) >> 2][(FL / 4) & 3] = __builtin_amdgcn_perm(cur[(FL / 4) >> 2][(FL / 4) & 3], pad_src, bnd);
            }
        } else if (act) {
            if constexpr (PT) pad_block_tab(cur, rem < 64 ? rem : 64, pad_src, ptab);
            else pad_block(cur, rem < 64 ? rem : 64, pad_src);
            const bool fin = rem <= 55; /* the bit length fits behind the pad */
            if (fin) {
                cur[3][2] = len << 3;
                cur[3][3] = len >> 29;
            }
        }
        uint32_t w[16];
#pragma unroll
        for (int t = 0; t < 16; t++) w[t] = cur[t >> 2][t & 3];
        if constexpr (LDS) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); /* the image's reads are done */
        load_blk(more ? cur_t : nxt_t, more ? b + 1u : 0u, nxt);
        /* offsets two tiles ahead, straight into `no` (consumed above: a copy
         * of a register whose load is in flight would make hipcc wait for
         * every outstanding load, this round's prefetch included); while this
         * tile still has blocks it re-reads the next tile's words, which
         * keeps the per-round load count fixed */
        no = wk.template load_off<0>(more ? tile + 1u : tile + 2u);
        if (fl_tile) {
            if constexpr (FL > 0) {
                if (act) { /* one block: from the initial state */
                    uint32_t v[4] = {NC_MD5_A0, NC_MD5_B0, NC_MD5_C0, NC_MD5_D0};
                    md5_steps_fl<FL>(v, w, std::make_integer_sequence<int, 61>{});
                    const rsrc_t rout = make_rsrc(out + wk.key0(tile), 256u);
                    __builtin_amdgcn_raw_buffer_store_b32(NC_MD5_A0 + v[0], rout, (int)(lane * 4u), 0, kAuxOut);
                }
            }
        }
        /* a tile's block 0 (wave-uniform b) starts from the constant state:
         * its own copy of the steps folds it in, and nothing resets st */
        auto gen = [&](auto first_c) __attribute__((always_inline)) {
            constexpr bool FIRST = decltype(first_c)::value;
            uint32_t v[4]; /* a queued key's X (run_tail) */
            if constexpr (FIRST) {
                v[0] = NC_MD5_A0;
                v[1] = NC_MD5_B0;
                v[2] = NC_MD5_C0;
                v[3] = NC_MD5_D0;
            } else {
                v[0] = st[0];
                v[1] = st[1];
                v[2] = st[2];
                v[3] = st[3];
            }
            if (act) {
                const bool fin = rem <= 55;
                /* steps 0..60 for every lane; a key that ends here is done (A's
                 * last update is step 60); a key of 56..64 bytes leaves steps
                 * 61..63 to its tail block's round (run_tail); longer keys run
                 * them here */
                if constexpr (FIRST) md5_steps_first61(v, w);
                else md5_steps(v, w, std::make_integer_sequence<int, 61>{});
                /* FS: a key whose last data block this is stores too, a
                 * placeholder when its padding needs a tail block (run_tail
                 * overwrites it): the tile's 256-byte store has no holes, so
                 * HBM sees whole lines, not partial writes */
                if (FS ? rem <= 64 : fin) {
                    const rsrc_t rout = make_rsrc(out + wk.key0(tile), 256u);
                    __builtin_amdgcn_raw_buffer_store_b32((FIRST ? NC_MD5_A0 : st[0]) + v[0], rout, (int)(lane * 4u),
                                                          0, kAuxOut);
                }
                if (fin || S) { /* (S: a key of 56..64 bytes queues its tail block) */
                } else if (len - 56u > 8u) {
                    md5_steps_from61(v, w, std::make_integer_sequence<int, 3>{});
                    st[0] = (FIRST ? NC_MD5_A0 : st[0]) + v[0];
                    st[1] = (FIRST ? NC_MD5_B0 : st[1]) + v[1];
                    st[2] = (FIRST ? NC_MD5_C0 : st[2]) + v[2];
                    st[3] = (FIRST ? NC_MD5_D0 : st[3]) + v[3];
                    v[0] = st[0];
                    v[1] = st[1];
                    v[2] = st[2];
                    v[3] = st[3];
                }
            }
            return std::array<uint32_t, 4>{v[0], v[1], v[2], v[3]};
        };
        if (!fl_tile) { /* (a fixed-length tile, FL <= 48, has no tail keys) */
            std::array<uint32_t, 4> v;
            if constexpr (FL > 0) { /* a fixed-length kernel's odd tile: one step copy (two spill at 64 VGPRs) */
                if (b == 0u) {
                    st[0] = NC_MD5_A0;
                    st[1] = NC_MD5_B0;
                    st[2] = NC_MD5_C0;
                    st[3] = NC_MD5_D0;
                }
                v = gen(std::false_type{});
            } else if constexpr (S) {
                v = gen(std::true_type{});
            } else {
                v = b == 0u ? gen(std::true_type{}) : gen(std::false_type{});
            }
            /* keys whose last data block could not take the length (or empty
             * keys) queue their state for a data-free tail block */

            if (tm != 0ull) {
                if (tail) {
                    const uint32_t slot = (q.head + q.count + lanemask_lt_popc(tm)) & (kQ - 1u);
                    q.w[0 * kQ + slot] = v[0];
                    q.w[1 * kQ + slot] = v[1];
                    q.w[2 * kQ + slot] = v[2];
                    q.w[3 * kQ + slot] = v[3];
                    q.w[4 * kQ + slot] = len;
                    q.w[5 * kQ + slot] = wk.key0(tile) + lane;
                    q.w[6 * kQ + slot] = w[11];
                    q.w[7 * kQ + slot] = w[2];
                    q.w[8 * kQ + slot] = w[9];
                }
                q.count += (uint32_t)__builtin_popcountll(tm);
                if (q.count >= 64u) {
                    /* FS: this round's placeholders land before the tail
                     * results that replace them */
                    if constexpr (FS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    run_tail(q, lane, out);
                }
            }
        }

        /* advance */
        if (more) {
            b++;
        } else {
            tile++;
            b = 0;
            cur_t = nxt_t;
        }
    };
    if constexpr (S64) {
        for (;;) {
            round(std::true_type{}, da, db);
            if (bail || tile >= tlast) break;
            round(std::true_type{}, db, da);
            if (bail || tile >= tlast) break;
        }
    }
    if (!S64 || bail) {
        if constexpr (S64) { /* the generic rounds from this tile: its offsets and block 0 again */
            cur_t = wk.keys_of(tile, wk.template load_off<0>(tile));
            no = wk.template load_off<0>(tile + 1u);
            load_blk(cur_t, 0u, da);
            b = 0u;
        }
        for (;;) {
            round(std::false_type{}, da, db);
            if (tile >= tlast) break;
            round(std::false_type{}, db, da);
            if (tile >= tlast) break;
        }
    }
    }
    /* (pooled for the generic kernel; the fixed-length instantiations queue
     * almost nothing, and the pooled flush there made hipcc spill) */
    if constexpr (FL == 0) flush_tails(qmem, qmeta, q, wave, lane, out);
    else while (q.count != 0u) run_tail(q, lane, out);
}

/*
 * Long keys: the same rounds, fed from an 8 KiB LDS line image per wave
 * (nc_direct.h dma_lines: 128 bytes of every key per round, whole lines, so a
 * line is fetched once). A round hashes up to two blocks of each key; keys
 * whose padding needs one more, data-free block get it in the same round
 * (with long keys every lane of a tile usually needs it at once, so there is
 * no queue).
 */
/* OA: the offsets' cache policy — the default, as the direct kernel's: a
 * lane's start and end dwords share lines that nt can evict between the two
 * loads (C4 shard 1.8063 -> 1.7884 ms, HBM reads 9.48 -> 9.29 GB per launch,
 * profiles/r06k_c4_offsets_policy_ab_md5.jsonl, pmc_r06k_c4_offsets_policy.json);
 * nt (kAuxNt, the round-5 form) by A/B bit 6 */
template <bool IL, int OA = 0>
__global__ __launch_bounds__(256) void nc_md5_lines_kernel(const uint8_t *__restrict__ keys,
                                                           const uint64_t *__restrict__ off, uint64_t nkeys,
                                                           uint32_t *__restrict__ out, uint64_t ntiles, uint32_t chunk)
{
    __shared__ __attribute__((aligned(16))) uint8_t kbuf[kWaves * kLineImage];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const Tiles<IL> tiles = wave_tiles<IL>(ntiles, chunk, kWaves, wave);
    uint32_t tile = 0; /* local tile index */
    const uint32_t tlast = tiles.n;
    if (tile >= tlast) return;
    Walker<IL> wk;
    wk.init(keys, off, nkeys, tiles, lane);
    uint8_t *const img = kbuf + wave * kLineImage;
    TileKeys cur_t = wk.keys_of(tile, wk.template load_off<OA>(tile));
    Offs no = wk.template load_off<OA>(tile + 1u);
    wk.dma_lines(cur_t, 0u, img);
    uint32_t b = 0;
    uint32_t st[4] = {NC_MD5_A0, NC_MD5_B0, NC_MD5_C0, NC_MD5_D0};
    uint32_t pad_src;
    asm volatile("v_mov_b32 %0, %1" : "=v"(pad_src) : "i"(kPadSrc));

    /* one 64-byte block holding rem (> 0) of the key's remaining bytes */
    auto block = [&](u32x4 (&d)[4], int32_t rem) __attribute__((always_inline)) {
        pad_block_u(d, rem < 64 ? rem : 64, pad_src); /* in place */
        const bool fin = rem <= 55;
        if (fin) {
            d[3][2] = cur_t.len << 3;
            d[3][3] = cur_t.len >> 29;
        }
        uint32_t w[16];
#pragma unroll
        for (int t = 0; t < 16; t++) w[t] = d[t >> 2][t & 3];
        uint32_t v[4] = {st[0], st[1], st[2], st[3]};
        md5_steps(v, w, std::make_integer_sequence<int, 61>{});
        if (fin) {
            const rsrc_t rout = make_rsrc(out + wk.key0(tile), 256u);
            __builtin_amdgcn_raw_buffer_store_b32(st[0] + v[0], rout, (int)(lane * 4u), 0, kAuxOut);
        } else {
            md5_steps_from61(v, w, std::make_integer_sequence<int, 3>{});
            st[0] += v[0];
            st[1] += v[1];
            st[2] += v[2];
            st[3] += v[3];
        }
    };
    for (;;) {
        const bool more = __ballot(cur_t.valid && cur_t.len > 128u * (b + 1u)) != 0ull;
        const TileKeys nxt_t = wk.keys_of(tile + 1u, no);
        u32x4 d0[4], d1[4];
        wk.read_lines(img, d0, d1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); /* the image's reads are done */
        wk.dma_lines(more ? cur_t : nxt_t, more ? b + 1u : 0u, img);
        no = wk.template load_off<OA>(more ? tile + 1u : tile + 2u);

        const int32_t rem = (int32_t)cur_t.len - 128 * (int32_t)b; /* key bytes from this line's start */
        if (cur_t.valid && rem > 0) block(d0, rem);
        if (__ballot(cur_t.valid && rem > 64) != 0ull && cur_t.valid && rem > 64) block(d1, rem - 64);
        /* the data-free last block: length % 64 in 56..63 or 0 (or an empty
         * key), ending in this line */
        const int32_t last = rem > 64 ? rem - 64 : rem; /* bytes in the line's last block with data */
        const bool tail = cur_t.valid && ((rem > 0 && rem <= 128 && last >= 56) || (b == 0u && cur_t.len == 0u));
        if (__ballot(tail) != 0ull && tail) {
            uint32_t w[16] = {};
            w[0] = (cur_t.len & 63u) == 0u ? 0x80u : 0u;
            w[14] = cur_t.len << 3;
            w[15] = cur_t.len >> 29;
            const rsrc_t rout = make_rsrc(out + wk.key0(tile), 256u);
            __builtin_amdgcn_raw_buffer_store_b32(md5_tail_final_a(st, w), rout, (int)(lane * 4u), 0, kAuxOut);
        }
        if (more) {
            b++;
        } else {
            tile++;
            b = 0;
            cur_t = nxt_t;
            st[0] = NC_MD5_A0;
            st[1] = NC_MD5_B0;
            st[2] = NC_MD5_C0;
            st[3] = NC_MD5_D0;
        }
        if (tile >= tlast) break;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); /* no LDS-DMA may outlive the workgroup */
}

namespace nc_md5 {

template <int FL, bool PT>
void launch_fl(const uint8_t *d_keys, const uint64_t *d_off, uint64_t nkeys, uint32_t *d_out, hipStream_t stream,
               uint64_t grid, uint64_t ntiles, uint32_t chunk)
{
    hipLaunchKernelGGL((nc_md5_direct_kernel<false, false, FL, PT>), dim3((unsigned)grid), dim3(256), 0, stream, d_keys,
                       d_off, nkeys, d_out, ntiles, chunk);
}

/* var: bits 0-1 tiles per wave (0: 16, 1: 8, 2: 32, 3: 64); bit 2: the LDS-DMA
 * variant (long keys); bit 3 tiles interleaved over the grid; bit 4 the
 * padding selectors from the LDS table (pad_block_tab); bit 5 whole-line
 * stores (placeholders for the tail keys, FS); bit 6 (A/B) the line kernel's
 * offsets non-temporal (OA, the round-5 form); bit 7 (A/B) no S64 form.
 * max_len: the caller's shape's longest key (0xffffffff: unknown); at most
 * 64 takes the S64 form (FS only).  fl: the batch's
 * fixed key length if the caller's shape says so (0: unknown or varying);
 * 16, 20, 24, 32, 40 and 48 have specialised instantiations (each tile still
 * checks its lengths) */
template <bool PT>
hipError_t launch_pt(const uint8_t *d_keys, const uint64_t *d_off, uint64_t nkeys, uint32_t *d_out,
                     hipStream_t stream, int var, uint32_t fl, uint32_t max_len)
{
    static const uint32_t kChunk[4] = {16, 8, 32, 64};
    const uint32_t chunk = kChunk[var & 3];
    const uint64_t ntiles = (nkeys + 63u) / 64u;
    const uint64_t grid = (ntiles + (uint64_t)kWaves * chunk - 1u) / ((uint64_t)kWaves * chunk);
    if (grid > 0x7fffffffu) return hipErrorInvalidValue;
    (void)hipGetLastError();
    const bool il = (var & 8) != 0;
    if (var & 4) {
        if (il && (var & 64))
            hipLaunchKernelGGL((nc_md5_lines_kernel<true, kAuxNt>), dim3((unsigned)grid), dim3(256), 0, stream,
                               d_keys, d_off, nkeys, d_out, ntiles, chunk);
        else if (il)
            hipLaunchKernelGGL(nc_md5_lines_kernel<true>, dim3((unsigned)grid), dim3(256), 0, stream, d_keys, d_off,
                               nkeys, d_out, ntiles, chunk);
        else
            hipLaunchKernelGGL(nc_md5_lines_kernel<false>, dim3((unsigned)grid), dim3(256), 0, stream, d_keys, d_off,
                               nkeys, d_out, ntiles, chunk);
    } else if (il) {
        hipLaunchKernelGGL((nc_md5_direct_kernel<false, true, 0, PT>), dim3((unsigned)grid), dim3(256), 0, stream,
                           d_keys, d_off, nkeys, d_out, ntiles, chunk);
    } else if (fl == 16 || fl == 20 || fl == 24 || fl == 32 || fl == 40 || fl == 48) {
        switch (fl) {
        case 16: launch_fl<16, PT>(d_keys, d_off, nkeys, d_out, stream, grid, ntiles, chunk); break;
        case 20: launch_fl<20, PT>(d_keys, d_off, nkeys, d_out, stream, grid, ntiles, chunk); break;
        case 24: launch_fl<24, PT>(d_keys, d_off, nkeys, d_out, stream, grid, ntiles, chunk); break;
        case 32: launch_fl<32, PT>(d_keys, d_off, nkeys, d_out, stream, grid, ntiles, chunk); break;
        case 40: launch_fl<40, PT>(d_keys, d_off, nkeys, d_out, stream, grid, ntiles, chunk); break;
        default: launch_fl<48, PT>(d_keys, d_off, nkeys, d_out, stream, grid, ntiles, chunk); break;
        }
    } else if ((var & 32) && max_len <= 64u && (var & 128) == 0) {
        hipLaunchKernelGGL((nc_md5_direct_kernel<false, false, 0, PT, true, true>), dim3((unsigned)grid), dim3(256), 0,
                           stream, d_keys, d_off, nkeys, d_out, ntiles, chunk);
    } else if (var & 32) {
        hipLaunchKernelGGL((nc_md5_direct_kernel<false, false, 0, PT, true>), dim3((unsigned)grid), dim3(256), 0,
                           stream, d_keys, d_off, nkeys, d_out, ntiles, chunk);
    } else {
        hipLaunchKernelGGL((nc_md5_direct_kernel<false, false, 0, PT>), dim3((unsigned)grid), dim3(256), 0, stream,
                           d_keys, d_off, nkeys, d_out, ntiles, chunk);
    }
    return hipGetLastError();
}

hipError_t launch(const uint8_t *d_keys, const uint64_t *d_off, uint64_t nkeys, uint32_t *d_out, hipStream_t stream,
                  int var, uint32_t fl, uint32_t max_len)
{
    return (var & 16) ? launch_pt<true>(d_keys, d_off, nkeys, d_out, stream, var, fl, max_len)
                      : launch_pt<false>(d_keys, d_off, nkeys, d_out, stream, var, fl, max_len);
}

} // namespace nc_md5
