/*
 * Diagnostics and benchmark tuning — NOT part of the drop-in boundary
 * (include/nc_gpuhash.h is). A proxy never needs these:
 *   - a STREAM-style read kernel that measures the achievable HBM read
 *     bandwidth in the same run as the hash kernels (SURVEY.md §8d asks for
 *     the roofline fraction against both the 8 TB/s spec and a measured read
 *     ceiling);
 *   - the shape policy's kernel choice, an event-timed launch loop, and the
 *     process-wide launch tuning used by tests and sweeps.
 */
#ifndef NC_GPUHASH_PROBE_H
#define NC_GPUHASH_PROBE_H

#include <stdint.h>
#include "nc_gpuhash.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Read `bytes` (multiple of 16) from device buffer d_buf with 16-byte
 * coalesced loads, `iters` times on `stream`; store the mean ms per pass.
 * d_sink receives one u32 per workgroup (keeps the loads live); it needs
 * 4 * 65536 bytes. */
rstatus_t nc_gpuhash_probe_read(const void *d_buf, uint64_t bytes, uint32_t *d_sink, void *stream, int iters,
                                float *avg_ms);
/* The same with non-temporal (nt) loads: the ceiling for a read-once stream
 * under the cache policy of launch variant bit 6. */
rstatus_t nc_gpuhash_probe_read_nt(const void *d_buf, uint64_t bytes, uint32_t *d_sink, void *stream, int iters,
                                   float *avg_ms);
/* The read/write mix of a hash kernel: the read of `bytes` plus one 16-byte
 * store per 128 bytes read (12.5 % of the bytes moved are writes; C2
 * fnv1a_64's are 12 %) into d_wout, which must hold
 * ceil(bytes / 32768) * 4096 bytes. policy: bit 0 the loads, bit 1 the stores
 * with the default cache policy instead of non-temporal (EINVAL otherwise). */
rstatus_t nc_gpuhash_probe_mix(const void *d_buf, uint64_t bytes, void *d_wout, uint64_t wout_bytes,
                               uint32_t *d_sink, void *stream, int policy, int iters, float *avg_ms);

/* The grouped C2 pipeline's store pattern against its reads (VERDICT r05
 * item 5): tiles of tile_read contiguous bytes (a multiple of 8 KiB) read
 * with nt 16-byte loads by 512-thread workgroups (`grid` of them, tiles
 * grid-strided in runs of `run` consecutive tiles), each tile's tile_write
 * output bytes at d_out + tile * tile_write — stored after its tile, or
 * (defer bit 0) once per run from LDS, run * tile_write <= 8 KiB contiguous;
 * defer bits 4-5 the stores' flavour: 0 nt, 1 plain, 2 sc1, 3 sc0 sc1 (2 and 3
 * need out_bytes < 2 GiB). Mean ms per pass of all bytes / tile_read tiles. */
rstatus_t nc_gpuhash_probe_tile_mix(const void *d_buf, uint64_t bytes, void *d_out, uint64_t out_bytes,
                                   uint32_t tile_read, uint32_t tile_write, uint32_t run, uint32_t grid, int defer,
                                   uint32_t *d_sink, void *stream, int iters, float *avg_ms);

/* Clock sampler: ONE wave on `stream` (launched before the kernels it
 * watches, so it holds its slot) records n samples of (s_memtime,
 * s_memrealtime) into d_out[2n], one every gap_ticks of the 100 MHz
 * real-time clock, then exits (n * gap_ticks <= 1 s). Asynchronous: the
 * shader clock the GPU ran at while the other streams' kernels ran is
 * (c[i+1] - c[i]) / (r[i+1] - r[i]) * 100 MHz (tools/clock_probe.py). */
rstatus_t nc_gpuhash_probe_clock_sampler(uint64_t *d_out, uint32_t n, uint32_t gap_ticks, void *stream);

/* The launch variant the auto policy picks for this mode and shape (the
 * variant bits of nc_gpuhash_set_tuning; bit 16 = the plain workgroup
 * pipeline); -1 with errno EINVAL for an invalid mode. */
int nc_gpuhash_pick_variant(int mode, uint64_t nkeys, const struct nc_gpuhash_shape *shape);

/* Same launch repeated `iters` times between two hipEvents recorded on
 * `stream`; blocks until done and stores the mean milliseconds per launch. */
rstatus_t nc_gpuhash_time_device(int mode, const uint8_t *d_keys, const uint64_t *d_offsets,
                                 uint64_t nkeys, uint32_t *d_out, void *stream,
                                 int iters, float *avg_ms);
rstatus_t nc_gpuhash_time_device_shaped(int mode, const uint8_t *d_keys, const uint64_t *d_offsets,
                                        uint64_t nkeys, uint32_t *d_out,
                                        const struct nc_gpuhash_shape *shape, void *stream,
                                        int iters, float *avg_ms);

/* Launch tuning (process-wide, atomic; for tests and benchmarks only; every setting gives
 * identical outputs; variant 0 = the shape-driven auto policy, any other
 * value is used as given). grid_cap: maximum workgroups per launch (0 = persistent,
 * one per resident slot; -1 = keep). sort: group a tile's keys by length
 * before hashing (1 on, 0 off, -1 keep). variant: kernel code variant bits
 * (bit 0: shift-add FNV-64 multiply; bit 3: DIAGNOSTIC no-hash build,
 * fnv1a_64 unsorted only, outputs are NOT hashes, with bits 1-2 its L2
 * prefetch distance code (0 off, 1..3 = 2..4 tiles ahead); bit 4: DIAGNOSTIC arithmetic offsets
 * for fixed 32-byte keys, fnv1a_64 unsorted only; bit 5: register-staged
 * pipeline, two tiles in flight; bit 6: default cache policy on the key,
 * offset and output streams instead of non-temporal, fnv1a_64 and md5 only;
 * bit 7: wave-ring pipeline, bits 8-10 its slab/look-ahead shape; bits 11-15:
 * wave-ring options (fnv1a_64, md5: 4 waves per workgroup, pair-interleaved
 * keys, 64-key tiles, 256-key tiles hashed in length-sorted rounds, 128-key
 * tiles in two sorted rounds); bit 16: the plain workgroup
 * pipeline as an explicit choice; bit 17: length-grouped tiles, as sort = 1;
 * bit 18: workgroup pipelines launch three resident sets of workgroups;
 * bit 19: the direct per-lane pipeline (md5 and the byte-serial modes), bits
 * 20-23 its options (tiles per wave, 128-byte line image, grid interleave),
 * and with it: bit 10 rounds of two lines (eight-wave line kernel, no crc),
 * bit 11 the short-key kernel for keys <= 32 B by the shape (bits 20-21 its
 * tiles in flight, 22-23 the crc tables; the word modes too), bit 12 eight-wave
 * line workgroups or, with bit 11, sixteen waves per CU, bit 13 slicing-by-8
 * crc tables, bit 14 DIAGNOSTIC no-hash build, bit 15 md5's LDS pad table;
 * bit 24: the wave-sorted pipeline (fnv x4, one_at_a_time), bits 20-21 its
 * tiles per wave, bit 22 DIAGNOSTIC no-hash build (fnv1a_64), bit 23 its
 * tiles interleaved over the grid; bit 25: the grouped workgroup pipeline
 * (each wave one length quartile of the tile), bit 20 its DIAGNOSTIC no-hash
 * build (fnv1a_64), bits 21-22 its resident sets (6, 1, 3, 8), bit 23 three
 * slab buffers, bit 27 one coalesced store per tile; bit 26: md5
 * without its fixed-length specialisation (A/B); -1 = keep). */
rstatus_t nc_gpuhash_set_tuning(int grid_cap, int sort, int variant);

/* Batch ring diagnostics (tests only). start_seq: number the ring's batches
 * from `seq` (a ring that has run for that long; EBUSY after the first
 * submit). hold: 1 = launch no worker until set back to 0 (a submitted batch
 * stays pending, so a poll must say NC_EAGAIN). */
rstatus_t nc_gpuhash_ring_debug_start_seq(nc_gpuhash_ring_t *r, uint64_t seq);
rstatus_t nc_gpuhash_ring_debug_hold(nc_gpuhash_ring_t *r, int hold);
/* timeline: on = 1 before the first submit makes every batch record its
 * device timeline in its slot (s_memrealtime, 100 MHz): [0] descriptor
 * found, [1] batch staged in LDS, [2] every hash store issued, [3] stores
 * acknowledged, written before the done word; [4] hashes released (or, with
 * write-through hashes, drained) and [5] the lane's batch count, stored just
 * before the done word and possibly landing just after it; [6] the shader
 * clock over the hash phase ([1] to [2]) in MHz; [7] when thread 0's wave
 * finished its own keys (s_memrealtime). on = -1 only reads
 * slot `slot`'s eight words into out (when out is not NULL). */
rstatus_t nc_gpuhash_ring_debug_timeline(nc_gpuhash_ring_t *r, int on, uint32_t slot, uint64_t out[8]);
/* where the ring stages its batches: 1 = device memory written through the
 * PCIe BAR (large-BAR devices), 0 = mapped host memory (no large BAR, or
 * NC_GPUHASH_RING_STAGING=host when the ring was created), -1 = NULL ring */
int nc_gpuhash_ring_debug_staging(const nc_gpuhash_ring_t *r);

#ifdef __cplusplus
}
#endif

#endif
