/*
 * Diagnostics: a STREAM-style read kernel that measures the achievable HBM
 * read bandwidth in the same run as the hash kernels (SURVEY.md §8d asks for
 * the roofline fraction against both the 8 TB/s spec and a measured
 * read ceiling). Not part of the hashing path.
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

#ifdef __cplusplus
}
#endif

#endif
