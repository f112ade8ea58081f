/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * A clean-room CPU restatement of twemproxy's src/hashkit key-hash functions,
 * used as the parity checker for the MI355X batched hasher. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The
 * product library (twemproxy_amd/csrc) never links, calls or falls back to it.
 *
 * Parity pinning: every function is checked against golden vectors produced by
 * the real reference hashkit compiled from /root/reference (oracle/Makefile
 * target `ref`, script tests/golden/make_golden.py) and against the reference's
 * own known-answer tests (src/test_all.c:41-60).
 *
 * Mode ids follow HASH_CODEC order (src/hashkit/nc_hashkit.h:24-36).
 */
#ifndef NC_ORACLE_H
#define NC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    ORACLE_ONE_AT_A_TIME = 0,
    ORACLE_MD5,
    ORACLE_CRC16,
    ORACLE_CRC32,
    ORACLE_CRC32A,
    ORACLE_FNV1_64,
    ORACLE_FNV1A_64,
    ORACLE_FNV1_32,
    ORACLE_FNV1A_32,
    ORACLE_HSIEH,
    ORACLE_MURMUR,
    ORACLE_JENKINS,
    ORACLE_NMODES
};

/* One key, one mode. Returns 0 for an invalid mode. */
uint32_t oracle_hash(int mode, const uint8_t *key, size_t len);

/* Full 16-byte MD5 digest (src/hashkit/nc_md5.c:301 md5_signature). */
void oracle_md5(const uint8_t *key, size_t len, uint8_t digest[16]);

/* ketama_hash (src/hashkit/nc_ketama.c:31-41). */
uint32_t oracle_ketama_hash(const uint8_t *key, size_t len, uint32_t alignment);

/*
 * Batch over a CSR: key i = keys[offsets[i] .. offsets[i+1]).
 * Every key goes through a hash_t-style function pointer, as
 * server_pool_hash does (src/nc_server.c:643). nthreads <= 1 runs on the
 * calling thread; otherwise contiguous byte-balanced ranges on pthreads.
 * Returns 0, or -1 on a bad mode.
 */
int oracle_hash_batch(int mode, const uint8_t *keys, const uint64_t *offsets,
                      uint64_t nkeys, uint32_t *out, int nthreads);

/* Best-of-`reps` wall seconds of oracle_hash_batch (CLOCK_MONOTONIC). */
double oracle_time_batch(int mode, const uint8_t *keys, const uint64_t *offsets,
                         uint64_t nkeys, uint32_t *out, int nthreads, int reps);

/*
 * Distribution restatements (next-row parity): ketama continuum build
 * (src/hashkit/nc_ketama.c:58-219, no ejection: every server live),
 * ketama_dispatch (:222-246) and modula_dispatch (src/hashkit/nc_modula.c:146-156).
 * names: nserver NUL-free strings given as (ptr,len) pairs.
 * Returns the number of continuum points written (<= cap), or -1.
 */
int oracle_ketama_build(const char *const *names, const uint32_t *name_lens,
                        const uint32_t *weights, uint32_t nserver,
                        uint32_t *values, uint32_t *indices, uint32_t cap);
int oracle_ketama_build_live(const char *const *names, const uint32_t *name_lens,
                             const uint32_t *weights, const uint8_t *live, uint32_t nserver,
                             uint32_t *values, uint32_t *indices, uint32_t cap);
uint32_t oracle_ketama_dispatch(const uint32_t *values, const uint32_t *indices,
                                uint32_t n, uint32_t hash);
/* modula_update (src/hashkit/nc_modula.c:34-143, all live): one point per
 * weight unit, server-major; returns points written or -1. */
int oracle_modula_build(const uint32_t *weights, uint32_t nserver,
                        uint32_t *indices, uint32_t cap);
uint32_t oracle_modula_dispatch(const uint32_t *indices, uint32_t n, uint32_t hash);

/* server_pool_idx (src/nc_server.c:647-700) over a CSR batch: dist 0 ketama
 * (values + indices), 1 modula (indices); tag NULL or 2 bytes. 0 or -1. */
int oracle_server_idx_batch(int mode, int dist, const uint32_t *values, const uint32_t *indices,
                            uint32_t ncont, uint32_t nserver, const char *tag,
                            const uint8_t *keys, const uint64_t *offsets, uint64_t nkeys, uint32_t *out);

/* memcache_parse_req (src/proto/nc_memcache.c) over a stream of retrieval
 * requests, sequentially; see nc_oracle.c. Returns 0, or -1 when a limit is hit. */
int oracle_mc_parse(const uint8_t *s, uint64_t n, uint64_t max_keys, uint64_t *kstart, uint32_t *klen,
                    uint32_t *kreq, int32_t *status, uint64_t max_reqs, uint64_t *nkeys, uint64_t *nreqs_parsed,
                    uint64_t *first_error, uint64_t *consumed);

/* redis_parse_req (src/proto/nc_redis.c) over a stream of RESP requests of
 * the key classes arg0 / arg1 / argn / argx / argkvx, sequentially; see
 * nc_oracle.c. max_key_len = mbuf_data_size(). 0, or -1 when a limit is hit. */
int oracle_redis_parse(const uint8_t *s, uint64_t n, uint32_t max_key_len, uint64_t max_keys, uint64_t *kstart,
                       uint32_t *klen, uint32_t *kreq, int32_t *status, uint64_t max_reqs, uint64_t *nkeys,
                       uint64_t *nreqs_parsed, uint64_t *first_error, uint64_t *consumed);
/* the key class of a command name (0 none, 1 arg0, 2 arg1, 3 argn, 4 argx, 5 argkvx) */
int oracle_redis_class(const uint8_t *m, uint64_t len);

#ifdef __cplusplus
}
#endif

#endif
