/*
 * nc_gpuhash — MI355X (gfx950) batched key hashing, a drop-in for twemproxy's
 * src/hashkit.
 *
 * C ABI only: plain pointers and sizes, no C++ or torch types. Link
 * libnc_gpuhash.so in place of libhashkit.a (src/hashkit/Makefile.am:8-23,
 * src/Makefile.am:58). Reference interfaces each entry point replaces are cited
 * as /root/reference/<path>:<line>.
 *
 * Four groups:
 *   1. Link-compatible per-key symbols with the exact prototypes of
 *      src/hashkit/nc_hashkit.h:57-69 (+ ketama_hash, src/hashkit/nc_ketama.c:31).
 *      These are host functions: a per-key GPU round trip costs more than the
 *      hash. The batched entry points below never call them.
 *   2. The hash: selector (src/nc_conf.c:1738-1764, hash_algos[] :30-35).
 *   3. Batched GPU hashing over an offset CSR: key i is
 *      keys[offsets[i] .. offsets[i+1]). Device-resident, synchronous host and
 *      asynchronous (ticket + poll) host forms. There is no CPU fallback: with
 *      no usable GPU they return NC_ERROR with errno ENODEV.
 *   4. Multi-GPU shard planning (byte-balanced key ranges).
 */
#ifndef NC_GPUHASH_H
#define NC_GPUHASH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* rstatus_t and its values, src/nc_core.h:61-69. Guarded so the header can be
 * included next to nc_core.h inside twemproxy. */
#ifndef _NC_CORE_H_
typedef int rstatus_t;
#define NC_OK     0
#define NC_ERROR -1
#define NC_EAGAIN -2
#define NC_ENOMEM -3
#endif

/* Mode ids are hash_type_t values in HASH_CODEC order
 * (src/hashkit/nc_hashkit.h:24-48). */
typedef enum nc_gpuhash_mode {
    NC_GPUHASH_ONE_AT_A_TIME = 0,
    NC_GPUHASH_MD5 = 1,
    NC_GPUHASH_CRC16 = 2,
    NC_GPUHASH_CRC32 = 3,
    NC_GPUHASH_CRC32A = 4,
    NC_GPUHASH_FNV1_64 = 5,
    NC_GPUHASH_FNV1A_64 = 6,   /* conf default, src/nc_conf.h:44 */
    NC_GPUHASH_FNV1_32 = 7,
    NC_GPUHASH_FNV1A_32 = 8,
    NC_GPUHASH_HSIEH = 9,
    NC_GPUHASH_MURMUR = 10,
    NC_GPUHASH_JENKINS = 11,
    NC_GPUHASH_NMODES = 12     /* HASH_SENTINEL */
} nc_gpuhash_mode_t;

/* Bytes that must stay readable after offsets[nkeys] in a device key buffer
 * handed to nc_gpuhash_batch_device (16-byte vector loads of the last key). */
#define NC_GPUHASH_PAD 32

/* ---- 1. per-key, link-compatible (src/hashkit/nc_hashkit.h:57-69) ---- */
uint32_t hash_one_at_a_time(const char *key, size_t key_length);
void md5_signature(const unsigned char *key, unsigned int length, unsigned char *result);
uint32_t hash_md5(const char *key, size_t key_length);
uint32_t hash_crc16(const char *key, size_t key_length);
uint32_t hash_crc32(const char *key, size_t key_length);
uint32_t hash_crc32a(const char *key, size_t key_length);
uint32_t hash_fnv1_64(const char *key, size_t key_length);
uint32_t hash_fnv1a_64(const char *key, size_t key_length);
uint32_t hash_fnv1_32(const char *key, size_t key_length);
uint32_t hash_fnv1a_32(const char *key, size_t key_length);
uint32_t hash_hsieh(const char *key, size_t key_length);
uint32_t hash_jenkins(const char *key, size_t length);
uint32_t hash_murmur(const char *key, size_t length);
/* src/hashkit/nc_ketama.c:31-41 */
uint32_t ketama_hash(const char *key, size_t key_length, uint32_t alignment);

/* ---- 2. hash: selector (src/nc_conf.c:1738-1764) ---- */
/* Name -> mode id; -1 with errno EINVAL for "is not a valid hash". */
int nc_gpuhash_mode_from_name(const char *name, size_t len);
/* Mode id -> HASH_CODEC name ("fnv1a_64", ...); NULL for an invalid id. */
const char *nc_gpuhash_mode_name(int mode);

/* ---- 3a. device-resident batch ----
 * d_keys, d_offsets (nkeys + 1 entries, non-decreasing) and d_out (nkeys)
 * are device pointers; d_keys must stay readable NC_GPUHASH_PAD bytes past
 * offsets[nkeys]. Enqueues on `stream` (a hipStream_t, NULL = default
 * stream) and returns without waiting. Output order is input key order
 * (frag_seq[] depends on it, src/proto/nc_memcache.c:1337). */
rstatus_t nc_gpuhash_batch_device(int mode, const uint8_t *d_keys, const uint64_t *d_offsets,
                                  uint64_t nkeys, uint32_t *d_out, void *stream);

/* What the packer of a batch knows about it (all host-side facts, no device
 * read): Σ key bytes = offsets[nkeys] - offsets[0], and the shortest and
 * longest key. It selects the kernel pipeline; every choice
 * gives identical outputs. Zero key_bytes (or a NULL shape) = unknown. */
struct nc_gpuhash_shape {
    uint64_t key_bytes;
    uint32_t min_len;
    uint32_t max_len;
};

/* nc_gpuhash_batch_device with the batch shape (NULL = unknown, the same as
 * nc_gpuhash_batch_device). */
rstatus_t nc_gpuhash_batch_device_shaped(int mode, const uint8_t *d_keys, const uint64_t *d_offsets,
                                         uint64_t nkeys, uint32_t *d_out,
                                         const struct nc_gpuhash_shape *shape, void *stream);

/* ---- 3a'. fused server_pool_idx on the device ----
 * Replaces the per-key server_pool_idx (src/nc_server.c:647-700) for a batch:
 * hash_tag trimming (:665-677), server_pool_hash's empty-key rule (:639-641),
 * the pool's hash (mode), then ketama_dispatch (src/hashkit/nc_ketama.c:222-246)
 * or modula_dispatch (src/hashkit/nc_modula.c:146-156) over the pool's
 * continuum, which the caller copies to the device once per rebuild (it
 * changes only in ketama_update / modula_update). d_out[i] = server index.
 * dist: NC_GPUHASH_DIST_KETAMA or _MODULA (DIST_RANDOM is libc random(),
 * src/hashkit/nc_random.c:136-146, nondeterministic: EINVAL). nserver ==
 * array_n(&pool->server); 1 gives all zeros without hashing (:655-658).
 * hash_tag: NULL (none) or the pool's two tag bytes. shape: NULL or the
 * batch shape (it picks the slab size, as for nc_gpuhash_batch_device_shaped).
 * d_offsets must be 16-byte aligned (hipMalloc'd buffers are), else EINVAL. */
#define NC_GPUHASH_DIST_KETAMA 0 /* DIST_CODEC order, src/hashkit/nc_hashkit.h:38-41 */
#define NC_GPUHASH_DIST_MODULA 1
/* struct continuum, src/nc_server.h:64-67 (same layout) */
struct nc_gpuhash_continuum {
    uint32_t index;
    uint32_t value;
};
rstatus_t nc_gpuhash_server_idx_device(int mode, int dist, const uint8_t *d_keys,
                                       const uint64_t *d_offsets, uint64_t nkeys,
                                       const struct nc_gpuhash_continuum *d_continuum,
                                       uint32_t ncontinuum, uint32_t nserver, const char *hash_tag,
                                       const struct nc_gpuhash_shape *shape, uint32_t *d_out,
                                       void *stream);

/* ketama_update (src/hashkit/nc_ketama.c:58-219) building the continuum
 * straight into device memory for nc_gpuhash_server_idx_device: servers with
 * live[s] == 0 are skipped as ejected (NULL = all live); points per server
 * from the weights in the reference's float arithmetic (:159-160); 4 points
 * per "<name>-<i>" md5 digest (:169-181, ketama_hash :31-41); sorted by value,
 * ties in build order (:197-198). Writes *ncontinuum points (<= 160 x live
 * servers for equal weights) to d_continuum; NC_ENOMEM if more than cap. A
 * zero weight is EINVAL (the reference asserts weight > 0, :100). Blocks until
 * the build is done (a cold path: once per rebuild). */
rstatus_t nc_gpuhash_ketama_build_device(const char *const *names, const uint32_t *name_lens,
                                         const uint32_t *weights, const uint8_t *live, uint32_t nserver,
                                         struct nc_gpuhash_continuum *d_continuum, uint32_t cap,
                                         uint32_t *ncontinuum, void *stream);

/* ---- 3a''. key extraction on the device ----
 * A stream of pipelined memcache retrieval requests ("get k1 k2 ...\r\n",
 * "gets ...\r\n": memcache_parse_req, src/proto/nc_memcache.c:219-447,
 * :709-717) into the key CSR the batch entry points take. Every complete
 * request line is parsed in parallel; keys are produced for the requests
 * before the first one that is malformed (the reference would close the
 * connection there) or is not a retrieval command (its data block is not a
 * line: the host parser takes over from `consumed`). */
typedef struct nc_gpuhash_mc_parser nc_gpuhash_mc_parser_t;

#define NC_GPUHASH_MC_OK            0
#define NC_GPUHASH_MC_EINVAL       -1 /* syntax the reference rejects */
#define NC_GPUHASH_MC_EKEYLEN      -2 /* empty key or longer than 250 bytes (nc_memcache.c:33) */
#define NC_GPUHASH_MC_EUNSUPPORTED -3 /* a request type other than get / gets */

struct nc_gpuhash_mc_result {
    uint64_t nreqs;       /* complete ("...\r\n") request lines in the stream */
    uint64_t nkeys;       /* keys written (requests [0, first_error)) */
    uint64_t first_error; /* index of the first request not parsed here, or nreqs */
    uint64_t consumed;    /* stream bytes of requests [0, first_error) */
};

/* Device workspace for streams up to max_bytes (< 2^31), max_reqs complete
 * requests and max_keys keys. NULL with errno on failure. */
nc_gpuhash_mc_parser_t *nc_gpuhash_mc_parser_create(uint64_t max_bytes, uint64_t max_reqs, uint64_t max_keys);
void nc_gpuhash_mc_parser_destroy(nc_gpuhash_mc_parser_t *ps);

/* Parse d_stream[0, nbytes). Writes the packed keys (d_keys, NULL = spans
 * only; needs result->nkeys's bytes + NC_GPUHASH_PAD), d_offsets (nkeys + 1),
 * the request index of each key (d_key_req, may be NULL) and each request's
 * NC_GPUHASH_MC_* status (d_req_status, room for max_reqs entries, may be
 * NULL). Blocks until done (the counts size the next launch). NC_ENOMEM when
 * a limit of the workspace is exceeded (more complete request lines than
 * max_reqs, more keys than max_keys, or more than max_bytes), with nothing
 * written past those limits. */
rstatus_t nc_gpuhash_mc_parse_device(nc_gpuhash_mc_parser_t *ps, const uint8_t *d_stream, uint64_t nbytes,
                                     uint8_t *d_keys, uint64_t *d_offsets, uint32_t *d_key_req,
                                     int32_t *d_req_status, struct nc_gpuhash_mc_result *result,
                                     void *stream);

/* Key extraction on the device from pipelined redis (RESP) requests of the
 * command classes whose keys redis_parse_req pushes (arg0 / arg1 / argn / argx
 * / argkvx: src/proto/nc_redis.c:64-334, :460-1900; AUTH excluded). The
 * boundaries of binary-safe requests are found by a speculative parse from
 * every position after a CR LF, then the chain from byte 0 (pointer jumping).
 * Keys are produced for the requests before the first one that fails or is of
 * another command class; an incomplete last request is left for the next
 * read, as the reference leaves it in the mbuf. */
typedef struct nc_gpuhash_redis_parser nc_gpuhash_redis_parser_t;

#define NC_GPUHASH_REDIS_OK            0
#define NC_GPUHASH_REDIS_EINVAL       -1 /* syntax the reference rejects */
#define NC_GPUHASH_REDIS_EKEYLEN      -2 /* key length >= mbuf_data_size() (nc_redis.c:1369-1375) */
#define NC_GPUHASH_REDIS_EUNSUPPORTED -3 /* a command outside these classes: the host parser decides */

struct nc_gpuhash_redis_result {
    uint64_t nreqs;       /* requests parsed: the ok ones plus the failing one, if any */
    uint64_t nkeys;       /* keys written (requests [0, first_error)) */
    uint64_t first_error; /* index of the failing request, or nreqs */
    uint64_t consumed;    /* stream bytes of requests [0, first_error) */
};

/* Device workspace for streams up to max_bytes (< 2^31), max_reqs requests and
 * max_keys keys (each < 2^31). NULL with errno on failure. */
nc_gpuhash_redis_parser_t *nc_gpuhash_redis_parser_create(uint64_t max_bytes, uint64_t max_reqs, uint64_t max_keys);
void nc_gpuhash_redis_parser_destroy(nc_gpuhash_redis_parser_t *ps);

/* Parse d_stream[0, nbytes); max_key_len is mbuf_data_size() (keys must be
 * shorter). Outputs as nc_gpuhash_mc_parse_device, with NC_GPUHASH_REDIS_*
 * statuses; d_req_status holds max_reqs + 1 entries. A stream of max_reqs ok
 * requests followed by a byte that starts no request is accepted: nreqs then
 * counts the failing request (max_reqs + 1), first_error names it and its
 * status goes to d_req_status[max_reqs]. Blocks until done. */
rstatus_t nc_gpuhash_redis_parse_device(nc_gpuhash_redis_parser_t *ps, const uint8_t *d_stream, uint64_t nbytes,
                                        uint32_t max_key_len, uint8_t *d_keys, uint64_t *d_offsets,
                                        uint32_t *d_key_req, int32_t *d_req_status,
                                        struct nc_gpuhash_redis_result *result, void *stream);

/* ---- 3b. host batches through a context (pinned staging, one stream per slot) ---- */
typedef struct nc_gpuhash_ctx nc_gpuhash_ctx_t;

/* A borrowed key span inside an mbuf, the shape of struct keypos
 * (src/nc_message.h:232-235). */
struct nc_keyspan {
    const uint8_t *start;
    const uint8_t *end;
};

/* Create a context on `device` able to take batches of up to max_keys keys
 * and max_key_bytes key bytes, with `nslots` in-flight batches (>= 1). */
nc_gpuhash_ctx_t *nc_gpuhash_ctx_create(int device, uint64_t max_keys, uint64_t max_key_bytes,
                                        int nslots);
void nc_gpuhash_ctx_destroy(nc_gpuhash_ctx_t *ctx);

/* Batches with at most max_key_bytes key bytes run zero-copy: the kernel
 * reads the keys from the slot's mapped pinned staging across PCIe and writes
 * the hashes back the same way, so no H2D/D2H copy is enqueued (one launch
 * instead of three operations). 0 = always copy. The default is 1 MiB
 * (environment NC_GPUHASH_ZERO_COPY=<bytes> overrides it at ctx_create). */
rstatus_t nc_gpuhash_ctx_set_zero_copy(nc_gpuhash_ctx_t *ctx, uint64_t max_key_bytes);

/* Pack a CSR batch into a free slot's pinned staging, enqueue H2D, kernel and
 * D2H, and return a ticket without blocking. NC_EAGAIN if every slot is busy,
 * NC_ENOMEM if the batch exceeds the context's limits. The caller may reuse
 * keys/offsets as soon as this returns (they are copied, as mbufs are
 * recycled after msg_put, src/nc_mbuf.c:118-128). */
rstatus_t nc_gpuhash_submit(nc_gpuhash_ctx_t *ctx, int mode, const uint8_t *keys,
                            const uint64_t *offsets, uint32_t nkeys, uint32_t *out, int *ticket);
/* The same from keypos-style spans (the fragment loops,
 * src/proto/nc_memcache.c:1324-1345, src/proto/nc_redis.c:2862-2901). */
rstatus_t nc_gpuhash_submit_spans(nc_gpuhash_ctx_t *ctx, int mode, const struct nc_keyspan *spans,
                                  uint32_t nkeys, uint32_t *out, int *ticket);
/* NC_OK once the ticket's hashes are in its `out`, NC_EAGAIN while pending. */
rstatus_t nc_gpuhash_poll(nc_gpuhash_ctx_t *ctx, int ticket);
/* Block until the ticket completes. */
rstatus_t nc_gpuhash_wait(nc_gpuhash_ctx_t *ctx, int ticket);

/* One synchronous host batch on a process-wide context (device 0), the
 * SURVEY.md §8b.2 shape. */
rstatus_t nc_hashkit_batch(int mode, const uint8_t *keys, const uint64_t *offsets,
                           uint32_t nkeys, uint32_t *out);

/* ---- 3c. whole host batches from caller-pinned memory (no repack) ----
 * The large-batch host path (SURVEY.md §8d end to end: host CSR (pinned) ->
 * hipMemcpyAsync H2D -> kernel -> D2H). The caller's CSR is used where it
 * lies: memory from hipHostMalloc, or registered once with
 * nc_gpuhash_host_register (a proxy pins its mbuf arena). A pipe holds
 * `depth` device chunk buffers and three streams (H2D, kernel, D2H): chunk
 * i+1's keys and offsets go up while chunk i hashes and chunk i-1's hashes
 * come back. Chunks are contiguous key ranges of at most chunk_keys keys and
 * chunk_bytes key bytes. */
typedef struct nc_gpuhash_pipe nc_gpuhash_pipe_t;

nc_gpuhash_pipe_t *nc_gpuhash_pipe_create(int device, uint64_t chunk_keys, uint64_t chunk_bytes, int depth);
void nc_gpuhash_pipe_destroy(nc_gpuhash_pipe_t *p);

/* Hash keys [0, nkeys) of a pinned host CSR into the pinned `out`; blocks
 * until every hash is in `out`. keys must be readable NC_GPUHASH_PAD bytes
 * past offsets[nkeys] (the device contract); shape may be NULL. A key longer
 * than chunk_bytes is NC_ENOMEM. Not thread-safe per pipe (one batch at a
 * time; use a pipe per thread). flags: 0 (reserved). */
rstatus_t nc_gpuhash_batch_pinned(nc_gpuhash_pipe_t *p, int mode, const uint8_t *keys, const uint64_t *offsets,
                                  uint64_t nkeys, uint32_t *out, const struct nc_gpuhash_shape *shape,
                                  int flags);

/* Page-lock (and map) an existing host range for the pinned path
 * (hipHostRegister), and undo it. */
rstatus_t nc_gpuhash_host_register(void *ptr, size_t bytes);
rstatus_t nc_gpuhash_host_unregister(void *ptr);

/* ---- 3d. small batches with no HIP call per batch: the batch ring ----
 * One mbuf's keys at a time (the batch site of src/nc_message.c:700-714 and
 * the fragment loops) without a kernel launch or an event per batch: the
 * ring's slots live in mapped, coherent host memory — a ring of 1 or 2 lanes
 * on a large-BAR device stages its batches in device memory the host writes
 * through the BAR instead (NC_GPUHASH_RING_STAGING=host|device at create
 * overrides) — and ONE resident launch
 * polls them (csrc/nc_ring.hip), one workgroup per lane: batch n belongs to
 * lane n % nlanes, each lane takes its batches in order, and the lanes'
 * PCIe round trips overlap. A submit copies the spans' bytes into the slot
 * (the mbufs may be recycled on return) and publishes it with one store; the
 * lane's worker hashes it and writes the hashes and a completion word back
 * to host memory; poll is one load. The launch starts on the first batch,
 * ends after 10 ms with no batch on any lane or after 2 s (checked after
 * every batch and honoured before the next one is taken, under load too),
 * and is relaunched by the next submit or
 * poll: a batch published while the launch ends is served on a later poll,
 * so poll (or wait) every ticket. Up to nslots batches in flight; lanes may
 * finish out of order. A live launch holds nlanes workgroup slots (one lane's
 * LDS holds its batch image) while it polls, which batch kernels on the same
 * GPU then run without. Limits per batch: max_keys <= 4095 keys,
 * max_key_bytes <= 32768 bytes (two mbufs' worth). NULL with errno on failure
 * (EINVAL limits, ENODEV no GPU). Thread-safe per ring (one mutex). */
#define NC_GPUHASH_RING_MAX_LANES 8
#define NC_GPUHASH_RING_DEFAULT_LANES 8    /* capped at nslots */
#define NC_GPUHASH_RING_DEFAULT_THREADS 1024
typedef struct nc_gpuhash_ring nc_gpuhash_ring_t;
/* nlanes = min(NC_GPUHASH_RING_DEFAULT_LANES, nslots) */
nc_gpuhash_ring_t *nc_gpuhash_ring_create(int device, uint32_t nslots, uint32_t max_keys, uint64_t max_key_bytes);
/* nlanes 1..NC_GPUHASH_RING_MAX_LANES (capped at nslots; 0 = default);
 * threads per lane's workgroup 256, 512 or 1024 (0 = default) */
nc_gpuhash_ring_t *nc_gpuhash_ring_create_ex(int device, uint32_t nslots, uint32_t max_keys, uint64_t max_key_bytes,
                                             uint32_t nlanes, uint32_t threads);
/* stops the workers (they return at their next poll) and frees the ring */
void nc_gpuhash_ring_destroy(nc_gpuhash_ring_t *r);
/* submit keypos-style spans; NC_EAGAIN when the next slot's batch is still in
 * flight, NC_ENOMEM past the limits, NC_ERROR/EINVAL for a NULL or inverted
 * span (end < start); *ticket (0 .. 2^31-1) identifies the batch among the
 * last 2^31 submitted */
rstatus_t nc_gpuhash_ring_submit_spans(nc_gpuhash_ring_t *r, int mode, const struct nc_keyspan *spans,
                                       uint32_t nkeys, uint32_t *out, int *ticket);
/* NC_OK once the batch's hashes are in its `out`, NC_EAGAIN before, and
 * NC_ERROR/EINVAL for a ticket this ring never issued. Lifetime: the ring
 * keeps `out` until the batch is delivered — by this poll, or by the submit
 * that reuses its slot — so `out` must stay valid until then, or be released
 * with nc_gpuhash_ring_forget first. */
rstatus_t nc_gpuhash_ring_poll(nc_gpuhash_ring_t *r, int ticket);
rstatus_t nc_gpuhash_ring_wait(nc_gpuhash_ring_t *r, int ticket);
/* the ticket's owner is going away (a client connection closed and freed
 * its msg, src/nc_message.c:372-396): the batch still runs, but its hashes
 * are never copied into its `out`, which may be freed on return. NC_OK
 * (also for a ticket already delivered), NC_ERROR/EINVAL for a ticket this
 * ring never issued */
rstatus_t nc_gpuhash_ring_forget(nc_gpuhash_ring_t *r, int ticket);
/* launches so far (the first submit's, and relaunches after idle or 2 s) */
uint64_t nc_gpuhash_ring_launches(const nc_gpuhash_ring_t *r);
/* the ring's lane count */
uint32_t nc_gpuhash_ring_lanes(const nc_gpuhash_ring_t *r);
/* the ring's per-batch limits and slot count, as created (any pointer may be
 * NULL); NC_ERROR/EINVAL for a NULL ring */
rstatus_t nc_gpuhash_ring_limits(const nc_gpuhash_ring_t *r, uint32_t *max_keys, uint64_t *max_key_bytes,
                                 uint32_t *nslots);

/* ---- 4. multi-GPU shard planning ----
 * Split keys [0, nkeys) into nshards contiguous ranges with about equal key
 * bytes: key_bounds[g] .. key_bounds[g+1] is shard g (nshards + 1 entries). */
rstatus_t nc_gpuhash_shard_bounds(const uint64_t *offsets, uint64_t nkeys, uint32_t nshards,
                                  uint64_t *key_bounds);

/* ---- 5. fragment plan (the batch sites' second half) ----
 * What memcache_fragment_retrieval (src/proto/nc_memcache.c:1283-1370) and
 * redis_fragment_argx (src/proto/nc_redis.c:2804-2898) make of ONE
 * multi-key request once its keys' server indices are known (batched:
 * nc_gpuhash_server_idx_device over the request's keys; the reference calls
 * msg_backend_idx per key, src/nc_message.c:461-467): one fragment per
 * distinct server, fragments in ascending server order (the reference walks
 * sub_msgs[0 .. nserver)), keys in request order inside each. For keys
 * 0 .. nkeys-1 with server indices sidx[]: frag_seq[i] = key i's fragment
 * (the position of r->frag_seq[i] in the fragment queue), frag_server[f] =
 * fragment f's server, frag_nkeys[f] = its key count; the frag_* arrays hold
 * min(nkeys, nserver) entries. The reference does not fragment a one-key
 * request (memcache_should_fragment, src/proto/nc_memcache.c:104-118;
 * redis_fragment, src/proto/nc_redis.c:2903): that stays the caller's test.
 * Returns the number of fragments (0 for no keys), or -1 with errno EINVAL
 * (NULL buffers, nserver 0, a server index >= nserver). Host code, no GPU. */
int nc_gpuhash_frag_plan(const uint32_t *sidx, uint32_t nkeys, uint32_t nserver, uint32_t *frag_seq,
                         uint32_t *frag_server, uint32_t *frag_nkeys);

/* ---- info ---- */
/* Number of visible GPUs (0 when none); never initialises more than HIP's
 * device query does. */
int nc_gpuhash_device_count(void);
/* Library version string. */
const char *nc_gpuhash_version(void);

#ifdef __cplusplus
}
#endif

#endif /* NC_GPUHASH_H */
