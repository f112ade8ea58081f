/*
 * The batch sites of a twemproxy built with libnc_gpuhash (INTEGRATION.md
 * §2): what a maintainer adds beside src/nc_server.c so that request keys get
 * their server index from ring batches instead of one server_pool_idx() call
 * per key. Compiled against the reference's own headers (nc_core.h,
 * nc_server.h, nc_message.h); oracle/Makefile target `batch-site` builds it
 * the way the reference builds its objects. Two sites:
 *
 *   multi-key requests: the fragment loops (src/proto/nc_memcache.c:
 *     1323-1344, src/proto/nc_redis.c:2862-2901) take every key's index from
 *     the msg's batch (msg_backend_hashes_*);
 *   pipelined single-key requests: the read loop of msg_recv_chain
 *     (src/nc_message.c:699-713) hands each parsed request to req_recv_done
 *     (src/nc_request.c:627-700), which forwards it at once (req_forward,
 *     :556, picking the server at :576 by server_pool_conn). Here
 *     req_recv_done DEFERS the forward into the connection's read batch
 *     (read_batch_defer), the end of the read submits one ring batch for
 *     the read (read_batch_submit), and the event loop's next turn forwards
 *     the read's requests in order once the batch is done (read_batch_poll,
 *     read_batch_server_idx).
 *
 * The split follows server_pool_idx (src/nc_server.c:647-700):
 *   host, before the batch: the one-server shortcut (:655-658) and the
 *     hash_tag trim (:665-677) -> one span per key;
 *   device, the batch: pool->key_hash of every span (the batch ring,
 *     nc_gpuhash_ring_*: no HIP call per batch);
 *   host, after it: the empty-key rule of server_pool_hash (:639-641) and the
 *     distribution step (:679-697).
 * Submit and poll are separate so the event loop never blocks (src/nc.c:
 * 525-531): keep the state in the msg (or the connection), return to
 * core_loop, poll on the next turn, resume once the poll says NC_OK.
 *
 * Limits: a ring batch holds at most the ring's max_keys keys and
 * max_key_bytes key bytes (nc_gpuhash_ring_limits). A request with more is
 * cut into several ring batches, up to NC_BATCH_SITE_INFLIGHT in flight at
 * once and the rest submitted as earlier ones finish (on later polls); a
 * single key longer than max_key_bytes (a redis key may be up to 512 MB) is
 * hashed by pool->key_hash — the library's link-compatible per-key symbol,
 * what server_pool_hash calls today — when its turn comes.
 *
 * Lifetime: the ring writes a batch's hashes into the caller's `hashes`
 * array when the batch is reaped, which may happen during a later submit of
 * another msg. A msg (or connection) torn down while its batches are in
 * flight (a client closing, src/nc_message.c:372-396) must call
 * msg_backend_hashes_forget / read_batch_forget first; the arrays may then be
 * freed.
 */
#ifndef NC_BATCH_SITE_H
#define NC_BATCH_SITE_H

#include <nc_core.h>
#include <nc_server.h>
#include <nc_message.h>

#include <nc_gpuhash.h>

/* ring batches of one msg (or one read) in flight at once */
#define NC_BATCH_SITE_INFLIGHT 4

/* the distribution step of server_pool_idx for an already computed hash
 * (src/nc_server.c:679-697); a one-server pool is 0 */
uint32_t server_pool_idx_of_hash(const struct server_pool *pool, uint32_t hash);

/* the span server_pool_idx hashes for key [key, key + keylen): the whole key,
 * or the part inside the pool's hash_tag (src/nc_server.c:665-677) */
void server_pool_hash_span(const struct server_pool *pool, const uint8_t *key, uint32_t keylen,
                           struct nc_keyspan *span);

/* the hashes of n spans, computed in ring batches (see Limits above): state
 * the caller keeps (in the msg) between submit and the poll that says NC_OK */
struct msg_hashes {
    nc_gpuhash_ring_t          *ring;
    const struct server_pool   *pool;
    const struct nc_keyspan    *span;
    uint32_t                   *hashes;
    uint32_t                   n;         /* keys */
    uint32_t                   next;      /* first key not yet submitted or hashed */
    uint32_t                   max_keys;  /* ring limits per batch */
    uint64_t                   max_bytes;
    uint32_t                   head, count; /* FIFO of batches in flight */
    int                        ticket[NC_BATCH_SITE_INFLIGHT];
    uint32_t                   batches;   /* ring batches submitted so far */
    uint32_t                   host_keys; /* keys longer than a batch holds, hashed by pool->key_hash */
};

/* start hashing span[0, n) for pool into hashes[0, n) (both caller-owned,
 * alive until the poll says NC_OK or msg_hashes_forget). A one-server or
 * random-dispatch pool needs no hash: hashes are 0 and the first poll says
 * NC_OK. NC_OK (started; some batches may wait for a free ring slot), or
 * NC_ERROR/NC_ENOMEM from the ring. */
rstatus_t msg_hashes_start(struct msg_hashes *h, const struct server_pool *pool, nc_gpuhash_ring_t *ring,
                           const struct nc_keyspan *span, uint32_t *hashes, uint32_t n);
/* NC_OK once every hash is in hashes[] (0 for a key that is empty after the
 * trim, server_pool_hash :639-641), NC_EAGAIN before; submits the batches
 * that were waiting for a ring slot */
rstatus_t msg_hashes_poll(struct msg_hashes *h);
/* the owner is going away: no batch in flight writes into hashes[] any more */
void msg_hashes_forget(struct msg_hashes *h);

/* ---- multi-key requests (the fragment loops) ---- */

/* submit the keys of r (array_n(r->keys) keypos spans, src/nc_message.h:232-
 * 235): span[] (caller's, array_n(r->keys) entries) gets the trimmed spans,
 * hashes[] the hashes once msg_backend_hashes_poll says NC_OK */
rstatus_t msg_backend_hashes_submit(struct msg *r, nc_gpuhash_ring_t *ring, struct msg_hashes *h,
                                    struct nc_keyspan *span, uint32_t *hashes);
rstatus_t msg_backend_hashes_poll(struct msg *r, struct msg_hashes *h);
void msg_backend_hashes_forget(struct msg *r, struct msg_hashes *h);

/* idx[i] = msg_backend_idx(r, key i) from the batch's hashes: the value the
 * fragment loop's per-key call returns (src/nc_message.c:461-467) */
void msg_backend_idx_batch(const struct msg *r, const uint32_t *hashes, uint32_t *idx);

/* ---- pipelined single-key requests (one read's forwards) ---- */

/* one read's requests of one client connection, in parse order. A request
 * that req_recv_done would forward by key 0 (no fragments, not noforward)
 * is `single`: its server comes from the read's batch. Every other request
 * parsed after the first deferred one is deferred too (single = 0) and
 * takes its unchanged path at flush time, so the client's outq order
 * (req_forward's enqueue_outq, src/nc_request.c:567-569) stays the parse
 * order. */
struct read_batch {
    const struct server_pool   *pool;
    nc_gpuhash_ring_t          *ring;
    uint32_t                   n, cap;    /* requests deferred; capacity */
    uint32_t                   nsingle;   /* of which single */
    struct msg                 **msg;     /* [cap] */
    uint32_t                   *slot;     /* [cap]: index into span/hashes, or UINT32_MAX (not single) */
    struct nc_keyspan          *span;     /* [cap]: key 0 of each single request, trimmed */
    uint32_t                   *hashes;   /* [cap] */
    struct msg_hashes          h;
    int                        submitted;
};

rstatus_t read_batch_init(struct read_batch *rb, const struct server_pool *pool, nc_gpuhash_ring_t *ring,
                          uint32_t cap);
void read_batch_deinit(struct read_batch *rb);
/* defer msg's forward (after req_filter, as req_forward would run next):
 * NC_ENOMEM when the batch is full or already submitted (submit, poll and
 * flush it first) */
rstatus_t read_batch_defer(struct read_batch *rb, struct msg *msg, int single);
/* end of the read: one ring batch (or several, Limits) for the read's
 * single requests */
rstatus_t read_batch_submit(struct read_batch *rb);
/* NC_OK once every single request's server is known, NC_EAGAIN before */
rstatus_t read_batch_poll(struct read_batch *rb);
/* request i of the read (i < rb->n, in parse order) and, when single, its
 * server index (server_pool_idx of its key 0); returns single */
int read_batch_server_idx(const struct read_batch *rb, uint32_t i, struct msg **msg, uint32_t *idx);
/* after the flush: empty for the connection's next read */
void read_batch_reset(struct read_batch *rb);
/* the connection closes with the batch in flight (see Lifetime) */
void read_batch_forget(struct read_batch *rb);

#endif
