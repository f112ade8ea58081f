/*
 * The batch site of a twemproxy built with libnc_gpuhash:
 * what a maintainer adds beside src/nc_server.c so that the fragment loops
 * (src/proto/nc_memcache.c:1323-1344, src/proto/nc_redis.c:2862-2901) get the
 * server index of every key of a multi-key request from ONE batch instead of
 * one server_pool_idx() call per key. Compiled against the reference's own
 * headers (nc_core.h, nc_server.h, nc_message.h); oracle/Makefile target
 * `batch-site` builds it the way the reference builds its objects.
 *
 * The split follows server_pool_idx (src/nc_server.c:647-700):
 *   host, before the batch: the one-server shortcut (:655-658) and the
 *     hash_tag trim (:665-677) -> one span per key;
 *   device, the batch: pool->key_hash of every span (the batch ring,
 *     nc_gpuhash_ring_*: no HIP call per batch);
 *   host, after it: the empty-key rule of server_pool_hash (:639-641) and the
 *     distribution step (:679-697).
 * Submit and poll are separate so the event loop never blocks (src/nc.c:
 * 525-531): keep the ticket in the msg, return to core_loop, poll on the next
 * turn, and resume the fragment step once the poll says NC_OK.
 */
#ifndef NC_BATCH_SITE_H
#define NC_BATCH_SITE_H

#include <nc_core.h>
#include <nc_server.h>
#include <nc_message.h>

#include <nc_gpuhash.h>

/* the distribution step of server_pool_idx for an already computed hash
 * (src/nc_server.c:679-697); a one-server pool is 0 */
uint32_t server_pool_idx_of_hash(const struct server_pool *pool, uint32_t hash);

/* the span server_pool_idx hashes for key [key, key + keylen): the whole key,
 * or the part inside the pool's hash_tag (src/nc_server.c:665-677) */
void server_pool_hash_span(const struct server_pool *pool, const uint8_t *key, uint32_t keylen,
                           struct nc_keyspan *span);

/* submit the keys of r (array_n(r->keys) keypos spans, src/nc_message.h:232-
 * 235) as one ring batch: span[] (caller's, array_n(r->keys) entries) gets
 * the trimmed spans, hashes[] the hashes once msg_backend_hashes_poll says
 * NC_OK. *ticket = -1 when no batch is needed (a one-server pool: every index
 * is 0). NC_EAGAIN: every ring slot is busy (poll an older ticket, retry). */
rstatus_t msg_backend_hashes_submit(struct msg *r, nc_gpuhash_ring_t *ring, struct nc_keyspan *span,
                                    uint32_t *hashes, int *ticket);

/* NC_OK once hashes[] holds the batch's hashes (with server_pool_hash's 0 for
 * a key that is empty after the trim), NC_EAGAIN before */
rstatus_t msg_backend_hashes_poll(struct msg *r, nc_gpuhash_ring_t *ring, const struct nc_keyspan *span,
                                  uint32_t *hashes, int ticket);

/* idx[i] = msg_backend_idx(r, key i) from the batch's hashes: the value the
 * fragment loop's per-key call returns (src/nc_message.c:461-467) */
void msg_backend_idx_batch(const struct msg *r, const uint32_t *hashes, uint32_t *idx);

#endif
