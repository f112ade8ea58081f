/*
 * The batch sites of a twemproxy built with libnc_gpuhash: see
 * nc_batch_site.h and INTEGRATION.md §2. Each function cites the reference
 * code it replaces or keeps. Hashing is the ring's, except a key longer than
 * one ring batch holds, which takes pool->key_hash (the library's per-key
 * symbol) exactly as server_pool_hash does today.
 */
#include "nc_batch_site.h"

#include <nc_hashkit.h>

uint32_t
server_pool_idx_of_hash(const struct server_pool *pool, uint32_t hash)
{
    if (array_n(&pool->server) == 1) {
        return 0; /* src/nc_server.c:655-658 */
    }

    switch (pool->dist_type) { /* src/nc_server.c:679-697 */
    case DIST_KETAMA:
        return ketama_dispatch(pool->continuum, pool->ncontinuum, hash);

    case DIST_MODULA:
        return modula_dispatch(pool->continuum, pool->ncontinuum, hash);

    case DIST_RANDOM:
        return random_dispatch(pool->continuum, pool->ncontinuum, 0);

    default:
        NOT_REACHED();
        return 0;
    }
}

void
server_pool_hash_span(const struct server_pool *pool, const uint8_t *key, uint32_t keylen, struct nc_keyspan *span)
{
    if (!string_empty(&pool->hash_tag)) { /* src/nc_server.c:665-677 */
        const struct string *tag = &pool->hash_tag;
        const uint8_t *tag_start, *tag_end;

        tag_start = nc_strchr(key, key + keylen, tag->data[0]);
        if (tag_start != NULL) {
            tag_end = nc_strchr(tag_start + 1, key + keylen, tag->data[1]);
            if ((tag_end != NULL) && (tag_end - tag_start > 1)) {
                key = tag_start + 1;
                keylen = (uint32_t)(tag_end - key);
            }
        }
    }
    span->start = key;
    span->end = key + keylen;
}

/* ---- the hashes of n spans in ring batches ---- */

static uint64_t
span_len(const struct nc_keyspan *s)
{
    return (uint64_t)(s->end - s->start);
}

/* submit batches of keys [next, ...) while a ring slot and an in-flight
 * entry are free; keys too long for any batch are hashed per key */
static rstatus_t
msg_hashes_pump(struct msg_hashes *h)
{
    while (h->next < h->n && h->count < NC_BATCH_SITE_INFLIGHT) {
        uint32_t first = h->next, end = first;
        uint64_t bytes = 0;
        rstatus_t status;
        int ticket;

        if (span_len(&h->span[first]) > h->max_bytes) {
            /* server_pool_hash's own call (src/nc_server.c:643) */
            h->hashes[first] = h->pool->key_hash((const char *)h->span[first].start,
                                                 (size_t)span_len(&h->span[first]));
            h->host_keys++;
            h->next++;
            continue;
        }
        while (end < h->n && end - first < h->max_keys && bytes + span_len(&h->span[end]) <= h->max_bytes) {
            bytes += span_len(&h->span[end]);
            end++;
        }
        status = nc_gpuhash_ring_submit_spans(h->ring, h->pool->key_hash_type, h->span + first, end - first,
                                              h->hashes + first, &ticket);
        if (status == NC_EAGAIN) {
            return NC_OK; /* every ring slot busy: submitted on a later poll */
        }
        if (status != NC_OK) {
            return status;
        }
        h->ticket[(h->head + h->count) % NC_BATCH_SITE_INFLIGHT] = ticket;
        h->count++;
        h->batches++;
        h->next = end;
    }
    return NC_OK;
}

rstatus_t
msg_hashes_start(struct msg_hashes *h, const struct server_pool *pool, nc_gpuhash_ring_t *ring,
                 const struct nc_keyspan *span, uint32_t *hashes, uint32_t n)
{
    uint32_t i, nslots;

    memset(h, 0, sizeof(*h));
    h->ring = ring;
    h->pool = pool;
    h->span = span;
    h->hashes = hashes;
    if (array_n(&pool->server) == 1 || pool->dist_type == DIST_RANDOM) {
        /* no hash is needed: one server (src/nc_server.c:655-658), or random
         * dispatch, which ignores it (:692-694) */
        for (i = 0; i < n; i++) {
            hashes[i] = 0;
        }
        return NC_OK;
    }
    if (nc_gpuhash_ring_limits(ring, &h->max_keys, &h->max_bytes, &nslots) != NC_OK) {
        return NC_ERROR;
    }
    h->n = n;
    return msg_hashes_pump(h);
}

rstatus_t
msg_hashes_poll(struct msg_hashes *h)
{
    rstatus_t status;
    uint32_t i;

    while (h->count > 0) { /* in submit order */
        status = nc_gpuhash_ring_poll(h->ring, h->ticket[h->head]);
        if (status != NC_OK) {
            return status; /* NC_EAGAIN: not yet */
        }
        h->head = (h->head + 1) % NC_BATCH_SITE_INFLIGHT;
        h->count--;
    }
    status = msg_hashes_pump(h);
    if (status != NC_OK) {
        return status;
    }
    if (h->next < h->n || h->count > 0) {
        return NC_EAGAIN;
    }
    for (i = 0; i < h->n; i++) {
        if (h->span[i].end == h->span[i].start) {
            h->hashes[i] = 0; /* server_pool_hash: keylen 0 (src/nc_server.c:639-641) */
        }
    }
    return NC_OK;
}

void
msg_hashes_forget(struct msg_hashes *h)
{
    while (h->count > 0) {
        (void)nc_gpuhash_ring_forget(h->ring, h->ticket[h->head]);
        h->head = (h->head + 1) % NC_BATCH_SITE_INFLIGHT;
        h->count--;
    }
    h->next = h->n;
}

/* ---- multi-key requests ---- */

rstatus_t
msg_backend_hashes_submit(struct msg *r, nc_gpuhash_ring_t *ring, struct msg_hashes *h, struct nc_keyspan *span,
                          uint32_t *hashes)
{
    const struct server_pool *pool = ((const struct conn *)r->owner)->owner;
    uint32_t i, n = array_n(r->keys);

    for (i = 0; i < n; i++) {
        const struct keypos *kp = array_get(r->keys, i);

        server_pool_hash_span(pool, kp->start, (uint32_t)(kp->end - kp->start), &span[i]);
    }
    return msg_hashes_start(h, pool, ring, span, hashes, n);
}

rstatus_t
msg_backend_hashes_poll(struct msg *r, struct msg_hashes *h)
{
    (void)r;
    return msg_hashes_poll(h);
}

void
msg_backend_hashes_forget(struct msg *r, struct msg_hashes *h)
{
    (void)r;
    msg_hashes_forget(h);
}

void
msg_backend_idx_batch(const struct msg *r, const uint32_t *hashes, uint32_t *idx)
{
    const struct server_pool *pool = ((const struct conn *)r->owner)->owner;
    uint32_t i, n = array_n(r->keys);

    for (i = 0; i < n; i++) {
        idx[i] = server_pool_idx_of_hash(pool, hashes[i]);
    }
}

/* ---- pipelined single-key requests ---- */

rstatus_t
read_batch_init(struct read_batch *rb, const struct server_pool *pool, nc_gpuhash_ring_t *ring, uint32_t cap)
{
    memset(rb, 0, sizeof(*rb));
    rb->pool = pool;
    rb->ring = ring;
    rb->cap = cap;
    rb->msg = nc_alloc(cap * sizeof(*rb->msg));
    rb->slot = nc_alloc(cap * sizeof(*rb->slot));
    rb->span = nc_alloc(cap * sizeof(*rb->span));
    rb->hashes = nc_alloc(cap * sizeof(*rb->hashes));
    if (rb->msg == NULL || rb->slot == NULL || rb->span == NULL || rb->hashes == NULL) {
        read_batch_deinit(rb);
        return NC_ENOMEM;
    }
    return NC_OK;
}

void
read_batch_deinit(struct read_batch *rb)
{
    if (rb->submitted) {
        msg_hashes_forget(&rb->h);
    }
    nc_free(rb->msg);
    nc_free(rb->slot);
    nc_free(rb->span);
    nc_free(rb->hashes);
    rb->msg = NULL;
    rb->slot = NULL;
    rb->span = NULL;
    rb->hashes = NULL;
    rb->n = rb->cap = 0;
}

rstatus_t
read_batch_defer(struct read_batch *rb, struct msg *msg, int single)
{
    if (rb->submitted || rb->n == rb->cap) {
        return NC_ENOMEM;
    }
    rb->msg[rb->n] = msg;
    rb->slot[rb->n] = UINT32_MAX;
    if (single) {
        /* the key req_forward routes by (src/nc_request.c:572-576) */
        const struct keypos *kp = array_get(msg->keys, 0);

        server_pool_hash_span(rb->pool, kp->start, (uint32_t)(kp->end - kp->start), &rb->span[rb->nsingle]);
        rb->slot[rb->n] = rb->nsingle++;
    }
    rb->n++;
    return NC_OK;
}

rstatus_t
read_batch_submit(struct read_batch *rb)
{
    rstatus_t status;

    if (rb->submitted) {
        return NC_OK;
    }
    status = msg_hashes_start(&rb->h, rb->pool, rb->ring, rb->span, rb->hashes, rb->nsingle);
    if (status == NC_OK) {
        rb->submitted = 1;
    }
    return status;
}

rstatus_t
read_batch_poll(struct read_batch *rb)
{
    if (!rb->submitted) {
        return rb->nsingle == 0 ? NC_OK : NC_EAGAIN;
    }
    return msg_hashes_poll(&rb->h);
}

int
read_batch_server_idx(const struct read_batch *rb, uint32_t i, struct msg **msg, uint32_t *idx)
{
    *msg = rb->msg[i];
    if (rb->slot[i] == UINT32_MAX) {
        return 0;
    }
    *idx = server_pool_idx_of_hash(rb->pool, rb->hashes[rb->slot[i]]);
    return 1;
}

void
read_batch_reset(struct read_batch *rb)
{
    rb->n = rb->nsingle = 0;
    rb->submitted = 0;
}

void
read_batch_forget(struct read_batch *rb)
{
    if (rb->submitted) {
        msg_hashes_forget(&rb->h);
    }
    read_batch_reset(rb);
}
