/*
 * The batch site of a twemproxy built with libnc_gpuhash: see nc_batch_site.h
 * and INTEGRATION.md §2. Each function cites the reference code it replaces
 * or keeps; none of it hashes on the host.
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

rstatus_t
msg_backend_hashes_submit(struct msg *r, nc_gpuhash_ring_t *ring, struct nc_keyspan *span, uint32_t *hashes,
                          int *ticket)
{
    const struct server_pool *pool = ((const struct conn *)r->owner)->owner;
    uint32_t i, n = array_n(r->keys);

    if (array_n(&pool->server) == 1 || pool->dist_type == DIST_RANDOM) {
        /* no hash is needed: one server (src/nc_server.c:655-658), or random
         * dispatch, which ignores it (:692-694) */
        for (i = 0; i < n; i++) {
            hashes[i] = 0;
        }
        *ticket = -1;
        return NC_OK;
    }
    for (i = 0; i < n; i++) {
        const struct keypos *kp = array_get(r->keys, i);

        server_pool_hash_span(pool, kp->start, (uint32_t)(kp->end - kp->start), &span[i]);
    }
    return nc_gpuhash_ring_submit_spans(ring, pool->key_hash_type, span, n, hashes, ticket);
}

rstatus_t
msg_backend_hashes_poll(struct msg *r, nc_gpuhash_ring_t *ring, const struct nc_keyspan *span, uint32_t *hashes,
                        int ticket)
{
    uint32_t i, n = array_n(r->keys);
    rstatus_t status;

    if (ticket < 0) {
        return NC_OK;
    }
    status = nc_gpuhash_ring_poll(ring, ticket);
    if (status != NC_OK) {
        return status;
    }
    for (i = 0; i < n; i++) {
        if (span[i].end == span[i].start) {
            hashes[i] = 0; /* server_pool_hash: keylen 0 (src/nc_server.c:639-641) */
        }
    }
    return NC_OK;
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
