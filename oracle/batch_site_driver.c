/*
 * ORACLE — TEST INFRASTRUCTURE ONLY: the batch site of INTEGRATION.md §2,
 * executed.
 *
 * Built by oracle/Makefile target `batch-site` into _ref/libbatch_site.so:
 * the reference's request parsers, message / mbuf / server code and
 * ketama / modula / random dispatch, compiled where they lie under
 * /root/reference (the set ref_proto_driver.c drives), the maintainer's
 * integration/nc_batch_site.c, and this driver — with NO reference hash
 * algorithm object: every hash_<name> and md5_signature resolves to
 * twemproxy_amd/libnc_gpuhash.so (as in `link-compat`).
 *
 * bs_request parses one multi-key request with the reference's own parser
 * into a struct msg owned by a client connection of a pool that the
 * reference's ketama_update / modula_update built, then computes every key's
 * server index twice:
 *   - the reference's way: msg_backend_idx per key (src/nc_message.c:461-467,
 *     the call the fragment loops make, src/proto/nc_memcache.c:1326,
 *     src/proto/nc_redis.c:2876), on the library's per-key symbols;
 *   - the batch site's way: msg_backend_hashes_submit on the batch ring, poll
 *     until done (the event loop's resume), msg_backend_idx_batch.
 * tests/test_gpu_batch_site.py checks both against the indices the pure
 * reference build's fragment loops produced (tests/golden/proto_ref.json
 * "fragments").
 */
#include "ref_proto_driver.c"

#include <time.h>

#include "../integration/nc_batch_site.h"

/* Returns the number of keys (ref_idx / batch_idx filled), -1 for a parse or
 * set-up failure, -2 when the ring refused the batch (every slot busy), -3
 * when the ring never finished it, -4 for a ring error. *polls counts the
 * NC_EAGAIN polls before the batch was done. */
int bs_request(int redis, const uint8_t *buf, uint32_t len, int mode, int dist, const char *const *names,
               const uint32_t *name_lens, const uint32_t *weights, uint32_t nserver, const uint8_t *tag,
               uint32_t taglen, nc_gpuhash_ring_t *ring, uint32_t *ref_idx, uint32_t *batch_idx, uint32_t kcap,
               uint32_t *polls)
{
    struct server_pool pool;
    struct conn fake_client;
    if (!rp_ready || len > mbuf_data_size()) return -1;
    if (rp_pool_init(&pool, mode, dist, names, name_lens, weights, nserver, tag, taglen) != 0) return -1;
    memset(&fake_client, 0, sizeof(fake_client));
    fake_client.owner = &pool;
    fake_client.redis = redis ? 1 : 0;
    int rc = -1;
    struct mbuf *m = mbuf_get();
    struct msg *req = m ? msg_get(&fake_client, 1, redis ? 1 : 0) : NULL;
    if (req == NULL) {
        if (m) mbuf_put(m);
        rp_pool_deinit(&pool);
        return -1;
    }
    req->state = 0;
    req->token = NULL;
    mbuf_copy(m, buf, len);
    STAILQ_INIT(&req->mhdr);
    mbuf_insert(&req->mhdr, m);
    req->pos = m->start;
    req->parser(req);
    const uint32_t nk = array_n(req->keys);
    struct nc_keyspan *span = malloc((nk + 1) * sizeof(*span));
    uint32_t *hashes = malloc((nk + 1) * sizeof(*hashes));
    *polls = 0;
    if (req->result == MSG_PARSE_OK && nk <= kcap && span != NULL && hashes != NULL) {
        for (uint32_t i = 0; i < nk; i++) {
            const struct keypos *kp = array_get(req->keys, i);
            ref_idx[i] = msg_backend_idx(req, kp->start, (uint32_t)(kp->end - kp->start));
        }
        int ticket;
        rstatus_t st = msg_backend_hashes_submit(req, ring, span, hashes, &ticket);
        if (st == NC_EAGAIN) {
            rc = -2;
        } else if (st != NC_OK) {
            rc = -4;
        } else {
            struct timespec t0, t1;
            clock_gettime(CLOCK_MONOTONIC, &t0);
            for (;;) {
                st = msg_backend_hashes_poll(req, ring, span, hashes, ticket);
                if (st != NC_EAGAIN) break;
                (*polls)++;
                clock_gettime(CLOCK_MONOTONIC, &t1);
                if (t1.tv_sec - t0.tv_sec > 5) break;
            }
            if (st == NC_OK) {
                msg_backend_idx_batch(req, hashes, batch_idx);
                rc = (int)nk;
            } else {
                rc = st == NC_EAGAIN ? -3 : -4;
            }
        }
    }
    free(span);
    free(hashes);
    msg_put(req);
    rp_pool_deinit(&pool);
    return rc;
}
