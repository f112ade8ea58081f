/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Driver over the REAL reference request parsers and server_pool_idx,
 * compiled from the sources where they lie under /root/reference (oracle/
 * Makefile, target `ref-proto`; output only into oracle/_ref/): the proto
 * library (src/proto/nc_redis.c, nc_memcache.c), src/nc_message.c,
 * src/nc_mbuf.c and src/nc_server.c, the files the reference's own test_all
 * links (src/Makefile.am:63-89). It calls them the way test_all does
 * (src/test_all.c:76-107: a zeroed client conn, one mbuf, msg_get, the
 * parser) so tools/gen_proto_golden.py can record what the reference itself
 * returns — parse result, message type, consumed bytes and the keypos spans —
 * and the server index server_pool_idx picks with a hash_tag, and what the
 * reference's fragment loops (memcache_fragment / redis_fragment) make of a
 * multi-key request over a pool. Nothing here parses, hashes or fragments by
 * itself. Used only here, never on the GPU box.
 */
#include <stdlib.h>
#include <string.h>

#include <nc_core.h>
#include <nc_server.h>
#include <nc_message.h>
#include <nc_mbuf.h>
#include <nc_hashkit.h>

#define DEFINE_ACTION(_hash, _name) hash_##_name,
static hash_t rp_algos[] = { HASH_CODEC(DEFINE_ACTION) NULL };
#undef DEFINE_ACTION

static int rp_ready;

/* mbufs of MBUF_SIZE (nc_mbuf.h:39), the conf default mbuf-size */
int rp_init(void)
{
    if (!rp_ready) {
        struct instance nci;
        memset(&nci, 0, sizeof(nci));
        nci.mbuf_chunk_size = MBUF_SIZE;
        log_init(LOG_EMERG, NULL);
        mbuf_init(&nci);
        msg_init();
        rp_ready = 1;
    }
    return (int)mbuf_data_size();
}

/*
 * One request from buf[0, len) (len <= mbuf_data_size()): result
 * (MSG_PARSE_*), type (msg_type_t), consumed bytes (req->pos - m->start),
 * the connection's err flag, and up to kcap keypos spans as offsets into buf.
 * Returns the number of keys the parser pushed, or -1.
 */
int rp_parse_one(int redis, const uint8_t *buf, uint32_t len, int32_t *result, int32_t *type,
                 uint32_t *consumed, int32_t *conn_err, uint32_t *kstart, uint32_t *kend, uint32_t kcap)
{
    struct conn fake_client;
    memset(&fake_client, 0, sizeof(fake_client));
    if (!rp_ready || len > mbuf_data_size()) return -1;
    struct mbuf *m = mbuf_get();
    if (m == NULL) return -1;
    struct msg *req = msg_get(&fake_client, 1, redis ? 1 : 0);
    if (req == NULL) {
        mbuf_put(m);
        return -1;
    }
    req->state = 0;
    req->token = NULL;
    mbuf_copy(m, buf, len);
    STAILQ_INIT(&req->mhdr);
    mbuf_insert(&req->mhdr, m);
    req->pos = m->start;

    req->parser(req);

    *result = (int32_t)req->result;
    *type = (int32_t)req->type;
    *consumed = (uint32_t)(req->pos - m->start);
    *conn_err = fake_client.err;
    uint32_t nk = array_n(req->keys);
    for (uint32_t i = 0; i < nk && i < kcap; i++) {
        const struct keypos *kp = array_get(req->keys, i);
        if (kp->start < m->start || kp->end > m->last || kp->start > kp->end) {
            /* a span outside the request (the reference's COMMAND / LOLWUT
             * parse pushes one into static memory): marked, not measured */
            kstart[i] = kend[i] = UINT32_MAX;
            continue;
        }
        kstart[i] = (uint32_t)(kp->start - m->start);
        kend[i] = (uint32_t)(kp->end - m->start);
    }
    msg_put(req);
    return (int)nk;
}

/* msg_type_string (src/nc_message.c:449) into out; returns its length */
int rp_type_name(int32_t type, char *out, uint32_t cap)
{
    const struct string *s = msg_type_string((msg_type_t)type);
    uint32_t n = s->len < cap - 1u ? s->len : cap - 1u;
    memcpy(out, s->data, n);
    out[n] = '\0';
    return (int)n;
}

/* a server_pool of nserver live servers over the reference's own
 * ketama_update / modula_update (dist 0 / 1); 0 or -1 */
static int rp_pool_init(struct server_pool *pool, int mode, int dist, const char *const *names,
                        const uint32_t *name_lens, const uint32_t *weights, uint32_t nserver, const uint8_t *tag,
                        uint32_t taglen)
{
    if (mode < 0 || mode >= HASH_SENTINEL || (dist != 0 && dist != 1) || nserver == 0) return -1;
    memset(pool, 0, sizeof(*pool));
    if (array_init(&pool->server, nserver, sizeof(struct server)) != NC_OK) return -1;
    for (uint32_t s = 0; s < nserver; s++) {
        struct server *srv = array_push(&pool->server);
        memset(srv, 0, sizeof(*srv));
        srv->idx = s;
        srv->owner = pool;
        srv->name.data = (uint8_t *)names[s];
        srv->name.len = name_lens[s];
        srv->weight = weights[s];
    }
    pool->dist_type = dist == 0 ? DIST_KETAMA : DIST_MODULA;
    pool->key_hash_type = mode;
    pool->key_hash = rp_algos[mode];
    pool->hash_tag.data = (uint8_t *)tag;
    pool->hash_tag.len = taglen;
    rstatus_t st = dist == 0 ? ketama_update(pool) : modula_update(pool);
    if (st != NC_OK) {
        array_deinit(&pool->server);
        return -1;
    }
    return 0;
}

static void rp_pool_deinit(struct server_pool *pool)
{
    free(pool->continuum);
    array_deinit(&pool->server);
}

/*
 * One multi-key request buf[0, len) parsed as rp_parse_one does, from a
 * client connection owned by a pool (rp_pool_init), then fragmented by the
 * reference's own msg->fragment (memcache_fragment, src/proto/nc_memcache.c:
 * 1283-1389, or redis_fragment, src/proto/nc_redis.c:2804-2924): per key i
 * the server msg_backend_idx picked (sidx[i], src/nc_message.c:461-467) and
 * the position of frag_seq[i] in the fragment queue (fseq[i]); the
 * fragments' bytes as they would be sent, back to back in payload with their
 * lengths in plen. *nfrag = 0 when the reference does not fragment (one key,
 * or a command it does not split). Returns the number of keys, or -1 (parse
 * failure, too small an output, fragmentation error).
 */
int rp_fragment(int redis, const uint8_t *buf, uint32_t len, int mode, int dist, const char *const *names,
                const uint32_t *name_lens, const uint32_t *weights, uint32_t nserver, const uint8_t *tag,
                uint32_t taglen, uint32_t *sidx, uint32_t *fseq, uint32_t kcap, uint8_t *payload, uint32_t pcap,
                uint32_t *plen, uint32_t fcap, uint32_t *nfrag)
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
    struct msg_tqh frags;
    TAILQ_INIT(&frags);
    if (req->result == MSG_PARSE_OK && nk <= kcap && req->fragment(req, nserver, &frags) == NC_OK) {
        rc = (int)nk;
        *nfrag = 0;
        uint32_t used = 0;
        struct msg *sub;
        TAILQ_FOREACH(sub, &frags, m_tqe) {
            uint32_t n = 0;
            struct mbuf *b;
            STAILQ_FOREACH(b, &sub->mhdr, next) {
                const uint32_t bl = (uint32_t)(b->last - b->pos);
                if (used + n + bl > pcap) { rc = -1; break; }
                memcpy(payload + used + n, b->pos, bl);
                n += bl;
            }
            if (rc < 0 || *nfrag >= fcap) { rc = -1; break; }
            plen[(*nfrag)++] = n;
            used += n;
        }
        for (uint32_t i = 0; rc >= 0 && i < nk; i++) {
            const struct keypos *kp = array_get(req->keys, i);
            sidx[i] = msg_backend_idx(req, kp->start, (uint32_t)(kp->end - kp->start));
            fseq[i] = UINT32_MAX;
            if (req->frag_seq != NULL) {
                uint32_t j = 0;
                TAILQ_FOREACH(sub, &frags, m_tqe) {
                    if (sub == req->frag_seq[i]) fseq[i] = j;
                    j++;
                }
            }
        }
    }
    while (!TAILQ_EMPTY(&frags)) {
        struct msg *sub = TAILQ_FIRST(&frags);
        TAILQ_REMOVE(&frags, sub, m_tqe);
        msg_put(sub);
    }
    msg_put(req);
    rp_pool_deinit(&pool);
    return rc;
}

/*
 * server_pool_idx (src/nc_server.c:647-700) for n keys (CSR keys/offsets)
 * over a pool of nserver live servers whose continuum the reference's own
 * ketama_update / modula_update built (dist 0 / 1), key hash `mode`
 * (hash_algos order), hash_tag tag[0..taglen) (taglen 0 = none). Returns 0,
 * or -1.
 */
int rp_server_idx(int mode, int dist, const char *const *names, const uint32_t *name_lens,
                  const uint32_t *weights, uint32_t nserver, const uint8_t *tag, uint32_t taglen,
                  const uint8_t *keys, const uint64_t *offsets, uint64_t n, uint32_t *out)
{
    struct server_pool pool;
    if (rp_pool_init(&pool, mode, dist, names, name_lens, weights, nserver, tag, taglen) != 0) return -1;
    for (uint64_t i = 0; i < n; i++)
        out[i] = server_pool_idx(&pool, keys + offsets[i], (uint32_t)(offsets[i + 1] - offsets[i]));
    rp_pool_deinit(&pool);
    return 0;
}
