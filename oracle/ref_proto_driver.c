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
 * and the server index server_pool_idx picks with a hash_tag. Nothing here
 * parses or hashes by itself. Used only here, never on the GPU box.
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
    if (mode < 0 || mode >= HASH_SENTINEL || (dist != 0 && dist != 1) || nserver == 0) return -1;
    struct server_pool pool;
    memset(&pool, 0, sizeof(pool));
    if (array_init(&pool.server, nserver, sizeof(struct server)) != NC_OK) return -1;
    for (uint32_t s = 0; s < nserver; s++) {
        struct server *srv = array_push(&pool.server);
        memset(srv, 0, sizeof(*srv));
        srv->idx = s;
        srv->owner = &pool;
        srv->name.data = (uint8_t *)names[s];
        srv->name.len = name_lens[s];
        srv->weight = weights[s];
    }
    pool.dist_type = dist == 0 ? DIST_KETAMA : DIST_MODULA;
    pool.key_hash_type = mode;
    pool.key_hash = rp_algos[mode];
    pool.hash_tag.data = (uint8_t *)tag;
    pool.hash_tag.len = taglen;
    rstatus_t st = dist == 0 ? ketama_update(&pool) : modula_update(&pool);
    if (st != NC_OK) {
        array_deinit(&pool.server);
        return -1;
    }
    for (uint64_t i = 0; i < n; i++)
        out[i] = server_pool_idx(&pool, keys + offsets[i], (uint32_t)(offsets[i + 1] - offsets[i]));
    free(pool.continuum);
    array_deinit(&pool.server);
    return 0;
}
