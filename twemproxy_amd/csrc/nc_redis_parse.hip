/*
 * Key extraction on the device for redis: a stream of
 * pipelined RESP requests into the key CSR the hash kernels take, plus the
 * request each key belongs to.
 *
 * Reference: redis_parse_req, /root/reference/src/proto/nc_redis.c:460-1900,
 * for the command classes whose keys it pushes one by one:
 *   arg0 redis_arg0 (:64-104, less AUTH), arg1 redis_arg1 (:106-140),
 *   argn redis_argn (:208-298), argx redis_argx (:300-319),
 *   argkvx redis_argkvx (:321-334).
 * States: SW_START (:478-490), SW_NARG (:492-509), SW_NARG_LF (:511-521),
 * SW_REQ_TYPE_LEN (:523-543), SW_REQ_TYPE (:557-1326), SW_REQ_TYPE_LF
 * (:1333-1360), SW_KEY_LEN (:1362-1389), SW_KEY (:1403-1435), SW_KEY_LF
 * (:1437-1490), SW_ARG1_LEN/ARG1/ARG1_LF (:1492-1589), SW_ARGN_* (:1807-1878).
 * The oracle's sequential restatement is oracle/nc_oracle.c:oracle_redis_parse;
 * statuses are the same (0 ok, -1 syntax, -2 key length >= mbuf data size,
 * -3 a command outside these classes: the host parser takes over).
 *
 * RESP requests are length-prefixed and binary-safe, so request boundaries are
 * not visible in the bytes. The device parses speculatively:
 *   1. every '*' after a CR LF (and position 0) is a candidate start
 *      (a two-pass count / scan / write select over 16-B blocks); a true request start is always one, except a
 *      start that is not '*': that request fails at its first byte
 *      (SW_START, :478-483), so an ok chain that stops short of the stream
 *      end is followed by one failing request;
 *   2. one thread per candidate runs the request state machine from there,
 *      one bulk string per step: status, end, key count. Bulk data is
 *      skipped by its length, so a thread touches O(tokens) bytes;
 *   3. next[c] = the candidate at c's end (binary search), or none when c
 *      failed, is incomplete or ends the stream;
 *   4. the chain from candidate 0 is marked by radix-4 pointer jumping
 *      (about log4(2 nc) rounds; after round r distances [0, 4^r) are marked);
 *   5. the marked candidates, compacted in order, are the requests the
 *      reference parses; then the key count scan, emit, length scan and
 *      gather of the memcache pipeline (nc_mc_parse.hip).
 */
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <errno.h>
#include <stdlib.h>

#include "nc_gpuhash.h"

namespace {

enum : uint8_t { RC_NONE, RC_ARG0, RC_ARG1, RC_ARGN, RC_ARGX, RC_ARGKVX };

struct CmdName {
    char name[18];
    uint8_t len;
    uint8_t cls;
};

#define A0(s) {s, sizeof(s) - 1, RC_ARG0}
#define A1(s) {s, sizeof(s) - 1, RC_ARG1}
#define AN(s) {s, sizeof(s) - 1, RC_ARGN}
#define AX(s) {s, sizeof(s) - 1, RC_ARGX}

/* lowercase command names of the key classes (redis_arg0/arg1/argn/argx/argkvx,
 * nc_redis.c:64-334); compared case-insensitively (str*icmp, nc_proto.h:87) */
__constant__ CmdName kCmds[] = {
    A0("persist"), A0("pttl"), A0("ttl"), A0("type"), A0("dump"), A0("decr"), A0("get"), A0("getdel"),
    A0("incr"), A0("strlen"), A0("hgetall"), A0("hkeys"), A0("hlen"), A0("hvals"), A0("llen"), A0("scard"),
    A0("smembers"), A0("zcard"),
    A1("expire"), A1("expireat"), A1("pexpire"), A1("pexpireat"), A1("move"), A1("append"), A1("decrby"),
    A1("getbit"), A1("getset"), A1("incrby"), A1("incrbyfloat"), A1("setnx"), A1("hexists"), A1("hget"),
    A1("hstrlen"), A1("lindex"), A1("rpoplpush"), A1("sismember"), A1("zrank"), A1("zrevrank"), A1("zscore"),
    AN("sort"), AN("copy"), AN("bitcount"), AN("bitpos"), AN("bitfield"), AN("exists"), AN("getex"), AN("set"),
    AN("hdel"), AN("hmget"), AN("hmset"), AN("hscan"), AN("hset"), AN("hrandfield"), AN("lpush"), AN("lpushx"),
    AN("rpush"), AN("rpushx"), AN("lpop"), AN("rpop"), AN("lpos"), AN("sadd"), AN("sdiff"), AN("sdiffstore"),
    AN("sinter"), AN("sinterstore"), AN("srem"), AN("sunion"), AN("sunionstore"), AN("srandmember"),
    AN("sscan"), AN("spop"), AN("smismember"), AN("pfadd"), AN("pfmerge"), AN("pfcount"), AN("zadd"),
    AN("zdiff"), AN("zdiffstore"), AN("zinter"), AN("zinterstore"), AN("zmscore"), AN("zpopmax"),
    AN("zpopmin"), AN("zrandmember"), AN("zrange"), AN("zrangebylex"), AN("zrangebyscore"), AN("zrangestore"),
    AN("zrem"), AN("zrevrange"), AN("zrevrangebylex"), AN("zrevrangebyscore"), AN("zscan"), AN("zunion"),
    AN("zunionstore"), AN("geodist"), AN("geopos"), AN("geohash"), AN("geoadd"), AN("georadius"),
    AN("georadiusbymember"), AN("geosearch"), AN("geosearchstore"), AN("restore"),
    AX("mget"), AX("del"), AX("unlink"), AX("touch"),
    {"mset", 4, RC_ARGKVX},
};
constexpr int kNumCmds = sizeof(kCmds) / sizeof(kCmds[0]);

__device__ uint8_t cmd_class(const uint8_t *__restrict__ m, uint32_t len)
{
    if (len < 3 || len > 17) return RC_NONE;
    for (int e = 0; e < kNumCmds; e++) {
        if (kCmds[e].len != len) continue;
        uint32_t i = 0;
        /* every table byte is a lowercase letter: m | 0x20 matches exactly its two cases */
        while (i < len && (uint8_t)(m[i] | 0x20u) == (uint8_t)kCmds[e].name[i]) i++;
        if (i == len) return kCmds[e].cls;
    }
    return RC_NONE;
}

constexpr int32_t kIncomplete = 1; /* the request runs past the stream end */

enum BulkKind { BK_TYPE, BK_KEY, BK_ARG };

/* One bulk string "$<len>\r\n<data>\r\n" from s[*pp]: SW_REQ_TYPE_LEN /
 * SW_KEY_LEN / SW_ARG*_LEN (:523-543, :1362-1389, :1492-1512, :1807-1825),
 * their LF states, the data and its CR (:557-, :1403-1435, :1526-1544), and
 * the LF after it. The checks run in the reference's byte order, so the first
 * failure (or the stream end) gives the same status as the byte machine. On
 * 0, *pp is past the LF, the data is s[*dp, *dp + *dl) and *cls the command
 * class (BK_TYPE). */
__device__ __forceinline__ int32_t bulk(const uint8_t *__restrict__ s, uint32_t n, uint32_t *pp, BulkKind kind,
                                        uint32_t max_key_len, uint32_t *rnarg, uint32_t *dp, uint32_t *dl,
                                        uint8_t *cls)
{
    const uint32_t token = *pp;
    if (token >= n) return kIncomplete;
    if (s[token] != '$') return NC_GPUHASH_REDIS_EINVAL;
    uint32_t q = token + 1, rlen = 0;
    for (;;) {
        if (q >= n) return kIncomplete;
        const uint8_t ch = s[q];
        if (ch >= '0' && ch <= '9') {
            rlen = rlen * 10u + (uint32_t)(ch - '0');
            q++;
            continue;
        }
        if (ch == '\r') break;
        return NC_GPUHASH_REDIS_EINVAL;
    }
    if (kind == BK_TYPE && (rlen == 0 || *rnarg == 0)) return NC_GPUHASH_REDIS_EINVAL;
    if (kind == BK_KEY && rlen >= max_key_len) return NC_GPUHASH_REDIS_EKEYLEN;
    if (kind == BK_KEY && *rnarg == 0) return NC_GPUHASH_REDIS_EINVAL;
    if (kind == BK_ARG && (q - token <= 1 || *rnarg == 0)) return NC_GPUHASH_REDIS_EINVAL;
    (*rnarg)--;
    if (q + 1 >= n) return kIncomplete;
    if (s[q + 1] != '\n') return NC_GPUHASH_REDIS_EINVAL;
    const uint32_t d = q + 2;
    if (d >= n) return kIncomplete;
    const uint64_t m = (uint64_t)d + rlen; /* rlen data bytes, then CR */
    if (m >= n) return kIncomplete;
    if (s[m] != '\r') return NC_GPUHASH_REDIS_EINVAL;
    if (kind == BK_TYPE) {
        *cls = cmd_class(s + d, rlen);
        if (*cls == RC_NONE) return NC_GPUHASH_REDIS_EUNSUPPORTED;
    }
    if (m + 1 >= n) return kIncomplete;
    if (s[m + 1] != '\n') return NC_GPUHASH_REDIS_EINVAL;
    *pp = (uint32_t)m + 2u;
    *dp = d;
    *dl = rlen;
    return NC_GPUHASH_REDIS_OK;
}

/* One request from s[p0]: redis_parse_req for the key classes, one bulk
 * string per step (lanes parsing same-shaped requests stay converged).
 * Returns the status; on 0, *end is one past its LF and *nkeys its key count.
 * EMIT writes each key's span at base + i; the count pass writes the first
 * key's span to *kstart, *klen. oracle_redis_parse is the byte-at-a-time
 * restatement it is tested against. */
template <bool EMIT>
__device__ int32_t parse_req(const uint8_t *__restrict__ s, uint32_t n, uint32_t p0, uint32_t max_key_len,
                             uint32_t *end, uint32_t *nkeys, uint32_t *kstart, uint32_t *klen, uint32_t *kreq,
                             uint32_t base, uint32_t req)
{
    if (s[p0] != '*') return NC_GPUHASH_REDIS_EINVAL; /* SW_START (:478-483) */
    uint32_t p = p0 + 1, rnarg = 0;
    for (;;) { /* SW_NARG (:492-509) */
        if (p >= n) return kIncomplete;
        const uint8_t ch = s[p];
        if (ch >= '0' && ch <= '9') {
            rnarg = rnarg * 10u + (uint32_t)(ch - '0');
            p++;
            continue;
        }
        if (ch == '\r' && rnarg != 0) break;
        return NC_GPUHASH_REDIS_EINVAL;
    }
    const uint32_t narg = rnarg;
    if (p + 1 >= n) return kIncomplete; /* SW_NARG_LF */
    if (s[p + 1] != '\n') return NC_GPUHASH_REDIS_EINVAL;
    p += 2;
    uint32_t dp = 0, dl = 0, kn = 0;
    uint8_t cls = RC_NONE;
    int32_t st = bulk(s, n, &p, BK_TYPE, max_key_len, &rnarg, &dp, &dl, &cls);
    if (st != NC_GPUHASH_REDIS_OK) return st;
    if (narg == 1) return NC_GPUHASH_REDIS_EINVAL; /* SW_REQ_TYPE_LF (:1347-1348) */
    BulkKind kind = BK_KEY;
    for (;;) {
        st = bulk(s, n, &p, kind, max_key_len, &rnarg, &dp, &dl, &cls);
        if (st != NC_GPUHASH_REDIS_OK) return st;
        bool fin = false;
        if (kind == BK_KEY) { /* SW_KEY_LF (:1437-1490) */
            if constexpr (EMIT) {
                kstart[base + kn] = dp;
                klen[base + kn] = dl;
                kreq[base + kn] = req;
            } else if (kn == 0) {
                *kstart = dp;
                *klen = dl;
            }
            kn++;
            if (cls == RC_ARG0) {
                if (rnarg != 0) return NC_GPUHASH_REDIS_EINVAL;
                fin = true;
            } else if (cls == RC_ARG1) {
                if (rnarg != 1) return NC_GPUHASH_REDIS_EINVAL;
                kind = BK_ARG;
            } else if (cls == RC_ARGN || cls == RC_ARGX) {
                if (rnarg == 0) fin = true;
                else kind = cls == RC_ARGX ? BK_KEY : BK_ARG;
            } else { /* argkvx */
                if (narg % 2 == 0) return NC_GPUHASH_REDIS_EINVAL;
                kind = BK_ARG;
            }
        } else { /* SW_ARG1_LF (:1546-1589), SW_ARGN_LF (:1858-1878) */
            if (cls == RC_ARG1) {
                if (rnarg != 0) return NC_GPUHASH_REDIS_EINVAL;
                fin = true;
            } else if (rnarg == 0) {
                fin = true;
            } else {
                kind = cls == RC_ARGN ? BK_ARG : BK_KEY;
            }
        }
        if (fin) {
            *end = p;
            *nkeys = kn;
            return NC_GPUHASH_REDIS_OK;
        }
    }
}

/* Candidate starts (position 0, or '*' right after CR LF) of the 16-B aligned
 * block `blk` of the stream as a bit mask; the stream starts `delta` bytes
 * into block 0. One 16-B load per block plus the 4 bytes before it: aligned
 * loads that hold a stream byte stay inside the stream's pages. */
__device__ __forceinline__ uint32_t cand_mask(const uint8_t *__restrict__ sa, uint32_t delta, uint32_t n, uint32_t blk)
{
    const uint4 v = *reinterpret_cast<const uint4 *>(sa + (uint64_t)blk * 16u);
    const uint32_t prev = blk ? *reinterpret_cast<const uint32_t *>(sa + (uint64_t)blk * 16u - 4u) : 0u;
    const uint32_t w[5] = {prev, v.x, v.y, v.z, v.w};
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int j = k + 4;
        const uint32_t c0 = (w[j >> 2] >> (8 * (j & 3))) & 0xffu;
        const uint32_t c1 = (w[(j - 1) >> 2] >> (8 * ((j - 1) & 3))) & 0xffu;
        const uint32_t c2 = (w[(j - 2) >> 2] >> (8 * ((j - 2) & 3))) & 0xffu;
        const int64_t i = (int64_t)blk * 16 + k - delta;
        const bool hit = i == 0 || (i >= 2 && i < (int64_t)n && c0 == '*' && c1 == '\n' && c2 == '\r');
        m |= hit ? (1u << k) : 0u;
    }
    return m;
}

/* pass 1: candidates per workgroup of 256 blocks (4 KiB of stream) */
__global__ void rd_cand_count_kernel(const uint8_t *__restrict__ sa, uint32_t delta, uint32_t n, uint32_t nblk,
                                     uint32_t *__restrict__ wg_count)
{
    using Reduce = hipcub::BlockReduce<uint32_t, 256>;
    __shared__ typename Reduce::TempStorage tmp;
    const uint32_t blk = blockIdx.x * 256u + threadIdx.x;
    const uint32_t c = blk < nblk ? (uint32_t)__popc(cand_mask(sa, delta, n, blk)) : 0u;
    const uint32_t tot = Reduce(tmp).Sum(c);
    if (threadIdx.x == 0) wg_count[blockIdx.x] = tot;
}

/* pass 2: after the exclusive scan of wg_count, write positions in order */
__global__ void rd_cand_write_kernel(const uint8_t *__restrict__ sa, uint32_t delta, uint32_t n, uint32_t nblk,
                                     const uint32_t *__restrict__ wg_base, uint32_t *__restrict__ cand)
{
    using Scan = hipcub::BlockScan<uint32_t, 256>;
    __shared__ typename Scan::TempStorage tmp;
    const uint32_t blk = blockIdx.x * 256u + threadIdx.x;
    uint32_t m = blk < nblk ? cand_mask(sa, delta, n, blk) : 0u;
    uint32_t at = 0;
    Scan(tmp).ExclusiveSum((uint32_t)__popc(m), at);
    at += wg_base[blockIdx.x];
    while (m) {
        const int k = __ffs(m) - 1;
        m &= m - 1u;
        cand[at++] = (uint32_t)((int64_t)blk * 16 + k - delta);
    }
}

/* candidate c: parse, then link to the candidate at its end */
__global__ void rd_cand_kernel(const uint8_t *__restrict__ s, uint32_t n, uint32_t max_key_len,
                               const uint32_t *__restrict__ cand, uint32_t nc, int8_t *__restrict__ status,
                               uint32_t *__restrict__ cend, uint32_t *__restrict__ cnk, uint32_t *__restrict__ ck0s,
                               uint32_t *__restrict__ ck0l, uint32_t *__restrict__ next, uint8_t *__restrict__ mark)
{
    const uint32_t c = blockIdx.x * 256u + threadIdx.x;
    if (c > nc) return;
    if (c == nc) { /* the sentinel: points at itself */
        next[nc] = nc;
        mark[nc] = 0;
        return;
    }
    uint32_t e = 0, k = 0, k0s = 0, k0l = 0;
    const int32_t st = parse_req<false>(s, n, cand[c], max_key_len, &e, &k, &k0s, &k0l, nullptr, 0, 0);
    status[c] = (int8_t)st;
    cend[c] = e;
    cnk[c] = k;
    ck0s[c] = k0s;
    ck0l[c] = k0l;
    uint32_t nx = nc;
    if (st == NC_GPUHASH_REDIS_OK && e < n && s[e] == '*') {
        uint32_t lo = c + 1, hi = nc; /* first candidate >= e; e follows a CR LF and holds '*': it is one */
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (cand[mid] < e) lo = mid + 1;
            else hi = mid;
        }
        nx = lo;
    }
    next[c] = nx;
    mark[c] = c == 0 ? 1u : 0u;
}

/* one pointer-jumping round of radix 4: with jin = next^d, a marked c marks
 * c + d, c + 2d, c + 3d along the chain; jout = next^(4d) */
__global__ void rd_jump_kernel(const uint32_t *__restrict__ jin, uint32_t *__restrict__ jout, uint8_t *mark,
                               uint32_t nc)
{
    const uint32_t c = blockIdx.x * 256u + threadIdx.x;
    if (c > nc) return;
    const uint32_t j1 = jin[c], j2 = jin[j1], j3 = jin[j2];
    if (c < nc && mark[c]) { /* marks land only on the chain: races only mark early */
        mark[j1] = 1u;
        mark[j2] = 1u;
        mark[j3] = 1u;
    }
    jout[c] = jin[j3];
}

/* the chain's last request: [1] its candidate, [2] its status, [3] its end */
__global__ void rd_tail_kernel(const uint32_t *__restrict__ req, const int8_t *__restrict__ cstatus,
                               const uint32_t *__restrict__ cend, uint64_t *misc)
{
    const uint64_t nm = misc[0];
    const uint32_t c = nm ? req[nm - 1] : 0u;
    misc[1] = c;
    misc[2] = (uint64_t)(int64_t)cstatus[c];
    misc[3] = cend[c];
}

/* the request after an ok chain whose next byte is not '*': SW_START fails (:478-483) */
__global__ void rd_bad_start_kernel(int32_t *__restrict__ rstatus, uint64_t r)
{
    rstatus[r] = NC_GPUHASH_REDIS_EINVAL;
}

/* per request r (the r-th marked candidate): key count (ok ones) and status */
__global__ void rd_req_kernel(const uint32_t *__restrict__ req, uint32_t nreq, const int8_t *__restrict__ cstatus,
                              const uint32_t *__restrict__ cnk, uint32_t *__restrict__ nk,
                              int32_t *__restrict__ rstatus)
{
    const uint32_t r = blockIdx.x * 256u + threadIdx.x;
    if (r >= nreq) return;
    const uint32_t c = req[r];
    const int32_t st = cstatus[c];
    nk[r] = st == NC_GPUHASH_REDIS_OK ? cnk[c] : 0u;
    if (rstatus) rstatus[r] = st;
}

__global__ void rd_emit_kernel(const uint8_t *__restrict__ s, uint32_t n, uint32_t max_key_len,
                               const uint32_t *__restrict__ cand, const uint32_t *__restrict__ req, uint32_t nok,
                               const uint32_t *__restrict__ cnk, const uint32_t *__restrict__ ck0s,
                               const uint32_t *__restrict__ ck0l, const uint64_t *__restrict__ kbase,
                               uint32_t *__restrict__ kstart, uint32_t *__restrict__ klen, uint32_t *__restrict__ kreq)
{
    const uint32_t r = blockIdx.x * 256u + threadIdx.x;
    if (r >= nok) return;
    const uint32_t c = req[r], nkc = cnk[c], b = (uint32_t)kbase[r];
    if (nkc == 1) { /* one key (get, set, ...): its span is known from the count pass */
        kstart[b] = ck0s[c];
        klen[b] = ck0l[c];
        kreq[b] = r;
    } else if (nkc > 1) { /* mget, del, mset, ...: parse again */
        uint32_t e = 0, k = 0;
        (void)parse_req<true>(s, n, cand[c], max_key_len, &e, &k, kstart, klen, kreq, b, r);
    }
}

/* 8 lanes per key copy its bytes (C2-like keys are ~19 B; longer ones loop) */
__global__ void rd_gather_kernel(const uint8_t *__restrict__ s, const uint32_t *__restrict__ kstart,
                                 const uint64_t *__restrict__ koff, uint32_t nk, uint8_t *__restrict__ keys)
{
    const uint32_t k = blockIdx.x * 32u + (threadIdx.x >> 3);
    if (k >= nk) return;
    const uint64_t src = kstart[k], dst = koff[k], len = koff[k + 1] - koff[k];
    for (uint64_t j = threadIdx.x & 7u; j < len; j += 8u) keys[dst + j] = s[src + j];
}

__global__ void rd_pad_kernel(uint8_t *__restrict__ keys, const uint64_t *__restrict__ koff, uint32_t nk)
{
    const uint64_t e = koff[nk];
    if (threadIdx.x < NC_GPUHASH_PAD) keys[e + threadIdx.x] = 0u;
}

struct Widen {
    __host__ __device__ uint64_t operator()(uint32_t v) const { return v; }
};

unsigned grid_of(uint64_t n, unsigned per = 256u)
{
    const uint64_t g = (n + per - 1u) / per;
    return (unsigned)(g == 0 ? 1u : g);
}

} // namespace

struct nc_gpuhash_redis_parser {
    uint64_t max_bytes, max_reqs, max_keys, max_cands;
    uint32_t *wgc, *wgb; /* candidates per workgroup of the select, and their exclusive scan */
    uint64_t max_wg;
    uint32_t *cand;   /* candidate start positions */
    int8_t *cstatus;  /* per candidate: status of its speculative parse */
    uint32_t *cend, *cnk;
    uint32_t *ck0s, *ck0l; /* per candidate: the first key's span */
    uint32_t *jmp[2]; /* pointer-jumping successor arrays (nc + 1: the sentinel) */
    uint8_t *mark;    /* on the chain from candidate 0 */
    uint32_t *req;    /* marked candidates in order = the requests */
    uint32_t *nk;     /* keys per request */
    uint64_t *kbase;
    uint32_t *kstart, *klen, *kreq;
    uint64_t *misc;   /* [0] selected count */
    void *tmp;
    size_t tmp_bytes;
};

static void rparser_free(nc_gpuhash_redis_parser_t *ps)
{
    void *bufs[] = {ps->wgc, ps->wgb, ps->cand, ps->cstatus, ps->cend, ps->cnk, ps->ck0s, ps->ck0l, ps->jmp[0], ps->jmp[1], ps->mark,
                    ps->req, ps->nk, ps->kbase, ps->kstart, ps->klen, ps->kreq, ps->misc, ps->tmp};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    free(ps);
}

extern "C" nc_gpuhash_redis_parser_t *nc_gpuhash_redis_parser_create(uint64_t max_bytes, uint64_t max_reqs,
                                                                     uint64_t max_keys)
{
    if (max_bytes == 0 || max_reqs == 0 || max_keys == 0 || max_bytes >= (1ull << 31) || max_reqs >= (1ull << 31) ||
        max_keys >= (1ull << 31)) {
        errno = EINVAL;
        return nullptr;
    }
    nc_gpuhash_redis_parser_t *ps = (nc_gpuhash_redis_parser_t *)calloc(1, sizeof(*ps));
    if (ps == nullptr) {
        errno = ENOMEM;
        return nullptr;
    }
    ps->max_bytes = max_bytes;
    ps->max_reqs = max_reqs;
    ps->max_keys = max_keys;
    ps->max_cands = max_bytes / 2u + 2u; /* position 0 and one per CR LF */
    const uint64_t nc1 = ps->max_cands + 1u;
    size_t t1 = 0, t2 = 0, t3 = 0, t4 = 0;
    ps->max_wg = (max_bytes + 15u) / 16u / 256u + 2u;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, t1, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                                    (int64_t)ps->max_wg + 1);
    if (e == hipSuccess)
        e = hipcub::DeviceSelect::Flagged(nullptr, t4, hipcub::CountingInputIterator<uint32_t>(0),
                                          (uint8_t *)nullptr, (uint32_t *)nullptr, (uint64_t *)nullptr,
                                          (int64_t)ps->max_cands);
    hipcub::TransformInputIterator<uint64_t, Widen, uint32_t *> w0(nullptr, Widen());
    if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(nullptr, t2, w0, (uint64_t *)nullptr, (int64_t)max_reqs + 1);
    if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(nullptr, t3, w0, (uint64_t *)nullptr, (int64_t)max_keys + 1);
    size_t t = t1;
    for (size_t x : {t2, t3, t4}) t = x > t ? x : t;
    ps->tmp_bytes = t;
    if (e == hipSuccess) e = hipMalloc((void **)&ps->wgc, (ps->max_wg + 1) * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->wgb, (ps->max_wg + 1) * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->cand, nc1 * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->cstatus, nc1);
    if (e == hipSuccess) e = hipMalloc((void **)&ps->cend, nc1 * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->cnk, nc1 * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->ck0s, nc1 * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->ck0l, nc1 * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->jmp[0], nc1 * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->jmp[1], nc1 * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->mark, nc1);
    if (e == hipSuccess) e = hipMalloc((void **)&ps->req, nc1 * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->nk, (max_reqs + 1) * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->kbase, (max_reqs + 1) * sizeof(uint64_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->kstart, max_keys * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->klen, (max_keys + 1) * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->kreq, max_keys * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->misc, 8 * sizeof(uint64_t));
    if (e == hipSuccess) e = hipMalloc(&ps->tmp, ps->tmp_bytes ? ps->tmp_bytes : 16u);
    if (e != hipSuccess) {
        rparser_free(ps);
        errno = e == hipErrorNoDevice ? ENODEV : ENOMEM;
        return nullptr;
    }
    return ps;
}

extern "C" void nc_gpuhash_redis_parser_destroy(nc_gpuhash_redis_parser_t *ps)
{
    if (ps) rparser_free(ps);
}

extern "C" rstatus_t nc_gpuhash_redis_parse_device(nc_gpuhash_redis_parser_t *ps, const uint8_t *d_stream,
                                                  uint64_t nbytes, uint32_t max_key_len, uint8_t *d_keys,
                                                  uint64_t *d_offsets, uint32_t *d_key_req, int32_t *d_req_status,
                                                  struct nc_gpuhash_redis_result *res, void *stream)
{
    if (ps == nullptr || res == nullptr || (nbytes && d_stream == nullptr) || d_offsets == nullptr ||
        max_key_len == 0) {
        errno = EINVAL;
        return NC_ERROR;
    }
    if (nbytes > ps->max_bytes) {
        errno = ENOMEM;
        return NC_ENOMEM;
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    res->nreqs = res->nkeys = res->consumed = res->first_error = 0;
    const uint32_t n = (uint32_t)nbytes;
    hipError_t e = hipSuccess;
    uint64_t nreq = 0, nk = 0, first_bad = 0, consumed = 0;
    if (n) {
        uint64_t nc = 0;
        const uint32_t delta = (uint32_t)(reinterpret_cast<uintptr_t>(d_stream) & 15u);
        const uint8_t *sa = d_stream - delta;
        const uint32_t nblk = (uint32_t)((n + delta + 15u) / 16u), nwg = (nblk + 255u) / 256u;
        hipLaunchKernelGGL(rd_cand_count_kernel, dim3(nwg), dim3(256), 0, st, sa, delta, n, nblk, ps->wgc);
        e = hipGetLastError();
        if (e == hipSuccess) e = hipMemsetAsync(ps->wgc + nwg, 0, sizeof(uint32_t), st);
        if (e == hipSuccess)
            e = hipcub::DeviceScan::ExclusiveSum(ps->tmp, ps->tmp_bytes, ps->wgc, ps->wgb, (int64_t)nwg + 1, st);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(rd_cand_write_kernel, dim3(nwg), dim3(256), 0, st, sa, delta, n, nblk,
                               ps->wgb, ps->cand);
            e = hipGetLastError();
        }
        uint32_t nc32 = 0;
        if (e == hipSuccess) e = hipMemcpyAsync(&nc32, ps->wgb + nwg, sizeof(uint32_t), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        nc = nc32;
        if (e == hipSuccess) {
            const uint32_t c32 = (uint32_t)nc;
            hipLaunchKernelGGL(rd_cand_kernel, dim3(grid_of(nc + 1)), dim3(256), 0, st, d_stream, n, max_key_len,
                               ps->cand, c32, ps->cstatus, ps->cend, ps->cnk, ps->ck0s, ps->ck0l, ps->jmp[0],
                               ps->mark);
            int cur = 0;
            for (uint64_t span = 1; span < 2u * (nc + 1); span <<= 2, cur ^= 1)
                hipLaunchKernelGGL(rd_jump_kernel, dim3(grid_of(nc + 1)), dim3(256), 0, st, ps->jmp[cur],
                                   ps->jmp[cur ^ 1], ps->mark, c32);
            e = hipGetLastError();
            if (e == hipSuccess)
                e = hipcub::DeviceSelect::Flagged(ps->tmp, ps->tmp_bytes, hipcub::CountingInputIterator<uint32_t>(0),
                                                  ps->mark, ps->req, ps->misc, (int64_t)nc, st);
        }
        uint64_t tail[4] = {0, 0, 0, 0}; /* marked count, last candidate, its status, its end */
        if (e == hipSuccess) {
            hipLaunchKernelGGL(rd_tail_kernel, dim3(1), dim3(1), 0, st, ps->req, ps->cstatus, ps->cend, ps->misc);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipMemcpyAsync(tail, ps->misc, sizeof(tail), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        const uint64_t nm = tail[0];
        const int64_t lasts = (int64_t)tail[2];
        /* an ok chain that stops before the stream end: the next byte is not '*', a failing request */
        const bool bad_start = nm && lasts == NC_GPUHASH_REDIS_OK && tail[3] < n;
        if (nm) {
            nreq = lasts == kIncomplete ? nm - 1 : nm + (bad_start ? 1u : 0u);
            first_bad = lasts != NC_GPUHASH_REDIS_OK ? nm - 1 : nm;
        }
        /* the synthetic failing request after an ok chain holds no key: it is
         * reported in nreqs but does not count against max_reqs (its status
         * takes d_req_status's extra slot, index max_reqs at most) */
        if (e == hipSuccess && nreq - (bad_start ? 1u : 0u) > ps->max_reqs) {
            errno = ENOMEM;
            return NC_ENOMEM;
        }
        if (e == hipSuccess && first_bad) {
            uint32_t lastok = (uint32_t)tail[1], endp = (uint32_t)tail[3];
            if (first_bad != nm) { /* the last marked one failed: the ok one before it */
                e = hipMemcpy(&lastok, ps->req + first_bad - 1, sizeof(uint32_t), hipMemcpyDeviceToHost);
                if (e == hipSuccess) e = hipMemcpy(&endp, ps->cend + lastok, sizeof(uint32_t), hipMemcpyDeviceToHost);
            }
            consumed = endp;
        }
        if (e == hipSuccess && nreq) {
            hipLaunchKernelGGL(rd_req_kernel, dim3(grid_of(nm)), dim3(256), 0, st, ps->req, (uint32_t)(nreq < nm ? nreq : nm),
                               ps->cstatus, ps->cnk, ps->nk, d_req_status);
            if (bad_start && d_req_status)
                hipLaunchKernelGGL(rd_bad_start_kernel, dim3(1), dim3(1), 0, st, d_req_status, nm);
            e = hipGetLastError();
            /* nk[first_bad] = 0 so the exclusive scan's last element is the key total */
            if (e == hipSuccess) e = hipMemsetAsync(ps->nk + first_bad, 0, sizeof(uint32_t), st);
            hipcub::TransformInputIterator<uint64_t, Widen, uint32_t *> wn(ps->nk, Widen());
            if (e == hipSuccess)
                e = hipcub::DeviceScan::ExclusiveSum(ps->tmp, ps->tmp_bytes, wn, ps->kbase, (int64_t)first_bad + 1, st);
            if (e == hipSuccess) e = hipMemcpyAsync(&nk, ps->kbase + first_bad, sizeof(uint64_t), hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e == hipSuccess && nk > ps->max_keys) {
                errno = ENOMEM;
                return NC_ENOMEM;
            }
        }
        if (e == hipSuccess && nk) {
            uint32_t *kreq = d_key_req ? d_key_req : ps->kreq;
            hipLaunchKernelGGL(rd_emit_kernel, dim3(grid_of(first_bad)), dim3(256), 0, st, d_stream, n, max_key_len,
                               ps->cand, ps->req, (uint32_t)first_bad, ps->cnk, ps->ck0s, ps->ck0l, ps->kbase,
                               ps->kstart, ps->klen, kreq);
            e = hipGetLastError();
            if (e == hipSuccess) e = hipMemsetAsync(ps->klen + nk, 0, sizeof(uint32_t), st);
            hipcub::TransformInputIterator<uint64_t, Widen, uint32_t *> wl(ps->klen, Widen());
            if (e == hipSuccess)
                e = hipcub::DeviceScan::ExclusiveSum(ps->tmp, ps->tmp_bytes, wl, d_offsets, (int64_t)nk + 1, st);
            if (e == hipSuccess && d_keys) {
                hipLaunchKernelGGL(rd_gather_kernel, dim3(grid_of(nk, 32u)), dim3(256), 0, st, d_stream, ps->kstart,
                                   d_offsets, (uint32_t)nk, d_keys);
                hipLaunchKernelGGL(rd_pad_kernel, dim3(1), dim3(64), 0, st, d_keys, d_offsets, (uint32_t)nk);
                e = hipGetLastError();
            }
        }
    }
    if (e == hipSuccess && nk == 0) e = hipMemsetAsync(d_offsets, 0, sizeof(uint64_t), st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        errno = e == hipErrorNoDevice ? ENODEV : EIO;
        return NC_ERROR;
    }
    res->nreqs = nreq;
    res->nkeys = nk;
    res->first_error = first_bad;
    res->consumed = consumed;
    return NC_OK;
}
