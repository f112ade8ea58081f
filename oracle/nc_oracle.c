/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see nc_oracle.h).
 *
 * Clean-room restatement of the twemproxy src/hashkit algorithms. It is
 * written from the published algorithm definitions (RFC 1321 for MD5, the
 * CRC polynomials evaluated bit by bit instead of through lookup tables,
 * Jenkins lookup3 / MurmurHash2 / SuperFastHash / FNV as specified) with every
 * quirk of the reference reproduced and cited. Citations are
 * /root/reference/<path>:<line>.
 *
 * "sx(b)" below is (uint32_t)(int32_t)(int8_t)b: x86-64 gcc treats `char` as
 * signed, so `(uint32_t)key[i]` sign-extends.
 */
#define _GNU_SOURCE
#include "nc_oracle.h"

#include <math.h>
#include <stdio.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static inline uint32_t sx32(uint8_t b) { return (uint32_t)(int32_t)(int8_t)b; }
static inline uint64_t sx64(uint8_t b) { return (uint64_t)(int64_t)(int8_t)b; }
static inline uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }
static inline uint32_t le32(const uint8_t *p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* src/hashkit/nc_one_at_a_time.c:35-51 — Jenkins one-at-a-time, signed bytes (:41). */
static uint32_t o_one_at_a_time(const uint8_t *k, size_t n)
{
    uint32_t v = 0;
    for (size_t i = 0; i < n; i++) {
        v += sx32(k[i]);
        v += v << 10;
        v ^= v >> 6;
    }
    v += v << 3;
    v ^= v >> 11;
    v += v << 15;
    return v;
}

/* ---- MD5, RFC 1321 section 3.4, written as the textbook 64-step loop ----
 * The reference (src/hashkit/nc_md5.c:89-194, :197-299) is an unrolled
 * OpenSSL-compatible variant; both are the same function. */
static uint32_t md5_T[64];
static const int md5_S[4][4] = { {7, 12, 17, 22}, {5, 9, 14, 20}, {4, 11, 16, 23}, {6, 10, 15, 21} };
static pthread_once_t md5_once = PTHREAD_ONCE_INIT;

static void md5_init_table(void)
{
    /* T[i] = floor(2^32 * |sin(i + 1)|) (RFC 1321 §3.4). */
    for (int i = 0; i < 64; i++) {
        md5_T[i] = (uint32_t)(uint64_t)floor(fabs(sin((double)(i + 1))) * 4294967296.0);
    }
}

static void md5_compress(uint32_t st[4], const uint8_t blk[64])
{
    uint32_t X[16];
    for (int i = 0; i < 16; i++) {
        X[i] = le32(blk + 4 * i);
    }
    uint32_t A = st[0], B = st[1], C = st[2], D = st[3];
    for (int i = 0; i < 64; i++) {
        uint32_t f;
        int g, r = i >> 4;
        switch (r) {
        case 0: f = (B & C) | (~B & D); g = i; break;
        case 1: f = (B & D) | (C & ~D); g = (5 * i + 1) & 15; break;
        case 2: f = B ^ C ^ D; g = (3 * i + 5) & 15; break;
        default: f = C ^ (B | ~D); g = (7 * i) & 15; break;
        }
        uint32_t t = D;
        D = C;
        C = B;
        B = B + rotl32(A + f + md5_T[i] + X[g], md5_S[r][i & 3]);
        A = t;
    }
    st[0] += A; st[1] += B; st[2] += C; st[3] += D;
}

void oracle_md5(const uint8_t *key, size_t len, uint8_t digest[16])
{
    pthread_once(&md5_once, md5_init_table);
    uint32_t st[4] = { 0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u };
    size_t full = len / 64;
    for (size_t b = 0; b < full; b++) {
        md5_compress(st, key + 64 * b);
    }
    /* Padding: 0x80, zeros, 64-bit little-endian bit length (nc_md5.c:249-274). */
    uint8_t tail[128];
    size_t rem = len - 64 * full;
    memset(tail, 0, sizeof(tail));
    memcpy(tail, key + 64 * full, rem);
    tail[rem] = 0x80;
    size_t tlen = (rem + 9 <= 64) ? 64 : 128;
    uint64_t bits = (uint64_t)len * 8u;
    for (int i = 0; i < 8; i++) {
        tail[tlen - 8 + i] = (uint8_t)(bits >> (8 * i));
    }
    md5_compress(st, tail);
    if (tlen == 128) {
        md5_compress(st, tail + 64);
    }
    for (int i = 0; i < 4; i++) {
        for (int j = 0; j < 4; j++) {
            digest[4 * i + j] = (uint8_t)(st[i] >> (8 * j));
        }
    }
}

/* src/hashkit/nc_md5.c:311-321 — digest bytes [0..3] as a little-endian u32. */
static uint32_t o_md5(const uint8_t *k, size_t n)
{
    uint8_t d[16];
    oracle_md5(k, n, d);
    return le32(d);
}

/* src/hashkit/nc_ketama.c:31-41 — digest word `alignment` (0..3), little-endian. */
uint32_t oracle_ketama_hash(const uint8_t *key, size_t len, uint32_t alignment)
{
    uint8_t d[16];
    oracle_md5(key, len, d);
    return le32(d + 4 * (alignment & 3));
}

/* src/hashkit/nc_crc16.c:56-66 — CRC-16/XMODEM step (poly 0x1021, MSB first)
 * with the running value kept in an unmasked u32: crc = (crc<<8) ^ T[idx].
 * The table entry T[idx] is evaluated here bit by bit. The index masks the
 * sign-extended char, so signedness does not matter. */
static uint32_t crc16_entry(uint32_t idx)
{
    uint32_t t = idx << 8;
    for (int i = 0; i < 8; i++) {
        t = (t & 0x8000u) ? ((t << 1) ^ 0x1021u) : (t << 1);
    }
    return t & 0xffffu;
}

static uint32_t o_crc16(const uint8_t *k, size_t n)
{
    uint32_t crc = 0;
    for (size_t i = 0; i < n; i++) {
        crc = (crc << 8) ^ crc16_entry(((crc >> 8) ^ sx32(k[i])) & 0xffu);
    }
    return crc;
}

/* Reflected CRC-32 (poly 0xEDB88320), init ~0, evaluated bit by bit. */
static uint32_t crc32_raw(const uint8_t *k, size_t n)
{
    uint32_t crc = 0xffffffffu;
    for (size_t i = 0; i < n; i++) {
        crc ^= k[i];
        for (int b = 0; b < 8; b++) {
            crc = (crc >> 1) ^ (0xEDB88320u & (0u - (crc & 1u)));
        }
    }
    return crc;
}

/* src/hashkit/nc_crc32.c:99-109 — libmemcached-compatible: 15 bits of ~crc. */
static uint32_t o_crc32(const uint8_t *k, size_t n) { return ((~crc32_raw(k, n)) >> 16) & 0x7fffu; }

/* src/hashkit/nc_crc32.c:112-123 — standard CRC-32/ISO-HDLC. */
static uint32_t o_crc32a(const uint8_t *k, size_t n) { return ~crc32_raw(k, n); }

/* src/hashkit/nc_fnv.c:26-37 — true 64-bit FNV-1, signed bytes, low 32 bits. */
static uint32_t o_fnv1_64(const uint8_t *k, size_t n)
{
    uint64_t h = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < n; i++) {
        h *= 0x100000001b3ull;
        h ^= sx64(k[i]);
    }
    return (uint32_t)h;
}

/* src/hashkit/nc_fnv.c:40-52 — 32-bit state seeded with the truncated 64-bit
 * offset basis; prime truncated to 0x1b3 (:42, :48). Signed bytes (:46). */
static uint32_t o_fnv1a_64(const uint8_t *k, size_t n)
{
    uint32_t h = (uint32_t)0xcbf29ce484222325ull;
    for (size_t i = 0; i < n; i++) {
        h ^= sx32(k[i]);
        h *= (uint32_t)0x100000001b3ull;
    }
    return h;
}

/* src/hashkit/nc_fnv.c:55-67. */
static uint32_t o_fnv1_32(const uint8_t *k, size_t n)
{
    uint32_t h = 2166136261u;
    for (size_t i = 0; i < n; i++) {
        h *= 16777619u;
        h ^= sx32(k[i]);
    }
    return h;
}

/* src/hashkit/nc_fnv.c:70-82. */
static uint32_t o_fnv1a_32(const uint8_t *k, size_t n)
{
    uint32_t h = 2166136261u;
    for (size_t i = 0; i < n; i++) {
        h ^= sx32(k[i]);
        h *= 16777619u;
    }
    return h;
}

/* src/hashkit/nc_hsieh.c:39-93 — SuperFastHash with the byte-form get16bits
 * (:33-36). len 0 -> 0 (:44). The rem==3 tail sign-extends key[2] (:65);
 * the rem==1 tail is unsigned (:76). */
static uint32_t o_hsieh(const uint8_t *k, size_t n)
{
    if (n == 0) {
        return 0;
    }
    uint32_t h = 0;
    size_t words = n >> 2, rem = n & 3;
    for (size_t i = 0; i < words; i++, k += 4) {
        uint32_t lo = (uint32_t)k[0] | ((uint32_t)k[1] << 8);
        uint32_t hi = (uint32_t)k[2] | ((uint32_t)k[3] << 8);
        h += lo;
        uint32_t tmp = (hi << 11) ^ h;
        h = (h << 16) ^ tmp;
        h += h >> 11;
    }
    if (rem == 3) {
        h += (uint32_t)k[0] | ((uint32_t)k[1] << 8);
        h ^= h << 16;
        h ^= sx32(k[2]) << 18;
        h += h >> 11;
    } else if (rem == 2) {
        h += (uint32_t)k[0] | ((uint32_t)k[1] << 8);
        h ^= h << 11;
        h += h >> 17;
    } else if (rem == 1) {
        h += k[0];
        h ^= h << 10;
        h += h >> 1;
    }
    h ^= h << 3;
    h += h >> 5;
    h ^= h << 4;
    h += h >> 17;
    h ^= h << 25;
    h += h >> 6;
    return h;
}

/* src/hashkit/nc_murmur.c:38-99 — MurmurHash2, seed 0xdeadbeef*len (:45),
 * h = seed ^ len (:52), little-endian words, unsigned tail bytes. */
static uint32_t o_murmur(const uint8_t *k, size_t n)
{
    const uint32_t m = 0x5bd1e995u;
    uint32_t h = (0xdeadbeefu * (uint32_t)n) ^ (uint32_t)n;
    size_t i = 0;
    for (; i + 4 <= n; i += 4) {
        uint32_t w = le32(k + i);
        w *= m;
        w ^= w >> 24;
        w *= m;
        h *= m;
        h ^= w;
    }
    size_t rem = n - i;
    if (rem) {
        if (rem >= 3) h ^= (uint32_t)k[i + 2] << 16;
        if (rem >= 2) h ^= (uint32_t)k[i + 1] << 8;
        h ^= k[i];
        h *= m;
    }
    h ^= h >> 13;
    h *= m;
    h ^= h >> 15;
    return h;
}

/* src/hashkit/nc_jenkins.c:76-230 — lookup3 hashlittle, initval 13 (:82).
 * Restated on little-endian words assembled from bytes; the reference's three
 * alignment paths agree on LE hosts. */
#define J_MIX(a, b, c) do {                              \
    a -= c; a ^= rotl32(c, 4);  c += b;                  \
    b -= a; b ^= rotl32(a, 6);  a += c;                  \
    c -= b; c ^= rotl32(b, 8);  b += a;                  \
    a -= c; a ^= rotl32(c, 16); c += b;                  \
    b -= a; b ^= rotl32(a, 19); a += c;                  \
    c -= b; c ^= rotl32(b, 4);  b += a; } while (0)
#define J_FINAL(a, b, c) do {                            \
    c ^= b; c -= rotl32(b, 14);                          \
    a ^= c; a -= rotl32(c, 11);                          \
    b ^= a; b -= rotl32(a, 25);                          \
    c ^= b; c -= rotl32(b, 16);                          \
    a ^= c; a -= rotl32(c, 4);                           \
    b ^= a; b -= rotl32(a, 14);                          \
    c ^= b; c -= rotl32(b, 24); } while (0)

static uint32_t o_jenkins(const uint8_t *k, size_t n)
{
    uint32_t a, b, c;
    a = b = c = 0xdeadbeefu + (uint32_t)n + 13u;
    if (n == 0) {
        return c;
    }
    while (n > 12) {
        a += le32(k);
        b += le32(k + 4);
        c += le32(k + 8);
        J_MIX(a, b, c);
        n -= 12;
        k += 12;
    }
    /* Last 1..12 bytes, zero-padded into three words. */
    uint8_t last[12] = { 0 };
    memcpy(last, k, n);
    a += le32(last);
    b += le32(last + 4);
    c += le32(last + 8);
    J_FINAL(a, b, c);
    return c;
}

typedef uint32_t (*o_hash_t)(const uint8_t *, size_t);

/* Function table in HASH_CODEC order (src/hashkit/nc_hashkit.h:24-36,
 * hash_algos[] src/nc_conf.c:30-35). */
static const o_hash_t o_algos[ORACLE_NMODES] = {
    o_one_at_a_time, o_md5, o_crc16, o_crc32, o_crc32a, o_fnv1_64,
    o_fnv1a_64, o_fnv1_32, o_fnv1a_32, o_hsieh, o_murmur, o_jenkins,
};

uint32_t oracle_hash(int mode, const uint8_t *key, size_t len)
{
    if (mode < 0 || mode >= ORACLE_NMODES) {
        return 0;
    }
    return o_algos[mode](key, len);
}

/* ---- batch driver (CPU baseline) ---- */

struct o_job {
    o_hash_t fn;
    const uint8_t *keys;
    const uint64_t *offsets;
    uint64_t lo, hi;
    uint32_t *out;
};

static void *o_run(void *arg)
{
    struct o_job *j = arg;
    /* volatile pointer: every key is hashed through the pointer, as
     * pool->key_hash is (src/nc_server.c:643), never inlined. */
    o_hash_t volatile fn = j->fn;
    for (uint64_t i = j->lo; i < j->hi; i++) {
        uint64_t s = j->offsets[i];
        j->out[i] = fn(j->keys + s, (size_t)(j->offsets[i + 1] - s));
    }
    return NULL;
}

/* First key index whose start offset is >= target (offsets is sorted). */
static uint64_t o_lower_bound(const uint64_t *offsets, uint64_t nkeys, uint64_t target)
{
    uint64_t lo = 0, hi = nkeys;
    while (lo < hi) {
        uint64_t mid = lo + (hi - lo) / 2;
        if (offsets[mid] < target) lo = mid + 1; else hi = mid;
    }
    return lo;
}

int oracle_hash_batch(int mode, const uint8_t *keys, const uint64_t *offsets,
                      uint64_t nkeys, uint32_t *out, int nthreads)
{
    if (mode < 0 || mode >= ORACLE_NMODES) {
        return -1;
    }
    pthread_once(&md5_once, md5_init_table);
    if (nthreads <= 1 || nkeys < 1024) {
        struct o_job j = { o_algos[mode], keys, offsets, 0, nkeys, out };
        o_run(&j);
        return 0;
    }
    if (nthreads > 256) {
        nthreads = 256;
    }
    struct o_job jobs[256];
    pthread_t tids[256];
    uint64_t total = offsets[nkeys] - offsets[0];
    uint64_t prev = 0;
    for (int t = 0; t < nthreads; t++) {
        uint64_t cut = (t == nthreads - 1) ? nkeys
            : o_lower_bound(offsets, nkeys, offsets[0] + total * (uint64_t)(t + 1) / (uint64_t)nthreads);
        /* keep a few keys per thread even for byte-degenerate inputs */
        uint64_t even = nkeys * (uint64_t)(t + 1) / (uint64_t)nthreads;
        if (total == 0) cut = even;
        if (cut < prev) cut = prev;
        jobs[t] = (struct o_job){ o_algos[mode], keys, offsets, prev, cut, out };
        prev = cut;
    }
    for (int t = 0; t < nthreads; t++) {
        pthread_create(&tids[t], NULL, o_run, &jobs[t]);
    }
    for (int t = 0; t < nthreads; t++) {
        pthread_join(tids[t], NULL);
    }
    return 0;
}

double oracle_time_batch(int mode, const uint8_t *keys, const uint64_t *offsets,
                         uint64_t nkeys, uint32_t *out, int nthreads, int reps)
{
    double best = 1e30;
    oracle_hash_batch(mode, keys, offsets, nkeys, out, nthreads); /* warm-up */
    for (int r = 0; r < (reps > 0 ? reps : 1); r++) {
        struct timespec a, b;
        clock_gettime(CLOCK_MONOTONIC, &a);
        if (oracle_hash_batch(mode, keys, offsets, nkeys, out, nthreads) != 0) {
            return -1.0;
        }
        clock_gettime(CLOCK_MONOTONIC, &b);
        double s = (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
        if (s < best) best = s;
    }
    return best;
}

/* ---- distributions ---- */

struct o_point { uint32_t value, index, order; };

static int o_point_cmp(const void *x, const void *y)
{
    const struct o_point *p = x, *q = y;
    if (p->value != q->value) return p->value < q->value ? -1 : 1;
    return p->order < q->order ? -1 : (p->order > q->order);
}

/* src/hashkit/nc_ketama.c:58-219 with every server live (auto_eject off). */
int oracle_ketama_build(const char *const *names, const uint32_t *name_lens,
                        const uint32_t *weights, uint32_t nserver,
                        uint32_t *values, uint32_t *indices, uint32_t cap)
{
    return oracle_ketama_build_live(names, name_lens, weights, NULL, nserver, values, indices, cap);
}

/* live[s] == 0: server s is ejected (auto_eject_hosts with next_retry > now,
 * :80-102): no points, not in the total weight or the live count. */
int oracle_ketama_build_live(const char *const *names, const uint32_t *name_lens,
                             const uint32_t *weights, const uint8_t *live, uint32_t nserver,
                             uint32_t *values, uint32_t *indices, uint32_t cap)
{
    uint32_t total = 0, nlive = 0;
    for (uint32_t s = 0; s < nserver; s++) {
        if (weights[s] == 0) return -1;
        if (live != NULL && !live[s]) continue;
        total += weights[s];
        nlive++;
    }
    if (nlive == 0) return 0;
    /* upper bound on points: each server gets <= 160*nlive points */
    size_t maxpts = (size_t)nlive * 160u * nlive + 4;
    struct o_point *pts = malloc(maxpts * sizeof(*pts));
    if (pts == NULL) return -1;
    uint32_t np = 0;
    for (uint32_t s = 0; s < nserver; s++) {
        if (live != NULL && !live[s]) continue;
        /* pointer_per_server: float arithmetic as written at :159-160. */
        float pct = (float)weights[s] / (float)total;
        float t = pct * 160.0f;
        t = t / 4.0f;
        t = t * (float)nlive;
        uint32_t pps = (uint32_t)(floorf((float)((double)t + 0.0000000001)) * 4.0f);
        for (uint32_t pi = 1; pi <= pps / 4; pi++) {
            char host[273];
            int hl = snprintf(host, sizeof(host), "%.*s-%u", (int)name_lens[s], names[s], pi - 1);
            size_t hostlen = (hl < 0) ? 0 : (size_t)hl;
            if (hostlen >= sizeof(host)) hostlen = sizeof(host) - 1;
            uint8_t d[16];
            oracle_md5((const uint8_t *)host, hostlen, d);
            for (uint32_t x = 0; x < 4; x++) {
                if (np >= maxpts) { free(pts); return -1; }
                pts[np].value = le32(d + 4 * x);
                pts[np].index = s;
                pts[np].order = np;
                np++;
            }
        }
    }
    qsort(pts, np, sizeof(*pts), o_point_cmp);
    if (np > cap) { free(pts); return -1; }
    for (uint32_t i = 0; i < np; i++) {
        values[i] = pts[i].value;
        indices[i] = pts[i].index;
    }
    free(pts);
    return (int)np;
}

/* src/hashkit/nc_ketama.c:222-246 — first point with value >= hash, wrapping. */
uint32_t oracle_ketama_dispatch(const uint32_t *values, const uint32_t *indices,
                                uint32_t n, uint32_t hash)
{
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        uint32_t mid = lo + (hi - lo) / 2;
        if (values[mid] < hash) lo = mid + 1; else hi = mid;
    }
    if (lo == n) lo = 0;
    return indices[lo];
}

/* src/hashkit/nc_modula.c:116-127 — one point per unit of weight. */
int oracle_modula_build(const uint32_t *weights, uint32_t nserver,
                        uint32_t *indices, uint32_t cap)
{
    uint32_t np = 0;
    for (uint32_t s = 0; s < nserver; s++) {
        for (uint32_t w = 0; w < weights[s]; w++) {
            if (np >= cap) return -1;
            indices[np++] = s;
        }
    }
    return (int)np;
}

/* src/hashkit/nc_modula.c:146-156. */
uint32_t oracle_modula_dispatch(const uint32_t *indices, uint32_t n, uint32_t hash)
{
    return indices[hash % n];
}

/*
 * server_pool_idx (src/nc_server.c:647-700) over a CSR batch, every server
 * live: nserver == 1 -> 0 (:655-658); hash_tag trimming (:665-677): the first
 * tag[0], then the first tag[1] after it, and with at least one byte between
 * them the key becomes those bytes; server_pool_hash's keylen 0 -> hash 0
 * (:639-641); then ketama_dispatch or modula_dispatch (:680-688).
 */
int oracle_server_idx_batch(int mode, int dist, const uint32_t *values, const uint32_t *indices,
                            uint32_t ncont, uint32_t nserver, const char *tag,
                            const uint8_t *keys, const uint64_t *offsets, uint64_t nkeys, uint32_t *out)
{
    if (mode < 0 || mode >= ORACLE_NMODES || (dist != 0 && dist != 1) || nserver == 0) return -1;
    for (uint64_t i = 0; i < nkeys; i++) {
        const uint8_t *key = keys + offsets[i];
        uint32_t keylen = (uint32_t)(offsets[i + 1] - offsets[i]);
        if (nserver == 1) {
            out[i] = 0;
            continue;
        }
        if (tag != NULL) {
            const uint8_t *s = memchr(key, (uint8_t)tag[0], keylen);
            if (s != NULL) {
                const uint8_t *e = memchr(s + 1, (uint8_t)tag[1], (size_t)(key + keylen - (s + 1)));
                if (e != NULL && e - s > 1) {
                    key = s + 1;
                    keylen = (uint32_t)(e - key);
                }
            }
        }
        const uint32_t h = keylen == 0 ? 0u : oracle_hash(mode, key, keylen);
        out[i] = dist == 0 ? oracle_ketama_dispatch(values, indices, ncont, h)
                           : oracle_modula_dispatch(indices, ncont, h);
    }
    return 0;
}

/*
 * memcache_parse_req (src/proto/nc_memcache.c) for a stream of retrieval
 * requests, sequentially, as the reference walks it: SW_START (:219-232),
 * SW_REQ_TYPE (:234-368; get :245, gets :268, CR after them :343-345),
 * SW_SPACES_BEFORE_KEY (:372-378), SW_KEY (:380-428; empty or > 250 bytes
 * :384-396; a CR is re-read :421-426), SW_SPACES_BEFORE_KEYS (:431-447),
 * SW_ALMOST_DONE (:709-717). Stops at the first request that is malformed
 * (-1: syntax, -2: key length) or not get/gets (-3), or at an incomplete
 * last request. Writes key spans of the accepted requests and each parsed
 * request's status; returns 0.
 */
int oracle_mc_parse(const uint8_t *s, uint64_t n, uint64_t max_keys, uint64_t *kstart, uint32_t *klen,
                    uint32_t *kreq, int32_t *status, uint64_t max_reqs, uint64_t *nkeys, uint64_t *nreqs_parsed,
                    uint64_t *first_error, uint64_t *consumed)
{
    uint64_t p = 0, nk = 0, nr = 0, done = 0;
    *first_error = UINT64_MAX;
    for (;;) {
        /* a request is complete only with its CR LF; find it (keys hold no CR) */
        uint64_t e = p;
        while (e + 1 < n && !(s[e] == '\r' && s[e + 1] == '\n')) e++;
        if (e + 1 >= n) break; /* incomplete: left for the next read */
        if (nr >= max_reqs) return -1;
        int32_t st = 0;
        uint64_t q = p, kn = 0;
        while (q < e && s[q] == ' ') q++;                            /* SW_START */
        const uint64_t t0 = q;
        while (q < e && s[q] >= 'a' && s[q] <= 'z') q++;            /* SW_REQ_TYPE */
        const uint64_t tl = q - t0;
        if (tl == 0 || (q < e && s[q] != ' ')) {
            st = -1;
        } else if (!((tl == 3 && memcmp(s + t0, "get", 3) == 0) || (tl == 4 && memcmp(s + t0, "gets", 4) == 0))) {
            st = -3;
        } else if (q == e) {
            st = -1; /* "get\r\n" */
        } else {
            while (q < e && s[q] == ' ') q++;                        /* SW_SPACES_BEFORE_KEY */
            for (;;) {
                if (q < e && s[q] == '\r') { st = -1; break; }      /* SW_ALMOST_DONE wants LF */
                const uint64_t k0 = q;                               /* SW_KEY */
                while (q < e && s[q] != ' ' && s[q] != '\r') q++;
                if (q - k0 == 0 || q - k0 > 250) { st = -2; break; }
                if (nk + kn >= max_keys) return -1;
                kstart[nk + kn] = k0;
                klen[nk + kn] = (uint32_t)(q - k0);
                kreq[nk + kn] = (uint32_t)nr;
                kn++;
                if (q < e && s[q] == '\r') { st = -1; break; }
                while (q < e && s[q] == ' ') q++;                    /* SW_SPACES_BEFORE_KEYS */
                if (q == e) break;
            }
        }
        status[nr] = st;
        nr++;
        if (st != 0) {
            *first_error = nr - 1;
            break;
        }
        nk += kn;
        p = e + 2;
        done = p;
    }
    *nkeys = nk;
    *nreqs_parsed = nr;
    if (*first_error == UINT64_MAX) *first_error = nr;
    *consumed = done;
    return 0;
}

/*
 * redis_parse_req (src/proto/nc_redis.c:460-1900) for a stream of pipelined
 * RESP requests, one byte at a time through the reference's states, for the
 * command classes whose keys the device extracts:
 *   arg0  redis_arg0 (:64-104, less AUTH, which the proxy answers itself),
 *   arg1  redis_arg1 (:106-140), argn redis_argn (:208-298),
 *   argx  redis_argx (:300-319), argkvx redis_argkvx (:321-334).
 * States: SW_START (:478-490), SW_NARG (:492-509), SW_NARG_LF (:511-521),
 * SW_REQ_TYPE_LEN (:523-543; rlen 0 is an error), SW_REQ_TYPE (:557-1326;
 * the name compares case-insensitively, nc_proto.h:87), SW_REQ_TYPE_LF
 * (:1333-1360; narg 1 is an error for these classes), SW_KEY_LEN
 * (:1362-1389; rlen >= mbuf_data_size() is an error, no digits is rlen 0),
 * SW_KEY (:1403-1435, a key is rlen bytes then CR), SW_KEY_LF (:1437-1490),
 * SW_ARG1_LEN (:1492-1512; no digits is an error), SW_ARG1 (:1526-1544),
 * SW_ARG1_LF (:1546-1589), SW_ARGN_LEN/ARGN/ARGN_LF (:1807-1878).
 * Lengths and counts accumulate in uint32_t like r->rlen / r->rnarg.
 * Statuses: 0 ok, -1 syntax error, -2 key length >= the mbuf data size,
 * -3 a command outside these classes (unknown to this table; the host parser
 * decides). Stops at the first non-ok request (recorded) or at an incomplete
 * last one (not recorded).
 */
enum { RC_NONE, RC_ARG0, RC_ARG1, RC_ARGN, RC_ARGX, RC_ARGKVX };

static const char *const rc_arg0[] = {"persist", "pttl", "ttl", "type", "dump", "decr", "get", "getdel", "incr",
                                      "strlen", "hgetall", "hkeys", "hlen", "hvals", "llen", "scard", "smembers",
                                      "zcard", NULL};
static const char *const rc_arg1[] = {"expire", "expireat", "pexpire", "pexpireat", "move", "append", "decrby",
                                      "getbit", "getset", "incrby", "incrbyfloat", "setnx", "hexists", "hget",
                                      "hstrlen", "lindex", "rpoplpush", "sismember", "zrank", "zrevrank", "zscore",
                                      NULL};
static const char *const rc_argn[] = {
    "sort", "copy", "bitcount", "bitpos", "bitfield", "exists", "getex", "set", "hdel", "hmget", "hmset", "hscan",
    "hset", "hrandfield", "lpush", "lpushx", "rpush", "rpushx", "lpop", "rpop", "lpos", "sadd", "sdiff",
    "sdiffstore", "sinter", "sinterstore", "srem", "sunion", "sunionstore", "srandmember", "sscan", "spop",
    "smismember", "pfadd", "pfmerge", "pfcount", "zadd", "zdiff", "zdiffstore", "zinter", "zinterstore", "zmscore",
    "zpopmax", "zpopmin", "zrandmember", "zrange", "zrangebylex", "zrangebyscore", "zrangestore", "zrem",
    "zrevrange", "zrevrangebylex", "zrevrangebyscore", "zscan", "zunion", "zunionstore", "geodist", "geopos",
    "geohash", "geoadd", "georadius", "georadiusbymember", "geosearch", "geosearchstore", "restore", NULL};
static const char *const rc_argx[] = {"mget", "del", "unlink", "touch", NULL};

static int rc_in(const char *const *tab, const uint8_t *m, uint64_t len)
{
    for (; *tab; tab++) {
        if (strlen(*tab) != len) continue;
        uint64_t i = 0;
        while (i < len && (m[i] == (uint8_t)(*tab)[i] || m[i] == (uint8_t)((*tab)[i] ^ 0x20))) i++;
        if (i == len) return 1;
    }
    return 0;
}

int oracle_redis_class(const uint8_t *m, uint64_t len)
{
    if (rc_in(rc_arg0, m, len)) return RC_ARG0;
    if (rc_in(rc_arg1, m, len)) return RC_ARG1;
    if (rc_in(rc_argn, m, len)) return RC_ARGN;
    if (rc_in(rc_argx, m, len)) return RC_ARGX;
    if (len == 4 && rc_in((const char *const[]){"mset", NULL}, m, len)) return RC_ARGKVX;
    return RC_NONE;
}

enum {
    RS_START, RS_NARG, RS_NARG_LF, RS_TYPE_LEN, RS_TYPE_LEN_LF, RS_TYPE, RS_TYPE_LF, RS_KEY_LEN, RS_KEY_LEN_LF,
    RS_KEY, RS_KEY_LF, RS_ARG_LEN, RS_ARG_LEN_LF, RS_ARG, RS_ARG_LF
};

int oracle_redis_parse(const uint8_t *s, uint64_t n, uint32_t max_key_len, uint64_t max_keys, uint64_t *kstart,
                       uint32_t *klen, uint32_t *kreq, int32_t *status, uint64_t max_reqs, uint64_t *nkeys,
                       uint64_t *nreqs_parsed, uint64_t *first_error, uint64_t *consumed)
{
    uint64_t nk = 0, nr = 0, done = 0, kn = 0, token = 0;
    uint32_t narg = 0, rnarg = 0, rlen = 0;
    int state = RS_START, cls = RC_NONE, have_token = 0, st = 0;
    *first_error = UINT64_MAX;
    for (uint64_t p = 0; p < n && st == 0; p++) {
        const uint8_t ch = s[p];
        int fin = 0;
        switch (state) {
        case RS_START:
            if (ch != '*') { st = -1; break; }
            rnarg = 0;
            kn = 0;
            state = RS_NARG;
            break;
        case RS_NARG:
            if (ch >= '0' && ch <= '9') rnarg = rnarg * 10u + (uint32_t)(ch - '0');
            else if (ch == '\r' && rnarg != 0) { narg = rnarg; state = RS_NARG_LF; }
            else st = -1;
            break;
        case RS_NARG_LF:
        case RS_TYPE_LEN_LF:
        case RS_KEY_LEN_LF:
        case RS_ARG_LEN_LF:
            if (ch != '\n') { st = -1; break; }
            state = state == RS_NARG_LF ? RS_TYPE_LEN : state == RS_TYPE_LEN_LF ? RS_TYPE
                  : state == RS_KEY_LEN_LF ? RS_KEY : RS_ARG;
            have_token = 0;
            break;
        case RS_TYPE_LEN:
        case RS_KEY_LEN:
        case RS_ARG_LEN:
            if (!have_token) {
                if (ch != '$') { st = -1; break; }
                have_token = 1;
                token = p;
                rlen = 0;
            } else if (ch >= '0' && ch <= '9') {
                rlen = rlen * 10u + (uint32_t)(ch - '0');
            } else if (ch == '\r') {
                if (state == RS_TYPE_LEN && (rlen == 0 || rnarg == 0)) { st = -1; break; }
                if (state == RS_KEY_LEN && rlen >= max_key_len) { st = -2; break; }
                if (state == RS_KEY_LEN && rnarg == 0) { st = -1; break; }
                if (state == RS_ARG_LEN && (p - token <= 1 || rnarg == 0)) { st = -1; break; }
                rnarg--;
                state = state == RS_TYPE_LEN ? RS_TYPE_LEN_LF : state == RS_KEY_LEN ? RS_KEY_LEN_LF : RS_ARG_LEN_LF;
            } else {
                st = -1;
            }
            break;
        case RS_TYPE:
        case RS_KEY:
        case RS_ARG: {
            /* rlen bytes of data, then CR: wait for the CR's byte to arrive */
            const uint64_t m = p + rlen;
            if (m >= n) { p = n; break; }
            if (s[m] != '\r') { st = -1; break; }
            if (state == RS_TYPE) {
                cls = oracle_redis_class(s + p, rlen);
                if (cls == RC_NONE) { st = -3; break; }
                state = RS_TYPE_LF;
            } else if (state == RS_KEY) {
                if (nk + kn >= max_keys) return -1;
                kstart[nk + kn] = p;
                klen[nk + kn] = rlen;
                kreq[nk + kn] = (uint32_t)nr;
                kn++;
                state = RS_KEY_LF;
            } else {
                state = RS_ARG_LF;
            }
            p = m;
            break;
        }
        case RS_TYPE_LF:
            if (ch != '\n' || narg == 1) { st = -1; break; }
            state = RS_KEY_LEN;
            have_token = 0;
            break;
        case RS_KEY_LF:
            if (ch != '\n') { st = -1; break; }
            have_token = 0;
            if (cls == RC_ARG0) {
                if (rnarg != 0) st = -1; else fin = 1;
            } else if (cls == RC_ARG1) {
                if (rnarg != 1) st = -1; else state = RS_ARG_LEN;
            } else if (cls == RC_ARGN || cls == RC_ARGX) {
                if (rnarg == 0) fin = 1; else state = cls == RC_ARGX ? RS_KEY_LEN : RS_ARG_LEN;
            } else { /* argkvx */
                if (narg % 2 == 0) st = -1; else state = RS_ARG_LEN;
            }
            break;
        case RS_ARG_LF:
            if (ch != '\n') { st = -1; break; }
            have_token = 0;
            if (cls == RC_ARG1) {
                if (rnarg != 0) st = -1; else fin = 1;
            } else if (cls == RC_ARGN) {
                if (rnarg == 0) fin = 1; else state = RS_ARG_LEN; /* SW_ARG1_LF then SW_ARGN_LF: same rule */
            } else { /* argkvx */
                if (rnarg == 0) fin = 1; else state = RS_KEY_LEN;
            }
            break;
        }
        if (st != 0) break;
        if (fin) {
            if (nr >= max_reqs) return -1;
            status[nr++] = 0;
            nk += kn;
            kn = 0;
            done = p + 1;
            state = RS_START;
        }
    }
    if (st != 0) {
        if (nr >= max_reqs) return -1;
        status[nr] = st;
        *first_error = nr;
        nr++;
    }
    *nkeys = nk;
    *nreqs_parsed = nr;
    if (*first_error == UINT64_MAX) *first_error = nr;
    *consumed = done;
    return 0;
}
