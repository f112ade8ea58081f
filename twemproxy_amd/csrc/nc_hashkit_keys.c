/*
 * Per-key, link-compatible hashkit symbols (src/hashkit/nc_hashkit.h:57-69,
 * src/hashkit/nc_ketama.c:31). These let libnc_gpuhash.so replace
 * libhashkit.a without touching twemproxy's hash_algos[] table
 * (src/nc_conf.c:30-35) or ketama_update's md5 (src/hashkit/nc_ketama.c:189).
 *
 * They are host code on purpose: a single key is hashed in tens of
 * nanoseconds, far below one host<->GPU round trip. The
 * batched GPU entry points (nc_gpuhash_host.c) never call into this file.
 */
#include <pthread.h>
#include <string.h>

#include "nc_gpuhash.h"
#include "nc_hash_algo.h"

static inline uint32_t ld_le32(const uint8_t *p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* Little-endian word of the n (< 4) bytes at p, rest zero. */
static inline uint32_t ld_le_partial(const uint8_t *p, size_t n)
{
    uint32_t w = 0;
    for (size_t i = 0; i < n; i++) {
        w |= (uint32_t)p[i] << (8 * i);
    }
    return w;
}

static uint32_t crc16_tab[256];
static uint32_t crc32_tab[256];
static pthread_once_t crc_once = PTHREAD_ONCE_INIT;

static void crc_tables_init(void)
{
    for (uint32_t i = 0; i < 256; i++) {
        crc16_tab[i] = nc_crc16_entry(i);
        crc32_tab[i] = nc_crc32_entry(i);
    }
}

uint32_t hash_one_at_a_time(const char *key, size_t key_length)
{
    const uint8_t *k = (const uint8_t *)key;
    uint32_t v = 0;
    for (size_t i = 0; i < key_length; i++) {
        v = nc_oaat_step(v, k[i]);
    }
    return nc_oaat_final(v);
}

void md5_signature(const unsigned char *key, unsigned int length, unsigned char *result)
{
    uint32_t st[4] = { NC_MD5_A0, NC_MD5_B0, NC_MD5_C0, NC_MD5_D0 };
    uint32_t w[16];
    size_t len = length, done = 0;
    while (len - done >= 64) {
        for (int t = 0; t < 16; t++) {
            w[t] = ld_le32(key + done + 4 * t);
        }
        nc_md5_block(st, w);
        done += 64;
    }
    uint32_t rem = (uint32_t)(len - done);
    for (uint32_t t = 0; t < 16; t++) {
        uint32_t lo = 4 * t;
        uint32_t raw = (lo < rem) ? ld_le_partial(key + done + lo, rem - lo < 4 ? rem - lo : 4) : 0;
        w[t] = nc_md5_pad_word(raw, t, rem);
    }
    uint64_t bits = (uint64_t)len << 3;
    if (rem >= 56) {
        nc_md5_block(st, w);
        memset(w, 0, sizeof(w));
    }
    w[14] = (uint32_t)bits;
    w[15] = (uint32_t)(bits >> 32);
    nc_md5_block(st, w);
    for (int i = 0; i < 4; i++) {
        for (int j = 0; j < 4; j++) {
            result[4 * i + j] = (unsigned char)(st[i] >> (8 * j));
        }
    }
}

uint32_t hash_md5(const char *key, size_t key_length)
{
    unsigned char d[16];
    md5_signature((const unsigned char *)key, (unsigned int)key_length, d);
    return ld_le32(d);
}

uint32_t ketama_hash(const char *key, size_t key_length, uint32_t alignment)
{
    unsigned char d[16];
    md5_signature((const unsigned char *)key, (unsigned int)key_length, d);
    return ld_le32(d + 4 * (alignment & 3));
}

uint32_t hash_crc16(const char *key, size_t key_length)
{
    pthread_once(&crc_once, crc_tables_init);
    const uint8_t *k = (const uint8_t *)key;
    uint32_t crc = 0;
    for (size_t i = 0; i < key_length; i++) {
        crc = NC_CRC16_NEXT(crc, crc16_tab[NC_CRC16_IDX(crc, k[i])]);
    }
    return crc;
}

static uint32_t crc32_run(const char *key, size_t key_length)
{
    pthread_once(&crc_once, crc_tables_init);
    const uint8_t *k = (const uint8_t *)key;
    uint32_t crc = 0xffffffffu;
    for (size_t i = 0; i < key_length; i++) {
        crc = NC_CRC32_NEXT(crc, crc32_tab[NC_CRC32_IDX(crc, k[i])]);
    }
    return crc;
}

uint32_t hash_crc32(const char *key, size_t key_length) { return nc_crc32_final(crc32_run(key, key_length)); }
uint32_t hash_crc32a(const char *key, size_t key_length) { return nc_crc32a_final(crc32_run(key, key_length)); }

#define NC_FNV_FN(name, init, step)                                   \
    uint32_t name(const char *key, size_t key_length)                 \
    {                                                                 \
        const uint8_t *k = (const uint8_t *)key;                      \
        uint32_t h = (init);                                          \
        for (size_t i = 0; i < key_length; i++) h = step(h, k[i]);    \
        return h;                                                     \
    }

NC_FNV_FN(hash_fnv1_64, NC_FNV64_INIT32, nc_fnv1_64_step)
NC_FNV_FN(hash_fnv1a_64, NC_FNV64_INIT32, nc_fnv1a_64_step)
NC_FNV_FN(hash_fnv1_32, NC_FNV32_INIT, nc_fnv1_32_step)
NC_FNV_FN(hash_fnv1a_32, NC_FNV32_INIT, nc_fnv1a_32_step)

uint32_t hash_hsieh(const char *key, size_t key_length)
{
    const uint8_t *k = (const uint8_t *)key;
    if (key_length == 0 || key == NULL) {
        return 0;
    }
    uint32_t h = 0;
    size_t nw = key_length >> 2;
    for (size_t i = 0; i < nw; i++) {
        h = nc_hsieh_word(h, ld_le32(k + 4 * i));
    }
    uint32_t rem = (uint32_t)(key_length & 3);
    h = nc_hsieh_tail(h, ld_le_partial(k + 4 * nw, rem), rem);
    return nc_hsieh_final(h);
}

uint32_t hash_murmur(const char *key, size_t length)
{
    const uint8_t *k = (const uint8_t *)key;
    uint32_t h = nc_murmur_init((uint32_t)length);
    size_t nw = length >> 2;
    for (size_t i = 0; i < nw; i++) {
        h = nc_murmur_word(h, ld_le32(k + 4 * i));
    }
    uint32_t rem = (uint32_t)(length & 3);
    h = nc_murmur_tail(h, ld_le_partial(k + 4 * nw, rem), rem);
    return nc_murmur_final(h);
}

uint32_t hash_jenkins(const char *key, size_t length)
{
    const uint8_t *k = (const uint8_t *)key;
    uint32_t a, b, c;
    a = b = c = nc_jenkins_init((uint32_t)length);
    if (length == 0) {
        return c;
    }
    while (length > 12) {
        a += ld_le32(k);
        b += ld_le32(k + 4);
        c += ld_le32(k + 8);
        NC_JENKINS_MIX(a, b, c);
        length -= 12;
        k += 12;
    }
    /* 1..12 bytes left: zero-extended words (the masked reads, :102-123). */
    a += ld_le_partial(k, length < 4 ? length : 4);
    if (length > 4) b += ld_le_partial(k + 4, length - 4 < 4 ? length - 4 : 4);
    if (length > 8) c += ld_le_partial(k + 8, length - 8);
    NC_JENKINS_FINAL(a, b, c);
    return c;
}
