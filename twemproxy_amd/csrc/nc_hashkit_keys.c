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
#include "nc_hash_key.h"

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

/* one key through the shared per-key implementation (nc_hash_key.h) */
static inline uint32_t key_hash(int mode, const char *key, size_t len)
{
    if (mode == NC_GPUHASH_CRC16 || mode == NC_GPUHASH_CRC32 || mode == NC_GPUHASH_CRC32A)
        pthread_once(&crc_once, crc_tables_init);
    return nc_key_hash(mode, (const uint8_t *)key, (uint64_t)len, crc16_tab, crc32_tab);
}

void md5_signature(const unsigned char *key, unsigned int length, unsigned char *result)
{
    uint32_t st[4];
    nc_key_md5(key, length, st);
    for (int i = 0; i < 4; i++) {
        for (int j = 0; j < 4; j++) {
            result[4 * i + j] = (unsigned char)(st[i] >> (8 * j));
        }
    }
}

uint32_t ketama_hash(const char *key, size_t key_length, uint32_t alignment)
{
    unsigned char d[16];
    md5_signature((const unsigned char *)key, (unsigned int)key_length, d);
    return nc_key_ld32(d + 4 * (alignment & 3));
}

uint32_t hash_one_at_a_time(const char *key, size_t key_length) { return key_hash(NC_GPUHASH_ONE_AT_A_TIME, key, key_length); }
uint32_t hash_md5(const char *key, size_t key_length) { return key_hash(NC_GPUHASH_MD5, key, key_length); }
uint32_t hash_crc16(const char *key, size_t key_length) { return key_hash(NC_GPUHASH_CRC16, key, key_length); }
uint32_t hash_crc32(const char *key, size_t key_length) { return key_hash(NC_GPUHASH_CRC32, key, key_length); }
uint32_t hash_crc32a(const char *key, size_t key_length) { return key_hash(NC_GPUHASH_CRC32A, key, key_length); }
uint32_t hash_fnv1_64(const char *key, size_t key_length) { return key_hash(NC_GPUHASH_FNV1_64, key, key_length); }
uint32_t hash_fnv1a_64(const char *key, size_t key_length) { return key_hash(NC_GPUHASH_FNV1A_64, key, key_length); }
uint32_t hash_fnv1_32(const char *key, size_t key_length) { return key_hash(NC_GPUHASH_FNV1_32, key, key_length); }
uint32_t hash_fnv1a_32(const char *key, size_t key_length) { return key_hash(NC_GPUHASH_FNV1A_32, key, key_length); }
uint32_t hash_murmur(const char *key, size_t length) { return key_hash(NC_GPUHASH_MURMUR, key, length); }
uint32_t hash_jenkins(const char *key, size_t length) { return key_hash(NC_GPUHASH_JENKINS, key, length); }

uint32_t hash_hsieh(const char *key, size_t key_length)
{
    if (key_length == 0 || key == NULL) { /* src/hashkit/nc_hsieh.c:44 */
        return 0;
    }
    return key_hash(NC_GPUHASH_HSIEH, key, key_length);
}
