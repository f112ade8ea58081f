/*
 * The 12 hashkit functions of src/hashkit/nc_hashkit.h:57-69 on ONE key at a
 * byte pointer, for the host and the device: the link-compatible per-key
 * symbols (nc_hashkit_keys.c) and the small-batch ring worker
 * (nc_ring.hip), which hashes each key of a batch from LDS. Byte loads only,
 * so any alignment and any address space (host memory, LDS, global) works.
 * The step functions and constants are nc_hash_algo.h's, shared with the
 * batch kernels; citations there.
 *
 * crc16t / crc32t are the 256-entry tables (nc_crc16_entry / nc_crc32_entry
 * of every index), which the caller keeps (static on the host, LDS in the
 * worker).
 */
#ifndef NC_HASH_KEY_H
#define NC_HASH_KEY_H

#include <stdint.h>

#include "nc_gpuhash.h"
#include "nc_hash_algo.h"

/* little-endian word of the 4 bytes at p */
NC_HD uint32_t nc_key_ld32(const uint8_t *p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* little-endian word of the n (< 4) bytes at p, rest zero */
NC_HD uint32_t nc_key_ld_partial(const uint8_t *p, uint64_t n)
{
    uint32_t w = 0;
    for (uint64_t i = 0; i < n; i++) w |= (uint32_t)p[i] << (8 * i);
    return w;
}

/* md5 state A, B, C, D after the whole padded message of len bytes
 * (src/hashkit/nc_md5.c:245-298; md5_signature's digest is st in LE) */
NC_HD void nc_key_md5(const uint8_t *key, uint64_t len, uint32_t st[4])
{
    uint32_t w[16];
    uint64_t done = 0;
    st[0] = NC_MD5_A0;
    st[1] = NC_MD5_B0;
    st[2] = NC_MD5_C0;
    st[3] = NC_MD5_D0;
    while (len - done >= 64) {
        for (int t = 0; t < 16; t++) w[t] = nc_key_ld32(key + done + 4 * t);
        nc_md5_block(st, w);
        done += 64;
    }
    const uint32_t rem = (uint32_t)(len - done);
    for (uint32_t t = 0; t < 16; t++) {
        const uint32_t lo = 4 * t;
        const uint32_t raw = lo < rem ? nc_key_ld_partial(key + done + lo, rem - lo < 4 ? rem - lo : 4) : 0;
        w[t] = nc_md5_pad_word(raw, t, rem);
    }
    const uint64_t bits = len << 3;
    if (rem >= 56) {
        nc_md5_block(st, w);
        for (int t = 0; t < 16; t++) w[t] = 0;
    }
    w[14] = (uint32_t)bits;
    w[15] = (uint32_t)(bits >> 32);
    nc_md5_block(st, w);
}

NC_HD uint32_t nc_key_crc32_run(const uint8_t *k, uint64_t len, const uint32_t *crc32t)
{
    uint32_t crc = 0xffffffffu;
    for (uint64_t i = 0; i < len; i++) crc = NC_CRC32_NEXT(crc, crc32t[NC_CRC32_IDX(crc, k[i])]);
    return crc;
}

NC_HD uint32_t nc_key_words(int murmur, const uint8_t *k, uint64_t len)
{
    /* hsieh (src/hashkit/nc_hsieh.c:39-93) and murmur (nc_murmur.c:38-99):
     * 4-byte words, then a 0..3-byte tail */
    if (!murmur && len == 0) return 0;
    uint32_t h = murmur ? nc_murmur_init((uint32_t)len) : 0u;
    const uint64_t nw = len >> 2;
    for (uint64_t i = 0; i < nw; i++) {
        const uint32_t w = nc_key_ld32(k + 4 * i);
        h = murmur ? nc_murmur_word(h, w) : nc_hsieh_word(h, w);
    }
    const uint32_t rem = (uint32_t)(len & 3);
    const uint32_t tw = nc_key_ld_partial(k + 4 * nw, rem);
    return murmur ? nc_murmur_final(nc_murmur_tail(h, tw, rem)) : nc_hsieh_final(nc_hsieh_tail(h, tw, rem));
}

NC_HD uint32_t nc_key_jenkins(const uint8_t *k, uint64_t length)
{
    uint32_t a, b, c;
    a = b = c = nc_jenkins_init((uint32_t)length);
    if (length == 0) return c;
    while (length > 12) {
        a += nc_key_ld32(k);
        b += nc_key_ld32(k + 4);
        c += nc_key_ld32(k + 8);
        NC_JENKINS_MIX(a, b, c);
        length -= 12;
        k += 12;
    }
    /* 1..12 bytes left: zero-extended words (src/hashkit/nc_jenkins.c:102-123) */
    a += nc_key_ld_partial(k, length < 4 ? length : 4);
    if (length > 4) b += nc_key_ld_partial(k + 4, length - 4 < 4 ? length - 4 : 4);
    if (length > 8) c += nc_key_ld_partial(k + 8, length - 8);
    NC_JENKINS_FINAL(a, b, c);
    return c;
}

/* hash_<mode>(key, len) of src/hashkit/nc_hashkit.h:57-69 (mode = hash_type_t) */
NC_HD uint32_t nc_key_hash(int mode, const uint8_t *k, uint64_t len, const uint32_t *crc16t, const uint32_t *crc32t)
{
    uint32_t h = 0;
    switch (mode) {
    case NC_GPUHASH_ONE_AT_A_TIME:
        for (uint64_t i = 0; i < len; i++) h = nc_oaat_step(h, k[i]);
        return nc_oaat_final(h);
    case NC_GPUHASH_MD5: {
        uint32_t st[4];
        nc_key_md5(k, len, st);
        return st[0]; /* digest bytes 0..3 (nc_md5.c:317-320) */
    }
    case NC_GPUHASH_CRC16:
        for (uint64_t i = 0; i < len; i++) h = NC_CRC16_NEXT(h, crc16t[NC_CRC16_IDX(h, k[i])]);
        return h;
    case NC_GPUHASH_CRC32: return nc_crc32_final(nc_key_crc32_run(k, len, crc32t));
    case NC_GPUHASH_CRC32A: return nc_crc32a_final(nc_key_crc32_run(k, len, crc32t));
    case NC_GPUHASH_FNV1_64:
        h = NC_FNV64_INIT32;
        for (uint64_t i = 0; i < len; i++) h = nc_fnv1_64_step(h, k[i]);
        return h;
    case NC_GPUHASH_FNV1A_64:
        h = NC_FNV64_INIT32;
        for (uint64_t i = 0; i < len; i++) h = nc_fnv1a_64_step(h, k[i]);
        return h;
    case NC_GPUHASH_FNV1_32:
        h = NC_FNV32_INIT;
        for (uint64_t i = 0; i < len; i++) h = nc_fnv1_32_step(h, k[i]);
        return h;
    case NC_GPUHASH_FNV1A_32:
        h = NC_FNV32_INIT;
        for (uint64_t i = 0; i < len; i++) h = nc_fnv1a_32_step(h, k[i]);
        return h;
    case NC_GPUHASH_HSIEH: return nc_key_words(0, k, len);
    case NC_GPUHASH_MURMUR: return nc_key_words(1, k, len);
    case NC_GPUHASH_JENKINS: return nc_key_jenkins(k, len);
    default: return 0;
    }
}

#endif
