/*
 * Step functions of the 12 twemproxy key hashes, shared by the host per-key
 * symbols (nc_hashkit_keys.c, gcc) and the gfx950 kernels
 * (nc_gpuhash_kernels.hip, hipcc). Everything is 32-bit integer arithmetic on
 * little-endian words; the loops that feed bytes/words live with the callers.
 *
 * Semantics follow /root/reference/src/hashkit (file:line per function);
 * SURVEY.md Appendix B lists the quirks reproduced here.
 */
#ifndef NC_HASH_ALGO_H
#define NC_HASH_ALGO_H

#include <stdint.h>

#if defined(__HIPCC__)
#define NC_HD static inline __host__ __device__ __attribute__((always_inline))
#else
#define NC_HD static inline __attribute__((always_inline))
#endif

/* signed-char promotion: (uint32_t)key[i] with x86-64's signed char. */
NC_HD uint32_t nc_sx8(uint32_t b) { return (uint32_t)(int32_t)(int8_t)(uint8_t)b; }
NC_HD uint32_t nc_rotl(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }

/* ---- FNV (src/hashkit/nc_fnv.c) ----
 * fnv1_64 keeps a 64-bit state but only its low 32 bits are returned, and the
 * low 32 bits of a product mod 2^64 depend only on the low 32 bits of the
 * factors, so the 64-bit form reduces to 32-bit arithmetic with the constants
 * truncated — which is literally what fnv1a_64 does (:42, :48). */
#define NC_FNV64_INIT32 0x84222325u   /* (uint32_t)0xcbf29ce484222325 */
#define NC_FNV64_PRIME32 0x000001b3u  /* (uint32_t)0x100000001b3 */
#define NC_FNV32_INIT 2166136261u
#define NC_FNV32_PRIME 16777619u

NC_HD uint32_t nc_fnv1_64_step(uint32_t h, uint32_t b) { return (h * NC_FNV64_PRIME32) ^ nc_sx8(b); }  /* :32-33 */
NC_HD uint32_t nc_fnv1a_64_step(uint32_t h, uint32_t b) { return (h ^ nc_sx8(b)) * NC_FNV64_PRIME32; } /* :46-48 */
NC_HD uint32_t nc_fnv1_32_step(uint32_t h, uint32_t b) { return (h * NC_FNV32_PRIME) ^ nc_sx8(b); }    /* :61-63 */
NC_HD uint32_t nc_fnv1a_32_step(uint32_t h, uint32_t b) { return (h ^ nc_sx8(b)) * NC_FNV32_PRIME; }   /* :76-78 */

/* ---- one_at_a_time (src/hashkit/nc_one_at_a_time.c:35-51) ---- */
NC_HD uint32_t nc_oaat_step(uint32_t v, uint32_t b)
{
    v += nc_sx8(b);
    v += v << 10;
    v ^= v >> 6;
    return v;
}
NC_HD uint32_t nc_oaat_final(uint32_t v)
{
    v += v << 3;
    v ^= v >> 11;
    v += v << 15;
    return v;
}

/* ---- CRC tables, generated from the polynomials ----
 * crc16: CRC-16/XMODEM (0x1021, MSB first), the table of
 * src/hashkit/nc_crc16.c:20-53; crc32/crc32a: reflected 0xEDB88320, the table
 * of src/hashkit/nc_crc32.c:27-92. */
NC_HD uint32_t nc_crc16_entry(uint32_t i)
{
    uint32_t t = i << 8;
    for (int k = 0; k < 8; k++) {
        t = (t & 0x8000u) ? ((t << 1) ^ 0x1021u) : (t << 1);
    }
    return t & 0xffffu;
}
NC_HD uint32_t nc_crc32_entry(uint32_t i)
{
    uint32_t c = i;
    for (int k = 0; k < 8; k++) {
        c = (c & 1u) ? ((c >> 1) ^ 0xEDB88320u) : (c >> 1);
    }
    return c;
}
/* crc16 state is an unmasked u32 (src/hashkit/nc_crc16.c:59-65). The index
 * masks the (sign-extended) byte, so signedness is irrelevant. */
#define NC_CRC16_IDX(crc, b) ((((crc) >> 8) ^ (b)) & 0xffu)
#define NC_CRC16_NEXT(crc, t) (((crc) << 8) ^ (t))
#define NC_CRC32_IDX(crc, b) (((crc) ^ (b)) & 0xffu)
#define NC_CRC32_NEXT(crc, t) (((crc) >> 8) ^ (t))
NC_HD uint32_t nc_crc32_final(uint32_t crc) { return ((~crc) >> 16) & 0x7fffu; } /* nc_crc32.c:108 */
NC_HD uint32_t nc_crc32a_final(uint32_t crc) { return ~crc; }                    /* nc_crc32.c:122 */

/* ---- hsieh SuperFastHash (src/hashkit/nc_hsieh.c:39-93) ----
 * w = one little-endian 4-byte word (get16bits byte form, :33-36). */
NC_HD uint32_t nc_hsieh_word(uint32_t h, uint32_t w)
{
    h += w & 0xffffu;
    uint32_t tmp = ((w >> 16) << 11) ^ h;
    h = (h << 16) ^ tmp;
    h += h >> 11;
    return h;
}
/* rem = len & 3 in 1..3, w = the remaining bytes (little-endian, rest ignored). */
NC_HD uint32_t nc_hsieh_tail(uint32_t h, uint32_t w, uint32_t rem)
{
    if (rem == 3) {
        h += w & 0xffffu;
        h ^= h << 16;
        h ^= nc_sx8(w >> 16) << 18; /* signed char, :65 */
        h += h >> 11;
    } else if (rem == 2) {
        h += w & 0xffffu;
        h ^= h << 11;
        h += h >> 17;
    } else if (rem == 1) {
        h += w & 0xffu;             /* unsigned char, :76 */
        h ^= h << 10;
        h += h >> 1;
    }
    return h;
}
NC_HD uint32_t nc_hsieh_final(uint32_t h)
{
    h ^= h << 3;
    h += h >> 5;
    h ^= h << 4;
    h += h >> 17;
    h ^= h << 25;
    h += h >> 6;
    return h;
}

/* ---- MurmurHash2 (src/hashkit/nc_murmur.c:38-99) ---- */
#define NC_MURMUR_M 0x5bd1e995u
NC_HD uint32_t nc_murmur_init(uint32_t len) { return (0xdeadbeefu * len) ^ len; } /* :45, :52 */
NC_HD uint32_t nc_murmur_word(uint32_t h, uint32_t k)
{
    k *= NC_MURMUR_M;
    k ^= k >> 24;
    k *= NC_MURMUR_M;
    h *= NC_MURMUR_M;
    return h ^ k;
}
/* rem in 0..3 tail bytes in w (unsigned, :74-87). */
NC_HD uint32_t nc_murmur_tail(uint32_t h, uint32_t w, uint32_t rem)
{
    if (rem != 0) {
        uint32_t mask = 0xffffffffu >> (32 - 8 * rem);
        h ^= w & mask;
        h *= NC_MURMUR_M;
    }
    return h;
}
NC_HD uint32_t nc_murmur_final(uint32_t h)
{
    h ^= h >> 13;
    h *= NC_MURMUR_M;
    h ^= h >> 15;
    return h;
}

/* ---- Jenkins lookup3 hashlittle (src/hashkit/nc_jenkins.c:76-230) ---- */
NC_HD uint32_t nc_jenkins_init(uint32_t len) { return 0xdeadbeefu + len + 13u; } /* :82 */
#define NC_JENKINS_MIX(a, b, c) do {                         \
    a -= c; a ^= nc_rotl(c, 4);  c += b;                     \
    b -= a; b ^= nc_rotl(a, 6);  a += c;                     \
    c -= b; c ^= nc_rotl(b, 8);  b += a;                     \
    a -= c; a ^= nc_rotl(c, 16); c += b;                     \
    b -= a; b ^= nc_rotl(a, 19); a += c;                     \
    c -= b; c ^= nc_rotl(b, 4);  b += a; } while (0)          /* :36-44 */
#define NC_JENKINS_FINAL(a, b, c) do {                       \
    c ^= b; c -= nc_rotl(b, 14);                             \
    a ^= c; a -= nc_rotl(c, 11);                             \
    b ^= a; b -= nc_rotl(a, 25);                             \
    c ^= b; c -= nc_rotl(b, 16);                             \
    a ^= c; a -= nc_rotl(c, 4);                              \
    b ^= a; b -= nc_rotl(a, 14);                             \
    c ^= b; c -= nc_rotl(b, 24); } while (0)                  /* :46-55 */

/* ---- MD5 (RFC 1321; src/hashkit/nc_md5.c:89-194) ----
 * One 64-byte block on 16 little-endian words; st[4] = A, B, C, D. */
#define NC_MD5_F(x, y, z) ((z) ^ ((x) & ((y) ^ (z))))
#define NC_MD5_G(x, y, z) ((y) ^ ((z) & ((x) ^ (y))))
#define NC_MD5_H(x, y, z) ((x) ^ (y) ^ (z))
#define NC_MD5_I(x, y, z) ((y) ^ ((x) | ~(z)))
#define NC_MD5_STEP(f, a, b, c, d, x, t, s) do { \
    (a) += f((b), (c), (d)) + (x) + (t);         \
    (a) = nc_rotl((a), (s));                     \
    (a) += (b); } while (0)

/* The 64 steps: (round function, a, b, c, d, message word, constant, shift). */
#define NC_MD5_ROUNDS(S) \
    S(NC_MD5_F, a, b, c, d, 0, 0xd76aa478u, 7) \
    S(NC_MD5_F, d, a, b, c, 1, 0xe8c7b756u, 12) \
    S(NC_MD5_F, c, d, a, b, 2, 0x242070dbu, 17) \
    S(NC_MD5_F, b, c, d, a, 3, 0xc1bdceeeu, 22) \
    S(NC_MD5_F, a, b, c, d, 4, 0xf57c0fafu, 7) \
    S(NC_MD5_F, d, a, b, c, 5, 0x4787c62au, 12) \
    S(NC_MD5_F, c, d, a, b, 6, 0xa8304613u, 17) \
    S(NC_MD5_F, b, c, d, a, 7, 0xfd469501u, 22) \
    S(NC_MD5_F, a, b, c, d, 8, 0x698098d8u, 7) \
    S(NC_MD5_F, d, a, b, c, 9, 0x8b44f7afu, 12) \
    S(NC_MD5_F, c, d, a, b, 10, 0xffff5bb1u, 17) \
    S(NC_MD5_F, b, c, d, a, 11, 0x895cd7beu, 22) \
    S(NC_MD5_F, a, b, c, d, 12, 0x6b901122u, 7) \
    S(NC_MD5_F, d, a, b, c, 13, 0xfd987193u, 12) \
    S(NC_MD5_F, c, d, a, b, 14, 0xa679438eu, 17) \
    S(NC_MD5_F, b, c, d, a, 15, 0x49b40821u, 22) \
    S(NC_MD5_G, a, b, c, d, 1, 0xf61e2562u, 5) \
    S(NC_MD5_G, d, a, b, c, 6, 0xc040b340u, 9) \
    S(NC_MD5_G, c, d, a, b, 11, 0x265e5a51u, 14) \
    S(NC_MD5_G, b, c, d, a, 0, 0xe9b6c7aau, 20) \
    S(NC_MD5_G, a, b, c, d, 5, 0xd62f105du, 5) \
    S(NC_MD5_G, d, a, b, c, 10, 0x02441453u, 9) \
    S(NC_MD5_G, c, d, a, b, 15, 0xd8a1e681u, 14) \
    S(NC_MD5_G, b, c, d, a, 4, 0xe7d3fbc8u, 20) \
    S(NC_MD5_G, a, b, c, d, 9, 0x21e1cde6u, 5) \
    S(NC_MD5_G, d, a, b, c, 14, 0xc33707d6u, 9) \
    S(NC_MD5_G, c, d, a, b, 3, 0xf4d50d87u, 14) \
    S(NC_MD5_G, b, c, d, a, 8, 0x455a14edu, 20) \
    S(NC_MD5_G, a, b, c, d, 13, 0xa9e3e905u, 5) \
    S(NC_MD5_G, d, a, b, c, 2, 0xfcefa3f8u, 9) \
    S(NC_MD5_G, c, d, a, b, 7, 0x676f02d9u, 14) \
    S(NC_MD5_G, b, c, d, a, 12, 0x8d2a4c8au, 20) \
    S(NC_MD5_H, a, b, c, d, 5, 0xfffa3942u, 4) \
    S(NC_MD5_H, d, a, b, c, 8, 0x8771f681u, 11) \
    S(NC_MD5_H, c, d, a, b, 11, 0x6d9d6122u, 16) \
    S(NC_MD5_H, b, c, d, a, 14, 0xfde5380cu, 23) \
    S(NC_MD5_H, a, b, c, d, 1, 0xa4beea44u, 4) \
    S(NC_MD5_H, d, a, b, c, 4, 0x4bdecfa9u, 11) \
    S(NC_MD5_H, c, d, a, b, 7, 0xf6bb4b60u, 16) \
    S(NC_MD5_H, b, c, d, a, 10, 0xbebfbc70u, 23) \
    S(NC_MD5_H, a, b, c, d, 13, 0x289b7ec6u, 4) \
    S(NC_MD5_H, d, a, b, c, 0, 0xeaa127fau, 11) \
    S(NC_MD5_H, c, d, a, b, 3, 0xd4ef3085u, 16) \
    S(NC_MD5_H, b, c, d, a, 6, 0x04881d05u, 23) \
    S(NC_MD5_H, a, b, c, d, 9, 0xd9d4d039u, 4) \
    S(NC_MD5_H, d, a, b, c, 12, 0xe6db99e5u, 11) \
    S(NC_MD5_H, c, d, a, b, 15, 0x1fa27cf8u, 16) \
    S(NC_MD5_H, b, c, d, a, 2, 0xc4ac5665u, 23) \
    S(NC_MD5_I, a, b, c, d, 0, 0xf4292244u, 6) \
    S(NC_MD5_I, d, a, b, c, 7, 0x432aff97u, 10) \
    S(NC_MD5_I, c, d, a, b, 14, 0xab9423a7u, 15) \
    S(NC_MD5_I, b, c, d, a, 5, 0xfc93a039u, 21) \
    S(NC_MD5_I, a, b, c, d, 12, 0x655b59c3u, 6) \
    S(NC_MD5_I, d, a, b, c, 3, 0x8f0ccc92u, 10) \
    S(NC_MD5_I, c, d, a, b, 10, 0xffeff47du, 15) \
    S(NC_MD5_I, b, c, d, a, 1, 0x85845dd1u, 21) \
    S(NC_MD5_I, a, b, c, d, 8, 0x6fa87e4fu, 6) \
    S(NC_MD5_I, d, a, b, c, 15, 0xfe2ce6e0u, 10) \
    S(NC_MD5_I, c, d, a, b, 6, 0xa3014314u, 15) \
    S(NC_MD5_I, b, c, d, a, 13, 0x4e0811a1u, 21) \
    S(NC_MD5_I, a, b, c, d, 4, 0xf7537e82u, 6) \
    S(NC_MD5_I, d, a, b, c, 11, 0xbd3af235u, 10) \
    S(NC_MD5_I, c, d, a, b, 2, 0x2ad7d2bbu, 15) \
    S(NC_MD5_I, b, c, d, a, 9, 0xeb86d391u, 21)

#define NC_MD5_S1(f, a, b, c, d, k, t, s) NC_MD5_STEP(f, a, b, c, d, w[k], t, s);
NC_HD void nc_md5_block(uint32_t st[4], const uint32_t w[16])
{
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    NC_MD5_ROUNDS(NC_MD5_S1)
    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
}

/* Two independent blocks with their steps alternating, so the two
 * dependency chains overlap on an in-order core (one lane, two keys). */
#define NC_MD5_S2(f, a, b, c, d, k, t, s) \
    NC_MD5_STEP(f, a##0, b##0, c##0, d##0, w0[k], t, s); NC_MD5_STEP(f, a##1, b##1, c##1, d##1, w1[k], t, s);
NC_HD void nc_md5_block2(uint32_t s0[4], const uint32_t w0[16], uint32_t s1[4], const uint32_t w1[16])
{
    uint32_t a0 = s0[0], b0 = s0[1], c0 = s0[2], d0 = s0[3];
    uint32_t a1 = s1[0], b1 = s1[1], c1 = s1[2], d1 = s1[3];
    NC_MD5_ROUNDS(NC_MD5_S2)
    s0[0] += a0;
    s0[1] += b0;
    s0[2] += c0;
    s0[3] += d0;
    s1[0] += a1;
    s1[1] += b1;
    s1[2] += c1;
    s1[3] += d1;
}

#define NC_MD5_A0 0x67452301u
#define NC_MD5_B0 0xefcdab89u
#define NC_MD5_C0 0x98badcfeu
#define NC_MD5_D0 0x10325476u

/* Word t (0..15) of the final padded block(s): `raw` holds message bytes
 * [4t, 4t+4) of this block where they exist, rem = message bytes left in the
 * block (0..63). Appends 0x80 after the message, zero after that
 * (src/hashkit/nc_md5.c:249-262). */
NC_HD uint32_t nc_md5_pad_word(uint32_t raw, uint32_t t, uint32_t rem)
{
    uint32_t lo = 4u * t;
    if (lo + 4u <= rem) return raw;
    if (lo >= rem + 1u) return 0u;
    uint32_t nb = rem - lo;                       /* 0..3 message bytes in this word */
    uint32_t keep = nb ? (raw & (0xffffffffu >> (32u - 8u * nb))) : 0u;
    return keep | (0x80u << (8u * nb));
}

#endif /* NC_HASH_ALGO_H */
