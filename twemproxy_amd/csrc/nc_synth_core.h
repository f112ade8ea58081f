/*
 * Counter-based key generator shared by the host (nc_synth.c) and device
 * (nc_synth_kernels.hip) forms; the spec is in include/nc_gpuhash_synth.h.
 */
#ifndef NC_SYNTH_CORE_H
#define NC_SYNTH_CORE_H

#include <stdint.h>
#include "nc_hash_algo.h" /* NC_HD */

#define NC_SYNTH_GAMMA 0x9E3779B97F4A7C15ull

NC_HD uint64_t nc_mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

NC_HD uint64_t nc_rnd(uint64_t stream, uint64_t ctr) { return nc_mix64(stream + (ctr + 1u) * NC_SYNTH_GAMMA); }
NC_HD uint64_t nc_stream_len(uint64_t seed) { return nc_mix64(seed ^ 0x6c656e67746873ull); }
NC_HD uint64_t nc_stream_key(uint64_t seed) { return nc_mix64(seed ^ 0x6b657962797465ull); }

/* Resolved generator parameters (thresholds precomputed on the host). */
struct nc_synth_plan {
    uint64_t s_len, s_key;
    int32_t dist;
    uint32_t a, b;
    int32_t charset;
    uint64_t thr[64]; /* ZIPF: r = 1 + #{k : thr[k] <= u}, k < b - 1 */
};

NC_HD uint32_t nc_synth_len(const struct nc_synth_plan *p, uint64_t i)
{
    if (p->dist == 0) return p->a;
    uint64_t r = nc_rnd(p->s_len, i);
    if (p->dist == 1) {
        uint64_t u = r >> 32;
        uint32_t k = 0;
        while (k + 1 < p->b && p->thr[k] <= u) k++;
        return p->a - 1u + (k + 1u);
    }
    return p->a + (uint32_t)(r % (uint64_t)(p->b - p->a + 1u));
}

NC_HD uint8_t nc_synth_byte(const struct nc_synth_plan *p, uint64_t i, uint32_t j)
{
    uint64_t w = nc_rnd(p->s_key, i * 4096u + (j >> 3));
    uint32_t b = (uint32_t)(w >> (8u * (j & 7u))) & 0xffu;
    return (uint8_t)(p->charset ? 0x21u + b % 94u : b);
}

#endif
