/* Host form of the synthetic key generator (include/nc_gpuhash_synth.h). */
#include <errno.h>
#include <math.h>
#include <string.h>

#include "nc_internal.h"

rstatus_t nc_synth_make_plan(const struct nc_synth_spec *spec, struct nc_synth_plan *plan)
{
    if (spec == NULL || plan == NULL) {
        errno = EINVAL;
        return NC_ERROR;
    }
    memset(plan, 0, sizeof(*plan));
    plan->s_len = nc_stream_len(spec->seed);
    plan->s_key = nc_stream_key(spec->seed);
    plan->dist = spec->len_dist;
    plan->a = spec->len_a;
    plan->b = spec->len_b;
    plan->charset = spec->charset ? 1 : 0;
    switch (spec->len_dist) {
    case NC_SYNTH_FIXED:
        if (spec->len_a > NC_SYNTH_MAX_KEY) goto bad;
        break;
    case NC_SYNTH_ZIPF: {
        /* len = a - 1 + r, r in [1, b], P(r) ~ r^-s. */
        if (spec->len_a < 1 || spec->len_b < 1 || spec->len_b > NC_SYNTH_MAX_ZIPF ||
            spec->len_a - 1 + spec->len_b > NC_SYNTH_MAX_KEY || !(spec->zipf_s >= 0.0)) {
            goto bad;
        }
        double h[NC_SYNTH_MAX_ZIPF + 1];
        h[0] = 0.0;
        for (uint32_t r = 1; r <= spec->len_b; r++) {
            h[r] = h[r - 1] + pow((double)r, -spec->zipf_s);
        }
        for (uint32_t k = 0; k + 1 < spec->len_b; k++) {
            plan->thr[k] = (uint64_t)floor(h[k + 1] / h[spec->len_b] * 4294967296.0);
        }
        break;
    }
    case NC_SYNTH_UNIFORM:
        if (spec->len_b < spec->len_a || spec->len_b > NC_SYNTH_MAX_KEY) goto bad;
        break;
    default:
        goto bad;
    }
    return NC_OK;
bad:
    errno = EINVAL;
    return NC_ERROR;
}

rstatus_t nc_synth_lengths_host(const struct nc_synth_spec *spec, uint64_t first, uint64_t n,
                                uint32_t *lens)
{
    struct nc_synth_plan p;
    if (nc_synth_make_plan(spec, &p) != NC_OK) return NC_ERROR;
    for (uint64_t i = 0; i < n; i++) {
        lens[i] = nc_synth_len(&p, first + i);
    }
    return NC_OK;
}

rstatus_t nc_synth_offsets_host(const struct nc_synth_spec *spec, uint64_t first, uint64_t n,
                                uint64_t *offsets)
{
    struct nc_synth_plan p;
    if (nc_synth_make_plan(spec, &p) != NC_OK) return NC_ERROR;
    offsets[0] = 0;
    for (uint64_t i = 0; i < n; i++) {
        offsets[i + 1] = offsets[i] + nc_synth_len(&p, first + i);
    }
    return NC_OK;
}

rstatus_t nc_synth_fill_host(const struct nc_synth_spec *spec, uint64_t first, uint64_t n,
                             const uint64_t *offsets, uint8_t *keys)
{
    struct nc_synth_plan p;
    if (nc_synth_make_plan(spec, &p) != NC_OK) return NC_ERROR;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t s = offsets[i], e = offsets[i + 1];
        uint64_t key = first + i;
        uint32_t len = (uint32_t)(e - s);
        uint32_t j = 0;
        /* eight bytes per generator word */
        for (; j + 8 <= len; j += 8) {
            uint64_t w = nc_rnd(p.s_key, key * 4096u + (j >> 3));
            for (uint32_t b = 0; b < 8; b++) {
                uint32_t v = (uint32_t)(w >> (8 * b)) & 0xffu;
                keys[s + j + b] = (uint8_t)(p.charset ? 0x21u + v % 94u : v);
            }
        }
        for (; j < len; j++) {
            keys[s + j] = nc_synth_byte(&p, key, j);
        }
    }
    return NC_OK;
}
