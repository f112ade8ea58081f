/*
 * ketama_update on the device: the continuum of a pool,
 * built where nc_gpuhash_server_idx_device reads it.
 *
 * Reference: ketama_update, /root/reference/src/hashkit/nc_ketama.c:58-219.
 *   - live servers only (auto_eject_hosts and next_retry, :80-102), total
 *     weight over live servers (:104-107);
 *   - points per server in float arithmetic exactly as written (:159-160);
 *   - one "<name>-<i>" string per 4 points (:169-181, KETAMA_MAX_HOSTLEN 273,
 *     truncated to 272 bytes);
 *   - 4 points per string: the 4 little-endian words of its md5 digest
 *     (ketama_hash :31-41, alignment x = 0..3);
 *   - sorted by value (qsort with ketama_item_cmp, :197-198). glibc's qsort
 *     is a merge sort here, so equal values keep their build order; the radix
 *     sort below is stable too.
 *
 * The host side (weights, strings: a few KB) is plain C++; the device side is
 * one md5-per-string kernel, a stable radix sort of (value, index) pairs
 * (hipCUB) and an interleave into struct continuum {index, value}.
 */
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <errno.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "nc_gpuhash.h"
#include "nc_hash_algo.h"

namespace {

constexpr uint32_t kPointsPerServer = 160; /* KETAMA_POINTS_PER_SERVER, nc_ketama.c:26 */
constexpr uint32_t kPointsPerHash = 4;
constexpr size_t kMaxHostLen = 273;        /* KETAMA_MAX_HOSTLEN, nc_ketama.c:27 */

/* one thread per string: md5 (RFC 1321 padding, nc_md5.c:245-274) of
 * str[off[s] .. off[s+1]), then its 4 digest words as 4 points */
__global__ __launch_bounds__(256) void nc_ketama_points_kernel(const uint8_t *__restrict__ str,
                                                               const uint32_t *__restrict__ off,
                                                               const uint32_t *__restrict__ sidx, uint32_t nstr,
                                                               uint32_t *__restrict__ vals, uint32_t *__restrict__ idx)
{
    const uint32_t s = blockIdx.x * 256u + threadIdx.x;
    if (s >= nstr) return;
    const uint8_t *p = str + off[s];
    const uint32_t len = off[s + 1] - off[s];
    uint32_t st[4] = {NC_MD5_A0, NC_MD5_B0, NC_MD5_C0, NC_MD5_D0};
    const uint32_t nblk = (len + 8u) / 64u + 1u;
    for (uint32_t b = 0; b < nblk; b++) {
        uint32_t w[16];
        for (uint32_t t = 0; t < 16u; t++) {
            uint32_t v = 0;
            for (uint32_t k = 0; k < 4u; k++) {
                const uint32_t i = 64u * b + 4u * t + k;
                const uint32_t byte = i < len ? p[i] : (i == len ? 0x80u : 0u);
                v |= byte << (8u * k);
            }
            w[t] = v;
        }
        if (b == nblk - 1u) {
            w[14] = len << 3;
            w[15] = 0u;
        }
        nc_md5_block(st, w);
    }
    for (uint32_t x = 0; x < kPointsPerHash; x++) {
        vals[kPointsPerHash * s + x] = st[x]; /* ketama_hash(host, hostlen, x), nc_ketama.c:36-40 */
        idx[kPointsPerHash * s + x] = sidx[s];
    }
}

__global__ __launch_bounds__(256) void nc_ketama_interleave_kernel(const uint32_t *__restrict__ vals,
                                                                   const uint32_t *__restrict__ idx, uint32_t n,
                                                                   nc_gpuhash_continuum *__restrict__ cont)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < n) {
        cont[i].index = idx[i];
        cont[i].value = vals[i];
    }
}

rstatus_t fail(int err, rstatus_t rc = NC_ERROR)
{
    errno = err;
    return rc;
}

struct DevBufs {
    void *p[8] = {};
    ~DevBufs()
    {
        for (void *q : p)
            if (q) (void)hipFree(q);
    }
};

} // namespace

extern "C" rstatus_t nc_gpuhash_ketama_build_device(const char *const *names, const uint32_t *name_lens,
                                                    const uint32_t *weights, const uint8_t *live, uint32_t nserver,
                                                    struct nc_gpuhash_continuum *d_continuum, uint32_t cap,
                                                    uint32_t *ncontinuum, void *stream)
{
    if (ncontinuum == nullptr || (nserver > 0 && (names == nullptr || name_lens == nullptr || weights == nullptr)))
        return fail(EINVAL);
    *ncontinuum = 0;
    uint32_t nlive = 0, total_weight = 0;
    for (uint32_t s = 0; s < nserver; s++) {
        if (weights[s] == 0) return fail(EINVAL); /* ASSERT(server->weight > 0), nc_ketama.c:100 */
        if (live != nullptr && !live[s]) continue;
        nlive++;
        total_weight += weights[s];
    }
    if (nlive == 0) return NC_OK; /* "no live servers" (nc_ketama.c:111-116) */

    /* host: the strings, server-major in build order (nc_ketama.c:150-189) */
    std::vector<uint8_t> bytes;
    std::vector<uint32_t> off(1, 0u), sidx;
    for (uint32_t s = 0; s < nserver; s++) {
        if (live != nullptr && !live[s]) continue;
        float pct = (float)weights[s] / (float)total_weight;
        uint32_t pointer_per_server =
            (uint32_t)((floorf((float)(pct * kPointsPerServer / 4 * (float)nlive + 0.0000000001))) * 4);
        for (uint32_t pi = 1; pi <= pointer_per_server / kPointsPerHash; pi++) {
            char host[kMaxHostLen] = "";
            int hl = snprintf(host, kMaxHostLen, "%.*s-%u", (int)name_lens[s], names[s], pi - 1);
            size_t hostlen = hl < 0 ? 0u : (size_t)hl;
            if (hostlen >= kMaxHostLen) hostlen = kMaxHostLen - 1;
            bytes.insert(bytes.end(), (const uint8_t *)host, (const uint8_t *)host + hostlen);
            off.push_back((uint32_t)bytes.size());
            sidx.push_back(s);
        }
    }
    const uint32_t nstr = (uint32_t)sidx.size();
    const uint32_t npts = nstr * kPointsPerHash;
    if (npts > cap) return fail(ENOMEM, NC_ENOMEM);
    if (npts == 0) return NC_OK;
    if (d_continuum == nullptr) return fail(EINVAL);

    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    DevBufs b;
    size_t temp_bytes = 0;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                                      (uint32_t *)nullptr, (uint32_t *)nullptr, (int)npts, 0, 32, st);
    const size_t sizes[7] = {bytes.size() + 1, off.size() * 4u, sidx.size() * 4u, npts * 4u, npts * 4u,
                             npts * 4u, npts * 4u};
    for (int i = 0; i < 7 && e == hipSuccess; i++) e = hipMalloc(&b.p[i], sizes[i]);
    if (e == hipSuccess) e = hipMalloc(&b.p[7], temp_bytes ? temp_bytes : 4u);
    uint8_t *d_str = (uint8_t *)b.p[0];
    uint32_t *d_off = (uint32_t *)b.p[1], *d_sidx = (uint32_t *)b.p[2];
    uint32_t *v0 = (uint32_t *)b.p[3], *i0 = (uint32_t *)b.p[4], *v1 = (uint32_t *)b.p[5], *i1 = (uint32_t *)b.p[6];
    if (e == hipSuccess) e = hipMemcpyAsync(d_str, bytes.data(), bytes.size(), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(d_off, off.data(), off.size() * 4u, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(d_sidx, sidx.data(), sidx.size() * 4u, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(nc_ketama_points_kernel, dim3((nstr + 255u) / 256u), dim3(256), 0, st, d_str, d_off, d_sidx,
                           nstr, v0, i0);
        e = hipGetLastError();
    }
    if (e == hipSuccess)
        e = hipcub::DeviceRadixSort::SortPairs(b.p[7], temp_bytes, v0, v1, i0, i1, (int)npts, 0, 32, st);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(nc_ketama_interleave_kernel, dim3((npts + 255u) / 256u), dim3(256), 0, st, v1, i1, npts,
                           d_continuum);
        e = hipGetLastError();
    }
    /* the temporaries are freed on return: the build must have finished */
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return fail(e == hipErrorNoDevice ? ENODEV : (e == hipErrorOutOfMemory ? ENOMEM : EIO));
    *ncontinuum = npts;
    return NC_OK;
}
