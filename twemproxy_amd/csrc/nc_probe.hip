/* STREAM-style HBM read probe (include/nc_gpuhash_probe.h). */
#include <hip/hip_runtime.h>

#include <errno.h>

#include "nc_gpuhash_probe.h"

namespace {

constexpr int kProbeBlock = 256;
constexpr int kProbeUnroll = 8;

/* Each workgroup streams contiguous 16-byte pieces, kProbeUnroll loads in
 * flight per lane, and xors everything into one word so nothing is dead.
 * WR (the mix probe): each lane also stores the xor of its kProbeUnroll pieces,
 * 16 bytes written per 128 read (a hash kernel's output-to-input ratio),
 * coalesced and streaming. */
template <bool NT, bool WR = false, bool WNT = true>
__global__ __launch_bounds__(kProbeBlock) void probe_read_kernel(const uint4 *__restrict__ p, uint64_t n16,
                                                                 uint32_t *__restrict__ sink,
                                                                 uint4 *__restrict__ wout = nullptr)
{
    uint32_t acc = 0;
    const uint64_t step = (uint64_t)gridDim.x * kProbeBlock * kProbeUnroll;
    for (uint64_t base = (uint64_t)blockIdx.x * kProbeBlock * kProbeUnroll + threadIdx.x; base < n16;
         base += step) {
        uint4 v[kProbeUnroll];
#pragma unroll
        for (int u = 0; u < kProbeUnroll; u++) {
            const uint64_t i = base + (uint64_t)u * kProbeBlock;
            if constexpr (NT) {
                typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                v4u x = {0u, 0u, 0u, 0u};
                if (i < n16) x = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(p) + i);
                v[u] = make_uint4(x.x, x.y, x.z, x.w);
            }
            else v[u] = i < n16 ? p[i] : make_uint4(0, 0, 0, 0);
        }
        if constexpr (WR) {
            uint4 x = v[0];
#pragma unroll
            for (int u = 1; u < kProbeUnroll; u++) x = make_uint4(x.x ^ v[u].x, x.y ^ v[u].y, x.z ^ v[u].z, x.w ^ v[u].w);
            typedef uint32_t v4u __attribute__((ext_vector_type(4)));
            const v4u y = {x.x, x.y, x.z, x.w};
            v4u *dst = reinterpret_cast<v4u *>(wout) + (base - threadIdx.x) / kProbeUnroll + threadIdx.x;
            if constexpr (WNT) __builtin_nontemporal_store(y, dst);
            else *dst = y;
        } else {
#pragma unroll
            for (int u = 0; u < kProbeUnroll; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
        }
    }
    for (int d = 32; d > 0; d >>= 1) acc ^= __shfl_xor(acc, d);
    if ((threadIdx.x & 63u) == 0) atomicXor(&sink[blockIdx.x], acc);
}

template <bool NT, bool WR = false, bool WNT = true>
rstatus_t probe_read(const void *d_buf, uint64_t bytes, uint32_t *d_sink, void *stream, int iters, float *avg_ms,
                     void *d_wout = nullptr)
{
    if (d_buf == nullptr || d_sink == nullptr || avg_ms == nullptr || iters <= 0 || (bytes & 15u) ||
        (WR && d_wout == nullptr)) {
        errno = EINVAL;
        return NC_ERROR;
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
        errno = ENODEV;
        return NC_ERROR;
    }
    unsigned grid = (unsigned)cus * 8u;
    if (grid > 65536u) grid = 65536u;
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess) {
        errno = ENODEV;
        return NC_ERROR;
    }
    if (hipEventCreate(&b) != hipSuccess) {
        (void)hipEventDestroy(a);
        errno = ENODEV;
        return NC_ERROR;
    }
    hipLaunchKernelGGL((probe_read_kernel<NT, WR, WNT>), dim3(grid), dim3(kProbeBlock), 0, st, (const uint4 *)d_buf,
                       bytes / 16, d_sink, (uint4 *)d_wout);
    (void)hipEventRecord(a, st);
    for (int i = 0; i < iters; i++) {
        hipLaunchKernelGGL((probe_read_kernel<NT, WR, WNT>), dim3(grid), dim3(kProbeBlock), 0, st, (const uint4 *)d_buf,
                           bytes / 16, d_sink, (uint4 *)d_wout);
    }
    (void)hipEventRecord(b, st);
    rstatus_t rc = NC_OK;
    float ms = 0.f;
    if (hipGetLastError() != hipSuccess || hipEventSynchronize(b) != hipSuccess ||
        hipEventElapsedTime(&ms, a, b) != hipSuccess) {
        errno = EIO;
        rc = NC_ERROR;
    } else {
        *avg_ms = ms / (float)iters;
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return rc;
}

} // namespace

extern "C" rstatus_t nc_gpuhash_probe_read(const void *d_buf, uint64_t bytes, uint32_t *d_sink, void *stream,
                                           int iters, float *avg_ms)
{
    return probe_read<false>(d_buf, bytes, d_sink, stream, iters, avg_ms);
}

extern "C" rstatus_t nc_gpuhash_probe_read_nt(const void *d_buf, uint64_t bytes, uint32_t *d_sink, void *stream,
                                              int iters, float *avg_ms)
{
    return probe_read<true>(d_buf, bytes, d_sink, stream, iters, avg_ms);
}

extern "C" rstatus_t nc_gpuhash_probe_mix(const void *d_buf, uint64_t bytes, void *d_wout, uint64_t wout_bytes,
                                         uint32_t *d_sink, void *stream, int policy, int iters, float *avg_ms)
{
    /* the last step's pieces land at most one workgroup step past bytes / 8 */
    const uint64_t need = ((bytes / 16 + (uint64_t)kProbeBlock * kProbeUnroll - 1) /
                           ((uint64_t)kProbeBlock * kProbeUnroll)) * kProbeBlock * 16u;
    if (wout_bytes < need) {
        errno = EINVAL;
        return NC_ERROR;
    }
    switch (policy) {
    case 0: return probe_read<true, true, true>(d_buf, bytes, d_sink, stream, iters, avg_ms, d_wout);
    case 1: return probe_read<false, true, true>(d_buf, bytes, d_sink, stream, iters, avg_ms, d_wout);
    case 2: return probe_read<true, true, false>(d_buf, bytes, d_sink, stream, iters, avg_ms, d_wout);
    case 3: return probe_read<false, true, false>(d_buf, bytes, d_sink, stream, iters, avg_ms, d_wout);
    default: errno = EINVAL; return NC_ERROR;
    }
}
