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

/* The grouped C2 pipeline's traffic shape without its hash: workgroups of
 * 512 threads walk "tiles" grid-strided (a run of `run` consecutive tiles
 * per step); a tile reads `rd` contiguous bytes (nt 16-byte loads, all
 * issued before use) and its `wr` output bytes go to out + tile * wr —
 * stored right after the tile (DEFER = false: 2 KiB pieces, the kernel's
 * coalesced store) or held in LDS and stored once per run (DEFER = true:
 * run * wr contiguous bytes at once). rd a multiple of 8 KiB, wr of 16 and
 * at most 8 KiB / run. SF: the output stores' flavour — 0 nt (the
 * kernels'), 1 plain, 2 sc1, 3 sc0 sc1 (write-through). */
template <int SF>
__device__ __forceinline__ void tile_mix_store(uint32_t __attribute__((ext_vector_type(4))) y, uint4 *out, uint64_t q)
{
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    if constexpr (SF == 0) {
        __builtin_nontemporal_store(y, reinterpret_cast<v4u *>(out) + q);
    } else if constexpr (SF == 1) {
        reinterpret_cast<v4u *>(out)[q] = y;
    } else { /* a buffer store, 16 B a lane, over the uniform base (offsets < 4 GiB: the probe's outputs) */
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(y, r, (int)(q * 16u), 0, SF == 2 ? 16 : 17);
    }
}

template <bool DEFER, int SF>
__global__ __launch_bounds__(512) void probe_tile_mix_kernel(const uint4 *__restrict__ in, uint64_t ntiles, uint32_t rd,
                                                             uint32_t wr, uint32_t run, uint4 *__restrict__ out,
                                                             uint32_t *__restrict__ sink)
{
    __shared__ uint4 stage[512];
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const uint32_t t = threadIdx.x;
    const uint32_t per = rd / (16u * 512u); /* 16-B loads per thread per tile */
    const uint32_t wq = wr / 16u;           /* 16-B output pieces per tile */
    uint32_t acc = 0;
    for (uint64_t r0 = (uint64_t)blockIdx.x * run; r0 < ntiles; r0 += (uint64_t)gridDim.x * run) {
        for (uint32_t k = 0; k < run && r0 + k < ntiles; k++) {
            const uint64_t tile = r0 + k;
            const v4u *src = reinterpret_cast<const v4u *>(in) + tile * (rd / 16u);
            v4u x = {0u, 0u, 0u, 0u};
            v4u v[8];
            for (uint32_t j0 = 0; j0 < per; j0 += 8u) {
#pragma unroll
                for (uint32_t j = 0; j < 8u; j++)
                    v[j] = j0 + j < per ? __builtin_nontemporal_load(src + (j0 + j) * 512u + t) : x;
#pragma unroll
                for (uint32_t j = 0; j < 8u; j++) x ^= v[j];
            }
            const v4u y = x;
            if constexpr (DEFER) {
                if (t < wq) stage[k * wq + t] = make_uint4(y.x, y.y, y.z, y.w);
            } else {
                if (t < wq) tile_mix_store<SF>(y, out, tile * wq + t);
            }
            acc ^= y.x;
        }
        if constexpr (DEFER) {
            __syncthreads();
            const uint32_t n = (uint32_t)((ntiles - r0 < run ? ntiles - r0 : run) * wq);
            for (uint32_t i = t; i < n; i += 512u) {
                const uint4 z = stage[i];
                const v4u y = {z.x, z.y, z.z, z.w};
                tile_mix_store<SF>(y, out, r0 * wq + i);
            }
            __syncthreads();
        }
    }
    if (acc == 0x9e3779b9u) sink[blockIdx.x] = acc;
}

/* One wave: lane 0 records (s_memtime, s_memrealtime) every `gap` ticks of
 * the 100 MHz real-time clock, n samples, then exits (bounded: n * gap
 * ticks). s_memtime counts shader-clock cycles, so consecutive samples give
 * the clock this CU ran at while other kernels filled the GPU. */
__global__ __launch_bounds__(64) void clock_sampler_kernel(uint64_t *__restrict__ out, uint32_t n, uint32_t gap)
{
    if (threadIdx.x != 0u) return;
    uint64_t next = wall_clock64();
    for (uint32_t i = 0; i < n; i++) {
        uint64_t r;
        do {
            __builtin_amdgcn_s_sleep(1);
            r = wall_clock64();
        } while (r < next);
        const uint64_t c = __builtin_readcyclecounter();
        out[2u * i] = c;
        out[2u * i + 1u] = r;
        next = r + gap;
    }
}

} // namespace

extern "C" rstatus_t nc_gpuhash_probe_clock_sampler(uint64_t *d_out, uint32_t n, uint32_t gap_ticks, void *stream)
{
    if (d_out == nullptr || n == 0u || gap_ticks == 0u || (uint64_t)n * gap_ticks > 100000000ull) {
        errno = EINVAL;
        return NC_ERROR;
    }
    (void)hipGetLastError();
    hipLaunchKernelGGL(clock_sampler_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), d_out, n,
                       gap_ticks);
    if (hipGetLastError() != hipSuccess) {
        errno = EIO;
        return NC_ERROR;
    }
    return NC_OK;
}

extern "C" rstatus_t nc_gpuhash_probe_tile_mix(const void *d_buf, uint64_t bytes, void *d_out, uint64_t out_bytes,
                                              uint32_t tile_read, uint32_t tile_write, uint32_t run, uint32_t grid,
                                              int defer, uint32_t *d_sink, void *stream, int iters, float *avg_ms)
{
    if (d_buf == nullptr || d_out == nullptr || d_sink == nullptr || avg_ms == nullptr || iters <= 0 ||
        tile_read == 0u || tile_read % 8192u || tile_write % 16u || run == 0u || (uint64_t)run * tile_write > 8192u ||
        grid == 0u || grid > 65536u) {
        errno = EINVAL;
        return NC_ERROR;
    }
    const uint64_t ntiles = bytes / tile_read;
    if (ntiles * tile_write > out_bytes || (((defer >> 4) & 3) >= 2 && out_bytes > 0x7fffffffull)) {
        errno = EINVAL;
        return NC_ERROR;
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    typedef void (*mix_fn)(const uint4 *, uint64_t, uint32_t, uint32_t, uint32_t, uint4 *, uint32_t *);
    static const mix_fn kinds[2][4] = {
        {probe_tile_mix_kernel<false, 0>, probe_tile_mix_kernel<false, 1>, probe_tile_mix_kernel<false, 2>,
         probe_tile_mix_kernel<false, 3>},
        {probe_tile_mix_kernel<true, 0>, probe_tile_mix_kernel<true, 1>, probe_tile_mix_kernel<true, 2>,
         probe_tile_mix_kernel<true, 3>}};
    const mix_fn k = kinds[(defer & 1) != 0][(defer >> 4) & 3];
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
    hipLaunchKernelGGL(k, dim3(grid), dim3(512), 0, st, (const uint4 *)d_buf, ntiles, tile_read, tile_write, run,
                       (uint4 *)d_out, d_sink);
    (void)hipEventRecord(a, st);
    for (int i = 0; i < iters; i++)
        hipLaunchKernelGGL(k, dim3(grid), dim3(512), 0, st, (const uint4 *)d_buf, ntiles, tile_read, tile_write, run,
                           (uint4 *)d_out, d_sink);
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
