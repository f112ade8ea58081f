/*
 * Device form of the synthetic key generator (include/nc_gpuhash_synth.h):
 * lengths -> inclusive scan (hipcub) -> offsets, then one thread per key
 * writes its bytes. Bench/test set-up only; not on the hashing path.
 */
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <errno.h>

#include "nc_internal.h"

namespace {

__global__ void synth_len_kernel(struct nc_synth_plan plan, uint64_t first, uint64_t n, uint64_t *d_off)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) d_off[0] = 0;
    if (i < n) d_off[i + 1] = nc_synth_len(&plan, first + i);
}

__global__ void synth_fill_kernel(struct nc_synth_plan plan, uint64_t first, uint64_t n,
                                  const uint64_t *__restrict__ d_off, uint8_t *__restrict__ d_keys)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t s = d_off[i];
    const uint32_t len = (uint32_t)(d_off[i + 1] - s);
    const uint64_t key = first + i;
    uint32_t j = 0;
    for (; j + 8 <= len; j += 8) {
        const uint64_t w = nc_rnd(plan.s_key, key * 4096u + (j >> 3));
#pragma unroll
        for (uint32_t b = 0; b < 8; b++) {
            const uint32_t v = (uint32_t)(w >> (8 * b)) & 0xffu;
            d_keys[s + j + b] = (uint8_t)(plan.charset ? 0x21u + v % 94u : v);
        }
    }
    for (; j < len; j++) d_keys[s + j] = nc_synth_byte(&plan, key, j);
}

rstatus_t fail(int err)
{
    errno = err;
    return NC_ERROR;
}

} // namespace

extern "C" rstatus_t nc_synth_offsets_device(const struct nc_synth_spec *spec, uint64_t first, uint64_t n,
                                             uint64_t *d_offsets, void *stream)
{
    struct nc_synth_plan plan;
    if (nc_synth_make_plan(spec, &plan) != NC_OK || d_offsets == nullptr) return fail(EINVAL);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const uint64_t blocks = (n + 1 + 255) / 256;
    hipLaunchKernelGGL(synth_len_kernel, dim3((unsigned)blocks), dim3(256), 0, st, plan, first, n, d_offsets);
    if (hipGetLastError() != hipSuccess) return fail(ENODEV);
    if (n == 0) return NC_OK;
    size_t tmp_bytes = 0;
    if (hipcub::DeviceScan::InclusiveSum(nullptr, tmp_bytes, d_offsets + 1, d_offsets + 1, (int64_t)n, st) !=
        hipSuccess)
        return fail(EIO);
    void *tmp = nullptr;
    if (hipMalloc(&tmp, tmp_bytes) != hipSuccess) return fail(ENOMEM);
    hipError_t e = hipcub::DeviceScan::InclusiveSum(tmp, tmp_bytes, d_offsets + 1, d_offsets + 1, (int64_t)n, st);
    (void)hipStreamSynchronize(st);
    (void)hipFree(tmp);
    return e == hipSuccess ? NC_OK : fail(EIO);
}

extern "C" rstatus_t nc_synth_fill_device(const struct nc_synth_spec *spec, uint64_t first, uint64_t n,
                                          const uint64_t *d_offsets, uint8_t *d_keys, void *stream)
{
    struct nc_synth_plan plan;
    if (nc_synth_make_plan(spec, &plan) != NC_OK || d_offsets == nullptr || d_keys == nullptr)
        return fail(EINVAL);
    if (n == 0) return NC_OK;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(synth_fill_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, plan, first, n,
                       d_offsets, d_keys);
    return hipGetLastError() == hipSuccess ? NC_OK : fail(ENODEV);
}
