/*
 * The direct pipeline's C3 memory pattern (per-lane 2 x 16-byte key loads at
 * a 32-byte lane stride, 2 x 4-byte offset loads, one 4-byte store per key;
 * tools/probes/direct_pattern.hip mode 2), no hash, at fewer resident waves
 * per CU with more tiles in flight per wave: is the read/write mix of 32
 * waves per CU the limit, as the line-image probe found for long keys
 * (6.2 TB/s at 8 waves per CU, 5.2-5.8 at 20)?
 *
 *   tools/probes/direct_depth [iters]      (one JSON line per shape)
 */
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <type_traits>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                             \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

template <int WPB, int DEPTH>
__global__ __launch_bounds__(64 * WPB) void pattern(const uint8_t *__restrict__ keys, const uint64_t *__restrict__ off,
                                                    uint32_t *__restrict__ out, uint32_t ntiles)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = blockIdx.x * WPB + (threadIdx.x >> 6);
    const uint32_t W = gridDim.x * WPB;
    const uint32_t n = w < ntiles ? (ntiles - w + W - 1u) / W : 0u; /* this wave's tiles */
    if (n == 0u) return;
    u32x4 a[DEPTH][2];
    uint32_t s[DEPTH], e[DEPTH];
    auto load = [&](uint32_t j, int q) __attribute__((always_inline)) {
        const uint32_t tile = w + (j < n ? j : n - 1u) * W;
        const uint32_t k = tile * 64u + lane;
        const u32x4 *p = reinterpret_cast<const u32x4 *>(keys + (uint64_t)k * 32u);
        a[q][0] = p[0];
        a[q][1] = p[1];
        const uint32_t *o32 = reinterpret_cast<const uint32_t *>(off);
        s[q] = __builtin_nontemporal_load(o32 + 2u * k);
        e[q] = __builtin_nontemporal_load(o32 + 2u * k + 2u);
    };
#pragma unroll
    for (int q = 0; q < DEPTH - 1; q++) load((uint32_t)q, q);
    for (uint32_t j0 = 0; j0 < n; j0 += DEPTH) {
#pragma unroll
        for (int q = 0; q < DEPTH; q++) {
            const uint32_t j = j0 + (uint32_t)q;
            if (j >= n) break;
            load(j + DEPTH - 1u, (q + DEPTH - 1) % DEPTH);
            const uint32_t h = a[q][0].x ^ a[q][0].y ^ a[q][0].z ^ a[q][0].w ^ a[q][1].x ^ a[q][1].y ^ a[q][1].z ^
                               a[q][1].w ^ s[q] ^ e[q];
            __builtin_nontemporal_store(h, out + (w + j * W) * 64u + lane);
        }
    }
}

template <int WPB, int DEPTH>
float run(const uint8_t *keys, const uint64_t *off, uint32_t *out, uint32_t ntiles, uint32_t grid, uint32_t pad,
          int iters, int *per_cu)
{
    auto k = pattern<WPB, DEPTH>;
    if (pad > 65536) CK(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pad));
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, k, 64 * WPB, pad));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; i++) hipLaunchKernelGGL(k, dim3(grid), dim3(64 * WPB), pad, 0, keys, off, out, ntiles);
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < iters; i++) hipLaunchKernelGGL(k, dim3(grid), dim3(64 * WPB), pad, 0, keys, off, out, ntiles);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / iters;
}

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 20;
    const uint64_t n = 1ull << 26;
    const uint32_t ntiles = (uint32_t)(n / 64u);
    uint8_t *keys;
    uint64_t *off;
    uint32_t *out;
    CK(hipMalloc(&keys, n * 32u + 64u));
    CK(hipMalloc(&off, (n + 1u) * 8u));
    CK(hipMalloc(&out, n * 4u));
    CK(hipMemset(keys, 1, n * 32u + 64u));
    CK(hipMemset(off, 0, (n + 1u) * 8u));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    struct Shape {
        int wpb, depth;
        uint32_t pad;
        uint32_t tiles_per_wave; /* 0: a persistent grid (every resident slot once) */
    } shapes[] = {{16, 2, 0, 32}, {16, 2, 0, 0}, {16, 3, 0, 0}, {16, 2, 90000, 0}, {16, 3, 90000, 0},
                  {16, 4, 90000, 0}, {8, 2, 90000, 0}, {8, 3, 90000, 0}, {8, 4, 90000, 0}, {8, 3, 90000, 16},
                  {8, 3, 90000, 32}, {8, 4, 60000, 0}, {4, 3, 70000, 0}, {4, 4, 40000, 0}};
    for (const Shape &sh : shapes) {
        int per_cu = 0;
        uint32_t grid;
        float ms = 0;
        auto go = [&](auto wpb_c, auto depth_c) {
            constexpr int WPB = decltype(wpb_c)::value, DEPTH = decltype(depth_c)::value;
            int occ = 0;
            CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, pattern<WPB, DEPTH>, 64 * WPB, sh.pad));
            if (sh.pad > 65536) occ = 1;
            grid = sh.tiles_per_wave ? (ntiles + WPB * sh.tiles_per_wave - 1u) / (WPB * sh.tiles_per_wave)
                                     : (uint32_t)(cus * (occ > 0 ? occ : 1));
            ms = run<WPB, DEPTH>(keys, off, out, ntiles, grid, sh.pad, iters, &per_cu);
        };
        if (sh.wpb == 16 && sh.depth == 2) go(std::integral_constant<int, 16>{}, std::integral_constant<int, 2>{});
        else if (sh.wpb == 16 && sh.depth == 3) go(std::integral_constant<int, 16>{}, std::integral_constant<int, 3>{});
        else if (sh.wpb == 16) go(std::integral_constant<int, 16>{}, std::integral_constant<int, 4>{});
        else if (sh.wpb == 8 && sh.depth == 2) go(std::integral_constant<int, 8>{}, std::integral_constant<int, 2>{});
        else if (sh.wpb == 8 && sh.depth == 3) go(std::integral_constant<int, 8>{}, std::integral_constant<int, 3>{});
        else if (sh.wpb == 4 && sh.depth == 3) go(std::integral_constant<int, 4>{}, std::integral_constant<int, 3>{});
        else if (sh.wpb == 8) go(std::integral_constant<int, 8>{}, std::integral_constant<int, 4>{});
        else go(std::integral_constant<int, 4>{}, std::integral_constant<int, 4>{});
        const double alg = n * 44.0;
        printf("{\"probe\": \"direct_depth\", \"waves_per_wg\": %d, \"tiles_in_flight\": %d, \"lds_pad\": %u, "
               "\"wg_per_cu\": %d, \"grid\": %u, \"ms\": %.4f, \"gb_s\": %.1f, \"c3_alg_frac\": %.4f}\n",
               sh.wpb, sh.depth - 1, sh.pad, per_cu, grid, ms, alg / ms / 1e6, alg / ms / 1e6 / 8000.0);
        fflush(stdout);
    }
    return 0;
}
