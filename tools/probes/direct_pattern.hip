/*
 * Which part of the direct per-lane pipeline's memory traffic limits it on
 * C3's shape (2^26 x 32-byte keys, u64 offsets, u32 outputs; DESIGN.md §5.4:
 * its no-hash build runs 0.587 ms where the wave ring hashes fnv1a_64 in
 * 0.52). The direct kernel's access pattern, piece by piece, with no hash:
 * 64-key tiles, one key per lane, 16 waves per workgroup, 32 tiles per wave
 * interleaved over the grid, the next tile's loads in flight while the
 * current one is consumed.
 *
 *   mode 0  keys only: two 16-byte loads per lane at a 32-byte lane stride
 *   mode 1  + the offsets: two 4-byte loads per lane (start, end low dwords)
 *   mode 2  + one 4-byte store per key (the direct kernel's traffic)
 *   mode 3  mode 2 with the keys as two coalesced 1 KiB wave loads
 *   mode 4  mode 2 with the offsets as one 8-byte load per lane (start) and
 *           the end from the next lane (DPP)
 *   mode 5  mode 2 with default-policy stores instead of non-temporal
 *   mode 6  mode 2 with each tile's 64 hashes stored as 16 bytes by 16 lanes
 *   mode 7  mode 6 with default-policy stores
 *
 *   tools/probes/direct_pattern [iters]      (one JSON line per mode)
 */
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                             \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

template <int MODE>
__global__ __launch_bounds__(1024) void pattern(const uint8_t *__restrict__ keys, const uint64_t *__restrict__ off,
                                                uint32_t *__restrict__ out, uint32_t ntiles, uint32_t *sink)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = blockIdx.x * 16u + (threadIdx.x >> 6);
    const uint32_t W = gridDim.x * 16u;
    uint32_t acc = 0;
    u32x4 a0, a1, b0, b1;
    uint32_t s0 = 0, e0 = 0, s1 = 0, e1 = 0;
    auto load = [&](uint32_t tile, u32x4 &x0, u32x4 &x1, uint32_t &s, uint32_t &e) __attribute__((always_inline)) {
        const uint32_t k = tile * 64u + lane;
        if constexpr (MODE == 3) {
            const u32x4 *p = reinterpret_cast<const u32x4 *>(keys + (uint64_t)tile * 2048u);
            x0 = p[lane];
            x1 = p[64 + lane];
        } else {
            const u32x4 *p = reinterpret_cast<const u32x4 *>(keys + (uint64_t)k * 32u);
            x0 = p[0];
            x1 = p[1];
        }
        if constexpr (MODE >= 1) {
            const uint32_t *o32 = reinterpret_cast<const uint32_t *>(off);
            if constexpr (MODE == 4) {
                s = __builtin_nontemporal_load(o32 + 2u * k);
                e = __shfl_down(s, 1);
            } else {
                s = __builtin_nontemporal_load(o32 + 2u * k);
                e = __builtin_nontemporal_load(o32 + 2u * k + 2u);
            }
        }
    };
    auto store = [&](uint32_t h, uint32_t tile) __attribute__((always_inline)) {
        if constexpr (MODE == 6 || MODE == 7) {
            /* lane l < 16 gathers hashes 4l .. 4l+3 */
            const uint32_t src = (lane & 15u) * 4u;
            u32x4 v;
            v.x = __shfl(h, (int)src);
            v.y = __shfl(h, (int)src + 1);
            v.z = __shfl(h, (int)src + 2);
            v.w = __shfl(h, (int)src + 3);
            u32x4 *dst = reinterpret_cast<u32x4 *>(out + tile * 64u) + lane;
            if (lane < 16u) {
                if constexpr (MODE == 6) __builtin_nontemporal_store(v, dst);
                else *dst = v;
            }
        } else if constexpr (MODE == 5) {
            out[tile * 64u + lane] = h;
        } else {
            __builtin_nontemporal_store(h, out + tile * 64u + lane);
        }
    };
    uint32_t tile = w;
    if (tile >= ntiles) return;
    load(tile, a0, a1, s0, e0);
    for (uint32_t j = 0;; j += 2) {
        const uint32_t t1 = tile + W;
        if (t1 < ntiles) load(t1, b0, b1, s1, e1);
        const uint32_t h = a0.x ^ a0.y ^ a0.z ^ a0.w ^ a1.x ^ a1.y ^ a1.z ^ a1.w ^ s0 ^ e0;
        if constexpr (MODE >= 2) store(h, tile);
        else acc ^= h;
        if (t1 >= ntiles) break;
        tile = t1;
        const uint32_t t2 = tile + W;
        if (t2 < ntiles) load(t2, a0, a1, s0, e0);
        const uint32_t h1 = b0.x ^ b0.y ^ b0.z ^ b0.w ^ b1.x ^ b1.y ^ b1.z ^ b1.w ^ s1 ^ e1;
        if constexpr (MODE >= 2) store(h1, tile);
        else acc ^= h1;
        if (t2 >= ntiles) break;
        tile = t2;
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

template <int MODE>
float run(const uint8_t *keys, const uint64_t *off, uint32_t *out, uint32_t ntiles, uint32_t *sink, int iters)
{
    const uint32_t grid = (ntiles + 16u * 32u - 1u) / (16u * 32u);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; i++) hipLaunchKernelGGL(pattern<MODE>, dim3(grid), dim3(1024), 0, 0, keys, off, out, ntiles, sink);
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < iters; i++)
        hipLaunchKernelGGL(pattern<MODE>, dim3(grid), dim3(1024), 0, 0, keys, off, out, ntiles, sink);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / iters;
}

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 20;
    const uint64_t n = 1ull << 26, ntiles = n / 64u;
    uint8_t *keys;
    uint64_t *off;
    uint32_t *out, *sink;
    CK(hipMalloc(&keys, n * 32u + 64u));
    CK(hipMalloc(&off, (n + 1u) * 8u));
    CK(hipMalloc(&out, n * 4u));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(keys, 1, n * 32u + 64u));
    CK(hipMemset(off, 0, (n + 1u) * 8u));
    const char *what[] = {"keys: per-lane 2 x 16 B", "+ offsets (2 x 4 B per lane)", "+ 4 B store per key",
                          "keys as coalesced 1 KiB wave loads", "offsets as one 4 B load + DPP",
                          "default-policy 4 B stores", "16 B stores by 16 lanes (nt)", "16 B stores by 16 lanes"};
    for (int m = 0; m < 8; m++) {
        float ms = 0;
        switch (m) {
        case 0: ms = run<0>(keys, off, out, (uint32_t)ntiles, sink, iters); break;
        case 1: ms = run<1>(keys, off, out, (uint32_t)ntiles, sink, iters); break;
        case 2: ms = run<2>(keys, off, out, (uint32_t)ntiles, sink, iters); break;
        case 3: ms = run<3>(keys, off, out, (uint32_t)ntiles, sink, iters); break;
        case 4: ms = run<4>(keys, off, out, (uint32_t)ntiles, sink, iters); break;
        case 5: ms = run<5>(keys, off, out, (uint32_t)ntiles, sink, iters); break;
        case 6: ms = run<6>(keys, off, out, (uint32_t)ntiles, sink, iters); break;
        default: ms = run<7>(keys, off, out, (uint32_t)ntiles, sink, iters); break;
        }
        const double bytes = m == 0 ? n * 32.0 : (m == 1 ? n * 40.0 : (m == 4 ? n * 44.0 : n * 44.0));
        printf("{\"probe\": \"direct_pattern\", \"mode\": %d, \"what\": \"%s\", \"ms\": %.4f, \"moved_bytes\": %.0f, "
               "\"gb_s\": %.1f, \"c3_alg_frac\": %.4f}\n",
               m, what[m], ms, bytes, bytes / ms / 1e6, (n * 44.0) / ms / 1e6 / 8000.0);
        fflush(stdout);
    }
    return 0;
}
