// Read-pattern probe for the long-key direct pipelines (C4 shard: 2^25 x 256 B
// keys, 8 GiB): does fetching a key's two 128-byte lines one ROUND apart — the
// lines kernels' order (nc_direct.h dma_lines: round r moves line r of a
// tile's 64 keys, stride 256 B) — cost HBM bandwidth against fetching the
// tile's 16 KiB contiguously?
//
// Every wave owns 64-key tiles interleaved over the grid (as the IL
// variants) and moves each tile by LDS-DMA in 1 KiB instructions into a
// per-wave image, like the kernels:
//   pattern 0 "pairs": one round per tile, 16 instructions covering the
//             tile's 16 KiB in address order (16 KiB image per wave);
//   pattern 1 "lines": two rounds per tile, round r = line r of every key
//             (8 instructions, 8 keys x 128 B each, 8 KiB image);
//   pattern 2 "lines, both rounds at once": the two rounds' 16 instructions
//             issued back to back (16 KiB image): the same addresses as 1,
//             each line pair fetched together.
// A round ends with a wait for its DMAs and a delay of dependent VALU work
// standing in for the hash (`spin` iterations per 16 KiB tile, split over the
// rounds), then one LDS word is read and folded so nothing is dead. Prints
// GB/s per pattern and spin.
//   hipcc -O3 --offload-arch=gfx950 -o tools/probes/line_pattern tools/probes/line_pattern.hip
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>

namespace {

constexpr int kWaves = 4; /* per workgroup */

__device__ __forceinline__ void dma16(const uint8_t *base, uint32_t voff, uint8_t *lds)
{
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(base), (short)0,
                                                                       0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)lds, 16, voff, 0, 0, 0);
}

template <int PAT>
__global__ __launch_bounds__(64 * kWaves) void probe(const uint8_t *__restrict__ keys, uint32_t ntiles, int spin,
                                                     uint32_t *__restrict__ sink)
{
    constexpr uint32_t kImg = PAT == 1 ? 8192u : 16384u;
    __shared__ __attribute__((aligned(16))) uint8_t img[kWaves * kImg];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t *my = img + wave * kImg;
    const uint32_t W = gridDim.x * kWaves;
    uint32_t acc = lane;
    for (uint32_t tile = blockIdx.x * kWaves + wave; tile < ntiles; tile += W) {
        const uint8_t *tb = keys + (uint64_t)tile * 16384u;
        const int rounds = PAT == 1 ? 2 : 1;
        for (int r = 0; r < rounds; r++) {
            if constexpr (PAT == 0) {
#pragma unroll
                for (int i = 0; i < 16; i++) dma16(tb, 1024u * i + 16u * lane, my + 1024 * i);
            } else {
#pragma unroll
                for (int rr = 0; rr < (PAT == 2 ? 2 : 1); rr++) {
                    const uint32_t line = PAT == 2 ? (uint32_t)rr : (uint32_t)r;
#pragma unroll
                    for (int i = 0; i < 8; i++) {
                        const uint32_t key = 8u * i + (lane >> 3);
                        dma16(tb, key * 256u + line * 128u + 16u * (lane & 7u), my + 8192 * rr + 1024 * i);
                    }
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            uint32_t x = acc;
            const int n = PAT == 1 ? spin / 2 : spin; /* the same work per byte in every pattern */
            for (int s = 0; s < n; s++) x = __builtin_amdgcn_alignbit(x, x, 7) + 0x9e3779b9u;
            acc = x ^ *reinterpret_cast<const uint32_t *>(my + 4u * lane);
        }
    }
    if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

template <int PAT>
float run(const uint8_t *d, uint32_t ntiles, int spin, uint32_t *sink, int grid)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(probe<PAT>, dim3(grid), dim3(64 * kWaves), 0, 0, d, ntiles, spin, sink);
    (void)hipEventRecord(a, 0);
    const int iters = 5;
    for (int i = 0; i < iters; i++)
        hipLaunchKernelGGL(probe<PAT>, dim3(grid), dim3(64 * kWaves), 0, 0, d, ntiles, spin, sink);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return ms / iters;
}

} // namespace

int main()
{
    const uint32_t ntiles = 1u << 19; /* 2^25 keys x 256 B = 8 GiB */
    const size_t bytes = (size_t)ntiles * 16384u;
    uint8_t *d = nullptr;
    uint32_t *sink = nullptr;
    if (hipMalloc((void **)&d, bytes) != hipSuccess || hipMalloc((void **)&sink, 1 << 20) != hipSuccess) {
        fprintf(stderr, "hipMalloc failed\n");
        return 1;
    }
    (void)hipMemset(d, 0x5a, bytes);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const char *names[3] = {"pairs (16 KiB tile in address order, one round)",
                            "lines (line r of 64 keys per round, two rounds)",
                            "lines, both rounds issued together"};
    for (int spin : {0, 200, 800}) {
        /* (pattern, workgroups per CU): LDS 4 x 16 KiB (8 KiB for lines) per
         * workgroup fits 2 (5); lines also at 2, the others' occupancy */
        const int cases[4][2] = {{0, 2}, {1, 5}, {1, 2}, {2, 2}};
        for (const auto &c : cases) {
            const int pat = c[0], per_cu = c[1];
            const int grid = cus * per_cu;
            float ms = pat == 0 ? run<0>(d, ntiles, spin, sink, grid)
                                : (pat == 1 ? run<1>(d, ntiles, spin, sink, grid) : run<2>(d, ntiles, spin, sink, grid));
            printf("{\"pattern\": %d, \"name\": \"%s\", \"spin\": %d, \"grid\": %d, \"ms\": %.4f, \"gb_s\": %.1f}\n", pat,
                   names[pat], spin, grid, ms, bytes / (ms * 1e6));
            fflush(stdout);
        }
    }
    (void)hipFree(d);
    (void)hipFree(sink);
    return 0;
}
