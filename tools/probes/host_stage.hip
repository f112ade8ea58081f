/*
 * Where the batch ring's host submit time goes: the cost of
 * staging one C5 mbuf (15.4 KB of keys + 585 span words) into host memory of
 * each kind the ring could use, with and without a GPU kernel reading the
 * staging between copies (as the ring's worker does).
 *
 *   tools/probes/host_stage            (one JSON line per memory kind)
 */
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now_s()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* reads the staged image across PCIe (16 B per thread), as the worker does */
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ void touch(const u32x4 *p, uint32_t n16, uint32_t *sink)
{
    uint32_t acc = 0;
    for (uint32_t i = threadIdx.x; i < n16; i += blockDim.x) {
        const u32x4 v = __builtin_nontemporal_load(p + i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main()
{
    const size_t kbytes = 15412, nspan = 585, reps = 20000;
    uint8_t *src = (uint8_t *)malloc(kbytes);
    for (size_t i = 0; i < kbytes; i++) src[i] = (uint8_t)(i * 7);
    uint32_t *sink;
    if (hipMalloc(&sink, 4) != hipSuccess) return 1;
    struct Kind {
        const char *name;
        unsigned flags;
        int host_malloc;
    } kinds[] = {{"malloc", 0, 1},
                 {"hipHostMalloc Mapped|Coherent", hipHostMallocMapped | hipHostMallocCoherent, 0},
                 {"hipHostMalloc Mapped|NonCoherent", hipHostMallocMapped | hipHostMallocNonCoherent, 0},
                 {"hipHostMalloc Mapped|WriteCombined", hipHostMallocMapped | hipHostMallocWriteCombined, 0}};
    for (const Kind &k : kinds) {
        uint8_t *dst = NULL;
        if (k.host_malloc) dst = (uint8_t *)aligned_alloc(4096, 65536);
        else if (hipHostMalloc((void **)&dst, 65536, k.flags) != hipSuccess) return 1;
        uint32_t *spans = (uint32_t *)(dst + 32768);
        for (int with_gpu = 0; with_gpu < (k.host_malloc ? 1 : 2); with_gpu++) {
            void *ddst = NULL;
            if (with_gpu && hipHostGetDevicePointer(&ddst, dst, 0) != hipSuccess) return 1;
            double best = 1e30;
            for (int round = 0; round < 5; round++) {
                double tot = 0.0;
                for (size_t r = 0; r < reps / 5; r++) {
                    const double a = now_s();
                    memcpy(dst, src, kbytes);
                    for (size_t i = 0; i < nspan; i++) spans[i] = (uint32_t)(i * 26) | ((uint32_t)(i * 26 + 20) << 16);
                    __atomic_thread_fence(__ATOMIC_SEQ_CST);
                    tot += now_s() - a;
                    if (with_gpu) {
                        hipLaunchKernelGGL(touch, dim3(1), dim3(1024), 0, 0, (const u32x4 *)ddst, (32768 + 2340) / 16, sink);
                        if (hipDeviceSynchronize() != hipSuccess) return 1;
                    }
                }
                const double us = tot / (reps / 5) * 1e6;
                if (us < best) best = us;
            }
            printf("{\"probe\": \"host_stage\", \"memory\": \"%s\", \"gpu_reads_between\": %d, \"bytes\": %zu, "
                   "\"span_words\": %zu, \"us_per_stage\": %.3f, \"gb_s\": %.2f}\n",
                   k.name, with_gpu, kbytes, nspan, best, (kbytes + 4 * nspan) / best / 1e3);
            fflush(stdout);
        }
        if (k.host_malloc) free(dst);
        else (void)hipHostFree(dst);
    }
    return 0;
}
