// Compute-only md5 ceiling on gfx950: every lane runs a 61-step final block
// on register-resident message words, no memory traffic, for three ways of
// writing a step's additions:
//   form 0 (the kernel's, nc_md5_steps.h): a+w (VOP2), +T (VOP2 literal), +f (VOP2)
//   form 1: hipcc's default: a+w (VOP2), s_mov T, v_add3(., f, sT) (VOP3)
//   form 2: v_add3(a, w, f) (VOP3), +T (VOP2 literal)
// Prints ns per 64-lane round per SIMD and the implied C3 time (2^20 rounds
// over 1024 SIMDs).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Itwemproxy_amd/csrc -Iinclude tools/probes/md5_rate.hip -o tools/probes/md5_rate
#include <hip/hip_runtime.h>

#include <stdio.h>

#include "nc_md5_steps.h"

using namespace nc_md5s;

template <int FORM, int I>
__device__ __forceinline__ void step(uint32_t (&v)[4], const uint32_t (&w)[16])
{
    if constexpr (FORM == 0) {
        md5_step<I>(v, w);
    } else {
        constexpr int u = (4 - (I & 3)) & 3;
        const uint32_t b = v[(u + 1) & 3], c = v[(u + 2) & 3], d = v[(u + 3) & 3];
        uint32_t f;
        if constexpr (I < 16) f = NC_MD5_F(b, c, d);
        else if constexpr (I < 32) f = NC_MD5_G(b, c, d);
        else if constexpr (I < 48) f = NC_MD5_H(b, c, d);
        else f = NC_MD5_I(b, c, d);
        uint32_t a;
        if constexpr (FORM == 1) {
            a = v[u] + w[kM[I]] + kT[I] + f;
        } else {
            uint32_t x;
            asm("v_add3_u32 %0, %1, %2, %3" : "=v"(x) : "v"(v[u]), "v"(w[kM[I]]), "v"(f));
            asm("v_add_u32_e32 %0, %1, %2" : "=v"(a) : "i"(kT[I]), "v"(x));
        }
        v[u] = nc_rotl(a, kS[I]) + b;
    }
}

template <int FORM, int... I>
__device__ __forceinline__ void steps(uint32_t (&v)[4], const uint32_t (&w)[16], std::integer_sequence<int, I...>)
{
    (step<FORM, I>(v, w), ...);
}

template <int FORM>
__global__ __launch_bounds__(256) void md5_rounds(unsigned *out, int rounds)
{
    uint32_t w[16];
#pragma unroll
    for (int t = 0; t < 16; t++) w[t] = threadIdx.x * 0x9e3779b9u + t;
    uint32_t acc = 0;
    for (int r = 0; r < rounds; r++) {
        uint32_t v[4] = {0x67452301u + acc, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
        steps<FORM>(v, w, std::make_integer_sequence<int, 61>{});
        acc += v[0];
        w[r & 15] ^= acc; /* keeps the rounds dependent on each other's data */
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

template <int FORM>
static void run(int wps, unsigned *o, int cus)
{
    const int rounds = 256;
    const int blocks = cus * wps;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 3; i++) hipLaunchKernelGGL(md5_rounds<FORM>, dim3(blocks), dim3(256), 0, 0, o, rounds);
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < 10; i++) hipLaunchKernelGGL(md5_rounds<FORM>, dim3(blocks), dim3(256), 0, 0, o, rounds);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    ms /= 10;
    const double ns_per_round = ms * 1e6 / ((double)wps * rounds);
    printf("{\"form\": %d, \"waves_per_simd\": %d, \"ms\": %.4f, \"ns_per_round_per_simd\": %.2f, \"c3_ms\": %.4f}\n",
           FORM, wps, ms, ns_per_round, ns_per_round * 1024 * 1e-6);
}

int main()
{
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    unsigned *o;
    (void)hipMalloc(&o, 1 << 20);
    for (int wps : {4, 8}) {
        run<0>(wps, o, p.multiProcessorCount);
        run<1>(wps, o, p.multiProcessorCount);
        run<2>(wps, o, p.multiProcessorCount);
    }
    return 0;
}
