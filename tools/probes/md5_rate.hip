// Compute-only md5 ceiling on gfx950: every lane runs a 61-step final block
// on register-resident message words, no memory traffic, for several ways of
// writing a step's additions:
//   form 0 (the kernel's, nc_md5_steps.h): w+T (VOP2 literal, off the step
//          chain), v_add3(a, wT, f) (VOP3)
//   form 1: hipcc's default: a+w (VOP2), s_mov T, v_add3(., f, sT) (VOP3)
//   form 2 (the round-2 kernel's): v_add3(a, w, f) (VOP3), +T (VOP2 literal)
//   form 3: form 0 written out here (a check of the header's form)
//   form 4: T in 64 SGPRs set before the loop, v_add3(a, w, sT), +f (VOP2)
//   form 5: form 2's ops, the 61 steps as one inline-asm statement
//           (md5_asm.inc, tools/gen_md5_asm.py): no hazard s_nops
//   form 6: form 0's ops as one inline-asm statement (w+T into two
//           alternating scratch registers), step i+1's w+T after step i's
//           v_add3; form 7: the same with each w+T first in its step
// Prints a check of form 5 against form 0, then ns per 64-lane round per SIMD
// and the implied C3 time (2^20 rounds over 1024 SIMDs). Built by
// twemproxy_amd/csrc/Makefile (target all).
#include <hip/hip_runtime.h>

#include <stdio.h>

#include "nc_md5_steps.h"

using namespace nc_md5s;

/* Steps 0..60 / 61..63 as ONE inline-asm statement each (nc_md5_asm.inc,
 * tools/gen_md5_asm.py): the same five VALU ops per step as md5_step, without
 * the s_nop hipcc's hazard recognizer puts after every inline-asm def
 * (measured slower than the kernel's form: the steps can no longer
 * interleave with hipcc's scheduling). */
#include "md5_asm.inc"

#define NC_MD5_ASM_OPERANDS(v, w, t)                                                                        \
    : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "=&v"(t)                                           \
    : "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(w[5]), "v"(w[6]), "v"(w[7]), "v"(w[8]), \
      "v"(w[9]), "v"(w[10]), "v"(w[11]), "v"(w[12]), "v"(w[13]), "v"(w[14]), "v"(w[15])

__device__ __forceinline__ void md5_steps_asm_0_61(uint32_t (&v)[4], const uint32_t (&w)[16])
{
    uint32_t t; /* scratch */
    asm(NC_MD5_ASM_STEPS_0_61 NC_MD5_ASM_OPERANDS(v, w, t));
}

#define NC_MD5_ASM6_OPERANDS(v, w, t, t5, t6)                                                               \
    : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "=&v"(t), "=&v"(t5), "=&v"(t6)                      \
    : "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(w[5]), "v"(w[6]), "v"(w[7]), "v"(w[8]), \
      "v"(w[9]), "v"(w[10]), "v"(w[11]), "v"(w[12]), "v"(w[13]), "v"(w[14]), "v"(w[15])

template <int FORM>
__device__ __forceinline__ void md5_steps_asm67_0_61(uint32_t (&v)[4], const uint32_t (&w)[16])
{
    uint32_t t, t5, t6;
    if constexpr (FORM == 6) asm(NC_MD5_ASM6_STEPS_0_61 NC_MD5_ASM6_OPERANDS(v, w, t, t5, t6));
    else asm(NC_MD5_ASM7_STEPS_0_61 NC_MD5_ASM6_OPERANDS(v, w, t, t5, t6));
}

__device__ __forceinline__ void md5_steps_asm_61_64(uint32_t (&v)[4], const uint32_t (&w)[16])
{
    uint32_t t;
    asm(NC_MD5_ASM_STEPS_61_64 NC_MD5_ASM_OPERANDS(v, w, t));
}


template <int FORM, int I>
__device__ __forceinline__ void step(uint32_t (&v)[4], const uint32_t (&w)[16], const uint32_t (&sT)[64])
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
        } else if constexpr (FORM == 3) {
            uint32_t wt = w[kM[I]] + kT[I];
            asm("" : "+v"(wt));
            a = v[u] + wt + f;
        } else if constexpr (FORM == 4) {
            uint32_t x;
            asm("v_add3_u32 %0, %1, %2, %3" : "=v"(x) : "v"(v[u]), "v"(w[kM[I]]), "s"(sT[I]));
            a = x + f;
        } else {
            uint32_t x;
            asm("v_add3_u32 %0, %1, %2, %3" : "=v"(x) : "v"(v[u]), "v"(w[kM[I]]), "v"(f));
            asm("v_add_u32_e32 %0, %1, %2" : "=v"(a) : "i"(kT[I]), "v"(x));
        }
        v[u] = nc_rotl(a, kS[I]) + b;
    }
}

template <int FORM, int... I>
__device__ __forceinline__ void steps(uint32_t (&v)[4], const uint32_t (&w)[16], const uint32_t (&sT)[64],
                                      std::integer_sequence<int, I...>)
{
    (step<FORM, I>(v, w, sT), ...);
}

template <int FORM>
__global__ __launch_bounds__(256) void md5_rounds(unsigned *out, int rounds, unsigned long long *clk)
{
    /* workgroup 0 (resident the whole launch: the grid is one wave set)
     * stamps the shader clock and the 100 MHz real-time clock at its start
     * and end: the clock this launch ran at */
    if (clk != nullptr && blockIdx.x == 0 && threadIdx.x == 0) {
        clk[0] = __builtin_readcyclecounter();
        clk[1] = wall_clock64();
    }
    uint32_t w[16];
#pragma unroll
    for (int t = 0; t < 16; t++) w[t] = threadIdx.x * 0x9e3779b9u + t;
    uint32_t acc = 0;
    uint32_t sT[64];
    if constexpr (FORM == 4) {
#pragma unroll
        for (int i = 0; i < 64; i++) asm volatile("s_mov_b32 %0, %1" : "=s"(sT[i]) : "i"(kT[i]));
    }
    for (int r = 0; r < rounds; r++) {
        uint32_t v[4] = {0x67452301u + acc, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
        if constexpr (FORM == 5) md5_steps_asm_0_61(v, w);
        else if constexpr (FORM >= 6) md5_steps_asm67_0_61<FORM>(v, w);
        else steps<FORM>(v, w, sT, std::make_integer_sequence<int, 61>{});
        acc += v[0];
        w[r & 15] ^= acc; /* keeps the rounds dependent on each other's data */
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
    if (clk != nullptr && blockIdx.x == 0 && threadIdx.x == 0) {
        __builtin_amdgcn_s_waitcnt(0);
        clk[2] = __builtin_readcyclecounter();
        clk[3] = wall_clock64();
    }
}

/* sustain_ms > 0: launches back to back for that long first (the power
 * controller settles the clock under a long VALU-bound load, as under the
 * hash kernels' timed loops), then times 10 more */
template <int FORM>
static void run(int wps, unsigned *o, int cus, unsigned long long *clk, double sustain_ms = 0.0)
{
    const int rounds = 256;
    const int blocks = cus * wps;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 3; i++) hipLaunchKernelGGL(md5_rounds<FORM>, dim3(blocks), dim3(256), 0, 0, o, rounds, nullptr);
    if (sustain_ms > 0.0) {
        float el = 0.f;
        (void)hipEventRecord(a, 0);
        while (el < sustain_ms) {
            for (int i = 0; i < 20; i++)
                hipLaunchKernelGGL(md5_rounds<FORM>, dim3(blocks), dim3(256), 0, 0, o, rounds, nullptr);
            (void)hipEventRecord(b, 0);
            (void)hipEventSynchronize(b);
            (void)hipEventElapsedTime(&el, a, b);
        }
    }
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < 10; i++)
        hipLaunchKernelGGL(md5_rounds<FORM>, dim3(blocks), dim3(256), 0, 0, o, rounds, i == 9 ? clk : nullptr);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    ms /= 10;
    unsigned long long c[4] = {0, 0, 0, 0};
    (void)hipMemcpy(c, clk, sizeof c, hipMemcpyDeviceToHost);
    const double mhz = c[3] > c[1] ? (double)(c[2] - c[0]) / (double)(c[3] - c[1]) * 100.0 : 0.0;
    const double ns_per_round = ms * 1e6 / ((double)wps * rounds);
    printf("{\"form\": %d, \"waves_per_simd\": %d, \"sustained\": %s, \"ms\": %.4f, \"ns_per_round_per_simd\": %.2f, "
           "\"c3_ms\": %.4f, \"clock_mhz\": %.1f}\n",
           FORM, wps, sustain_ms > 0.0 ? "true" : "false", ms, ns_per_round, ns_per_round * 1024 * 1e-6, mhz);
}

template <int FORM>
__global__ void md5_check(unsigned *out)
{
    uint32_t w[16];
#pragma unroll
    for (int t = 0; t < 16; t++) w[t] = (threadIdx.x + 1u) * 0x9e3779b9u ^ (t * 0x85ebca6bu);
    uint32_t v[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    if constexpr (FORM == 5) {
        md5_steps_asm_0_61(v, w);
        md5_steps_asm_61_64(v, w);
    } else if constexpr (FORM >= 6) {
        md5_steps_asm67_0_61<FORM>(v, w);
        md5_steps_from61(v, w, std::make_integer_sequence<int, 3>{});
    } else {
        md5_steps(v, w, std::make_integer_sequence<int, 61>{});
        md5_steps_from61(v, w, std::make_integer_sequence<int, 3>{});
    }
    for (int i = 0; i < 4; i++) out[threadIdx.x * 4 + i] = v[i];
}

int main()
{
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    unsigned *o;
    (void)hipMalloc(&o, 1 << 20);
    unsigned long long *clk;
    (void)hipMalloc(&clk, 64);
    {
        unsigned h0[256], h5[256], h6[256], h7[256];
        hipLaunchKernelGGL(md5_check<0>, dim3(1), dim3(64), 0, 0, o);
        (void)hipMemcpy(h0, o, sizeof h0, hipMemcpyDeviceToHost);
        hipLaunchKernelGGL(md5_check<5>, dim3(1), dim3(64), 0, 0, o);
        (void)hipMemcpy(h5, o, sizeof h5, hipMemcpyDeviceToHost);
        hipLaunchKernelGGL(md5_check<6>, dim3(1), dim3(64), 0, 0, o);
        (void)hipMemcpy(h6, o, sizeof h6, hipMemcpyDeviceToHost);
        hipLaunchKernelGGL(md5_check<7>, dim3(1), dim3(64), 0, 0, o);
        (void)hipMemcpy(h7, o, sizeof h7, hipMemcpyDeviceToHost);
        int bad = 0, bad6 = 0, bad7 = 0;
        for (int i = 0; i < 256; i++) {
            bad += h0[i] != h5[i];
            bad6 += h0[i] != h6[i];
            bad7 += h0[i] != h7[i];
        }
        printf("{\"asm_steps_match\": %s, \"mismatches\": %d, \"form6_mismatches\": %d, \"form7_mismatches\": %d}\n",
               bad ? "false" : "true", bad, bad6, bad7);
    }
    for (int wps : {4, 8}) {
        run<0>(wps, o, p.multiProcessorCount, clk);
        run<1>(wps, o, p.multiProcessorCount, clk);
        run<2>(wps, o, p.multiProcessorCount, clk);
        run<3>(wps, o, p.multiProcessorCount, clk);
        run<4>(wps, o, p.multiProcessorCount, clk);
        run<5>(wps, o, p.multiProcessorCount, clk);
        run<6>(wps, o, p.multiProcessorCount, clk);
        run<7>(wps, o, p.multiProcessorCount, clk);
    }
    /* the kernel's form at 8 waves per SIMD after 300 ms of back-to-back
     * launches: the rate at the clock a long md5 load settles at */
    run<0>(8, o, p.multiProcessorCount, clk, 300.0);
    return 0;
}
