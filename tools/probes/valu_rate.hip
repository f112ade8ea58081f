// VALU issue-rate probe for the integer ops the hash kernels use (gfx950).
// For each op: a grid of 256-thread workgroups (WAVES/SIMD resident), every
// lane running CH independent chains of ITERS dependent instructions of that
// op (inline asm, so the instruction is exactly the one named). Prints
// wave-instructions per cycle per SIMD from hipEvents and the device clock.
//   hipcc -O3 --offload-arch=gfx950 tools/probes/valu_rate.hip -o /tmp/valu_rate && /tmp/valu_rate
#include <hip/hip_runtime.h>

#include <stdio.h>

#define ITERS 4096

#define OP_ADD(x, y) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(x) : "v"(y))
#define OP_ADD3(x, y) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x) : "v"(y))
#define OP_ALIGNBIT(x, y) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(x) : "v"(y))
#define OP_BITOP3(x, y) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0xac" : "+v"(x) : "v"(y))
#define OP_PERM(x, y) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(x) : "v"(y))
#define OP_MED3(x, y) asm volatile("v_med3_i32 %0, %0, %1, %1" : "+v"(x) : "v"(y))
#define OP_XOR(x, y) asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(x) : "v"(y))
#define OP_LSHLADD(x, y) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x) : "v"(y))
#define OP_MULLO(x, y) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(y))
#define OP_BFE(x, y) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(x) : "v"(y))
#define OP_XAD(x, y) asm volatile("v_xad_u32 %0, %0, %1, %1" : "+v"(x) : "v"(y))
#define OP_XORSDWA(x, y) asm volatile("v_xor_b32_sdwa %0, %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(x) : "v"(y))
#define OP_FNV(x, y) asm volatile("v_xor_b32_sdwa %0, %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n\tv_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(y))
#define OP_FNVSA(x, y) asm volatile("v_xor_b32_sdwa %0, %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n\tv_lshl_add_u32 v40, %0, 1, %0\n\tv_lshl_add_u32 v41, v40, 3, v40\n\tv_lshl_add_u32 %0, v41, 4, v40" : "+v"(x) : "v"(y) : "v40", "v41")
#define OP_MULU24(x, y) asm volatile("v_mul_u32_u24_e32 %0, %1, %0" : "+v"(x) : "v"(y))
#define OP_CNDMASK(x, y) asm volatile("v_cmp_lt_u32_e32 vcc, %0, %1\n\tv_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(x) : "v"(y) : "vcc")
#define OP_ADD_SGPR(x, y) asm volatile("s_mov_b32 s40, 0x12345\n\tv_add3_u32 %0, %0, %1, s40" : "+v"(x) : "v"(y) : "s40")

#define KERNEL(NAME, OP)                                                                   \
    template <int CH>                                                                      \
    __global__ __launch_bounds__(256) void k_##NAME(unsigned *out, unsigned seed)          \
    {                                                                                      \
        unsigned x[CH];                                                                    \
        const unsigned y = threadIdx.x ^ seed;                                             \
        _Pragma("unroll") for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c;             \
        for (int i = 0; i < ITERS; i++) {                                                  \
            _Pragma("unroll") for (int c = 0; c < CH; c++) OP(x[c], y);                    \
        }                                                                                  \
        unsigned s = 0;                                                                    \
        _Pragma("unroll") for (int c = 0; c < CH; c++) s ^= x[c];                          \
        if (s == 0x9e3779b9u) out[blockIdx.x] = s;                                         \
    }

KERNEL(add, OP_ADD)
KERNEL(add3, OP_ADD3)
KERNEL(alignbit, OP_ALIGNBIT)
KERNEL(bitop3, OP_BITOP3)
KERNEL(perm, OP_PERM)
KERNEL(med3, OP_MED3)
KERNEL(xor, OP_XOR)
KERNEL(lshladd, OP_LSHLADD)
KERNEL(mullo, OP_MULLO)
KERNEL(bfe, OP_BFE)
KERNEL(xad, OP_XAD)
KERNEL(add3s, OP_ADD_SGPR)
KERNEL(xorsdwa, OP_XORSDWA)
KERNEL(fnv, OP_FNV)
KERNEL(fnvsa, OP_FNVSA)
KERNEL(mulu24, OP_MULU24)
KERNEL(cndmask, OP_CNDMASK)

static int g_cus;
static unsigned *g_out;

template <int CH>
static void run(const char *name, void (*k)(unsigned *, unsigned), int waves_per_simd, int clock_khz)
{
    const int blocks = g_cus * waves_per_simd; /* 4 waves per block = one per SIMD */
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int w = 0; w < 3; w++) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, g_out, 1u);
    hipEventRecord(a, 0);
    const int reps = 5;
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, g_out, 1u);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    const double insts_per_simd = (double)waves_per_simd * CH * ITERS; /* wave-instructions per SIMD */
    const double cycles = ms * 1e-3 * clock_khz * 1e3;
    printf("{\"op\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"ms\": %.4f, \"inst_per_cycle_per_simd_at_max_clock\": %.4f, \"cycles_per_inst\": %.3f}\n",
           name, CH, waves_per_simd, ms, insts_per_simd / cycles, cycles / insts_per_simd);
}

#define RUN(NAME)                                                 \
    run<8>(#NAME, k_##NAME<8>, 8, clk);                           \
    run<8>(#NAME, k_##NAME<8>, 2, clk);                           \
    run<1>(#NAME "_chain", k_##NAME<1>, 1, clk);                  \
    run<1>(#NAME "_chain", k_##NAME<1>, 8, clk);

int main()
{
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    g_cus = p.multiProcessorCount;
    const int clk = p.clockRate; /* kHz, the max shader clock */
    hipMalloc(&g_out, 1 << 20);
    printf("# %s CUs %d clock %d kHz\n", p.gcnArchName, g_cus, clk);
    RUN(add) RUN(add3) RUN(alignbit) RUN(bitop3) RUN(perm) RUN(med3) RUN(xor) RUN(lshladd) RUN(mullo) RUN(bfe) RUN(xad)
    RUN(add3s)
    RUN(xorsdwa) RUN(fnv) RUN(fnvsa) RUN(mulu24) RUN(cndmask)
    return 0;
}
