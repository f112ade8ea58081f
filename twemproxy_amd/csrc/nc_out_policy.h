/*
 * The hash outputs' store policy, one place for every kernel: the cache
 * policy of the 4-byte (and 16-byte) stores of the hashes into `out`.
 * NC_OUT_POLICY (A/B builds, tools/build_ablib.sh): 0 nt (streaming), 1 plain,
 * 2 sc1 (write-through, the line dropped from L2). The stores share the HBM
 * with a read stream about eight times their size, and their flavour moves
 * what that read/write mix sustains (tools/probe_tile_mix.py --flavours).
 */
#ifndef NC_OUT_POLICY_H
#define NC_OUT_POLICY_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef NC_OUT_POLICY
#define NC_OUT_POLICY 0
#endif

/* buffer-store aux bits: 2 = nt (slc), 16 = sc1 */
constexpr int kAuxOut = NC_OUT_POLICY == 0 ? 2 : NC_OUT_POLICY == 1 ? 0 : 16;

__device__ __forceinline__ void out_st32(uint32_t *p, uint32_t v)
{
    if constexpr (NC_OUT_POLICY == 0) __builtin_nontemporal_store(v, p);
    else if constexpr (NC_OUT_POLICY == 1) *p = v;
    else __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); /* global_store_dword sc1 */
}

/* the same as inline asm, for kernels that count their own vmcnt */
__device__ __forceinline__ void out_asm_st32(void *p, uint32_t v)
{
    if constexpr (NC_OUT_POLICY == 0) asm volatile("global_store_dword %0, %1, off nt" : : "v"(p), "v"(v) : "memory");
    else if constexpr (NC_OUT_POLICY == 1) asm volatile("global_store_dword %0, %1, off" : : "v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dword %0, %1, off sc1" : : "v"(p), "v"(v) : "memory");
}

#endif
