/*
 * Can the host write device memory directly (the BAR), and what would the
 * batch ring gain from it (one batch in flight spends ~1.7 us
 * fetching the staged image across PCIe and ~2.2 us detecting the
 * descriptor, publishing the done word and reaping)?
 *
 * For each kind of allocation (hipMalloc, hipExtMallocWithFlags fine-grained
 * and uncached, and the ring's own hipHostMalloc Mapped|Coherent host memory):
 *   - whether a host store / load through the pointer works (a SIGSEGV is
 *     caught and reported, nothing else is attempted on that kind);
 *   - the host's cost of staging one C5 mbuf (15.4 KB) there by memcpy;
 *   - a ping-pong: one wave polls a flag word in that memory (system-scope
 *     relaxed loads) and answers in mapped host memory; the host writes the
 *     flag and spins on the answer: the round trip per message.
 * The polling kernel ends on a stop value or after 2 s of s_memrealtime,
 * whichever comes first, so a lost message cannot hang the GPU.
 *
 *   tools/probes/bar_probe      (one JSON line per memory kind)
 */
#include <hip/hip_runtime.h>

#include <setjmp.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <immintrin.h>

/* copies into write-combined BAR memory: 32-byte non-temporal stores (the
 * destination 32-byte aligned, the source any) and plain 32-byte stores */
__attribute__((target("avx2"))) static void copy_nt32(uint8_t *dst, const uint8_t *src, size_t n)
{
    size_t i = 0;
    for (; i + 32 <= n; i += 32)
        _mm256_stream_si256((__m256i *)(dst + i), _mm256_loadu_si256((const __m256i *)(src + i)));
    if (i < n) memcpy(dst + i, src + i, n - i);
    _mm_sfence();
}
__attribute__((target("avx2"))) static void copy_st32(uint8_t *dst, const uint8_t *src, size_t n)
{
    size_t i = 0;
    for (; i + 32 <= n; i += 32)
        _mm256_store_si256((__m256i *)(dst + i), _mm256_loadu_si256((const __m256i *)(src + i)));
    if (i < n) memcpy(dst + i, src + i, n - i);
}

static double now_s()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static sigjmp_buf g_jb;
static void on_segv(int) { siglongjmp(g_jb, 1); }

/* host access test: 1 if a store and a load through p work */
static int host_access(volatile uint32_t *p)
{
    struct sigaction sa, old_segv, old_bus;
    memset(&sa, 0, sizeof(sa));
    sa.sa_handler = on_segv;
    sigaction(SIGSEGV, &sa, &old_segv);
    sigaction(SIGBUS, &sa, &old_bus);
    int ok = 0;
    if (sigsetjmp(g_jb, 1) == 0) {
        p[0] = 0x5a5a1234u;
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
        ok = p[0] == 0x5a5a1234u;
    }
    sigaction(SIGSEGV, &old_segv, NULL);
    sigaction(SIGBUS, &old_bus, NULL);
    return ok;
}

/* one wave: wait for flag == i (i = 1..n), answer ack = i; stop on flag ==
 * 0xffffffff or after 2 s (200 M ticks of the 100 MHz s_memrealtime) */
__global__ void pong(const uint32_t *flag, uint32_t *ack, uint32_t n, uint32_t *polls)
{
    if (threadIdx.x != 0) return;
    const uint64_t t0 = wall_clock64();
    uint32_t want = 1, npoll = 0;
    while (want <= n) {
        const uint32_t f = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        npoll++;
        if (f == 0xffffffffu) break;
        if (f == want) {
            __hip_atomic_store(ack, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            want++;
            continue;
        }
        if (wall_clock64() - t0 > 200000000ull) break;
    }
    polls[0] = npoll;
}

int main()
{
    const size_t kbytes = 15412, stage_reps = 20000;
    const uint32_t msgs = 20000;
    uint8_t *src = (uint8_t *)malloc(kbytes);
    for (size_t i = 0; i < kbytes; i++) src[i] = (uint8_t)(i * 7);
    uint32_t *ack_h = NULL, *ack_d = NULL, *polls = NULL;
    if (hipHostMalloc((void **)&ack_h, 4096, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 1;
    if (hipHostGetDevicePointer((void **)&ack_d, ack_h, 0) != hipSuccess) return 1;
    if (hipMalloc((void **)&polls, 4) != hipSuccess) return 1;
    struct Kind {
        const char *name;
        int how; /* 0 hipMalloc, 1 ext flags, 2 hipHostMalloc mapped coherent */
        unsigned flags;
    } kinds[] = {{"hipMalloc", 0, 0},
                 {"hipExtMallocWithFlags Finegrained", 1, hipDeviceMallocFinegrained},
                 {"hipExtMallocWithFlags Uncached", 1, hipDeviceMallocUncached},
                 {"hipHostMalloc Mapped|Coherent (the ring's)", 2, 0}};
    {
        int v1 = -1, v2 = -1, v3 = -1, v4 = -1;
        (void)hipDeviceGetAttribute(&v1, hipDeviceAttributeDirectManagedMemAccessFromHost, 0);
        (void)hipDeviceGetAttribute(&v2, hipDeviceAttributePageableMemoryAccess, 0);
        (void)hipDeviceGetAttribute(&v3, hipDeviceAttributeHostNativeAtomicSupported, 0);
        (void)hipDeviceGetAttribute(&v4, hipDeviceAttributeCanUseHostPointerForRegisteredMem, 0);
        printf("{\"probe\": \"bar_dev_attr\", \"direct_managed_from_host\": %d, \"pageable\": %d, "
               "\"host_native_atomic\": %d, \"host_ptr_registered\": %d}\n", v1, v2, v3, v4);
    }
    for (const Kind &k : kinds) {
        void *p = NULL, *pd = NULL;
        hipError_t e = hipSuccess;
        if (k.how == 0) e = hipMalloc(&p, 1 << 20);
        else if (k.how == 1) e = hipExtMallocWithFlags(&p, 1 << 20, k.flags);
        else e = hipHostMalloc(&p, 1 << 20, hipHostMallocMapped | hipHostMallocCoherent);
        if (e != hipSuccess) {
            printf("{\"probe\": \"bar\", \"memory\": \"%s\", \"alloc\": \"%s\"}\n", k.name, hipGetErrorString(e));
            fflush(stdout);
            continue;
        }
        pd = p;
        if (k.how == 2 && hipHostGetDevicePointer(&pd, p, 0) != hipSuccess) return 1;
        if (hipMemset(pd, 0, 1 << 20) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 1;
        const int acc = host_access((volatile uint32_t *)p);
        hipPointerAttribute_t pa;
        memset(&pa, 0, sizeof(pa));
        const hipError_t pe = hipPointerGetAttributes(&pa, p);
        printf("{\"probe\": \"bar_attr\", \"memory\": \"%s\", \"rc\": %d, \"type\": %d, \"device_ptr\": %d, "
               "\"host_ptr\": %d, \"host_eq_dev\": %d, \"is_managed\": %d, \"alloc_flags\": %u}\n",
               k.name, (int)pe, (int)pa.type, pa.devicePointer != NULL, pa.hostPointer != NULL,
               pa.hostPointer == pa.devicePointer, pa.isManaged, pa.allocationFlags);
        double stage_us = -1.0, rt_us = -1.0;
        uint32_t got = 0, npoll = 0;
        if (acc) {
            uint8_t *dst = (uint8_t *)p + 4096;
            double best = 1e30;
            for (int round = 0; round < 5; round++) {
                const double a = now_s();
                for (size_t r = 0; r < stage_reps / 5; r++) {
                    memcpy(dst, src, kbytes);
                    __atomic_thread_fence(__ATOMIC_SEQ_CST);
                }
                const double us = (now_s() - a) / (stage_reps / 5) * 1e6;
                if (us < best) best = us;
            }
            stage_us = best;
            /* the same copy as 32-byte non-temporal and plain AVX stores */
            double best_nt = 1e30, best_st = 1e30;
            for (int round = 0; round < 5; round++) {
                double a = now_s();
                for (size_t r = 0; r < stage_reps / 5; r++) {
                    copy_nt32(dst, src, kbytes);
                    __atomic_thread_fence(__ATOMIC_SEQ_CST);
                }
                double us = (now_s() - a) / (stage_reps / 5) * 1e6;
                if (us < best_nt) best_nt = us;
                a = now_s();
                for (size_t r = 0; r < stage_reps / 5; r++) {
                    copy_st32(dst, src, kbytes);
                    __atomic_thread_fence(__ATOMIC_SEQ_CST);
                }
                us = (now_s() - a) / (stage_reps / 5) * 1e6;
                if (us < best_st) best_st = us;
            }
            printf("{\"probe\": \"bar_copy\", \"memory\": \"%s\", \"bytes\": %zu, \"memcpy_us\": %.3f, "
                   "\"avx_nt32_us\": %.3f, \"avx_st32_us\": %.3f}\n", k.name, kbytes, stage_us, best_nt, best_st);
            /* ping-pong: flag in this memory, answer in mapped host memory */
            volatile uint32_t *flag = (volatile uint32_t *)p;
            flag[0] = 0;
            __atomic_store_n(ack_h, 0u, __ATOMIC_SEQ_CST);
            __atomic_thread_fence(__ATOMIC_SEQ_CST);
            hipLaunchKernelGGL(pong, dim3(1), dim3(64), 0, 0, (const uint32_t *)pd, ack_d, msgs, polls);
            /* the kernel's start: wait until it has answered message 1 */
            const double t_start = now_s();
            flag[0] = 1;
            while (__atomic_load_n(ack_h, __ATOMIC_ACQUIRE) != 1u && now_s() - t_start < 1.0) {
            }
            const double a = now_s();
            uint32_t i = 2;
            for (; i <= msgs; i++) {
                flag[0] = i;
                __atomic_thread_fence(__ATOMIC_SEQ_CST);
                const double w0 = now_s();
                while (__atomic_load_n(ack_h, __ATOMIC_ACQUIRE) != i) {
                    if (now_s() - w0 > 0.1) break; /* lost: stop measuring */
                }
                if (__atomic_load_n(ack_h, __ATOMIC_ACQUIRE) != i) break;
            }
            got = i - 1;
            rt_us = got > 1 ? (now_s() - a) / (double)(got - 1) * 1e6 : -1.0;
            flag[0] = 0xffffffffu;
            __atomic_thread_fence(__ATOMIC_SEQ_CST);
            if (hipDeviceSynchronize() != hipSuccess) return 1;
            if (hipMemcpy(&npoll, polls, 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        }
        printf("{\"probe\": \"bar\", \"memory\": \"%s\", \"host_access\": %d, \"stage_bytes\": %zu, "
               "\"host_stage_us\": %.3f, \"pingpong_msgs\": %u, \"pingpong_round_trip_us\": %.3f, "
               "\"device_polls\": %u}\n",
               k.name, acc, kbytes, stage_us, got, rt_us, npoll);
        fflush(stdout);
        if (k.how == 2) (void)hipHostFree(p);
        else (void)hipFree(p);
    }
    return 0;
}
