// signal_probe.hip -- how the copy kernel's completion reaches the host
// (tuning tool, not part of the library).
//   hipcc --offload-arch=gfx950 -O2 tools/signal_probe.hip -o tools/signal_probe
//
// One "call" = launch a streaming copy (the library's copy_segments shape:
// UNROLL 4, pipelined, nt sc1 stores, one block per CU or fewer) on a
// blocking stream, then spin on host-coherent memory until the kernel says it
// is done. Completion variants:
//   counter : every block adds 1 to a device counter (agent scope); the last
//             one resets it and stores the epoch to the host flag (library)
//   hostadd : every block adds 1 to a host-coherent counter (system scope,
//             no return value used); the host waits for the call's total
//   slots   : every block stores the epoch to its own host-coherent slot;
//             the host scans the slots
// Prints the mean per-call time over K calls after warmup, per size.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kBlock = 256, U = 4;

struct P {
    u32x4 *dst;
    const u32x4 *src;
    unsigned long long nvec;
    unsigned *count;     // device counter (counter) / host counter (hostadd) / host slots (slots)
    unsigned *flag;      // host flag (counter)
    unsigned epoch;
};

__device__ __forceinline__ void st16(u32x4 *p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void copy_k(P p) {
    const unsigned long long step = (unsigned long long)gridDim.x * kBlock * U;
    unsigned long long base = (unsigned long long)blockIdx.x * kBlock * U + threadIdx.x;
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const unsigned long long i = base + (unsigned long long)u * kBlock;
        if (i < p.nvec) x[u] = p.src[i];
    }
    while (base < p.nvec) {
        const unsigned long long next = base + step;
        u32x4 y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned long long i = next + (unsigned long long)u * kBlock;
            if (i < p.nvec) y[u] = p.src[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned long long i = base + (unsigned long long)u * kBlock;
            if (i < p.nvec) st16(p.dst + i, x[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = y[u];
        base = next;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x != 0) return;
    if constexpr (MODE == 0) {
        const unsigned prev = __hip_atomic_fetch_add(p.count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev + 1 == gridDim.x) {
            __hip_atomic_store(p.count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(p.flag, p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    } else if constexpr (MODE == 1) {
        __hip_atomic_fetch_add(p.count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
        __hip_atomic_store(p.count + blockIdx.x, p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double now() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

int main(int argc, char **argv) {
    const size_t big = 256ull << 20;
    void *src, *dst;
    CHECK(hipMalloc(&src, big));
    CHECK(hipMalloc(&dst, big));
    CHECK(hipMemset(src, 1, big));
    unsigned *dcount, *hflag, *hcount, *hslots;
    CHECK(hipMalloc(&dcount, 64));
    CHECK(hipMemset(dcount, 0, 64));
    CHECK(hipHostMalloc((void **)&hflag, 64, hipHostMallocCoherent | hipHostMallocMapped));
    CHECK(hipHostMalloc((void **)&hcount, 64, hipHostMallocCoherent | hipHostMallocMapped));
    CHECK(hipHostMalloc((void **)&hslots, 4096 * 4, hipHostMallocCoherent | hipHostMallocMapped));
    *hflag = 0;
    *hcount = 0;
    for (int i = 0; i < 4096; ++i) hslots[i] = 0;
    hipStream_t st;
    CHECK(hipStreamCreateWithFlags(&st, hipStreamDefault));
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    unsigned epoch = 0;
    unsigned long long hc_target = 0;
    const size_t sizes[] = {65536, 1 << 20, 16 << 20, big};
    for (int rep = 0; rep < 2; ++rep)
        for (size_t bytes : sizes) {
            const unsigned long long nvec = bytes / 16;
            unsigned long long g = (nvec + kBlock * U - 1) / (kBlock * U);
            if (g > (unsigned long long)cus) g = cus;
            const int calls = bytes <= (1 << 20) ? 4000 : bytes <= (16 << 20) ? 1000 : 200;
            for (int mode = 0; mode < 3; ++mode) {
                double t0 = 0;
                for (int c = -20; c < calls; ++c) {
                    if (c == 0) t0 = now();
                    ++epoch;
                    P p{(u32x4 *)dst, (const u32x4 *)src, nvec, mode == 0 ? dcount : mode == 1 ? hcount : hslots,
                        hflag, epoch};
                    if (mode == 0)
                        hipExtLaunchKernelGGL(copy_k<0>, dim3(g), dim3(kBlock), 0, st, nullptr, nullptr, 0, p);
                    else if (mode == 1)
                        hipExtLaunchKernelGGL(copy_k<1>, dim3(g), dim3(kBlock), 0, st, nullptr, nullptr, 0, p);
                    else
                        hipExtLaunchKernelGGL(copy_k<2>, dim3(g), dim3(kBlock), 0, st, nullptr, nullptr, 0, p);
                    const double tw = now();
                    unsigned spins = 0;
#define WAIT(cond)                                                                          \
    while (!(cond)) {                                                                       \
        __builtin_ia32_pause();                                                             \
        if ((++spins & 4095u) == 0 && now() - tw > 1.0) {                                   \
            fprintf(stderr, "mode %d: completion not seen within 1 s (%zu bytes)\n", mode, bytes); \
            CHECK(hipStreamSynchronize(st));                                                \
            return 1;                                                                       \
        }                                                                                   \
    }
                    if (mode == 0) {
                        WAIT(__atomic_load_n(hflag, __ATOMIC_ACQUIRE) == epoch);
                    } else if (mode == 1) {
                        hc_target += g;
                        WAIT(__atomic_load_n(hcount, __ATOMIC_ACQUIRE) == (unsigned)hc_target);
                    } else {
                        for (unsigned long long b = 0; b < g; ++b)
                            WAIT(__atomic_load_n(hslots + b, __ATOMIC_ACQUIRE) == epoch);
                    }
                }
                const double t = (now() - t0) / calls;
                CHECK(hipStreamSynchronize(st));
                if (rep == 1)
                    printf("%-8s %10zu bytes  %4llu blocks  %8.2f us per call\n",
                           mode == 0 ? "counter" : mode == 1 ? "hostadd" : "slots", bytes, g, t * 1e6);
            }
        }
    return 0;
}
