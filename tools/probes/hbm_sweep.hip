// hbm_sweep.hip -- launch-geometry / cache-policy sweep for the streaming
// kernels of the reduction path (copy = the PE_size 1 identity fold, and the
// k-source double-sum fold of the reduce-scatter leg). Standalone tuning tool,
// not part of the library.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/hbm_sweep.hip -o tools/probes/hbm_sweep
// run:   tools/probes/hbm_sweep [MiB]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

template <int POL>
__device__ __forceinline__ u32x4 ld(const u32x4 *p) {
    if constexpr ((POL < 4 || POL == 7) && (POL & 1)) return __builtin_nontemporal_load(p);
    else return *p;
}
template <int POL>
__device__ __forceinline__ void st(u32x4 *p, u32x4 v) {
    if constexpr (POL == 4) asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
    else if constexpr (POL == 5) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
    else if constexpr (POL == 6 || POL == 7) asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
    else if constexpr (POL & 2) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// grid-stride copy, UNROLL vectors per lane spaced one block apart
template <int BS, int U, int POL>
__global__ __launch_bounds__(BS) void copy_gs(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, uint64_t nvec) {
    const uint64_t step = (uint64_t)gridDim.x * BS * U;
    for (uint64_t base = (uint64_t)blockIdx.x * BS * U + threadIdx.x; base < nvec; base += step) {
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            uint64_t i = base + (uint64_t)u * BS;
            if (i < nvec) x[u] = ld<POL>(s + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            uint64_t i = base + (uint64_t)u * BS;
            if (i < nvec) st<POL>(d + i, x[u]);
        }
    }
}

// k-source fold (double sum), same geometry
template <int BS, int U, int K, int POL>
__global__ __launch_bounds__(BS) void fold_gs(const u32x4 *const *__restrict__ srcs_unused,
                                              const u32x4 *s0, const u32x4 *s1, const u32x4 *s2, const u32x4 *s3,
                                              const u32x4 *s4, const u32x4 *s5, const u32x4 *s6, const u32x4 *s7,
                                              u32x4 *__restrict__ d, uint64_t nvec) {
    const u32x4 *s[8] = {s0, s1, s2, s3, s4, s5, s6, s7};
    const uint64_t step = (uint64_t)gridDim.x * BS * U;
    for (uint64_t base = (uint64_t)blockIdx.x * BS * U + threadIdx.x; base < nvec; base += step) {
        u32x4 x[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            uint64_t i = base + (uint64_t)u * BS;
            if (i < nvec) {
#pragma unroll
                for (int k = 0; k < K; ++k) x[u][k] = ld<POL>(s[k] + i);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            uint64_t i = base + (uint64_t)u * BS;
            if (i < nvec) {
                f64x2 acc = __builtin_bit_cast(f64x2, x[u][0]);
#pragma unroll
                for (int k = 1; k < K; ++k) acc += __builtin_bit_cast(f64x2, x[u][k]);
                st<POL>(d + i, __builtin_bit_cast(u32x4, acc));
            }
        }
    }
}

struct Res { const char *name; int bs, u, pol, bpc; double us, gbs; };

template <typename F>
double time_it(F launch, int reps) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) launch();
    CHECK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(a));
        launch();
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms; CHECK(hipEventElapsedTime(&ms, a, b));
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2] * 1e3;  // median us
}

int g_cus = 256;
std::vector<Res> results;

template <int BS, int U, int POL>
void run_copy(const u32x4 *s, u32x4 *d, uint64_t nvec, size_t bytes) {
    for (int bpc : {1, 2, 4, 8, 16, 32}) {
        uint64_t want = (nvec + (uint64_t)BS * U - 1) / ((uint64_t)BS * U);
        uint64_t cap = (uint64_t)g_cus * bpc;
        unsigned grid = (unsigned)std::min(want, cap);
        double us = time_it([&] { hipLaunchKernelGGL((copy_gs<BS, U, POL>), dim3(grid), dim3(BS), 0, 0, s, d, nvec); }, 20);
        results.push_back({"copy", BS, U, POL, bpc, us, 2.0 * bytes / (us * 1e-6) / 1e9});
    }
}

template <int BS, int U, int K, int POL>
void run_fold(const u32x4 *const *s, u32x4 *d, uint64_t nvec, size_t bytes) {
    for (int bpc : {1, 2, 4, 8}) {
        uint64_t want = (nvec + (uint64_t)BS * U - 1) / ((uint64_t)BS * U);
        uint64_t cap = (uint64_t)g_cus * bpc;
        unsigned grid = (unsigned)std::min(want, cap);
        double us = time_it([&] {
            hipLaunchKernelGGL((fold_gs<BS, U, K, POL>), dim3(grid), dim3(BS), 0, 0, nullptr,
                               s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7], d, nvec); }, 10);
        static char nm[8][16];
        snprintf(nm[K - 1], 16, "fold%d", K);
        results.push_back({nm[K - 1], BS, U, POL, bpc, us, (K + 1.0) * bytes / (us * 1e-6) / 1e9});
    }
}

int main(int argc, char **argv) {
    size_t mib = argc > 1 ? atol(argv[1]) : 256;
    size_t bytes = mib << 20;
    uint64_t nvec = bytes / 16;
    CHECK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, 0));
    u32x4 *bufs[9];
    for (int i = 0; i < 9; ++i) {
        CHECK(hipMalloc(&bufs[i], bytes));
        CHECK(hipMemset(bufs[i], i + 1, bytes));
    }
    // hipMemcpy D2D for reference
    double us_memcpy = time_it([&] { CHECK(hipMemcpyAsync(bufs[1], bufs[0], bytes, hipMemcpyDeviceToDevice, 0)); }, 20);
    printf("hipMemcpyAsync D2D %zu MiB: %.1f us  %.0f GB/s (read+write)\n", mib, us_memcpy, 2.0 * bytes / (us_memcpy * 1e-6) / 1e9);

    const u32x4 *srcs[8];
    for (int k = 0; k < 8; ++k) srcs[k] = bufs[k];
    // folds with the library's store (nt sc1): pol 6 = plain loads, 7 = nt loads
#define FOLDS(K)                                              \
    run_fold<256, 1, K, 6>(srcs, bufs[8], nvec, bytes);       \
    run_fold<256, 1, K, 7>(srcs, bufs[8], nvec, bytes);       \
    run_fold<256, 2, K, 6>(srcs, bufs[8], nvec, bytes);       \
    run_fold<256, 2, K, 7>(srcs, bufs[8], nvec, bytes);       \
    run_fold<256, 4, K, 6>(srcs, bufs[8], nvec, bytes);       \
    run_fold<256, 4, K, 7>(srcs, bufs[8], nvec, bytes);       \
    run_fold<512, 1, K, 7>(srcs, bufs[8], nvec, bytes);       \
    run_fold<512, 2, K, 7>(srcs, bufs[8], nvec, bytes);
    FOLDS(2)
    FOLDS(3)
    FOLDS(4)
    FOLDS(8)

    std::sort(results.begin(), results.end(), [](const Res &a, const Res &b) {
        int c = strcmp(a.name, b.name);
        return c != 0 ? c < 0 : a.gbs > b.gbs;
    });
    printf("%-6s %5s %3s %4s %4s %9s %8s\n", "kernel", "block", "U", "pol", "b/CU", "us", "GB/s");
    for (auto &r : results)
        printf("%-6s %5d %3d %4d %4d %9.1f %8.0f\n", r.name, r.bs, r.u, r.pol, r.bpc, r.us, r.gbs);
    return 0;
}
