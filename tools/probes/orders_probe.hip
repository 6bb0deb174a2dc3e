// orders_probe.hip -- launch shapes of the every-member-order fold
// (combine_orders_vec: K sources -> K outputs, output q = src q first, then the
// others in order) on one GPU, 256 MiB per PE split into K shards as in an
// N = K PE call; double sum, `sc1` stores, non-temporal loads; HIP events,
// median of 7 (tuning tool, not part of the library).
//   build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/probes/orders_probe.hip -o tools/probes/orders_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <stdint.h>

#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
union P2 {
    u32x4 v;
    double e[2];
};
struct Ptrs {
    const u32x4 *s[8];
    u32x4 *d[8];
};

__device__ __forceinline__ void st_sc1(u32x4 *p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

template <int K, int U>
__global__ __launch_bounds__(256) void orders(Ptrs p, size_t nvec) {
    const size_t step = (size_t)gridDim.x * 256 * U;
    for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < nvec; base += step) {
        P2 x[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * 256;
            if (i < nvec) {
#pragma unroll
                for (int k = 0; k < K; ++k) x[u][k].v = __builtin_nontemporal_load(p.s[k] + i);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * 256;
            if (i >= nvec) continue;
#pragma unroll
            for (int q = 0; q < K; ++q) {
                P2 a = x[u][q];
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    if (k == q) continue;
                    a.e[0] = a.e[0] + x[u][k].e[0];
                    a.e[1] = a.e[1] + x[u][k].e[1];
                }
                st_sc1(p.d[q] + i, a.v);
            }
        }
    }
}

template <typename F>
double time_us(F launch) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    launch();
    launch();
    CHECK(hipDeviceSynchronize());
    std::vector<double> ts;
    for (int r = 0; r < 7; ++r) {
        CHECK(hipEventRecord(a, 0));
        launch();
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms * 1e3);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main() {
    const size_t S = 256ull << 20;
    int cus = 256;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    char *src, *dst;
    CHECK(hipMalloc(&src, S));
    CHECK(hipMalloc(&dst, S));
    CHECK(hipMemset(src, 0x3f, S));
    CHECK(hipMemset(dst, 0, S));
    auto ptrs = [&](int k) {
        Ptrs p{};
        for (int i = 0; i < k; ++i) {
            p.s[i] = (const u32x4 *)(src + i * (S / k));
            p.d[i] = (u32x4 *)(dst + i * (S / k));
        }
        return p;
    };
#define RUN(K, U, BPC) do {                                                                       \
        Ptrs p_ = ptrs(K);                                                                        \
        const size_t nvec = S / K / 16;                                                           \
        double us = time_us([&] { hipLaunchKernelGGL((orders<K, U>), dim3(cus * BPC), dim3(256), 0, 0, p_, nvec); }); \
        printf("orders<K=%d,U=%d> %d blocks/CU %8.2f us %6.0f GB/s\n", K, U, BPC, us, 2.0 * S / us / 1e3); \
        fflush(stdout);                                                                           \
    } while (0)
    for (int r = 0; r < 4; ++r) {
        if (r == 2) {  // passes 2-3: random full-mantissa doubles instead of a memset pattern
            std::vector<double> h(S / 8);
            uint64_t x = 88172645463325252ull;
            for (auto &v : h) {
                x ^= x << 13; x ^= x >> 7; x ^= x << 17;
                v = (double)(int64_t)x * 0x1p-63;
            }
            CHECK(hipMemcpy(src, h.data(), S, hipMemcpyHostToDevice));
            printf("--- random source data\n");
        }
        RUN(2, 1, 2); RUN(2, 1, 4); RUN(2, 1, 8); RUN(2, 2, 2); RUN(2, 2, 4); RUN(2, 4, 2); RUN(2, 4, 4);
        RUN(3, 1, 4); RUN(3, 2, 1); RUN(3, 2, 4); RUN(3, 4, 4);
        RUN(4, 1, 1); RUN(4, 1, 4); RUN(4, 1, 8); RUN(4, 2, 4); RUN(4, 2, 8); RUN(4, 4, 4);
        RUN(8, 4, 8); RUN(8, 2, 8); RUN(8, 4, 4); RUN(8, 1, 8);
    }
    return 0;
}
