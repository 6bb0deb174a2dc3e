// fold_variants.hip -- k-source double-sum fold (the reduce-scatter kernel),
// grid-stride as in the library vs software-pipelined, 256 MiB per source,
// timed with HIP events (tuning tool, not part of the library).
//   build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/probes/fold_variants.hip -o tools/probes/fold_variants
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
union P2 {
    u32x4 v;
    double e[2];
};

__device__ __forceinline__ void st16(u32x4 *p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

struct Srcs {
    const u32x4 *s[8];
};

template <int K, int U>
__global__ __launch_bounds__(256) void fold_gs(Srcs in, u32x4 *d, size_t nvec) {
    const size_t step = (size_t)gridDim.x * 256 * U;
    for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < nvec; base += step) {
        P2 x[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * 256;
            if (i < nvec) {
#pragma unroll
                for (int k = 0; k < K; ++k) x[u][k].v = __builtin_nontemporal_load(in.s[k] + i);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * 256;
            if (i < nvec) {
                P2 a = x[u][0];
#pragma unroll
                for (int k = 1; k < K; ++k) {
                    a.e[0] = a.e[0] + x[u][k].e[0];
                    a.e[1] = a.e[1] + x[u][k].e[1];
                }
                st16(d + i, a.v);
            }
        }
    }
}

template <int K, int U>
__global__ __launch_bounds__(256) void fold_pipe(Srcs in, u32x4 *d, size_t nvec) {
    const size_t step = (size_t)gridDim.x * 256 * U;
    size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    P2 x[U][K];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        size_t i = base + (size_t)u * 256;
        if (i < nvec) {
#pragma unroll
            for (int k = 0; k < K; ++k) x[u][k].v = __builtin_nontemporal_load(in.s[k] + i);
        }
    }
    while (base < nvec) {
        const size_t nb = base + step;
        P2 y[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = nb + (size_t)u * 256;
            if (i < nvec) {
#pragma unroll
                for (int k = 0; k < K; ++k) y[u][k].v = __builtin_nontemporal_load(in.s[k] + i);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * 256;
            if (i < nvec) {
                P2 a = x[u][0];
#pragma unroll
                for (int k = 1; k < K; ++k) {
                    a.e[0] = a.e[0] + x[u][k].e[0];
                    a.e[1] = a.e[1] + x[u][k].e[1];
                }
                st16(d + i, a.v);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < K; ++k) x[u][k] = y[u][k];
        base = nb;
    }
}

template <typename F>
static double time_us(F launch) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    std::vector<float> t;
    for (int r = 0; r < 15; ++r) {
        CHECK(hipEventRecord(a, 0));
        launch();
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (r >= 3) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2] * 1e3;
}

int main() {
    const size_t bytes = 256ull << 20, nvec = bytes / 16;
    Srcs in{};
    for (int k = 0; k < 8; ++k) {
        void *p;
        CHECK(hipMalloc(&p, bytes));
        CHECK(hipMemset(p, 0x11 * (k + 1), bytes));
        in.s[k] = (const u32x4 *)p;
    }
    u32x4 *d;
    CHECK(hipMalloc(&d, bytes));
    CHECK(hipMemset(d, 0, bytes));
    CHECK(hipDeviceSynchronize());
    int cus = 256;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    auto rep = [&](const char *name, int k, int bpc, double us) {
        printf("%-14s k=%d blocks/CU %d  %8.2f us  %6.0f GB/s\n", name, k, bpc, us, (k + 1.0) * bytes / us / 1e3);
    };
#define RUN(KERNEL, K, U, BPC) rep(#KERNEL "<" #U ">", K, BPC, time_us([&] { \
        hipLaunchKernelGGL((KERNEL<K, U>), dim3(cus * BPC), dim3(256), 0, 0, in, d, nvec); }))
    for (int r = 0; r < 2; ++r) {
        RUN(fold_gs, 2, 1, 2);   // library shape for k = 2
        RUN(fold_pipe, 2, 1, 1);
        RUN(fold_pipe, 2, 1, 2);
        RUN(fold_pipe, 2, 2, 1);
        RUN(fold_pipe, 2, 2, 2);
        RUN(fold_gs, 4, 1, 1);   // library shape for k = 4
        RUN(fold_pipe, 4, 1, 1);
        RUN(fold_pipe, 4, 1, 2);
        RUN(fold_gs, 8, 4, 8);   // library shape for k = 8
        RUN(fold_pipe, 8, 1, 1);
        RUN(fold_pipe, 8, 1, 2);
        RUN(fold_pipe, 8, 2, 1);
        RUN(fold_pipe, 8, 2, 2);
    }
    return 0;
}
