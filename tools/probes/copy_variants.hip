// copy_variants.hip -- layouts of the 256 MiB streaming copy (the PE_size = 1
// identity fold, the bench's dominant kernel), timed with HIP events
// (tuning tool, not part of the library).
//   build: hipcc --offload-arch=gfx950 -O3 tools/probes/copy_variants.hip -o tools/probes/copy_variants
//
//   gs      the library's copy_segments: grid-stride, U vectors per lane spaced
//           one block apart, all loads then all stores, `nt sc1` stores
//   part    each block owns one contiguous 1/G of the buffer (same inner loop)
//   pipe    grid-stride, software-pipelined: the loads of pass p+1 are issued
//           before the stores of pass p
//   plain   gs with plain stores (no nt/sc1), for reference
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st_nt_sc1(u32x4 *p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

template <int BS, int U, bool NT>
__global__ __launch_bounds__(BS) void copy_gs(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, size_t nvec) {
    const size_t step = (size_t)gridDim.x * BS * U;
    for (size_t base = (size_t)blockIdx.x * BS * U + threadIdx.x; base < nvec; base += step) {
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * BS;
            if (i < nvec) x[u] = s[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * BS;
            if (i < nvec) {
                if (NT) st_nt_sc1(d + i, x[u]);
                else d[i] = x[u];
            }
        }
    }
}

template <int BS, int U>
__global__ __launch_bounds__(BS) void copy_part(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, size_t nvec) {
    const size_t per = (nvec + gridDim.x - 1) / gridDim.x;
    const size_t lo = (size_t)blockIdx.x * per, hi = lo + per < nvec ? lo + per : nvec;
    for (size_t base = lo + threadIdx.x; base < hi; base += (size_t)BS * U) {
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * BS;
            if (i < hi) x[u] = s[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * BS;
            if (i < hi) st_nt_sc1(d + i, x[u]);
        }
    }
}

template <int BS, int U>
__global__ __launch_bounds__(BS) void copy_pipe(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, size_t nvec) {
    const size_t step = (size_t)gridDim.x * BS * U;
    size_t base = (size_t)blockIdx.x * BS * U + threadIdx.x;
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        size_t i = base + (size_t)u * BS;
        if (i < nvec) x[u] = s[i];
    }
    while (base < nvec) {
        const size_t nb = base + step;
        u32x4 y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = nb + (size_t)u * BS;
            if (i < nvec) y[u] = s[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * BS;
            if (i < nvec) st_nt_sc1(d + i, x[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = y[u];
        base = nb;
    }
}

template <typename K>
static double time_us(K kernel, unsigned grid, unsigned bs, const u32x4 *s, u32x4 *d, size_t nvec) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    std::vector<float> t;
    for (int r = 0; r < 25; ++r) {
        CHECK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(kernel, dim3(grid), dim3(bs), 0, 0, s, d, nvec);
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (r >= 5) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return t[t.size() / 2] * 1e3;
}

int main() {
    const size_t bytes = 256ull << 20, nvec = bytes / 16;
    u32x4 *s, *d;
    CHECK(hipMalloc(&s, bytes));
    CHECK(hipMalloc(&d, bytes));
    CHECK(hipMemset(s, 0x3c, bytes));
    CHECK(hipMemset(d, 0x5a, bytes));
    CHECK(hipDeviceSynchronize());
    int cus = 256;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    auto report = [&](const char *name, int bpc, double us) {
        printf("%-22s blocks/CU %2d  %7.2f us  %6.0f GB/s\n", name, bpc, us, 2.0 * bytes / us / 1e3);
    };
    for (int rep = 0; rep < 2; ++rep) {
        for (int bpc : {1, 2, 4}) {
            const unsigned g = cus * bpc;
            report("gs 256x8 (library)", bpc, time_us(copy_gs<256, 8, true>, g, 256, s, d, nvec));
            report("gs 256x16", bpc, time_us(copy_gs<256, 16, true>, g, 256, s, d, nvec));
            report("gs 512x8", bpc, time_us(copy_gs<512, 8, true>, g, 512, s, d, nvec));
            report("gs 256x8 plain store", bpc, time_us(copy_gs<256, 8, false>, g, 256, s, d, nvec));
            report("part 256x8", bpc, time_us(copy_part<256, 8>, g, 256, s, d, nvec));
            report("part 256x4", bpc, time_us(copy_part<256, 4>, g, 256, s, d, nvec));
            report("pipe 256x4", bpc, time_us(copy_pipe<256, 4>, g, 256, s, d, nvec));
            report("pipe 256x8", bpc, time_us(copy_pipe<256, 8>, g, 256, s, d, nvec));
        }
        // many small blocks, one pass each
        const unsigned gfull = (unsigned)(nvec / (256 * 8));
        report("gs 256x8 one pass", (int)(gfull / cus), time_us(copy_gs<256, 8, true>, gfull, 256, s, d, nvec));
        report("gs 256x4 one pass", (int)(2 * gfull / cus),
               time_us(copy_gs<256, 4, true>, 2 * gfull, 256, s, d, nvec));
    }
    return 0;
}
