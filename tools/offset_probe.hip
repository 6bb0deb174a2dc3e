// offset_probe.hip -- does the relative placement of source and target in HBM
// change the copy rate? (tuning tool, not part of the library)
//   hipcc --offload-arch=gfx950 -O2 -Iinclude tools/offset_probe.hip -Losss-gasnet_amd/lib -lshmem_reduce \
//       -Wl,-rpath,'$ORIGIN/../osss-gasnet_amd/lib' -o tools/offset_probe
// Copies 256 MiB with the library's copy kernel (mi355_copy_segments) from
// base to base + 256 MiB + delta for a range of deltas, and reads/writes
// only, timed with HIP events (median of 30 launches each).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "mi355_reduce.h"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void read_k(const u32x4 *s, unsigned long long n, unsigned *out) {
    u32x4 acc = {0, 0, 0, 0};
    for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * 256)
        acc ^= s[i];
    if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x12345678u) out[0] = 1;
}

__global__ __launch_bounds__(256) void write_k(u32x4 *d, unsigned long long n) {
    const u32x4 v = {1, 2, 3, 4};
    for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * 256)
        __builtin_nontemporal_store(v, d + i);
}

int main() {
    const size_t S = 256ull << 20;
    char *base;
    const size_t total = 2 * S + (128ull << 20);  // room for every delta below
    CHECK(hipMalloc((void **)&base, total));
    CHECK(hipMemset(base, 1, total));
    unsigned *out;
    CHECK(hipMalloc((void **)&out, 64));
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    auto timed = [&](auto fn) {
        std::vector<float> t;
        for (int r = 0; r < 33; ++r) {
            CHECK(hipEventRecord(a, st));
            fn();
            CHECK(hipEventRecord(b, st));
            CHECK(hipEventSynchronize(b));
            float ms;
            CHECK(hipEventElapsedTime(&ms, a, b));
            if (r >= 3) t.push_back(ms * 1e3f);
        }
        std::sort(t.begin(), t.end());
        return t[t.size() / 2];
    };
    int ncu = 256;
    for (int blocks : {ncu, 2 * ncu, 4 * ncu, 8 * ncu}) {
        float us = timed([&] { hipLaunchKernelGGL(read_k, dim3(blocks), dim3(256), 0, st, (const u32x4 *)base, S / 16, out); });
        printf("read-only  256 MiB, %4d blocks: %7.2f us  %6.0f GB/s\n", blocks, us, S / (us * 1e-6) / 1e9);
    }
    for (int blocks : {ncu, 2 * ncu, 4 * ncu, 8 * ncu}) {
        float us = timed([&] { hipLaunchKernelGGL(write_k, dim3(blocks), dim3(256), 0, st, (u32x4 *)base, S / 16); });
        printf("write-only 256 MiB, %4d blocks: %7.2f us  %6.0f GB/s\n", blocks, us, S / (us * 1e-6) / 1e9);
    }
    const long long deltas[] = {0, 256, 4096, 8192, 16384, 65536, 1 << 20, (2 << 20) + 4096, (16 << 20) + 12288,
                                -4096, -(1 << 20)};
    for (long long d : deltas) {
        void *dst = base + S + (32ll << 20) + d;
        if ((char *)dst + S > base + total) exit(3);  // stay inside the allocation
        const void *src = base;
        size_t nb = S;
        float us = timed([&] {
            if (mi355_copy_segments(&dst, &src, &nb, 1, st) != 0) exit(2);
        });
        printf("copy 256 MiB, dst - src = 288 MiB %+9lld B: %7.2f us  %6.0f GB/s\n", d, us, 2.0 * S / (us * 1e-6) / 1e9);
    }
    return 0;
}
