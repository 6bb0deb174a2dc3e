// copy_tail.hip -- where the 1-PE identity copy's time goes across its blocks
// (round 6 probe). The library's copy loop (combine.hip copy_segments<4,1>:
// grid-stride, one block per CU, 4 vectors per lane software-pipelined, plain
// loads, `nt sc1` stores) with each block's start and end stamped with
// s_memrealtime (100 MHz), 256 MiB, warm (one pair) and cold (5 pairs in
// turn). If the last block ends well after the median one, a balanced
// distribution of the work (a work queue) would shorten the call.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/copy_tail.hip -o tools/probes/copy_tail
// run:   tools/probes/copy_tail      (one JSON line per configuration)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int kBlock = 256;

__device__ __forceinline__ void st16(u32x4 *p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

template <int UNROLL>
__global__ __launch_bounds__(kBlock) void copy_stamped(const u32x4 *s, u32x4 *d, uint64_t nvec, uint64_t *stamps) {
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    const uint64_t step = (uint64_t)gridDim.x * kBlock * UNROLL;
    uint64_t base = (uint64_t)blockIdx.x * kBlock * UNROLL + threadIdx.x;
    u32x4 x[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
        const uint64_t i = base + (uint64_t)u * kBlock;
        if (i < nvec) x[u] = s[i];
    }
    while (base < nvec) {
        const uint64_t next = base + step;
        u32x4 y[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = next + (uint64_t)u * kBlock;
            if (i < nvec) y[u] = s[i];
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = base + (uint64_t)u * kBlock;
            if (i < nvec) st16(d + i, x[u]);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) x[u] = y[u];
        base = next;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = t_start;
        stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

int main() {
    const size_t S = 256ull << 20;
    const uint64_t nvec = S / 16;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int pairs = 5;
    std::vector<char *> bufs(2 * pairs);
    for (auto &b : bufs) {
        CHECK(hipMalloc((void **)&b, S));
        CHECK(hipMemset(b, 1, S));
    }
    for (int bpc : {1, 2}) {
        const unsigned grid = (unsigned)cus * bpc;
        uint64_t *stamps;
        CHECK(hipMalloc((void **)&stamps, 2 * grid * sizeof(uint64_t)));
        std::vector<uint64_t> h(2 * grid);
        hipEvent_t e0, e1;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        for (int cold = 0; cold < 2; ++cold) {
            std::vector<double> span, med_end, last_end, first_end, kern;
            for (int r = 0; r < 60; ++r) {
                const int p = cold ? r % pairs : 0;
                CHECK(hipEventRecord(e0, 0));
                copy_stamped<4><<<grid, kBlock>>>((const u32x4 *)bufs[2 * p], (u32x4 *)bufs[2 * p + 1], nvec, stamps);
                CHECK(hipEventRecord(e1, 0));
                CHECK(hipDeviceSynchronize());
                float ms = 0;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                if (r < 10) continue;
                CHECK(hipMemcpy(h.data(), stamps, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
                uint64_t t0 = UINT64_MAX;
                std::vector<uint64_t> ends(grid);
                for (unsigned b = 0; b < grid; ++b) {
                    t0 = std::min(t0, h[2 * b]);
                    ends[b] = h[2 * b + 1];
                }
                for (auto &e : ends) e -= t0;
                std::sort(ends.begin(), ends.end());
                first_end.push_back(ends.front() * 0.01);
                med_end.push_back(ends[grid / 2] * 0.01);
                last_end.push_back(ends.back() * 0.01);
                kern.push_back(ms * 1e3);
            }
            auto mean = [](const std::vector<double> &v) {
                double s = 0;
                for (double x : v) s += x;
                return s / v.size();
            };
            printf("{\"blocks_per_cu\": %d, \"grid\": %u, \"cold\": %s, \"kernel_event_us\": %.2f, "
                   "\"first_block_end_us\": %.2f, \"median_block_end_us\": %.2f, \"last_block_end_us\": %.2f, "
                   "\"tail_us\": %.2f, \"frac_event\": %.4f}\n",
                   bpc, grid, cold ? "true" : "false", mean(kern), mean(first_end), mean(med_end), mean(last_end),
                   mean(last_end) - mean(med_end), 2.0 * S / (mean(kern) * 1e-6) / 8e12);
            fflush(stdout);
        }
        CHECK(hipFree(stamps));
    }
    for (auto b : bufs) CHECK(hipFree(b));
    return 0;
}
