// doorbell_probe.hip -- round trip of a host -> resident-kernel doorbell on
// MI355X (tuning tool for the persistent fused server, not part of the
// library): the host stores k into a doorbell word, a resident kernel that
// polls it stores k into a host-coherent reply word, the host spins on the
// reply. Doorbell placements: host-coherent pinned memory (GPU polls over
// PCIe) and device memory the host writes through its mapping (GPU polls its
// own HBM). Pollers: one lane of block 0, or one lane of each of 32 blocks
// (the last to see it replies). Every kernel exits after `iters` rounds or
// a 2 s timeout.
//   build: hipcc --offload-arch=gfx950 -O3 tools/doorbell_probe.hip -o tools/doorbell_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ unsigned ld_sys(const unsigned *p) {
    return __hip_atomic_load(const_cast<unsigned *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void poller(const unsigned *bell, unsigned *reply, unsigned *count, int iters, int sleep) {
    if (threadIdx.x != 0) return;
    const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 200000000ull;  // 2 s
    for (unsigned k = 1; k <= (unsigned)iters; ++k) {
        while (ld_sys(bell) != k) {
            if (__builtin_amdgcn_s_memrealtime() > t_end) return;
            if (sleep) __builtin_amdgcn_s_sleep(1);
        }
        // count the blocks in: the last one replies and resets the counter
        const unsigned prev = __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev + 1 == gridDim.x) {
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(reply, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

static double run(const char *what, unsigned *bell_host_view, const unsigned *bell_dev, unsigned *reply,
                  unsigned *count, int blocks, int sleep) {
    const int iters = 3000;
    *bell_host_view = 0;
    __atomic_store_n(reply, 0u, __ATOMIC_RELEASE);
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    hipStream_t st;
    CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipLaunchKernelGGL(poller, dim3(blocks), dim3(64), 0, st, bell_dev, reply, count, iters, sleep);
    CHECK(hipGetLastError());
    std::vector<double> ts;
    auto t_fail = std::chrono::steady_clock::now() + std::chrono::seconds(2);
    for (unsigned k = 1; k <= (unsigned)iters; ++k) {
        auto t0 = std::chrono::steady_clock::now();
        __atomic_store_n(bell_host_view, k, __ATOMIC_RELEASE);
        while (__atomic_load_n(reply, __ATOMIC_ACQUIRE) != k) {
            if (std::chrono::steady_clock::now() > t_fail) {
                printf("%-44s blocks %2d sleep %d: no reply at round %u\n", what, blocks, sleep, k);
                CHECK(hipStreamSynchronize(st));
                CHECK(hipStreamDestroy(st));
                return -1;
            }
        }
        ts.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    CHECK(hipStreamSynchronize(st));
    CHECK(hipStreamDestroy(st));
    std::sort(ts.begin() + 100, ts.end());
    const double med = ts[100 + (ts.size() - 100) / 2];
    printf("%-44s blocks %2d sleep %d: median %.2f us  p90 %.2f us\n", what, blocks, sleep, med,
           ts[100 + (ts.size() - 100) * 9 / 10]);
    fflush(stdout);
    return med;
}

int main() {
    unsigned *reply, *hbell, *count;
    CHECK(hipHostMalloc((void **)&reply, 64, hipHostMallocCoherent | hipHostMallocMapped));
    CHECK(hipHostMalloc((void **)&hbell, 64, hipHostMallocCoherent | hipHostMallocMapped));
    CHECK(hipMalloc((void **)&count, 64));
    CHECK(hipMemset(count, 0, 64));
    CHECK(hipDeviceSynchronize());
    for (int blocks : {1, 32})
        for (int sleep : {0, 1}) run("doorbell in host-coherent pinned memory", hbell, hbell, reply, count, blocks, sleep);
    // device memory the host may be able to write through a mapping
    struct { const char *name; unsigned flags; } kinds[] = {
        {"doorbell in fine-grained device memory", hipDeviceMallocFinegrained},
        {"doorbell in uncached device memory", hipDeviceMallocUncached}};
    for (auto &kd : kinds) {
        unsigned *dbell = nullptr;
        if (hipExtMallocWithFlags((void **)&dbell, 4096, kd.flags) != hipSuccess) {
            printf("%s: allocation failed\n", kd.name);
            continue;
        }
        hipPointerAttribute_t attr;
        void *hp = nullptr;
        if (hipPointerGetAttributes(&attr, dbell) == hipSuccess) hp = attr.hostPointer;
        printf("%s: device %p host view %p\n", kd.name, (void *)dbell, hp);
        fflush(stdout);
        if (hp == nullptr) continue;
        for (int blocks : {1, 32})
            for (int sleep : {0, 1}) run(kd.name, (unsigned *)hp, dbell, reply, count, blocks, sleep);
        CHECK(hipFree(dbell));
    }
    return 0;
}
