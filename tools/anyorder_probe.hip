// anyorder_probe.hip -- where the fixed per-call cost of a blocking 1-PE call
// goes (tuning tool, not part of the library).
//   build: hipcc --offload-arch=gfx950 -O2 tools/anyorder_probe.hip -o tools/anyorder_probe
//
// A call = launch one streaming copy kernel (256 MiB or 64 KiB) whose last
// block stores a host-coherent flag, then spin on the flag (the library's
// protocol). Each kernel stamps s_memrealtime (100 MHz) when its first block
// starts and when its last block finishes, so per call:
//   busy = last-block end - first-block start      (kernel time)
//   gap  = next call's first-block start - this end (host sees flag, returns,
//          launches again, the CP dispatches)
// Variants: plain hipLaunchKernel on a blocking stream; hipExtLaunchKernel
// with hipExtAnyOrderLaunch (AQL barrier bit clear); a non-blocking stream.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

static double now() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

struct Args {
    const u32x4 *s;
    u32x4 *d;
    unsigned long long nvec;
    unsigned *cnt;
    unsigned *flag;
    unsigned epoch;
    unsigned long long *stamps;  // [2 * call]: start, end
    unsigned call;
};

__global__ __launch_bounds__(256) void copy_k(Args a) {
    if (blockIdx.x == 0 && threadIdx.x == 0) a.stamps[2 * a.call] = wall_clock64();
    const unsigned long long step = (unsigned long long)gridDim.x * 256 * 8;
    for (unsigned long long base = (unsigned long long)blockIdx.x * 256 * 8 + threadIdx.x; base < a.nvec;
         base += step) {
        u32x4 x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            unsigned long long i = base + (unsigned long long)u * 256;
            if (i < a.nvec) x[u] = a.s[i];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            unsigned long long i = base + (unsigned long long)u * 256;
            if (i < a.nvec) __builtin_nontemporal_store(x[u], a.d + i);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        unsigned prev = atomicAdd(a.cnt, 1u);
        if (prev == gridDim.x - 1) {
            *a.cnt = 0;
            a.stamps[2 * a.call + 1] = wall_clock64();
            __threadfence_system();
            __hip_atomic_store(a.flag, a.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

static void run(const char *name, size_t bytes, hipStream_t st, int mode, int calls, Args a, unsigned blocks) {
    a.nvec = bytes / 16;
    std::vector<unsigned long long> h(2 * calls);
    double t0 = 0;
    for (int c = 0; c < calls; ++c) {
        if (c == 10) t0 = now();
        a.call = c;
        a.epoch = a.epoch + 1;
        if (mode == 0)
            hipLaunchKernelGGL(copy_k, dim3(blocks), dim3(256), 0, st, a);
        else
            hipExtLaunchKernelGGL(copy_k, dim3(blocks), dim3(256), 0, st, nullptr, nullptr,
                                  mode == 1 ? hipExtAnyOrderLaunch : 0, a);
        while (__atomic_load_n(a.flag, __ATOMIC_ACQUIRE) != a.epoch) {
        }
    }
    double per = (now() - t0) / (calls - 10) * 1e6;
    CHECK(hipStreamSynchronize(st));
    CHECK(hipMemcpy(h.data(), a.stamps, h.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> busy, gap;
    for (int c = 10; c < calls - 1; ++c) {
        busy.push_back((h[2 * c + 1] - h[2 * c]) * 0.01);
        gap.push_back((h[2 * c + 2] - h[2 * c + 1]) * 0.01);
    }
    std::sort(busy.begin(), busy.end());
    std::sort(gap.begin(), gap.end());
    printf("%-34s %9zu B  call %7.2f us  busy(med) %7.2f us  gap(med) %6.2f us  gap(p10) %6.2f\n", name, bytes,
           per, busy[busy.size() / 2], gap[gap.size() / 2], gap[gap.size() / 10]);
}

int main() {
    hipStream_t blk, nblk;
    CHECK(hipStreamCreateWithFlags(&blk, hipStreamDefault));
    CHECK(hipStreamCreateWithFlags(&nblk, hipStreamNonBlocking));
    const size_t big = 256ull << 20;
    Args a{};
    void *s, *d;
    CHECK(hipMalloc(&s, big));
    CHECK(hipMalloc(&d, big));
    CHECK(hipMemset(s, 1, big));
    CHECK(hipMemset(d, 2, big));
    CHECK(hipMalloc(&a.cnt, 64));
    CHECK(hipMemset(a.cnt, 0, 64));
    CHECK(hipMalloc(&a.stamps, 2 * 8 * 4096));
    CHECK(hipHostMalloc((void **)&a.flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
    *a.flag = 0;
    a.s = (const u32x4 *)s;
    a.d = (u32x4 *)d;
    CHECK(hipDeviceSynchronize());
    int cus = 256;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    for (int rep = 0; rep < 2; ++rep) {
        run("256MiB blocking, hipLaunchKernel", big, blk, 0, 200, a, 2 * cus);
        a.epoch += 1000;
        run("256MiB blocking, ExtLaunch", big, blk, 2, 200, a, 2 * cus);
        a.epoch += 1000;
        run("256MiB blocking, ExtLaunch anyorder", big, blk, 1, 200, a, 2 * cus);
        a.epoch += 1000;
        run("256MiB nonblocking, hipLaunchKernel", big, nblk, 0, 200, a, 2 * cus);
        a.epoch += 1000;
        run("256MiB nonblocking, anyorder", big, nblk, 1, 200, a, 2 * cus);
        a.epoch += 1000;
        run("64KiB blocking, hipLaunchKernel", 65536, blk, 0, 2000, a, 16);
        a.epoch += 10000;
        run("64KiB blocking, anyorder", 65536, blk, 1, 2000, a, 16);
        a.epoch += 10000;
        run("64KiB nonblocking, anyorder", 65536, nblk, 1, 2000, a, 16);
        a.epoch += 10000;
    }
    return 0;
}
