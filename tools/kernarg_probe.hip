// kernarg_probe.hip -- host round trip of a blocking launch (launch, the
// kernel's last block stores a flag in host-coherent memory, the host spins on
// it) against the size of the kernel's by-value argument, on MI355X (tuning
// tool, not part of the library): is it worth moving the fused kernel's
// per-member pointer tables (~1.2 KB of kernarg) into device memory?
//   build: hipcc --offload-arch=gfx950 -O3 tools/kernarg_probe.hip -o tools/kernarg_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int BYTES>
struct Arg {
    unsigned *flag;
    unsigned epoch;
    unsigned pad[(BYTES - 16) / 4 > 0 ? (BYTES - 16) / 4 : 1];
};

template <int BYTES>
__global__ void k(Arg<BYTES> a) {
    if (threadIdx.x == 0 && blockIdx.x == 0)
        __hip_atomic_store(a.flag, a.epoch + a.pad[0] * 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int BYTES>
void run(unsigned *flag, hipStream_t st, int grid) {
    Arg<BYTES> a{};
    a.flag = flag;
    std::vector<double> ts;
    for (int r = 0; r < 5; ++r) {
        const int calls = 2000;
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < calls; ++i) {
            a.epoch = r * calls + i + 1 + BYTES * 100000u;
            hipLaunchKernelGGL(k<BYTES>, dim3(grid), dim3(256), 0, st, a);
            while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != a.epoch) {
            }
        }
        auto t1 = std::chrono::steady_clock::now();
        ts.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count() / calls);
    }
    std::sort(ts.begin(), ts.end());
    printf("kernarg %5zu B  grid %4d  %6.2f us per blocking launch (median of 5 x 2000)\n", sizeof(Arg<BYTES>), grid,
           ts[2]);
    fflush(stdout);
}

int main() {
    unsigned *flag;
    CHECK(hipHostMalloc((void **)&flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
    *flag = 0;
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    for (int pass = 0; pass < 2; ++pass)
        for (int grid : {1, 256}) {
            run<16>(flag, st, grid);
            run<128>(flag, st, grid);
            run<512>(flag, st, grid);
            run<1280>(flag, st, grid);
            run<2560>(flag, st, grid);
        }
    return 0;
}
