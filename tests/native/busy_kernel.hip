// busy_kernel.hip -- TEST HELPER (tests/test_gpu_multipe.py): a grid that
// fills every CU of the GPU for a given time on a caller's stream, so a test
// can start a reduction while another kernel holds the CUs. Built by
// osss-gasnet_amd/csrc/Makefile into osss-gasnet_amd/lib/libtestbusy.so.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <time.h>

// Every block counts itself in; the last one to start tells the host (a
// page-locked word), so test_busy_launch returns only once the whole grid
// holds the CUs (a launch on another stream is otherwise dispatched whenever
// the command processor gets to it, possibly after the collective the test
// wants to delay has already run).
__global__ __launch_bounds__(256) void busy_k(uint64_t ticks, unsigned *started, unsigned total,
                                              unsigned *host_flag) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(started, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev + 1 == total) __hip_atomic_store(host_flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

// Occupy the GPU for `ms` milliseconds (100 MHz real-time ticks) with
// blocks_per_cu 256-thread blocks per CU on `stream`, and return once every
// block has started: 0, a hipError_t, or -1 when the grid was not all
// resident within 2 s (the caller's assumption of a full GPU does not hold).
extern "C" int test_busy_launch(double ms, int blocks_per_cu, void *stream) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    static unsigned *started = nullptr, *flag = nullptr;
    if (started == nullptr) {
        if (hipMalloc((void **)&started, sizeof(unsigned)) != hipSuccess) return (int)hipGetLastError();
        if (hipHostMalloc((void **)&flag, sizeof(unsigned), hipHostMallocCoherent | hipHostMallocMapped) !=
            hipSuccess)
            return (int)hipGetLastError();
    }
    hipError_t e = hipMemsetAsync(started, 0, sizeof(unsigned), (hipStream_t)stream);
    if (e != hipSuccess) return (int)e;
    if ((e = hipStreamSynchronize((hipStream_t)stream)) != hipSuccess) return (int)e;
    __atomic_store_n(flag, 0u, __ATOMIC_RELEASE);
    const unsigned total = (unsigned)(cus * blocks_per_cu);
    hipLaunchKernelGGL(busy_k, dim3(total), dim3(256), 0, (hipStream_t)stream, (uint64_t)(ms * 1e5), started,
                       total, flag);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    const double t0 = now_s();
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == 0)
        if (now_s() - t0 > 2.0) return -1;
    return 0;
}
