// busy_kernel.hip -- TEST HELPER (tests/test_gpu_multipe.py): a grid that
// fills every CU of the GPU for a given time on a caller's stream, so a test
// can start a reduction while another kernel holds the CUs. Built by
// osss-gasnet_amd/csrc/Makefile into osss-gasnet_amd/lib/libtestbusy.so.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void busy_k(uint64_t ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

// Occupy the GPU for `ms` milliseconds (100 MHz real-time ticks) with
// blocks_per_cu 256-thread blocks per CU on `stream`; 0 or a hipError_t.
extern "C" int test_busy_launch(double ms, int blocks_per_cu, void *stream) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    hipLaunchKernelGGL(busy_k, dim3(cus * blocks_per_cu), dim3(256), 0, (hipStream_t)stream,
                       (uint64_t)(ms * 1e5));
    return (int)hipGetLastError();
}
