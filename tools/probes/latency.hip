// latency.hip -- host<->GPU round-trip costs that bound a small reduction call
// (tuning tool, not part of the library).
//   build: hipcc --offload-arch=gfx950 -O2 tools/probes/latency.hip -o tools/probes/latency
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include <atomic>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

static double now() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

__global__ void empty_k() {}

__global__ void flag_k(volatile unsigned *flag, unsigned v) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store((unsigned *)flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// last-block-done: every block bumps a device counter; the last one signals the host
__global__ void copy_flag_k(const float4 *s, float4 *d, size_t n, unsigned *cnt, volatile unsigned *flag,
                            unsigned v) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) d[i] = s[i];
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        unsigned prev = atomicAdd(cnt, 1u);
        if (prev == gridDim.x - 1) {
            *cnt = 0;
            __threadfence_system();
            __hip_atomic_store((unsigned *)flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

template <typename F>
double per_call_us(F f, int reps) {
    for (int i = 0; i < 50; ++i) f(i);
    double t0 = now();
    for (int i = 0; i < reps; ++i) f(i + 1000);
    return (now() - t0) / reps * 1e6;
}

int main(int argc, char **argv) {
    int flags = argc > 1 ? atoi(argv[1]) : -1;
    if (flags >= 0) CHECK(hipSetDeviceFlags(flags));
    hipStream_t st;
    CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const int reps = 2000;
    printf("device flags %d\n", flags);
    printf("launch only (async)            %7.2f us\n", per_call_us([&](int) {
        hipLaunchKernelGGL(empty_k, dim3(1), dim3(64), 0, st); }, reps));
    CHECK(hipStreamSynchronize(st));
    printf("hipDeviceSynchronize (idle)    %7.2f us\n", per_call_us([&](int) { CHECK(hipDeviceSynchronize()); }, reps));
    printf("hipStreamSynchronize (idle)    %7.2f us\n", per_call_us([&](int) { CHECK(hipStreamSynchronize(st)); }, reps));
    printf("launch + streamSync            %7.2f us\n", per_call_us([&](int) {
        hipLaunchKernelGGL(empty_k, dim3(1), dim3(64), 0, st); CHECK(hipStreamSynchronize(st)); }, reps));
    printf("devSync + launch + streamSync  %7.2f us\n", per_call_us([&](int) {
        CHECK(hipDeviceSynchronize());
        hipLaunchKernelGGL(empty_k, dim3(1), dim3(64), 0, st); CHECK(hipStreamSynchronize(st)); }, reps));
    hipEvent_t ev;
    CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    printf("launch + event + eventSync     %7.2f us\n", per_call_us([&](int) {
        hipLaunchKernelGGL(empty_k, dim3(1), dim3(64), 0, st); CHECK(hipEventRecord(ev, st)); CHECK(hipEventSynchronize(ev)); }, reps));

    unsigned *hflag;
    CHECK(hipHostMalloc((void **)&hflag, 64, hipHostMallocCoherent | hipHostMallocMapped));
    *hflag = 0;
    printf("launch + spin on host flag     %7.2f us\n", per_call_us([&](int i) {
        hipLaunchKernelGGL(flag_k, dim3(1), dim3(64), 0, st, (volatile unsigned *)hflag, (unsigned)i);
        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != (unsigned)i) {} }, reps));
    CHECK(hipStreamSynchronize(st));

    printf("devSync + launch + spin flag   %7.2f us\n", per_call_us([&](int i) {
        CHECK(hipDeviceSynchronize());
        hipLaunchKernelGGL(flag_k, dim3(1), dim3(64), 0, st, (volatile unsigned *)hflag, (unsigned)i);
        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != (unsigned)i) {} }, reps));
    hipStream_t bst;
    CHECK(hipStreamCreateWithFlags(&bst, hipStreamDefault));
    printf("blocking stream launch + spin  %7.2f us\n", per_call_us([&](int i) {
        hipLaunchKernelGGL(flag_k, dim3(1), dim3(64), 0, bst, (volatile unsigned *)hflag, (unsigned)i);
        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != (unsigned)i) {} }, reps));
    printf("null stream launch + spin      %7.2f us\n", per_call_us([&](int i) {
        hipLaunchKernelGGL(flag_k, dim3(1), dim3(64), 0, 0, (volatile unsigned *)hflag, (unsigned)i);
        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != (unsigned)i) {} }, reps));
    CHECK(hipDeviceSynchronize());
    printf("null launch+spin, null memset  %7.2f us\n", per_call_us([&](int i) {
        hipMemsetAsync(hflag + 8, 0, 4, 0);
        hipLaunchKernelGGL(flag_k, dim3(1), dim3(64), 0, 0, (volatile unsigned *)hflag, (unsigned)i);
        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != (unsigned)i) {} }, reps));
    CHECK(hipDeviceSynchronize());
    // 64 KiB copy with last-block flag vs stream sync
    size_t n = 65536 / 16;
    float4 *a, *b;
    unsigned *cnt;
    CHECK(hipMalloc(&a, 65536)); CHECK(hipMalloc(&b, 65536)); CHECK(hipMalloc(&cnt, 64));
    CHECK(hipMemset(cnt, 0, 64));
    printf("64KiB copy + streamSync        %7.2f us\n", per_call_us([&](int i) {
        hipLaunchKernelGGL(copy_flag_k, dim3(16), dim3(256), 0, st, a, b, n, cnt, (volatile unsigned *)hflag, (unsigned)i);
        CHECK(hipStreamSynchronize(st)); }, reps));
    printf("64KiB copy + spin host flag    %7.2f us\n", per_call_us([&](int i) {
        hipLaunchKernelGGL(copy_flag_k, dim3(16), dim3(256), 0, st, a, b, n, cnt, (volatile unsigned *)hflag, (unsigned)i);
        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != (unsigned)i) {} }, reps));
    CHECK(hipStreamSynchronize(st));
    // graph of one kernel
    hipGraph_t g; hipGraphExec_t ge;
    CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    hipLaunchKernelGGL(empty_k, dim3(1), dim3(64), 0, st);
    CHECK(hipStreamEndCapture(st, &g));
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    printf("graphLaunch + streamSync       %7.2f us\n", per_call_us([&](int) {
        CHECK(hipGraphLaunch(ge, st)); CHECK(hipStreamSynchronize(st)); }, reps));
    return 0;
}
