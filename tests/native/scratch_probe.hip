// scratch_probe.hip -- tests/test_residency.py: one kernel that needs scratch
// memory (a register array indexed by a value only known at run time) and one
// that does not, for tools/check_residency.py --no-scratch.
#include <hip/hip_runtime.h>

__global__ void with_scratch(const int *in, int *out, int k) {
    int a[64];
#pragma unroll 1
    for (int i = 0; i < 64; ++i) a[i] = in[threadIdx.x + i * 256];
    out[threadIdx.x] = a[(k + threadIdx.x) & 63];
}

__global__ void without_scratch(const int *in, int *out) { out[threadIdx.x] = in[threadIdx.x] + 1; }
