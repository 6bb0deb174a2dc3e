// peer_shapes.hip -- launch-shape variants of the library's every-member fold
// for bench.py's `peer_fold_shapes` leg (a measurement probe, not part of the
// library; tools/libpeershapes.so, built by tools/Makefile `peershapes`).
//
// Why: the fold's launch shape (combine_kernels.h OrdersShape: 1 vector per
// lane, 1 block per CU at 4 and 8 sources) was tuned with all sources in local
// HBM. In BASELINE config 3 at N = 8 each GPU folds its shard with 7 of its 8
// sources on other GPUs, read over xGMI with several times HBM's latency, so
// the bytes in flight per CU that hide it may differ. This library
// instantiates the library's own kernel template (combine_orders_vec<sum,
// double, 8, U, non-temporal loads, every output>) at other (U, blocks per
// CU) shapes; bench.py times them beside the library's own launch
// (mi355_combine_orders) on the same peer-mapped sources and checks every
// variant's outputs against the library's.
//
// C ABI:
//   int peer_shapes_count(void);
//   int peer_shapes_describe(int v, int *unroll, int *blocks_per_cu);
//   int peer_shapes_orders_double_sum(int v, int nsrc, void *const *dsts, const void *const *srcs,
//                                     size_t n, hipEvent_t start, hipEvent_t stop, hipStream_t st);
// nsrc = 4 or 8 (BASELINE config 3 at N = 4 / 8).
// Sources and outputs 16-byte aligned, n a multiple of 2 (whole vectors);
// returns 0 or a HIP error code / -1 for an unsupported call.
#include "combine_kernels.h"

namespace {

using namespace mi355k;

struct Variant {
    int unroll, bpc, pipe;  // pipe: the pipelined loop (orders_vectors_pipe), a probe-only kernel
};
// the library's shape is one vector per lane and one block per CU at 4 and
// (since round 6) 8 sources: the 8-source shape of rounds 1-5 (4, 8), then
// more bytes in flight per CU in steps -- more blocks, more vectors per lane
// -- for xGMI's latency
// (a probe build may pass its own list: -DPEER_SHAPES_VARIANTS='{1, 1}, {2, 1}')
#ifndef PEER_SHAPES_VARIANTS
#define PEER_SHAPES_VARIANTS {4, 8}, {1, 2}, {1, 4}, {2, 8}, {1, 16}
#endif
constexpr Variant kVariants[] = {PEER_SHAPES_VARIANTS};
constexpr int kCount = sizeof(kVariants) / sizeof(kVariants[0]);

// combine_kernels.h orders_vectors with the next pass's loads issued before
// this pass's folds and stores (the copy loop's pipelining, copy_segments): a
// wave keeps loads in flight while it folds (round 6 probe: no faster than
// the library's loop at one block per CU, profiles/r06/orders_window/pipelined.jsonl).
template <int OP, typename T, int NSRC, int UNROLL, int POL, bool ALL, bool SHIFT>
__device__ __forceinline__ void orders_vectors_pipe(const OrdersParams &p) {
    const uint64_t nvec = p.nvec;
    const uint64_t step = (uint64_t)gridDim.x * kBlock * UNROLL;
    const u32x4 *sb[NSRC];
#pragma unroll
    for (int k = 0; k < NSRC; ++k) sb[k] = (const u32x4 *)p.src[k];
    uint64_t base = (uint64_t)blockIdx.x * kBlock * UNROLL + threadIdx.x;
    Pack<T> x[UNROLL][NSRC];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
        const uint64_t i = base + (uint64_t)u * kBlock;
        if (i < nvec) {
#pragma unroll
            for (int k = 0; k < NSRC; ++k) x[u][k].v = ld16_src<POL, SHIFT>(sb[k], i);
        }
    }
    while (base < nvec) {
        const uint64_t next = base + step;
        Pack<T> y[UNROLL][NSRC];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = next + (uint64_t)u * kBlock;
            if (i < nvec) {
#pragma unroll
                for (int k = 0; k < NSRC; ++k) y[u][k].v = ld16_src<POL, SHIFT>(sb[k], i);
            }
        }
        __builtin_amdgcn_sched_barrier(0);   // the next pass's loads first
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = base + (uint64_t)u * kBlock;
            if (i < nvec) orders_one<OP, T, NSRC, ALL>(p, x[u], i);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int k = 0; k < NSRC; ++k) x[u][k] = y[u][k];
        base = next;
    }
}

template <int OP, typename T, int NSRC, int U>
__global__ __launch_bounds__(kBlock) void orders_pipe_kernel(OrdersParams p) {
    orders_vectors_pipe<OP, T, NSRC, U, POL_NT_LOAD, true, false>(p);
}

template <int OP, typename T, int NSRC, int U>
int run(int bpc, int pipe, void *const *dsts, const void *const *srcs, size_t n, hipEvent_t e0, hipEvent_t e1,
        hipStream_t st) {
    OrdersParams p{};
    for (int k = 0; k < NSRC; ++k) {
        p.src[k] = srcs[k];
        p.dst[k] = dsts[k];
    }
    p.nvec = n / (16 / sizeof(T));
    auto kern = pipe ? orders_pipe_kernel<OP, T, NSRC, U> : combine_orders_vec<OP, T, NSRC, U, POL_NT_LOAD, true>;
    const unsigned grid = grid_for((uint64_t)kBlock * U, p.nvec, bpc);
    hipExtLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, st, e0, e1, 0, p);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

template <int OP, typename T, int NSRC>
int dispatch(int v, void *const *dsts, const void *const *srcs, size_t n, hipEvent_t e0, hipEvent_t e1,
             hipStream_t st) {
    switch (kVariants[v].unroll) {
    case 1: return run<OP, T, NSRC, 1>(kVariants[v].bpc, kVariants[v].pipe, dsts, srcs, n, e0, e1, st);
    case 2: return run<OP, T, NSRC, 2>(kVariants[v].bpc, kVariants[v].pipe, dsts, srcs, n, e0, e1, st);
    case 4: return run<OP, T, NSRC, 4>(kVariants[v].bpc, kVariants[v].pipe, dsts, srcs, n, e0, e1, st);
    default: return -1;
    }
}

}  // namespace

extern "C" int peer_shapes_count(void) { return kCount; }

extern "C" int peer_shapes_pipe(int v) { return v < 0 || v >= kCount ? -1 : kVariants[v].pipe; }

extern "C" int peer_shapes_describe(int v, int *unroll, int *blocks_per_cu) {
    if (v < 0 || v >= kCount) return -1;
    *unroll = kVariants[v].unroll;
    *blocks_per_cu = kVariants[v].bpc;
    return 0;
}

extern "C" int peer_shapes_orders_double_sum(int v, int nsrc, void *const *dsts, const void *const *srcs, size_t n,
                                             hipEvent_t e0, hipEvent_t e1, hipStream_t st) {
    if (v < 0 || v >= kCount || n % 2 != 0 || (nsrc != 4 && nsrc != 8)) return -1;
    for (int k = 0; k < nsrc; ++k)
        if (((uintptr_t)dsts[k] | (uintptr_t)srcs[k]) & 15) return -1;
    return nsrc == 4 ? dispatch<MI355_OP_SUM, double, 4>(v, dsts, srcs, n, e0, e1, st)
                     : dispatch<MI355_OP_SUM, double, 8>(v, dsts, srcs, n, e0, e1, st);
}

// The same shapes for BASELINE config 4's float max (8 sources): the
// library runs it at one vector per lane (combine_kernels.h OrdersShape, min/
// max chains); n a multiple of 4.
extern "C" int peer_shapes_orders_float_max(int v, void *const *dsts, const void *const *srcs, size_t n, hipEvent_t e0,
                                            hipEvent_t e1, hipStream_t st) {
    if (v < 0 || v >= kCount || n % 4 != 0) return -1;
    for (int k = 0; k < 8; ++k)
        if (((uintptr_t)dsts[k] | (uintptr_t)srcs[k]) & 15) return -1;
    return dispatch<MI355_OP_MAX, float, 8>(v, dsts, srcs, n, e0, e1, st);
}

// More pairs for the every-member fold's shape probe (tools/probes/orders_shapes_cold.py):
// 8 sources, n a whole number of 16-byte vectors.
#define PEER_SHAPES_PAIR(NAME, OP, T)                                                                             \
    extern "C" int NAME(int v, void *const *dsts, const void *const *srcs, size_t n, hipEvent_t e0, hipEvent_t e1, \
                        hipStream_t st) {                                                                          \
        if (v < 0 || v >= kCount || n % (16 / sizeof(T)) != 0) return -1;                                         \
        for (int k = 0; k < 8; ++k)                                                                                \
            if (((uintptr_t)dsts[k] | (uintptr_t)srcs[k]) & 15) return -1;                                         \
        return dispatch<OP, T, 8>(v, dsts, srcs, n, e0, e1, st);                                                   \
    }
PEER_SHAPES_PAIR(peer_shapes_orders_double_max, MI355_OP_MAX, double)
PEER_SHAPES_PAIR(peer_shapes_orders_float_sum, MI355_OP_SUM, float)
PEER_SHAPES_PAIR(peer_shapes_orders_double_prod, MI355_OP_PROD, double)
PEER_SHAPES_PAIR(peer_shapes_orders_int_sum, MI355_OP_SUM, int)

// The plain k-source fold (one output; combine_vec) at the same shapes, for the order-free
// operators' shard at N = 8 (BASELINE config 4's longlong and: 8 x 8 MiB -> 1); probe only.
namespace {
template <int U>
int fold_run(int bpc, void *dst, const void *const *srcs, size_t n, hipEvent_t e0, hipEvent_t e1, hipStream_t st) {
    CombineParams p{};
    p.dst = dst;
    for (int k = 0; k < 8; ++k) p.src[k] = srcs[k];
    p.nvec = n / 2;
    auto kern = combine_vec<MI355_OP_AND, long, 8, U, POL_NT_LOAD>;
    const unsigned grid = grid_for((uint64_t)kBlock * U, p.nvec, bpc);
    hipExtLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, st, e0, e1, 0, p);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}
}  // namespace

extern "C" int peer_shapes_fold_long_and(int v, void *dst, const void *const *srcs, size_t n, hipEvent_t e0,
                                         hipEvent_t e1, hipStream_t st) {
    if (v < 0 || v >= kCount || n % 2 != 0 || kVariants[v].pipe) return -1;
    if ((uintptr_t)dst & 15) return -1;
    for (int k = 0; k < 8; ++k)
        if ((uintptr_t)srcs[k] & 15) return -1;
    switch (kVariants[v].unroll) {
    case 1: return fold_run<1>(kVariants[v].bpc, dst, srcs, n, e0, e1, st);
    case 2: return fold_run<2>(kVariants[v].bpc, dst, srcs, n, e0, e1, st);
    case 4: return fold_run<4>(kVariants[v].bpc, dst, srcs, n, e0, e1, st);
    default: return -1;
    }
}
