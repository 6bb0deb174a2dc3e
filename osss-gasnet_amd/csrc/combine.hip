// combine.hip -- element-wise combine kernels for the *_to_all reductions (gfx950).
//
// Replaces the scalar, indirect-call combine loops of the reference schedule
// (src/reduce/reduce-op.c:241-261, element functions :79-158) with streaming
// HIP kernels. The work is bandwidth-bound vector arithmetic: every output
// element costs NSRC loads and one store and a handful of VALU ops, so the
// design target is the HBM (or xGMI) roofline, not MFMA:
//   * 16-byte loads/stores per lane (1 KiB per wave instruction),
//   * UNROLL independent 16-byte vectors per lane x NSRC sources issued
//     before the first use, so each lane keeps NSRC*UNROLL loads in flight,
//   * grid-stride over a grid capped at a few blocks per CU (256 CUs),
//   * no LDS: nothing is re-used, staging through LDS would only add traffic.
//
// Numerics follow the reference operators exactly (compiled with
// -ffp-contract=off so no a*b+c is fused):
//   sum/prod      a + b, a * b (integers wrap two's-complement, like gcc's
//                 code for reduce-op.c:79-101; short promotes to int and
//                 truncates)
//   and/or/xor    bitwise (reduce-op.c:108-131)
//   min/max       a < b ? a : b / a > b ? a : b  -- a select, NOT v_min/v_max,
//                 so NaN and signed-zero cases pick the same operand as the
//                 reference (reduce-op.c:138-158)
//   complex prod  the C99 Annex G algorithm of libgcc __muldc3/__mulsc3, which
//                 is what gcc emits for `a * b` on double/float complex
//   long double   x87 80-bit extended arithmetic in software (x80.h)
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#include "mi355_reduce.h"
#include "ops.h"

namespace {

using namespace mi355;

constexpr int kBlock = 256;
constexpr int kMaxSrc = 8;

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
// Completion signal (mi355_signal_next_launch): the last block to finish
// stores `epoch` into a host-visible word, so the host learns the result is
// in memory ~4 us sooner than through hipStreamSynchronize (tools/latency.hip:
// 6.9 vs 10.7 us for a launch round trip on MI355X).
struct Signal {
    unsigned *count;  // device word, 0 between launches (the last block resets it)
    unsigned *flag;   // host-coherent word the host spins on; nullptr = no signal
    unsigned epoch;
};

// Publish recipe of MI355X_MICROARCH.md (inter-workgroup visibility, valid
// form "sc1 payload + drained waves + flag"): the bulk stores are
// write-through (`nt sc1`, st16), so once every wave has drained its stores
// they are in memory for any agent; a block that also made plain stores (an
// element tail, an unaligned kernel) first writes its XCD's L2 back with an
// agent-scope release. One lane per block counts the block in; the last
// block resets the counter and stores the epoch to the host-coherent flag.
__device__ __forceinline__ void signal_done(const Signal &sg, bool plain_stores) {
    if (sg.flag == nullptr) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        if (plain_stores) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const unsigned total = gridDim.x * gridDim.y;
        const unsigned prev = __hip_atomic_fetch_add(sg.count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev + 1 == total) {
            __hip_atomic_store(sg.count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(sg.flag, sg.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

struct CombineParams {
    void *dst;
    const void *src[kMaxSrc];
    uint64_t nvec;   // vector kernel: whole 16-byte vectors; scalar kernel: elements
    uint32_t tail;   // vector kernel: elements after nvec*V (< V)
    uint32_t head;   // vector kernel: elements just BEFORE dst/src (pointers advanced to 16-byte alignment)
    Signal sig;
};

// Cache policy (tools/hbm_sweep.hip, MI355X, 256 MiB per buffer):
//   stores: write-through to memory at agent scope, which makes the completion
//     signal cheap: no per-block L2 write-back (that cost 60 us on a 256 MiB
//     copy with 2048 blocks). The copy: `nt sc1`, as fast as plain
//     non-temporal stores (6.82 TB/s); the folds: `sc1` (st16_fold), 3-10 %
//     faster than `nt sc1` beside their non-temporal loads.
//   loads: plain for the copy (6.8 TB/s vs 6.1 non-temporal), non-temporal
//     for folds (Shape<NSRC>::policy).
enum { POL_PLAIN = 0, POL_NT_LOAD = 1 };

template <int POL>
__device__ __forceinline__ u32x4 ld16(const u32x4 *p) {
    if constexpr ((POL & POL_NT_LOAD) != 0) return __builtin_nontemporal_load(p);
    else return *p;
}
__device__ __forceinline__ void st16(u32x4 *p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
// The folds' stores: write-through at agent scope WITHOUT the non-temporal
// hint. Beside non-temporal loads this is the faster form (tools/fold_probe.hip,
// profiles/r02/fold_probe_copy.txt, 256 MiB per source: k = 2 116.4 vs 127.9 us,
// k = 3 158.7 vs 177.1, k = 8 393.5 vs 422); the copy keeps `nt sc1` (with
// its plain loads `sc1` alone is 18 % slower).
__device__ __forceinline__ void st16_fold(u32x4 *p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

// Vector path: every pointer 16-byte aligned. Each lane owns UNROLL vectors
// spaced one block apart (so a wave touches contiguous 1 KiB per source per
// step) and issues all NSRC*UNROLL loads before combining.
template <int OP, typename T, int NSRC, int UNROLL, int POL>
__global__ __launch_bounds__(kBlock) void combine_vec(CombineParams p) {
    constexpr int V = 16 / sizeof(T);
    const u32x4 *s[NSRC];
#pragma unroll
    for (int k = 0; k < NSRC; ++k) s[k] = (const u32x4 *)p.src[k];
    u32x4 *d = (u32x4 *)p.dst;
    const uint64_t nvec = p.nvec;
    const uint64_t step = (uint64_t)gridDim.x * kBlock * UNROLL;
    for (uint64_t base = (uint64_t)blockIdx.x * kBlock * UNROLL + threadIdx.x; base < nvec;
         base += step) {
        Pack<T> x[UNROLL][NSRC];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = base + (uint64_t)u * kBlock;
            if (i < nvec) {
#pragma unroll
                for (int k = 0; k < NSRC; ++k) x[u][k].v = ld16<POL>(s[k] + i);
            }
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = base + (uint64_t)u * kBlock;
            if (i < nvec) {
                Pack<T> acc = x[u][0];
#pragma unroll
                for (int k = 1; k < NSRC; ++k) {
#pragma unroll
                    for (int e = 0; e < V; ++e) acc.e[e] = apply<OP>(acc.e[e], x[u][k].e[e]);
                }
                st16_fold(d + i, acc.v);
            }
        }
    }
    const bool tail_block = V > 1 && p.tail != 0 && blockIdx.x == 0;
    if (tail_block && threadIdx.x < p.tail) {
        const uint64_t i = nvec * V + threadIdx.x;
        T acc = ((const T *)p.src[0])[i];
#pragma unroll
        for (int k = 1; k < NSRC; ++k) acc = apply<OP>(acc, ((const T *)p.src[k])[i]);
        ((T *)p.dst)[i] = acc;
    }
    const bool head_block = V > 1 && p.head != 0 && blockIdx.x == 0;
    if (head_block && threadIdx.x < p.head) {
        const int64_t i = (int64_t)threadIdx.x - (int64_t)p.head;
        T acc = ((const T *)p.src[0])[i];
#pragma unroll
        for (int k = 1; k < NSRC; ++k) acc = apply<OP>(acc, ((const T *)p.src[k])[i]);
        ((T *)p.dst)[i] = acc;
    }
    signal_done(p.sig, tail_block || head_block);
}

// Scalar path for pointers that are not 16-byte aligned (user offsets into
// arrays). Coalesced element loads, grid-stride.
template <int OP, typename T, int NSRC>
__global__ __launch_bounds__(kBlock) void combine_scalar(CombineParams p) {
    const T *s[NSRC];
#pragma unroll
    for (int k = 0; k < NSRC; ++k) s[k] = (const T *)p.src[k];
    T *d = (T *)p.dst;
    const uint64_t n = p.nvec;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * kBlock) {
        T v[NSRC];
#pragma unroll
        for (int k = 0; k < NSRC; ++k) v[k] = s[k][i];
        T acc = v[0];
#pragma unroll
        for (int k = 1; k < NSRC; ++k) acc = apply<OP>(acc, v[k]);
        d[i] = acc;
    }
    signal_done(p.sig, true);
}

// Every member's reference order in one pass (mi355_combine_orders). On
// member q the reference folds its OWN source first and then the others in
// active-set order (reduce-op.c:226-264), so for order-sensitive operators (FP
// rounding; the NaN and +-0 selects of min/max) the members' results differ.
// The owner of a shard loads the NSRC sources once and computes every fold
// from registers: dst[q] = fold(src[q], src[0], .., src[q-1], src[q+1], ..).
// A null dst[q] skips fold q (a kernel argument: the branch is uniform).
struct OrdersParams {
    void *dst[kMaxSrc];
    const void *src[kMaxSrc];
    uint64_t nvec;  // as CombineParams
    uint32_t tail;
    uint32_t head;
    Signal sig;
};

template <int OP, typename T, int NSRC>
__device__ __forceinline__ void orders_element(const OrdersParams &p, int64_t i) {
    T v[NSRC];
#pragma unroll
    for (int k = 0; k < NSRC; ++k) v[k] = ((const T *)p.src[k])[i];
#pragma unroll
    for (int q = 0; q < NSRC; ++q) {
        if (p.dst[q] == nullptr) continue;
        T acc = v[q];
#pragma unroll
        for (int k = 0; k < NSRC; ++k)
            if (k != q) acc = apply<OP>(acc, v[k]);
        ((T *)p.dst[q])[i] = acc;
    }
}

template <int OP, typename T, int NSRC, int UNROLL, int POL>
__global__ __launch_bounds__(kBlock) void combine_orders_vec(OrdersParams p) {
    constexpr int V = 16 / sizeof(T);
    const uint64_t nvec = p.nvec;
    const uint64_t step = (uint64_t)gridDim.x * kBlock * UNROLL;
    for (uint64_t base = (uint64_t)blockIdx.x * kBlock * UNROLL + threadIdx.x; base < nvec;
         base += step) {
        Pack<T> x[UNROLL][NSRC];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = base + (uint64_t)u * kBlock;
            if (i < nvec) {
#pragma unroll
                for (int k = 0; k < NSRC; ++k) x[u][k].v = ld16<POL>((const u32x4 *)p.src[k] + i);
            }
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = base + (uint64_t)u * kBlock;
            if (i >= nvec) continue;
#pragma unroll
            for (int q = 0; q < NSRC; ++q) {
                if (p.dst[q] == nullptr) continue;
                Pack<T> acc = x[u][q];
#pragma unroll
                for (int k = 0; k < NSRC; ++k) {
                    if (k == q) continue;
#pragma unroll
                    for (int e = 0; e < V; ++e) acc.e[e] = apply<OP>(acc.e[e], x[u][k].e[e]);
                }
                st16_fold((u32x4 *)p.dst[q] + i, acc.v);
            }
        }
    }
    const bool tail_block = V > 1 && p.tail != 0 && blockIdx.x == 0;
    if (tail_block && threadIdx.x < p.tail) orders_element<OP, T, NSRC>(p, (int64_t)(nvec * V + threadIdx.x));
    const bool head_block = V > 1 && p.head != 0 && blockIdx.x == 0;
    if (head_block && threadIdx.x < p.head) orders_element<OP, T, NSRC>(p, (int64_t)threadIdx.x - (int64_t)p.head);
    signal_done(p.sig, tail_block || head_block);
}

template <int OP, typename T, int NSRC>
__global__ __launch_bounds__(kBlock) void combine_orders_scalar(OrdersParams p) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < p.nvec; i += (uint64_t)gridDim.x * kBlock)
        orders_element<OP, T, NSRC>(p, (int64_t)i);
    signal_done(p.sig, true);
}

// Byte copy of up to NS segments in one launch; blockIdx.y = segment. NS = 1
// (the 1-PE identity, the bench's call) keeps the kernel arguments at 48
// bytes instead of 1.5 KiB for the 64-segment form (the all-gather leg).
constexpr int kMaxSeg = 64;
template <int NS>
struct SegParams {
    void *dst[NS];
    const void *src[NS];
    uint64_t nbytes[NS];
    Signal sig;
};

template <int UNROLL, int NS>
__global__ __launch_bounds__(kBlock) void copy_segments(SegParams<NS> p) {
    const int sg = blockIdx.y;
    const uint64_t nb = p.nbytes[sg];
    const char *src = (const char *)p.src[sg];
    char *dst = (char *)p.dst[sg];
    // 16-byte vectors where both ends are aligned: pointers with the same
    // misalignment (a user offset into two arrays) peel a head so that both
    // start on a 128-byte line (or at least on 16 bytes); different
    // misalignments take the narrow path below
    const unsigned mis128 = (unsigned)((uintptr_t)dst & 127);
    const unsigned mis = mis128 & 15u;
    const bool coaligned = mis == (unsigned)((uintptr_t)src & 15);
    uint64_t head = !coaligned ? nb
                    : mis128 == (unsigned)((uintptr_t)src & 127) ? (128u - mis128) & 127u
                                                                  : (16u - mis) & 15u;
    if (head > nb) head = nb;
    uint64_t vec_end = head;  // bytes [head, vec_end) go as vectors
    if (coaligned) {
        const u32x4 *s = (const u32x4 *)(src + head);
        u32x4 *d = (u32x4 *)(dst + head);
        const uint64_t nvec = (nb - head) / 16;
        const uint64_t step = (uint64_t)gridDim.x * kBlock * UNROLL;
        // software-pipelined: the loads of pass k+1 are in flight while the
        // stores of pass k issue (tools/copy_variants.hip: 78.3 vs 80.0 us for
        // 256 MiB at UNROLL 4, one block per CU, over all-loads-then-stores)
        uint64_t base = (uint64_t)blockIdx.x * kBlock * UNROLL + threadIdx.x;
        u32x4 x[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = base + (uint64_t)u * kBlock;
            if (i < nvec) x[u] = ld16<POL_PLAIN>(s + i);
        }
        while (base < nvec) {
            const uint64_t next = base + step;
            u32x4 y[UNROLL];
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                const uint64_t i = next + (uint64_t)u * kBlock;
                if (i < nvec) y[u] = ld16<POL_PLAIN>(s + i);
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
        vec_end = head + nvec * 16;
    }
    bool plain = false;
    if (!coaligned) {
        // narrow path: the widest unit both ends are aligned to (8, 4, 2 or 1 bytes)
        const unsigned both = (unsigned)(((uintptr_t)dst | (uintptr_t)src) & 7);
        const uint64_t stride = (uint64_t)gridDim.x * kBlock;
        const uint64_t t0 = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
        uint64_t done = 0;
        if ((both & 7) == 0) {
            const uint64_t nw = nb / 8;
            for (uint64_t i = t0; i < nw; i += stride) ((uint64_t *)dst)[i] = ((const uint64_t *)src)[i];
            done = nw * 8;
        } else if ((both & 3) == 0) {
            const uint64_t nw = nb / 4;
            for (uint64_t i = t0; i < nw; i += stride) ((uint32_t *)dst)[i] = ((const uint32_t *)src)[i];
            done = nw * 4;
        } else if ((both & 1) == 0) {
            const uint64_t nw = nb / 2;
            for (uint64_t i = t0; i < nw; i += stride) ((uint16_t *)dst)[i] = ((const uint16_t *)src)[i];
            done = nw * 2;
        }
        for (uint64_t i = done + t0; i < nb; i += stride) dst[i] = src[i];
        plain = nb > 0;
    } else {
        // the bytes outside the vector part: [0, head) and [vec_end, nb)
        const uint64_t nrest = head + (nb - vec_end);
        for (uint64_t r = (uint64_t)blockIdx.x * kBlock + threadIdx.x; r < nrest;
             r += (uint64_t)gridDim.x * kBlock) {
            const uint64_t i = r < head ? r : vec_end + (r - head);
            dst[i] = src[i];
            plain = true;
        }
    }
    signal_done(p.sig, __syncthreads_or(plain));
}

// One block that only carries the completion signal: tells the host when the
// stream has reached this point (everything queued before it has finished).
struct EmptyParams {
    Signal sig;
};
__global__ __launch_bounds__(kBlock) void signal_only(EmptyParams p) { signal_done(p.sig, false); }

// ---------------------------------------------------------------------------
// launch helpers
// ---------------------------------------------------------------------------
int g_cus[64];

// events and completion signal for the next launch (mi355_time_next_launch,
// mi355_signal_next_launch), consumed by it
thread_local hipEvent_t t_ev_start = nullptr, t_ev_stop = nullptr;
thread_local Signal t_sig = {nullptr, nullptr, 0};

// A host-visible word the host can also write: an armed signal that no kernel
// will carry (nothing to launch) is fired right here, in stream order.
void fire_on_host(hipStream_t st) {
    if (t_sig.flag == nullptr) return;
    if (hipStreamSynchronize(st) == hipSuccess)
        __atomic_store_n(t_sig.flag, t_sig.epoch, __ATOMIC_RELEASE);
    t_sig = Signal{nullptr, nullptr, 0};
}

// `final`: the last launch of an API call, the one that carries the signal
template <typename K, typename P>
int launch(K kernel, dim3 grid, hipStream_t st, P p, bool final = true) {
    p.sig = Signal{nullptr, nullptr, 0};
    if (final) {
        p.sig = t_sig;
        t_sig = Signal{nullptr, nullptr, 0};
    }
    if (t_ev_start != nullptr || t_ev_stop != nullptr) {
        hipExtLaunchKernelGGL(kernel, grid, dim3(kBlock), 0, st, t_ev_start, t_ev_stop, 0, p);
        t_ev_start = t_ev_stop = nullptr;
    } else {
        hipLaunchKernelGGL(kernel, grid, dim3(kBlock), 0, st, p);
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

int device_cus() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (g_cus[dev] == 0) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            cus <= 0)
            cus = 256;
        g_cus[dev] = cus;
    }
    return g_cus[dev];
}

// Blocks for a streaming launch: enough to cover the work once, capped at
// kBlocksPerCU resident blocks per CU (grid-stride covers the rest).
constexpr int kBlocksPerCU = 8;

unsigned grid_for(uint64_t units_per_block_pass, uint64_t units, int blocks_per_cu = kBlocksPerCU) {
    uint64_t want = (units + units_per_block_pass - 1) / units_per_block_pass;
    uint64_t cap = (uint64_t)device_cus() * blocks_per_cu;
    if (want < 1) want = 1;
    return (unsigned)(want < cap ? want : cap);
}

// Launch shape per source count, from tools/hbm_sweep.hip and
// tools/fold_bench.py on MI355X (256 MiB per source, double sums,
// non-temporal loads + `nt sc1` stores; GB/s counts (k+1) x 256 MiB;
// profiles/r01/hbm_sweep_v5.txt, fold_bench_k_sources.jsonl):
//   k=2: 1 vector/lane,  2 blocks/CU     6.4 TB/s
//   k=3: 2 vectors/lane, 1 block/CU      6.5 TB/s
//   k=4: 1 vector/lane,  1 block/CU      6.2-6.3 TB/s
//   k=8: 4 vectors/lane, 8 blocks/CU     5.8-5.9 TB/s (k=5..7 take k=8's
//        depth at half the blocks)
// Box-to-box spread is +-3 %, so neighbours within that band are ties.
// Long double is VALU-bound (x87 arithmetic in software): it wants many
// waves to hide ALU latency, not deep per-lane load queues.
template <int NSRC, typename T> struct Shape {
    static constexpr bool alu_heavy = std::is_same<T, x80>::value;
    static constexpr int unroll =
        alu_heavy ? 1 : NSRC == 2 ? 1 : NSRC == 3 ? 2 : NSRC == 4 ? 1 : NSRC < 8 ? 2 : 4;
    static constexpr int blocks_per_cu =
        alu_heavy ? 8 : NSRC == 2 ? 2 : NSRC == 3 ? 1 : NSRC == 4 ? 1 : NSRC < 8 ? 4 : 8;
    static constexpr int policy = POL_NT_LOAD;
};

// mi355_combine_orders: NSRC loads and up to NSRC stores per vector (every
// member's fold); the loads in flight per lane are those of the fold of the
// same width. Complex types: one vector per lane (NSRC*(NSRC-1) complex
// products per vector do not fit the registers of deeper unrolling; the
// loads in flight come from more blocks instead).
template <int NSRC, typename T> struct OrdersShape {
    static constexpr bool cplx = std::is_same<T, cplxf>::value || std::is_same<T, cplxd>::value;
    using S = Shape<NSRC, T>;
    static constexpr int unroll = cplx ? 1 : S::unroll;
    static constexpr int blocks_per_cu = cplx ? (S::blocks_per_cu * S::unroll < 8 ? S::blocks_per_cu * S::unroll : 8)
                                              : S::blocks_per_cu;
    static constexpr int policy = POL_NT_LOAD;
};

// How a launch over these pointers can run as 16-byte vectors: 0 = every
// pointer aligned; h > 0 = every pointer equally misaligned by whole elements
// (a user offset into the arrays): fold the first h elements element-wise and
// the rest as vectors from the advanced pointers (peeled to a 128-byte line
// when all share the misalignment within the line, else to 16 bytes); -1 =
// element-wise kernel.
template <typename T>
long vector_head(const void *const *ptrs, int np, size_t n) {
    constexpr int V = 16 / sizeof(T);
    uintptr_t orbits = 0;
    for (int k = 0; k < np; ++k) orbits |= (uintptr_t)ptrs[k];
    if ((orbits & 15) == 0) return 0;
    if (V == 1) return -1;
    uintptr_t mis = (uintptr_t)ptrs[0] & 127;
    bool line = true;
    for (int k = 1; k < np; ++k) line = line && ((uintptr_t)ptrs[k] & 127) == mis;
    if (!line) mis &= 15;
    bool same = mis % sizeof(T) == 0;
    for (int k = 1; k < np; ++k) same = same && ((uintptr_t)ptrs[k] & (line ? 127 : 15)) == mis;
    const size_t head = ((line ? 128 : 16) - mis) / sizeof(T);
    return same && n > head ? (long)head : -1;
}

template <int OP, typename T, int NSRC>
int launch_fixed(void *dst, const void *const *srcs, size_t n, hipStream_t st, bool final) {
    CombineParams p{};
    const void *ptrs[kMaxSrc + 1];
    p.dst = dst;
    ptrs[0] = dst;
    for (int k = 0; k < NSRC; ++k) p.src[k] = ptrs[1 + k] = srcs[k];
    constexpr int V = 16 / sizeof(T);
    const long head = vector_head<T>(ptrs, NSRC + 1, n);
    if (head >= 0) {
        if (head > 0) {
            p.head = (uint32_t)head;
            p.dst = (char *)dst + head * sizeof(T);
            for (int k = 0; k < NSRC; ++k) p.src[k] = (const char *)srcs[k] + head * sizeof(T);
            n -= (size_t)head;
        }
        using S = Shape<NSRC, T>;
        p.nvec = n / V;
        p.tail = (uint32_t)(n % V);
        const unsigned grid = grid_for((uint64_t)kBlock * S::unroll, p.nvec, S::blocks_per_cu);
        return launch(combine_vec<OP, T, NSRC, S::unroll, S::policy>, dim3(grid), st, p, final);
    }
    p.nvec = n;
    p.tail = 0;
    const unsigned grid = grid_for((uint64_t)kBlock * 4, n);
    return launch(combine_scalar<OP, T, NSRC>, dim3(grid), st, p, final);
}

// mi355_combine_orders for NSRC <= kMaxSrc sources: one launch
template <int OP, typename T, int NSRC>
int launch_orders_fixed(void *const *dsts, const void *const *srcs, size_t n, hipStream_t st) {
    OrdersParams p{};
    const void *ptrs[2 * kMaxSrc];
    int np = 0;
    for (int k = 0; k < NSRC; ++k) {
        p.src[k] = ptrs[np++] = srcs[k];
        p.dst[k] = dsts[k];
        if (dsts[k] != nullptr) ptrs[np++] = dsts[k];
    }
    constexpr int V = 16 / sizeof(T);
    const long head = vector_head<T>(ptrs, np, n);
    if (head >= 0) {
        if (head > 0) {
            p.head = (uint32_t)head;
            for (int k = 0; k < NSRC; ++k) {
                p.src[k] = (const char *)srcs[k] + head * sizeof(T);
                if (dsts[k] != nullptr) p.dst[k] = (char *)dsts[k] + head * sizeof(T);
            }
            n -= (size_t)head;
        }
        using S = OrdersShape<NSRC, T>;
        p.nvec = n / V;
        p.tail = (uint32_t)(n % V);
        const unsigned grid = grid_for((uint64_t)kBlock * S::unroll, p.nvec, S::blocks_per_cu);
        return launch(combine_orders_vec<OP, T, NSRC, S::unroll, S::policy>, dim3(grid), st, p);
    }
    p.nvec = n;
    p.tail = 0;
    const unsigned grid = grid_for((uint64_t)kBlock * 4, n);
    return launch(combine_orders_scalar<OP, T, NSRC>, dim3(grid), st, p);
}

template <int OP, typename T>
int launch_n(int nsrc, void *dst, const void *const *srcs, size_t n, hipStream_t st, bool final) {
    switch (nsrc) {
    case 1: return launch_fixed<OP, T, 1>(dst, srcs, n, st, final);
    case 2: return launch_fixed<OP, T, 2>(dst, srcs, n, st, final);
    case 3: return launch_fixed<OP, T, 3>(dst, srcs, n, st, final);
    case 4: return launch_fixed<OP, T, 4>(dst, srcs, n, st, final);
    case 5: return launch_fixed<OP, T, 5>(dst, srcs, n, st, final);
    case 6: return launch_fixed<OP, T, 6>(dst, srcs, n, st, final);
    case 7: return launch_fixed<OP, T, 7>(dst, srcs, n, st, final);
    case 8: return launch_fixed<OP, T, 8>(dst, srcs, n, st, final);
    default: return MI355_E_INVAL;
    }
}

// Left fold of any number of sources: first kMaxSrc into dst, then dst
// stays the accumulator (first operand) of every following launch. `final`:
// the last launch carries the armed completion signal.
template <int OP, typename T>
int launch_fold(void *dst, const void *const *srcs, int nsrc, size_t n, hipStream_t st, bool final = true) {
    if constexpr (!valid_pair<OP, T>()) {
        return MI355_E_UNSUP;
    } else {
        int first = nsrc < kMaxSrc ? nsrc : kMaxSrc;
        int rc = launch_n<OP, T>(first, dst, srcs, n, st, final && first == nsrc);
        int done = first;
        while (rc == 0 && done < nsrc) {
            const void *chunk[kMaxSrc];
            chunk[0] = dst;
            int take = nsrc - done < kMaxSrc - 1 ? nsrc - done : kMaxSrc - 1;
            for (int k = 0; k < take; ++k) chunk[1 + k] = srcs[done + k];
            done += take;
            rc = launch_n<OP, T>(1 + take, dst, chunk, n, st, final && done == nsrc);
        }
        return rc;
    }
}

template <typename T>
int dispatch_op(int op, void *dst, const void *const *srcs, int nsrc, size_t n, hipStream_t st) {
    switch (op) {
    case MI355_OP_SUM: return launch_fold<MI355_OP_SUM, T>(dst, srcs, nsrc, n, st);
    case MI355_OP_PROD: return launch_fold<MI355_OP_PROD, T>(dst, srcs, nsrc, n, st);
    case MI355_OP_AND: return launch_fold<MI355_OP_AND, T>(dst, srcs, nsrc, n, st);
    case MI355_OP_OR: return launch_fold<MI355_OP_OR, T>(dst, srcs, nsrc, n, st);
    case MI355_OP_XOR: return launch_fold<MI355_OP_XOR, T>(dst, srcs, nsrc, n, st);
    case MI355_OP_MIN: return launch_fold<MI355_OP_MIN, T>(dst, srcs, nsrc, n, st);
    case MI355_OP_MAX: return launch_fold<MI355_OP_MAX, T>(dst, srcs, nsrc, n, st);
    default: return MI355_E_INVAL;
    }
}

// Every member's order (mi355_combine_orders): one launch up to kMaxSrc
// sources. Beyond that, each member's fold is its own multi-launch left fold
// in that member's order; a fold whose target is its own source (in place)
// runs last, since the other folds still read that source.
template <int OP, typename T>
int launch_orders(void *const *dsts, const void *const *srcs, int nsrc, size_t n, hipStream_t st) {
    if constexpr (!valid_pair<OP, T>()) {
        return MI355_E_UNSUP;
    } else {
        switch (nsrc) {
        case 2: return launch_orders_fixed<OP, T, 2>(dsts, srcs, n, st);
        case 3: return launch_orders_fixed<OP, T, 3>(dsts, srcs, n, st);
        case 4: return launch_orders_fixed<OP, T, 4>(dsts, srcs, n, st);
        case 5: return launch_orders_fixed<OP, T, 5>(dsts, srcs, n, st);
        case 6: return launch_orders_fixed<OP, T, 6>(dsts, srcs, n, st);
        case 7: return launch_orders_fixed<OP, T, 7>(dsts, srcs, n, st);
        case 8: return launch_orders_fixed<OP, T, 8>(dsts, srcs, n, st);
        default: break;
        }
        int alias = -1, last = -1;
        for (int q = 0; q < nsrc; ++q) {
            if (dsts[q] == nullptr) continue;
            if (dsts[q] == srcs[q]) alias = q;
            else last = q;
        }
        const int final_q = alias >= 0 ? alias : last;
        const void *order[MI355_ORDERS_MAX_SOURCES];
        int rc = 0;
        for (int j = 0; j <= nsrc && rc == 0; ++j) {
            const int q = j < nsrc ? j : alias;  // the in-place fold, if any, after all others
            if (q < 0 || dsts[q] == nullptr || (j < nsrc && q == alias)) continue;
            order[0] = srcs[q];
            int m = 1;
            for (int k = 0; k < nsrc; ++k)
                if (k != q) order[m++] = srcs[k];
            rc = launch_fold<OP, T>(dsts[q], order, nsrc, n, st, q == final_q);
        }
        return rc;
    }
}

template <typename T>
int dispatch_orders(int op, void *const *dsts, const void *const *srcs, int nsrc, size_t n, hipStream_t st) {
    switch (op) {
    case MI355_OP_SUM: return launch_orders<MI355_OP_SUM, T>(dsts, srcs, nsrc, n, st);
    case MI355_OP_PROD: return launch_orders<MI355_OP_PROD, T>(dsts, srcs, nsrc, n, st);
    case MI355_OP_AND: return launch_orders<MI355_OP_AND, T>(dsts, srcs, nsrc, n, st);
    case MI355_OP_OR: return launch_orders<MI355_OP_OR, T>(dsts, srcs, nsrc, n, st);
    case MI355_OP_XOR: return launch_orders<MI355_OP_XOR, T>(dsts, srcs, nsrc, n, st);
    case MI355_OP_MIN: return launch_orders<MI355_OP_MIN, T>(dsts, srcs, nsrc, n, st);
    case MI355_OP_MAX: return launch_orders<MI355_OP_MAX, T>(dsts, srcs, nsrc, n, st);
    default: return MI355_E_INVAL;
    }
}

}  // namespace

extern "C" size_t mi355_dtype_size(int dtype) {
    switch (dtype) {
    case MI355_SHORT: return 2;
    case MI355_INT: return 4;
    case MI355_LONG:
    case MI355_LONGLONG: return 8;
    case MI355_FLOAT: return 4;
    case MI355_DOUBLE: return 8;
    case MI355_LONGDOUBLE: return 16;
    case MI355_COMPLEXF: return 8;
    case MI355_COMPLEXD: return 16;
    default: return 0;
    }
}

extern "C" int mi355_op_supported(int op, int dtype) {
    if (op < 0 || op >= MI355_NUM_OPS || dtype < 0 || dtype >= MI355_NUM_DTYPES) return 0;
    const bool is_int = dtype <= MI355_LONGLONG;
    const bool is_cplx = dtype == MI355_COMPLEXF || dtype == MI355_COMPLEXD;
    if (op == MI355_OP_SUM || op == MI355_OP_PROD) return 1;
    if (op == MI355_OP_AND || op == MI355_OP_OR || op == MI355_OP_XOR) return is_int ? 1 : 0;
    return is_cplx ? 0 : 1;
}

static int combine_impl(int op, int dtype, void *dst, const void *const *srcs, int nsrc, size_t n,
                        void *stream);
static int copy_segments_impl(void *const *dsts, const void *const *srcs, const size_t *nbytes, int nseg,
                              void *stream);
static int combine_orders_impl(int op, int dtype, void *const *dsts, const void *const *srcs, int nsrc, size_t n,
                               void *stream);

// Every error return cancels an armed signal/timing request (nothing carries them).
extern "C" int mi355_combine(int op, int dtype, void *dst, const void *const *srcs, int nsrc,
                             size_t n, void *stream) {
    const int rc = combine_impl(op, dtype, dst, srcs, nsrc, n, stream);
    if (rc != 0) {
        t_sig = Signal{nullptr, nullptr, 0};
        t_ev_start = t_ev_stop = nullptr;
    }
    return rc;
}

extern "C" int mi355_combine_orders(int op, int dtype, void *const *dsts, const void *const *srcs, int nsrc,
                                    size_t n, void *stream) {
    const int rc = combine_orders_impl(op, dtype, dsts, srcs, nsrc, n, stream);
    if (rc != 0) {
        t_sig = Signal{nullptr, nullptr, 0};
        t_ev_start = t_ev_stop = nullptr;
    }
    return rc;
}

extern "C" int mi355_copy_segments(void *const *dsts, const void *const *srcs, const size_t *nbytes,
                                   int nseg, void *stream) {
    const int rc = copy_segments_impl(dsts, srcs, nbytes, nseg, stream);
    if (rc != 0) {
        t_sig = Signal{nullptr, nullptr, 0};
        t_ev_start = t_ev_stop = nullptr;
    }
    return rc;
}

static int combine_impl(int op, int dtype, void *dst, const void *const *srcs, int nsrc, size_t n,
                        void *stream) {
    if (!mi355_op_supported(op, dtype)) return MI355_E_UNSUP;
    if (nsrc < 1 || dst == nullptr || srcs == nullptr) return MI355_E_INVAL;
    for (int k = 0; k < nsrc; ++k)
        if (srcs[k] == nullptr) return MI355_E_INVAL;
    hipStream_t st = (hipStream_t)stream;
    if (n == 0 || (nsrc == 1 && dst == srcs[0])) {
        fire_on_host(st);
        return 0;
    }
    if (nsrc == 1) {
        // a one-source fold is a copy: byte copy, independent of op/type
        void *d[1] = {dst};
        size_t nb[1] = {n * mi355_dtype_size(dtype)};
        return mi355_copy_segments(d, srcs, nb, 1, stream);
    }
    switch (dtype) {
    case MI355_SHORT: return dispatch_op<int16_t>(op, dst, srcs, nsrc, n, st);
    case MI355_INT: return dispatch_op<int32_t>(op, dst, srcs, nsrc, n, st);
    case MI355_LONG:
    case MI355_LONGLONG: return dispatch_op<int64_t>(op, dst, srcs, nsrc, n, st);
    case MI355_FLOAT: return dispatch_op<float>(op, dst, srcs, nsrc, n, st);
    case MI355_DOUBLE: return dispatch_op<double>(op, dst, srcs, nsrc, n, st);
    case MI355_LONGDOUBLE: return dispatch_op<x80>(op, dst, srcs, nsrc, n, st);
    case MI355_COMPLEXF: return dispatch_op<cplxf>(op, dst, srcs, nsrc, n, st);
    case MI355_COMPLEXD: return dispatch_op<cplxd>(op, dst, srcs, nsrc, n, st);
    default: return MI355_E_INVAL;
    }
}

static int combine_orders_impl(int op, int dtype, void *const *dsts, const void *const *srcs, int nsrc, size_t n,
                               void *stream) {
    if (!mi355_op_supported(op, dtype)) return MI355_E_UNSUP;
    if (nsrc < 1 || nsrc > MI355_ORDERS_MAX_SOURCES || dsts == nullptr || srcs == nullptr) return MI355_E_INVAL;
    int ndst = 0, nalias = 0;
    for (int k = 0; k < nsrc; ++k) {
        if (srcs[k] == nullptr) return MI355_E_INVAL;
        if (dsts[k] != nullptr) {
            ++ndst;
            if (dsts[k] == srcs[k]) ++nalias;
        }
    }
    // beyond one launch's sources the folds run one after another: only one may be in place
    if (nsrc > kMaxSrc && nalias > 1) return MI355_E_INVAL;
    hipStream_t st = (hipStream_t)stream;
    if (n == 0 || ndst == 0) {
        fire_on_host(st);
        return 0;
    }
    if (nsrc == 1) return combine_impl(op, dtype, dsts[0], srcs, 1, n, stream);
    switch (dtype) {
    case MI355_SHORT: return dispatch_orders<int16_t>(op, dsts, srcs, nsrc, n, st);
    case MI355_INT: return dispatch_orders<int32_t>(op, dsts, srcs, nsrc, n, st);
    case MI355_LONG:
    case MI355_LONGLONG: return dispatch_orders<int64_t>(op, dsts, srcs, nsrc, n, st);
    case MI355_FLOAT: return dispatch_orders<float>(op, dsts, srcs, nsrc, n, st);
    case MI355_DOUBLE: return dispatch_orders<double>(op, dsts, srcs, nsrc, n, st);
    case MI355_LONGDOUBLE: return dispatch_orders<x80>(op, dsts, srcs, nsrc, n, st);
    case MI355_COMPLEXF: return dispatch_orders<cplxf>(op, dsts, srcs, nsrc, n, st);
    case MI355_COMPLEXD: return dispatch_orders<cplxd>(op, dsts, srcs, nsrc, n, st);
    default: return MI355_E_INVAL;
    }
}

static int copy_segments_impl(void *const *dsts, const void *const *srcs, const size_t *nbytes, int nseg,
                              void *stream) {
    if (nseg < 0 || nseg > kMaxSeg) return MI355_E_INVAL;
    if (nseg == 0) {
        fire_on_host((hipStream_t)stream);
        return 0;
    }
    if (dsts == nullptr || srcs == nullptr || nbytes == nullptr) return MI355_E_INVAL;
    SegParams<kMaxSeg> p{};
    uint64_t maxv = 0;
    int used = 0;
    for (int k = 0; k < nseg; ++k) {
        if (nbytes[k] == 0 || dsts[k] == srcs[k]) continue;
        if (dsts[k] == nullptr || srcs[k] == nullptr) return MI355_E_INVAL;
        p.dst[used] = dsts[k];
        p.src[used] = srcs[k];
        p.nbytes[used] = nbytes[k];
        uint64_t v = (nbytes[k] + 15) / 16;
        if (v > maxv) maxv = v;
        ++used;
    }
    if (used == 0) {
        fire_on_host((hipStream_t)stream);
        return 0;
    }
    // pipelined UNROLL 4, one block per CU (tools/copy_variants.hip,
    // profiles/r01/copy_variants.txt: 78.2-78.5 us for 256 MiB, the best of
    // grid-stride / per-block partition / 1-4 blocks per CU / UNROLL 4-16)
    constexpr int U = 4;
    unsigned gx = grid_for((uint64_t)kBlock * U, maxv, 1);
    // keep total blocks ~ cap when many segments share the chip
    unsigned cap = (unsigned)device_cus();
    if ((uint64_t)gx * used > cap) gx = cap / used > 0 ? cap / used : 1;
    if (used == 1) {
        SegParams<1> p1{};
        p1.dst[0] = p.dst[0];
        p1.src[0] = p.src[0];
        p1.nbytes[0] = p.nbytes[0];
        return launch(copy_segments<U, 1>, dim3(gx, 1), (hipStream_t)stream, p1);
    }
    return launch(copy_segments<U, kMaxSeg>, dim3(gx, used), (hipStream_t)stream, p);
}

// System-scope acquire on every XCD of this GPU (`buffer_inv sc0 sc1`): drops
// L2 copies of lines another agent may have rewritten since they were read.
// Peer GPUs' memory reached through IPC mappings is cached in this GPU's L2
// without coherence (non-coherent MTYPE), and a kernel boundary on the same
// stream only acquires at agent scope, so a fold or copy that reads peers'
// buffers a second time (the next call on the same buffers) could otherwise
// hit the first call's lines. 32 one-wave blocks: blocks are dealt
// round-robin over the 8 XCDs, so every XCD's L2 gets invalidated (4 times);
// the next kernel on the stream starts after all of them. (One block per CU
// cost ~8 us per call at 4 PEs on one GPU: the invalidates queue up.)
__global__ __launch_bounds__(64) void acquire_system_k() {
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

extern "C" int mi355_acquire_system(void *stream) {
    hipLaunchKernelGGL(acquire_system_k, dim3(32), dim3(64), 0, (hipStream_t)stream);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

extern "C" int mi355_signal_launch(void *stream) {
    if (t_sig.flag == nullptr) return MI355_E_INVAL;
    return launch(signal_only, dim3(1), (hipStream_t)stream, EmptyParams{});
}

extern "C" void mi355_signal_next_launch(unsigned *count, unsigned *flag, unsigned epoch) {
    t_sig = Signal{count, flag, epoch};
}

extern "C" void mi355_time_next_launch(void *start_event, void *stop_event) {
    t_ev_start = (hipEvent_t)start_event;
    t_ev_stop = (hipEvent_t)stop_event;
}

// For fused.hip (same library): take the event pair armed for the next
// launch, if any, so its kernels carry the stamps too.
extern "C" void mi355i_take_launch_events(void **start_event, void **stop_event) {
    *start_event = t_ev_start;
    *stop_event = t_ev_stop;
    t_ev_start = t_ev_stop = nullptr;
}

// short <-> int32 for the RCCL schedule (RCCL has no 16-bit integer type):
// sum/prod wrap mod 2^32 in int32, and truncating to 16 bits afterwards gives
// the same bits as the reference's per-step promote-and-truncate (truncation
// is a ring homomorphism); min/max are exact on widened values.
__global__ __launch_bounds__(256) void widen_short_k(const int16_t *s, int32_t *d, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        d[i] = s[i];
}
__global__ __launch_bounds__(256) void narrow_int_k(const int32_t *s, int16_t *d, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        d[i] = (int16_t)s[i];
}

extern "C" int mi355_convert_short(int widen, const void *src, void *dst, size_t n, void *stream) {
    if (n == 0) return 0;
    if (src == nullptr || dst == nullptr) return MI355_E_INVAL;
    const unsigned grid = grid_for(256, n, 2);
    if (widen)
        hipLaunchKernelGGL(widen_short_k, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const int16_t *)src,
                           (int32_t *)dst, (uint64_t)n);
    else
        hipLaunchKernelGGL(narrow_int_k, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const int32_t *)src,
                           (int16_t *)dst, (uint64_t)n);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}
