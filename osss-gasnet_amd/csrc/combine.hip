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
#include <cxxabi.h>
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <type_traits>

#include "combine_kernels.h"
#include "mi355_reduce.h"
#include "ops.h"

namespace mi355k {

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

// Where a segment's vector part starts: `head` bytes peeled so the target
// starts on a 128-byte line (whole-line stores: a target 16 bytes off its
// line cost the copy 96 us against 77 per 256 MiB, profiles/r05/cold/
// linepeel_*.jsonl), then the source's phase against it (0: 16-byte aligned
// too; otherwise copy_segments_shift).
struct SegPlan {
    uint64_t head;
    unsigned delta;
};
__host__ __device__ inline SegPlan seg_plan(const void *dst, const void *src, uint64_t nb) {
    uint64_t head = (128u - (unsigned)((uintptr_t)dst & 127)) & 127u;
    if (head > nb) head = nb;
    return {head, (unsigned)(((uintptr_t)src + head) & 15)};
}

template <int UNROLL, int NS>
__global__ __launch_bounds__(kBlock) void copy_segments(SegParams<NS> p) {
    const int sg = blockIdx.y;
    const uint64_t nb = p.nbytes[sg];
    const char *src = (const char *)p.src[sg];
    char *dst = (char *)p.dst[sg];
    // 16-byte vectors where both ends are aligned: pointers with the same
    // misalignment within 16 bytes (a user offset into two arrays) peel a
    // head so that the target starts on a 128-byte line (seg_plan); different
    // misalignments take the narrow path below (the launcher sends them to
    // copy_segments_shift)
    const unsigned mis128 = (unsigned)((uintptr_t)dst & 127);
    const unsigned mis = mis128 & 15u;
    const bool coaligned = mis == (unsigned)((uintptr_t)src & 15);
    uint64_t head = !coaligned ? nb : (128u - mis128) & 127u;
    if (head > nb) head = nb;
    uint64_t vec_end = head;  // bytes [head, vec_end) go as vectors
    if (coaligned) {
        const u32x4 *s = (const u32x4 *)(src + head);
        u32x4 *d = (u32x4 *)(dst + head);
        const uint64_t nvec = (nb - head) / 16;
        const uint64_t step = (uint64_t)gridDim.x * kBlock * UNROLL;
        // software-pipelined: the loads of pass k+1 are in flight while the
        // stores of pass k issue (tools/probes/copy_variants.hip: 78.3 vs 80.0 us for
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

// A launch with a segment whose source is at another 16-byte phase than its
// target (a byte offset into one of the buffers): the target peeled to its
// 128-byte line (seg_plan), then copy_segments' pipelined loop with unaligned source loads
// (combine_kernels.h ld16_src; 0.87 of peak with the target on its line,
// against 0.24 in 8-byte words). Only such launches take this kernel, so
// copy_segments' code stays as measured.
template <int UNROLL, int NS>
__global__ __launch_bounds__(kBlock) void copy_segments_shift(SegParams<NS> p) {
    const int sg = blockIdx.y;
    const uint64_t nb = p.nbytes[sg];
    const char *src = (const char *)p.src[sg];
    char *dst = (char *)p.dst[sg];
    const uint64_t head = seg_plan(dst, src, nb).head;
    const u32x4 *s = (const u32x4 *)(src + head);   // not 16-byte aligned: read with ld16_src<.., true>
    u32x4 *d = (u32x4 *)(dst + head);
    const uint64_t nvec = (nb - head) / 16;
    // copy_segments' pipelined loop, two blocks per CU (cold_probe linepeel,
    // 256 MiB: 77 us = 0.87 of peak, 87 us before the target was peeled to
    // its line; one vector per lane per pass: 119 us)
    const uint64_t step = (uint64_t)gridDim.x * kBlock * UNROLL;
    uint64_t base = (uint64_t)blockIdx.x * kBlock * UNROLL + threadIdx.x;
    u32x4 x[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
        const uint64_t i = base + (uint64_t)u * kBlock;
        if (i < nvec) x[u] = ld16_src<POL_PLAIN, true>(s, i);
    }
    while (base < nvec) {
        const uint64_t next = base + step;
        u32x4 y[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = next + (uint64_t)u * kBlock;
            if (i < nvec) y[u] = ld16_src<POL_PLAIN, true>(s, i);
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
    // the bytes outside the vector part: [0, head) and [head + 16 nvec, nb)
    const uint64_t vec_end = head + nvec * 16;
    const uint64_t nrest = head + (nb - vec_end);
    bool plain = false;
    for (uint64_t r = (uint64_t)blockIdx.x * kBlock + threadIdx.x; r < nrest; r += (uint64_t)gridDim.x * kBlock) {
        const uint64_t i = r < head ? r : vec_end + (r - head);
        dst[i] = src[i];
        plain = true;
    }
    signal_done(p.sig, __syncthreads_or(plain));
}

// The two-member all-gather of a float/double sum or product (reduce.c,
// nan_pair): member q copies the other member p's shard, which p folded in
// ITS order, x86(a_p op a_q), and needs x86(a_q op a_p). The two are the same
// bits except where both operands are NaNs: SSE returns the first NaN
// operand, quieted (ops.h x86_result) -- a_q for q. So wherever q's own
// source a_q is a NaN the result is a_q quieted, elsewhere the copied value:
//   dst[i] = isnan(own[i]) ? quiet(own[i]) : peer[i]
// (own may alias dst: element-wise read-then-write). Plain loads and `nt sc1`
// stores as the copy kernel; one more local read stream than the copy.
// dst and peer share their 16-byte phase (one symmetric offset): the host
// peels `head` elements so both are aligned; own, at another phase when the
// target is offset against the source, is read unaligned (SHIFT, ld16_src).
// nvec == 0: every element through the element loop.
struct PatchParams {
    void *dst;
    const void *peer;
    const void *own;
    const unsigned long long *nan_flag;   // the other member's NaN word, or nullptr (patch)
    uint64_t nvec;   // whole 16-byte vectors
    uint64_t n;      // elements from dst (after the head)
    uint32_t head;   // elements just before dst / peer / own (peeled)
    Signal sig;
};

template <typename R>
__device__ __forceinline__ R nan_keep_own(R own, R peer) {
    using N = X86Nan<R>;
    using U = typename N::U;
    return __builtin_isnan(own) ? __builtin_bit_cast(R, __builtin_bit_cast(U, own) | N::quiet) : peer;
}

template <typename R, bool SHIFT>
__global__ __launch_bounds__(kBlock) void nan_patch_copy(PatchParams p) {
    constexpr int V = 16 / sizeof(R);
    constexpr int U = 4;
    // no NaN came out of the other member's fold: no result to patch, a copy
    // (the word is wave-uniform: one load, then a uniform branch)
    const bool patch = p.nan_flag == nullptr ||
                       __hip_atomic_load(const_cast<unsigned long long *>(p.nan_flag), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_SYSTEM) != 0;
    const u32x4 *pe = (const u32x4 *)p.peer;
    const u32x4 *ow = (const u32x4 *)p.own;
    u32x4 *d = (u32x4 *)p.dst;
    const uint64_t step = (uint64_t)gridDim.x * kBlock * U;
    for (uint64_t base = (uint64_t)blockIdx.x * kBlock * U + threadIdx.x; base < p.nvec; base += step) {
        Pack<R> x[U], o[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = base + (uint64_t)u * kBlock;
            if (i < p.nvec) {
                x[u].v = ld16<POL_PLAIN>(pe + i);
                if (patch) o[u].v = ld16_src<POL_PLAIN, SHIFT>(ow, i);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = base + (uint64_t)u * kBlock;
            if (i < p.nvec) {
                if (patch) {
#pragma unroll
                    for (int e = 0; e < V; ++e) x[u].e[e] = nan_keep_own(o[u].e[e], x[u].e[e]);
                }
                st16(d + i, x[u].v);
            }
        }
    }
    // the elements outside the vectors: [-head, 0) and [V nvec, n)
    bool plain = false;
    const uint64_t rest = p.head + (p.n - p.nvec * V);
    for (uint64_t r = (uint64_t)blockIdx.x * kBlock + threadIdx.x; r < rest; r += (uint64_t)gridDim.x * kBlock) {
        const int64_t i = r < p.head ? (int64_t)r - (int64_t)p.head : (int64_t)(p.nvec * V + (r - p.head));
        const R v = ((const R *)p.peer)[i];
        ((R *)p.dst)[i] = patch ? nan_keep_own(((const R *)p.own)[i], v) : v;
        plain = true;
    }
    signal_done(p.sig, __syncthreads_or(plain));
}

// One block that only carries the completion signal: tells the host when the
// stream has reached this point (everything queued before it has finished).
struct EmptyParams {
    Signal sig;
};
__global__ __launch_bounds__(kBlock) void signal_only(EmptyParams p) { signal_done(p.sig, false); }

}  // namespace mi355k

using namespace mi355k;

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
    t_nan_set = t_nan_clear = nullptr;  // a call that launched no fold consumes them too
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
    case MI355_SHORT: return combine_short(op, dst, srcs, nsrc, n, st);
    case MI355_INT: return combine_int(op, dst, srcs, nsrc, n, st);
    case MI355_LONG:
    case MI355_LONGLONG: return combine_long(op, dst, srcs, nsrc, n, st);
    case MI355_FLOAT: return combine_float(op, dst, srcs, nsrc, n, st);
    case MI355_DOUBLE: return combine_double(op, dst, srcs, nsrc, n, st);
    case MI355_LONGDOUBLE: return combine_longdouble(op, dst, srcs, nsrc, n, st);
    case MI355_COMPLEXF: return combine_complexf(op, dst, srcs, nsrc, n, st);
    case MI355_COMPLEXD: return combine_complexd(op, dst, srcs, nsrc, n, st);
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
    case MI355_SHORT: return orders_short(op, dsts, srcs, nsrc, n, st);
    case MI355_INT: return orders_int(op, dsts, srcs, nsrc, n, st);
    case MI355_LONG:
    case MI355_LONGLONG: return orders_long(op, dsts, srcs, nsrc, n, st);
    case MI355_FLOAT: return orders_float(op, dsts, srcs, nsrc, n, st);
    case MI355_DOUBLE: return orders_double(op, dsts, srcs, nsrc, n, st);
    case MI355_LONGDOUBLE: return orders_longdouble(op, dsts, srcs, nsrc, n, st);
    case MI355_COMPLEXF: return orders_complexf(op, dsts, srcs, nsrc, n, st);
    case MI355_COMPLEXD: return orders_complexd(op, dsts, srcs, nsrc, n, st);
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
    // pipelined UNROLL 4, one block per CU (tools/probes/copy_variants.hip,
    // profiles/r01/copy_variants.txt: 78.2-78.5 us for 256 MiB, the best of
    // grid-stride / per-block partition / 1-4 blocks per CU / UNROLL 4-16);
    // a segment whose source is at another phase than its target: the
    // unaligned-load kernel, two blocks per CU
    constexpr int U = 4;
    bool shifted = false;
    for (int k = 0; k < used; ++k) shifted = shifted || seg_plan(p.dst[k], p.src[k], p.nbytes[k]).delta != 0;
    unsigned gx = grid_for((uint64_t)kBlock * U, maxv, shifted ? 2 : 1);
    // keep total blocks ~ cap when many segments share the chip
    unsigned cap = (unsigned)device_cus() * (shifted ? 2 : 1);
    if ((uint64_t)gx * used > cap) gx = cap / used > 0 ? cap / used : 1;
    if (used == 1) {
        SegParams<1> p1{};
        p1.dst[0] = p.dst[0];
        p1.src[0] = p.src[0];
        p1.nbytes[0] = p.nbytes[0];
        return launch(shifted ? copy_segments_shift<U, 1> : copy_segments<U, 1>, dim3(gx, 1), (hipStream_t)stream, p1);
    }
    return launch(shifted ? copy_segments_shift<U, kMaxSeg> : copy_segments<U, kMaxSeg>, dim3(gx, used),
                  (hipStream_t)stream, p);
}

extern "C" void mi355_nan_flag_next_launch(unsigned long long *set, unsigned long long *clear) {
    t_nan_set = set;
    t_nan_clear = clear;
}

extern "C" int mi355_nan_patch_copy(int dtype, void *dst, const void *peer, const void *own, size_t n,
                                    const unsigned long long *nan_flag, void *stream) {
    const int rc = [&]() -> int {
        if (dtype != MI355_FLOAT && dtype != MI355_DOUBLE) return MI355_E_UNSUP;
        if (n == 0) {
            fire_on_host((hipStream_t)stream);
            return 0;
        }
        if (dst == nullptr || peer == nullptr || own == nullptr) return MI355_E_INVAL;
        const size_t es = mi355_dtype_size(dtype);
        // 16-byte vectors from the element where dst (and peer, at the same
        // phase) is aligned; own read unaligned if its phase differs. Element
        // by element when dst and peer differ in phase or dst is not
        // element-aligned.
        // dst is peeled to its 128-byte line (whole-line stores, see
        // combine_kernels.h vector_head) when n reaches it, else to 16 bytes.
        const uintptr_t pd = (uintptr_t)dst & 15;
        const bool vec = pd == ((uintptr_t)peer & 15) && pd % es == 0;
        const size_t lh = ((128 - ((uintptr_t)dst & 127)) & 127) / es;
        const size_t head = !vec ? 0 : n >= lh ? lh : ((16 - pd) & 15) / es;
        const bool use_vec = vec && n >= head;
        PatchParams p{};
        p.nan_flag = nan_flag;
        if (use_vec) {
            p.dst = (char *)dst + head * es;
            p.peer = (const char *)peer + head * es;
            p.own = (const char *)own + head * es;
            p.n = n - head;
            p.head = (uint32_t)head;
            p.nvec = p.n * es / 16;
        } else {
            p.dst = dst;
            p.peer = peer;
            p.own = own;
            p.n = n;
        }
        const bool shift = use_vec && ((uintptr_t)p.own & 15) != 0;
        const unsigned grid = grid_for((uint64_t)kBlock * 4, p.nvec > 0 ? p.nvec : p.n + p.head, 1);
        auto k = dtype == MI355_FLOAT ? (shift ? nan_patch_copy<float, true> : nan_patch_copy<float, false>)
                                      : (shift ? nan_patch_copy<double, true> : nan_patch_copy<double, false>);
        return launch(k, dim3(grid), (hipStream_t)stream, p);
    }();
    if (rc != 0) {
        t_sig = Signal{nullptr, nullptr, 0};
        t_ev_start = t_ev_stop = nullptr;
    }
    return rc;
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

// For fused.hip: its launches count as this layer's last kernel too.
extern "C" void mi355i_note_launch(const void *kernel) { t_last_kernel = kernel; }

extern "C" const void *mi355_last_kernel(void) { return t_last_kernel; }

// The kernel's demangled name, as rocprofv3 prints it ("void
// mi355k::copy_segments<4, 1>(mi355k::SegParams<1>)"). Not on the hot path:
// the runtime keeps the stub pointer per call and resolves it on request.
extern "C" int mi355_kernel_name(const void *kernel, char *buf, size_t len) {
    if (kernel == nullptr || buf == nullptr || len == 0) return MI355_E_INVAL;
    const char *mangled = hipKernelNameRefByPtr(kernel, nullptr);
    (void)hipGetLastError();
    if (mangled == nullptr) return MI355_E_INVAL;
    int status = 0;
    char *dem = abi::__cxa_demangle(mangled, nullptr, nullptr, &status);
    snprintf(buf, len, "%s", status == 0 && dem != nullptr ? dem : mangled);
    free(dem);
    return 0;
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
