// combine_kernels.h -- the fold kernels (combine.hip's k-source left fold and
// every-member-order fold) and their launch templates, shared by the
// per-element-type translation units combine_t_*.hip (one per type, so the
// 8 x 7 x 8 instantiations compile in parallel) and combine.hip (the C ABI,
// the copy and signal kernels). See combine.hip for the design notes.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <mutex>
#include <type_traits>

#include "mi355_reduce.h"
#include "ops.h"

namespace mi355k {

using namespace mi355;

constexpr int kBlock = 256;
constexpr int kMaxSrc = 8;

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
// Completion signal (mi355_signal_next_launch): the last block to finish
// stores `epoch` into a host-visible word, so the host learns the result is
// in memory ~4 us sooner than through hipStreamSynchronize (tools/probes/latency.hip:
// 6.9 vs 10.7 us for a launch round trip on MI355X).
struct Signal {
    unsigned *count;  // device word, 0 between launches (the last block resets it)
    unsigned *flag;   // host-coherent word the host spins on; nullptr = no signal
    unsigned epoch;
};

// Publish recipe of MI355X_MICROARCH.md (inter-workgroup visibility, valid
// form "sc1 payload + drained waves + flag"): the bulk stores are
// write-through (`nt sc1` st16 in the copy, `sc1` st16_fold in the folds), so
// once every wave has drained its stores they are in memory for any agent; a
// block that also made plain stores (an
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
    unsigned long long *nan_set;    // mi355_nan_flag_next_launch: 1 here if a result is NaN
    unsigned long long *nan_clear;  // ... and 0 here first
    Signal sig;
};

// The two-member schedule's NaN word (reduce.c nan_pair): written at system
// scope, read by the other member's gather kernel over the peer mapping.
__device__ __forceinline__ void nan_flag_store(unsigned long long *w, unsigned long long v) {
    __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Cache policy (tools/probes/hbm_sweep.hip, MI355X, 256 MiB per buffer):
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
// hint. Beside non-temporal loads this is the faster form (tools/probes/fold_probe.hip,
// profiles/r02/fold_probe_copy.txt, 256 MiB per source: k = 2 116.4 vs 127.9 us,
// k = 3 158.7 vs 177.1, k = 8 393.5 vs 422); the copy keeps `nt sc1` (with
// its plain loads `sc1` alone is 18 % slower).
__device__ __forceinline__ void st16_fold(u32x4 *p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

// Sources at another 16-byte phase than the outputs (a user offset into one
// of the arrays, e.g. target = &t[1], source = &s[0]): the outputs are still
// written as aligned vectors and each source vector is read with one 16-byte
// load from its unaligned address. gfx950 runs in unaligned access mode (the
// loads stay global_load_dwordx4; the type below only tells the compiler the
// alignment it may assume). Measured (tools/probes/cold_probe unal / shift / dpp,
// 256 MiB double sum of two sources, target aligned, sources 8 bytes off):
// 0.84 of peak warm / 0.76 cold -- against 0.59 element-wise, 0.73 / 0.70
// assembling each vector from two aligned loads (v_alignbyte), 0.77 / 0.71
// with the neighbour's vector through a DPP wave shift, 0.42 through
// ds_bpermute; the copy 0.86 / 0.72 against 0.24 in 8-byte words. Every byte
// offset 1-15 reads the right bytes (cold_probe unal's check).
typedef unsigned u32x4_any __attribute__((ext_vector_type(4), aligned(1)));
template <int POL, bool SHIFT>
__device__ __forceinline__ u32x4 ld16_src(const u32x4 *s, uint64_t i) {
    if constexpr (!SHIFT) return ld16<POL>(s + i);
    const u32x4_any *p = (const u32x4_any *)s + i;
    if constexpr ((POL & POL_NT_LOAD) != 0) return __builtin_nontemporal_load(p);
    else return *p;
}

// The vector loop of combine_vec (SHIFT: sources at another phase than the
// target, read unaligned).
template <int OP, typename T, int NSRC, int UNROLL, int POL, bool SHIFT>
__device__ __forceinline__ void fold_vectors(const CombineParams &p) {
    constexpr int V = 16 / sizeof(T);
    const uint64_t nvec = p.nvec;
    const u32x4 *s[NSRC];
#pragma unroll
    for (int k = 0; k < NSRC; ++k) s[k] = (const u32x4 *)p.src[k];
    u32x4 *d = (u32x4 *)p.dst;
    const uint64_t step = (uint64_t)gridDim.x * kBlock * UNROLL;
    for (uint64_t base = (uint64_t)blockIdx.x * kBlock * UNROLL + threadIdx.x; base < nvec;
         base += step) {
        Pack<T> x[UNROLL][NSRC];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = base + (uint64_t)u * kBlock;
            if (i < nvec) {
#pragma unroll
                for (int k = 0; k < NSRC; ++k) x[u][k].v = ld16_src<POL, SHIFT>(s[k], i);
            }
        }
        // every load issued before the first use: left alone, the scheduler
        // placed a register copy of one load's data (and its wait) before
        // the next load (float sum, two sources: 174 vs 125 us per 256 MiB)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = base + (uint64_t)u * kBlock;
            if (i < nvec) {
                Pack<T> acc = x[u][0];
#pragma unroll
                for (int k = 1; k < NSRC; ++k) {
#pragma unroll
                    for (int e = 0; e < V; ++e) acc.e[e] = apply_fast<OP>(acc.e[e], x[u][k].e[e]);
                }
                if constexpr (has_fast_form<OP, T>()) {
                    // a NaN came out somewhere: the reference's operator, step by step
                    bool redo = false;
#pragma unroll
                    for (int e = 0; e < V; ++e) redo |= redo_needed<OP>(acc.e[e]);
                    if (redo) {
                        acc = x[u][0];
#pragma unroll
                        for (int k = 1; k < NSRC; ++k) {
#pragma unroll
                            for (int e = 0; e < V; ++e) acc.e[e] = apply<OP>(acc.e[e], x[u][k].e[e]);
                        }
                        if (p.nan_set != nullptr) nan_flag_store(p.nan_set, 1);
                    }
                }
                st16_fold(d + i, acc.v);
            }
        }
    }
}

// Vector path: every output 16-byte aligned, the sources too or (SHIFT) all
// at one other phase. Each lane owns UNROLL vectors
// spaced one block apart (so a wave touches contiguous 1 KiB per source per
// step) and issues all NSRC*UNROLL loads before combining.
template <int OP, typename T, int NSRC, int UNROLL, int POL, bool SHIFT = false>
__global__ __launch_bounds__(kBlock) void combine_vec(CombineParams p) {
    constexpr int V = 16 / sizeof(T);
    if (p.nan_clear != nullptr && blockIdx.x == 0 && threadIdx.x == 0) nan_flag_store(p.nan_clear, 0);
    fold_vectors<OP, T, NSRC, UNROLL, POL, SHIFT>(p);
    const uint64_t nvec = p.nvec;
    const bool tail_block = V > 1 && p.tail != 0 && blockIdx.x == 0;
    if (tail_block && threadIdx.x < p.tail) {
        const uint64_t i = nvec * V + threadIdx.x;
        T acc = ((const T *)p.src[0])[i];
#pragma unroll
        for (int k = 1; k < NSRC; ++k) acc = apply<OP>(acc, ((const T *)p.src[k])[i]);
        ((T *)p.dst)[i] = acc;
        if (p.nan_set != nullptr && redo_needed<OP>(acc)) nan_flag_store(p.nan_set, 1);
    }
    const bool head_block = V > 1 && p.head != 0 && blockIdx.x == 0;
    if (head_block && threadIdx.x < p.head) {
        const int64_t i = (int64_t)threadIdx.x - (int64_t)p.head;
        T acc = ((const T *)p.src[0])[i];
#pragma unroll
        for (int k = 1; k < NSRC; ++k) acc = apply<OP>(acc, ((const T *)p.src[k])[i]);
        ((T *)p.dst)[i] = acc;
        if (p.nan_set != nullptr && redo_needed<OP>(acc)) nan_flag_store(p.nan_set, 1);
    }
    signal_done(p.sig, tail_block || head_block);
}

// Scalar path for pointers that are not 16-byte aligned (user offsets into
// arrays). Coalesced element loads, grid-stride.
template <int OP, typename T, int NSRC>
__global__ __launch_bounds__(kBlock) void combine_scalar(CombineParams p) {
    if (p.nan_clear != nullptr && blockIdx.x == 0 && threadIdx.x == 0) nan_flag_store(p.nan_clear, 0);
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
        if (p.nan_set != nullptr && redo_needed<OP>(acc)) nan_flag_store(p.nan_set, 1);
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

// ALL: every dst[q] is set (the P2P schedule's case). Without the per-output
// null tests the compiler keeps the next pass's loads ahead of this pass's
// stores; with them it placed `s_waitcnt vmcnt` on the previous pass's stores
// before the loads (the stores' data registers are reused as load addresses
// across the branches), which halved the kernel's rate at 2-4 sources
// (tools/probes/orders_probe.hip; rocprofv3 160 vs 82 us at 4 x 64 MiB).
// The software x87 sum/product: NSRC * (NSRC - 1) soft-float operations per
// element are too much code to unroll over the members, and a register array
// indexed by a rolled loop's variable lives in scratch memory. So the NSRC
// sources are loaded once into registers and only the member loop q stays
// rolled: member q's operands -- its own source first, then the others in
// member order -- are picked from the registers with compile-time indices
// and masks (x80d::pick): the first operand is v[q], the j-th after it v[j]
// for j < q and v[j + 1] otherwise. All loads precede every store, so an
// output that aliases its source (in place) is safe. (Round 2 before this:
// each member's fold re-read the sources from L2 one dependent load per
// operation.)
template <int NSRC>
__device__ __forceinline__ void x80_load(const OrdersParams &p, uint64_t i, x80 (&v)[NSRC]) {
#pragma unroll
    for (int k = 0; k < NSRC; ++k) {
        Pack<x80> w;
        w.v = ld16<POL_NT_LOAD>((const u32x4 *)p.src[k] + i);
        v[k] = w.e[0];
    }
}

template <int OP, int NSRC, bool ALL>
__device__ __forceinline__ void x80_orders_vector(const OrdersParams &p, uint64_t i, const x80 (&v)[NSRC]) {
    // Member 1's order (s1, s0, s2, ...) gives member 0's value (s0, s1, s2,
    // ...): x87 + and * commute, NaN and signed-zero rules included, and the
    // rest of the two chains is the same -- one chain fewer per element.
    // Fast chains, unrolled over the members (operands picked at compile
    // time), on the unpacked form of x80.h's add_fast_u/mul_fast_u: the
    // sources' domain is checked once (x80d::chain_operand: exponents that
    // keep every step in range), each step checks only its alignment,
    // cancellation and rounding, and
    // one wave vote decides for all the element's chains: every lane stayed
    // in the fast domain, or the whole wave redoes the chains on the general
    // path (the same x87 results either way; the choice is wave-uniform).
    x80d::xu u[NSRC], res[NSRC];
    int ok = 1;
#pragma unroll
    for (int k = 0; k < NSRC; ++k) {
        u[k] = x80d::unpack(v[k]);
        ok &= x80d::chain_operand<OP, NSRC - 1>(v[k]);
    }
#pragma unroll
    for (int q = 0; q < NSRC; ++q) {
        if (q == 1) {
            res[1] = res[0];
            continue;
        }
        x80d::xu a = u[q];
        // one chain after the other: interleaved by the scheduler, the
        // chains' select masks outgrow the SGPRs and spill to VGPR lanes
        if (q > 0) asm volatile("" : "+v"(a.m) : "v"(res[q - 1].m));
#pragma unroll
        for (int j = 0; j + 1 < NSRC; ++j) {
            x80d::xu r;
            const x80d::xu &b = u[j < q ? j : j + 1];
            ok &= OP == MI355_OP_SUM ? x80d::add_fast_u<false>(a, b, r) : x80d::mul_fast_u<false>(a, b, r);
            a = r;
        }
        res[q] = a;
        // the fast result goes out now (its registers free for the next
        // chain); a wave that fails the vote below rewrites every output
        // from the general path (which works from v[], in registers, so an
        // output aliasing its source is still safe)
#pragma unroll
        for (int w = 0; w < (q == 0 && NSRC > 1 ? 2 : 1); ++w) {
            if (!ALL && p.dst[q + w] == nullptr) continue;
            Pack<x80> o;
            o.e[0] = x80d::pack(a, v[q + w]);
            st16_fold((u32x4 *)p.dst[q + w] + i, o.v);
        }
        asm volatile("" : "+v"(ok));  // a VGPR, not lane masks kept (and spilled) across the chains
    }
    if (__all(ok)) return;
    x80 first = v[0];
    bool have_first = false;
#pragma unroll 1
    for (int q = 0; q < NSRC; ++q) {
        // member q's output, picked with compile-time indices: p.dst[q] with
        // the rolled loop's q made the compiler copy the kernel arguments'
        // pointer array into scratch memory (24 bytes per lane at NSRC = 2)
        u32x4 *dq = (u32x4 *)p.dst[0];
#pragma unroll
        for (int k = 1; k < NSRC; ++k) dq = q == k ? (u32x4 *)p.dst[k] : dq;
        if (!ALL && dq == nullptr) continue;
        x80 acc = v[0];
#pragma unroll
        for (int k = 1; k < NSRC; ++k) acc = x80d::pick(q == k, v[k], acc);
        const x80 own = acc;
        if (q == 1 && have_first) {
            acc = first;
        } else {
#pragma unroll
            for (int j = 0; j + 1 < NSRC; ++j) {
                const x80 b = x80d::pick(j < q, v[j], v[j + 1]);
                acc = OP == MI355_OP_SUM ? x80d::add_general(acc, b) : x80d::mul_general(acc, b);
            }
            if (q == 0) {
                first = acc;
                have_first = true;
            }
        }
#pragma unroll
        for (int w = 0; w < 3; ++w) acc.pad[w] = own.pad[w];  // the padding of the member's own slot
        Pack<x80> o;
        o.e[0] = acc;
        st16_fold(dq + i, o.v);
    }
}

// Operand classes on which min/max selects are order-independent (above).
template <typename T>
__device__ __forceinline__ bool single_fold_ok(const T &v) {
    if constexpr (std::is_same<T, x80>::value) {
        const int e = v.se & 0x7FFF;
        return (e >= 1) & (e <= 0x7FFE) & ((v.m >> 63) != 0);
    } else {
        return (v == v) & (v != T(0));
    }
}

// Member q's chain with the reference's operator over one vector of every
// source held in registers, q a run-time value: operands picked with
// compile-time indices and selects (q's own vector first, then the others in
// member order), so the rolled member loop of the rare NaN path indexes no
// register array (which would live in scratch memory).
template <int OP, typename T, int NSRC>
__device__ __forceinline__ Pack<T> member_chain(const Pack<T> (&x)[NSRC], int q) {
    constexpr int V = 16 / sizeof(T);
    Pack<T> acc = x[0];
#pragma unroll
    for (int k = 1; k < NSRC; ++k) acc.v = q == k ? x[k].v : acc.v;
#pragma unroll
    for (int j = 0; j + 1 < NSRC; ++j) {
        Pack<T> b;
        b.v = j < q ? x[j].v : x[j + 1].v;
#pragma unroll
        for (int e = 0; e < V; ++e) acc.e[e] = apply<OP>(acc.e[e], b.e[e]);
    }
    return acc;
}

// Vector i of every member's fold, the sources' vectors of that position in x.
template <int OP, typename T, int NSRC, bool ALL>
__device__ __forceinline__ void orders_one(const OrdersParams &p, const Pack<T> (&x)[NSRC], uint64_t i) {
    constexpr int V = 16 / sizeof(T);
    if constexpr ((OP == MI355_OP_MIN || OP == MI355_OP_MAX) &&
                  (std::is_floating_point<T>::value || std::is_same<T, x80>::value)) {
        // When no operand is a NaN or a zero (long double: every operand
        // a normal number), `a < b ? a : b` picks the same value bits in
        // every order (equal numbers of these classes have one
        // encoding): one fold serves every member. The members' orders
        // only differ on NaNs, +-0 ties and (x87) equal values with
        // different encodings (reduce-op.c:138-150), which take the
        // per-member folds below (wave-uniform choice).
        bool plain = true;
#pragma unroll
        for (int k = 0; k < NSRC; ++k)
#pragma unroll
            for (int e = 0; e < V; ++e) plain &= single_fold_ok(x[k].e[e]);
        if (__all(plain)) {
            Pack<T> m = x[0];
#pragma unroll
            for (int k = 1; k < NSRC; ++k)
#pragma unroll
                for (int e = 0; e < V; ++e) m.e[e] = apply<OP>(m.e[e], x[k].e[e]);
#pragma unroll
            for (int q = 0; q < NSRC; ++q)
                if (ALL || p.dst[q] != nullptr) st16_fold((u32x4 *)p.dst[q] + i, m.v);
            return;
        }
    }
    // every member's chain with the fast operator forms (ops.h
    // apply_fast), each output stored as its chain ends; a lane where
    // any chain had a NaN come out redoes every chain with the
    // reference's operator (member_chain, from registers, so an output
    // aliasing its source is safe) and rewrites the outputs -- the
    // same bits either way. For complex products this is also Annex G's recovery (the
    // former float-only wave vote, now per lane and for every type).
    bool redo = false;
#pragma unroll
    for (int q = 0; q < NSRC; ++q) {
        if (!ALL && p.dst[q] == nullptr) continue;
        Pack<T> acc = x[q];
#pragma unroll
        for (int k = 0; k < NSRC; ++k) {
            if (k == q) continue;
#pragma unroll
            for (int e = 0; e < V; ++e) acc.e[e] = apply_fast<OP>(acc.e[e], x[k].e[e]);
        }
#pragma unroll
        for (int e = 0; e < V; ++e) redo |= redo_needed<OP>(acc.e[e]);
        st16_fold((u32x4 *)p.dst[q] + i, acc.v);
    }
    if constexpr (has_fast_form<OP, T>()) {
        if (redo) {
#pragma unroll 1
            for (int q = 0; q < NSRC; ++q) {
                u32x4 *dq = (u32x4 *)p.dst[0];
#pragma unroll
                for (int k = 1; k < NSRC; ++k) dq = q == k ? (u32x4 *)p.dst[k] : dq;
                if (!ALL && dq == nullptr) continue;
                st16_fold(dq + i, member_chain<OP, T, NSRC>(x, q).v);
            }
        }
    }
}

// The vector loop of combine_orders_vec (SHIFT: as fold_vectors).
template <int OP, typename T, int NSRC, int UNROLL, int POL, bool ALL, bool SHIFT>
__device__ __forceinline__ void orders_vectors(const OrdersParams &p) {
    const uint64_t nvec = p.nvec;
    const uint64_t step = (uint64_t)gridDim.x * kBlock * UNROLL;
    const u32x4 *sb[NSRC];
#pragma unroll
    for (int k = 0; k < NSRC; ++k) sb[k] = (const u32x4 *)p.src[k];
    for (uint64_t base = (uint64_t)blockIdx.x * kBlock * UNROLL + threadIdx.x; base < nvec;
         base += step) {
        Pack<T> x[UNROLL][NSRC];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = base + (uint64_t)u * kBlock;
            if (i < nvec) {
#pragma unroll
                for (int k = 0; k < NSRC; ++k) x[u][k].v = ld16_src<POL, SHIFT>(sb[k], i);
            }
        }
        __builtin_amdgcn_sched_barrier(0);   // loads first (fold_vectors)
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = base + (uint64_t)u * kBlock;
            if (i < nvec) orders_one<OP, T, NSRC, ALL>(p, x[u], i);
        }
    }
}

template <int OP, typename T, int NSRC, int UNROLL, int POL, bool ALL, bool SHIFT = false>
__global__ __launch_bounds__(kBlock) void combine_orders_vec(OrdersParams p) {
    constexpr int V = 16 / sizeof(T);
    const uint64_t nvec = p.nvec;
    static_assert(!SHIFT || !std::is_same<T, x80>::value, "long double runs aligned or element-wise");
    if constexpr (std::is_same<T, x80>::value && (OP == MI355_OP_SUM || OP == MI355_OP_PROD)) {
        const uint64_t stride = (uint64_t)gridDim.x * kBlock;
        uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
        for (; i < nvec; i += stride) {
            x80 v[NSRC];
            x80_load<NSRC>(p, i, v);
            x80_orders_vector<OP, NSRC, ALL>(p, i, v);
        }
        signal_done(p.sig, false);
        return;
    }
    orders_vectors<OP, T, NSRC, UNROLL, POL, ALL, SHIFT>(p);
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

// ---------------------------------------------------------------------------
// launch helpers
// ---------------------------------------------------------------------------
inline int g_cus[64];

// events and completion signal for the next launch (mi355_time_next_launch,
// mi355_signal_next_launch), consumed by it
inline thread_local hipEvent_t t_ev_start = nullptr, t_ev_stop = nullptr;
inline thread_local Signal t_sig = {nullptr, nullptr, 0};
// host stub of the kernel this layer launched last (mi355_last_kernel)
inline thread_local const void *t_last_kernel = nullptr;
// NaN words for the next fold (mi355_nan_flag_next_launch), consumed by it
inline thread_local unsigned long long *t_nan_set = nullptr, *t_nan_clear = nullptr;

// A host-visible word the host can also write: an armed signal that no kernel
// will carry (nothing to launch) is fired right here, in stream order.
inline void fire_on_host(hipStream_t st) {
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
    t_last_kernel = (const void *)kernel;
    if (t_ev_start != nullptr || t_ev_stop != nullptr) {
        hipExtLaunchKernelGGL(kernel, grid, dim3(kBlock), 0, st, t_ev_start, t_ev_stop, 0, p);
        t_ev_start = t_ev_stop = nullptr;
    } else {
        hipLaunchKernelGGL(kernel, grid, dim3(kBlock), 0, st, p);
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

inline int device_cus() {
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

// Blocks of `fn` one CU holds at once (occupancy API, cached per kernel).
// A grid-stride launch larger than what is resident runs in rounds, the last
// one partly empty. The VALU-bound x87 folds cap their grids at this (the
// every-member x87 sum at 8 sources: 80 VGPRs, 6 blocks per CU instead of
// the 8 asked: 271 -> 263 us at 8 x 32 MiB, profiles/r03/orders_grid_cap.jsonl).
// The HBM-bound folds do not: capped at their residency (the 8-source fold
// holds 152 VGPRs, 3 blocks per CU) they ran 1-4 % slower -- the queued
// blocks refill CUs as others finish.
// Several host threads may launch folds (the launch state is per thread):
// readers see an entry only once its key and value are written (release /
// acquire on `used`), writers append under a mutex.
inline int resident_blocks(const void *fn) {
    static const void *keys[512];
    static int vals[512];
    static std::atomic<int> used{0};
    static std::mutex mu;
    const int seen = used.load(std::memory_order_acquire);
    for (int i = 0; i < seen; ++i)
        if (keys[i] == fn) return vals[i];
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, kBlock, 0) != hipSuccess || n < 1) n = 1;
    (void)hipGetLastError();
    std::lock_guard<std::mutex> lock(mu);
    const int u = used.load(std::memory_order_relaxed);
    for (int i = seen; i < u; ++i)
        if (keys[i] == fn) return vals[i];  // another thread added it meanwhile
    if (u < 512) {
        keys[u] = fn;
        vals[u] = n;
        used.store(u + 1, std::memory_order_release);
    }
    return n;
}

inline unsigned grid_for(uint64_t units_per_block_pass, uint64_t units, int blocks_per_cu = kBlocksPerCU) {
    uint64_t want = (units + units_per_block_pass - 1) / units_per_block_pass;
    uint64_t cap = (uint64_t)device_cus() * blocks_per_cu;
    if (want < 1) want = 1;
    return (unsigned)(want < cap ? want : cap);
}

// Launch shape per source count, from tools/probes/hbm_sweep.hip and
// tools/probes/fold_bench.py on MI355X (256 MiB per source, double sums,
// non-temporal loads + `nt sc1` stores at the time; the folds store `sc1`
// since round 2, see st16_fold; GB/s counts (k+1) x 256 MiB;
// profiles/r01/hbm_sweep_v5.txt, fold_bench_k_sources.jsonl):
//   k=2: 1 vector/lane,  2 blocks/CU     6.4 TB/s
//   k=3: 2 vectors/lane, 1 block/CU      6.5 TB/s
//   k=4: 1 vector/lane,  1 block/CU      6.2-6.3 TB/s
//   k=8: 4 vectors/lane, 8 blocks/CU     5.8-5.9 TB/s (k=5..7 take k=8's
//        depth at half the blocks)
// Box-to-box spread is +-3 %, so neighbours within that band are ties.
// Long double is VALU-bound (x87 arithmetic in software): it wants many
// waves to hide ALU latency, not deep per-lane load queues. Round 5
// (tools/probes/cold_probe k2types, 256 MiB): the float two-source fold at 4 blocks
// per CU, 115 vs 122 us (its NaN checks cover four lanes per vector); the
// float complex product's at 8 (ShapeOp), 131 vs 162 us -- its sum is faster
// at 2 (120 vs 123 us), so that one is per operator.
template <int NSRC, typename T> struct Shape {
    static constexpr bool alu_heavy = std::is_same<T, x80>::value;
    static constexpr int unroll =
        alu_heavy ? 1 : NSRC == 2 ? 1 : NSRC == 3 ? 2 : NSRC == 4 ? 1 : NSRC < 8 ? 2 : 4;
    static constexpr int blocks_per_cu =
        alu_heavy ? 8 : NSRC == 2 ? (std::is_same<T, float>::value ? 4 : 2) : NSRC == 3 ? 1 : NSRC == 4 ? 1 : NSRC < 8 ? 4 : 8;
    static constexpr int policy = POL_NT_LOAD;
};

template <int OP, int NSRC, typename T> struct ShapeOp : Shape<NSRC, T> {
    static constexpr int blocks_per_cu =
        NSRC == 2 && std::is_same<T, cplxf>::value && OP == MI355_OP_PROD ? 8 : Shape<NSRC, T>::blocks_per_cu;
};

// mi355_combine_orders: NSRC loads and up to NSRC stores per vector (every
// member's fold); the loads in flight per lane are those of the fold of the
// same width. Complex types: one vector per lane (NSRC*(NSRC-1) complex
// products per vector do not fit the registers of deeper unrolling; the
// loads in flight come from more blocks instead).
// min/max at 8 sources: one vector per lane (the compare-select chains of
// every member's fold hold more registers than the adds; at four vectors per
// lane double min at 8 sources ran at 5.1 TB/s against 6.5 for the sum; float
// max 86.2 -> 82.7 us at two -> one, profiles/r02/orders_vs_fold_alu_shapes.jsonl).
// 3-4 sources of min/max or complex products: eight blocks per CU (alu4:
// float max 95.2 -> 81.2 us, complex double product 102.7 -> 80.7 at 4 x 64 MiB).
// 8 sources (every PE's shard at N = 8) of sums, products and bitwise
// operators on real and integer types: one vector per lane and one block per
// CU, as the 4-source fold and the copy -- the 8 loads and 8 stores per
// vector are 16 streams, and a small resident grid sweeping them in order
// keeps HBM's rows open: 8 x 32 MiB -> 8 from HBM 93.5 -> 90.3 us (double
// sum), 93.1 -> 89.8 (float sum), 93.1 -> 89.6 (double product); at 8 x 8
// MiB within +-2 % (profiles/r06/orders_window/; the k-source fold's shape,
// 4 vectors per lane at 8 blocks per CU, was tuned with one output). Min/max
// at 8 sources: two blocks per CU -- their per-member chains run whenever a
// vector holds a NaN or a zero, and one wave per SIMD does not hide those
// (doubles' bytes read as floats, 8 x 8 MiB: 20.7 -> 25.2 us warm at one
// block), two do: 8 x 8 MiB float max 20.7 -> 19.7 us warm with NaNs, 19.5
// -> 18.4 finite, cold within 1-3 %; 8 x 32 MiB cold 102.2 -> 95.9 with NaNs
// (profiles/r06/orders_window/minmax_*.jsonl).
template <int OP, int NSRC, typename T> struct OrdersShape {
    static constexpr bool cplx = std::is_same<T, cplxf>::value || std::is_same<T, cplxd>::value;
    static constexpr bool sel = (OP == MI355_OP_MIN || OP == MI355_OP_MAX) && NSRC >= 5;
    using S = Shape<NSRC, T>;
    static constexpr bool alu_heavy = S::alu_heavy;
    static constexpr bool stream8 = NSRC == 8 && !S::alu_heavy && !cplx && !sel;
    static constexpr bool sel8 = NSRC == 8 && !S::alu_heavy && sel;
    // 3-4 sources with compare-select chains or complex products: the sum's
    // shape there (one block per CU) leaves too few waves to hide their ALU
    // latency; eight blocks per CU
    static constexpr bool alu4 = !S::alu_heavy && NSRC >= 3 && NSRC <= 4 &&
                                 (OP == MI355_OP_MIN || OP == MI355_OP_MAX || (cplx && OP == MI355_OP_PROD));
    static constexpr int unroll = cplx || stream8 ? 1 : alu4 ? 2 : sel && S::unroll > 2 ? 1 : S::unroll;
    static constexpr int blocks_per_cu = alu4      ? 8
                                         : stream8 ? 1
                                         : sel8    ? 2
                                         : cplx    ? (S::blocks_per_cu * S::unroll < 8 ? S::blocks_per_cu * S::unroll : 8)
                                                   : S::blocks_per_cu;
    static constexpr int policy = POL_NT_LOAD;
};

// Elements to peel so that every output starts on a 128-byte line, when the
// outputs share their offset within one (the symmetric target on each PE)
// and n reaches past it; else so that they start on 16 bytes. Outputs off
// their line store partial lines at both ends of every wave's span: a fold
// or copy whose target sits 16 bytes off its line ran 3-25 % slower warm and
// up to 30 % slower from HBM (profiles/r05/cold/linepeel_*.jsonl). pd: the
// outputs' common phase within 16 bytes (a multiple of the element size).
// 16-byte elements: no head (the kernels fold a head only for V > 1).
template <typename T>
size_t line_head(const void *const *outs, int nout, uintptr_t pd, size_t n) {
    if (sizeof(T) >= 16) return 0;
    const uintptr_t pl = (uintptr_t)outs[0] & 127;
    bool line = true;
    for (int k = 1; k < nout; ++k) line = line && ((uintptr_t)outs[k] & 127) == pl;
    const size_t h = ((128 - pl) & 127) / sizeof(T);
    return line && n > h ? h : ((16 - pd) & 15) / sizeof(T);
}

// How a launch over these pointers can run as 16-byte vectors: h >= 0 =
// every pointer at one phase within 16 bytes, by whole elements (0 or a user
// offset into the arrays): fold the first h elements (line_head) element-wise
// and the rest as vectors from the advanced pointers; -1 = not vectorisable
// this way (shift_head below, else the element-wise kernel).
template <typename T>
long vector_head(const void *const *outs, int nout, const void *const *ins, int nin, size_t n) {
    constexpr int V = 16 / sizeof(T);
    const uintptr_t pd = (uintptr_t)(nout > 0 ? outs[0] : ins[0]) & 15;
    bool same = pd % sizeof(T) == 0;
    for (int k = 0; k < nout; ++k) same = same && ((uintptr_t)outs[k] & 15) == pd;
    for (int k = 0; k < nin; ++k) same = same && ((uintptr_t)ins[k] & 15) == pd;
    if (!same) return -1;
    if (V == 1 || nout == 0) return pd == 0 ? 0 : -1;
    const size_t head = line_head<T>(outs, nout, pd, n);
    if (head == 0 || n > head) return (long)head;
    return pd == 0 ? 0 : -1;
}

// Outputs 16-byte aligned after peeling whole elements and the sources at
// any phases, one or several (an offset into some of the arrays): the vector
// kernels with unaligned source loads (SHIFT; an unaligned-form load of an
// aligned address is the same instruction). Returns the elements to peel,
// or -1 (outputs at different phases or not element-aligned, no whole
// vector, long double). The aligned launch shapes (cold_probe unal: the
// same rates at 2 or 4 blocks per CU).
template <typename T>
long shift_head(const void *const *outs, int nout, const void *const *srcs, int nsrc, size_t n) {
    if constexpr (std::is_same<T, x80>::value) {
        return -1;
    } else {
        constexpr size_t es = sizeof(T);
        constexpr size_t V = 16 / es;
        const uintptr_t pd = (uintptr_t)outs[0] & 15;
        for (int k = 1; k < nout; ++k)
            if (((uintptr_t)outs[k] & 15) != pd) return -1;
        if (pd % es != 0) return -1;
        const size_t head = line_head<T>(outs, nout, pd, n);
        bool aligned = true;
        for (int k = 0; k < nsrc; ++k) aligned = aligned && (((uintptr_t)srcs[k] + head * es) & 15) == 0;
        if (aligned || n < head + V) return -1;
        return (long)head;
    }
}
template <int OP, typename T, int NSRC>
int launch_fixed(void *dst, const void *const *srcs, size_t n, hipStream_t st, bool final) {
    CombineParams p{};
    p.nan_set = t_nan_set;
    p.nan_clear = t_nan_clear;
    t_nan_set = t_nan_clear = nullptr;
    const void *ptrs[kMaxSrc + 1];
    p.dst = dst;
    ptrs[0] = dst;
    for (int k = 0; k < NSRC; ++k) p.src[k] = ptrs[1 + k] = srcs[k];
    constexpr int V = 16 / sizeof(T);
    const long head = vector_head<T>(&ptrs[0], 1, &ptrs[1], NSRC, n);
    if (head >= 0) {
        if (head > 0) {
            p.head = (uint32_t)head;
            p.dst = (char *)dst + head * sizeof(T);
            for (int k = 0; k < NSRC; ++k) p.src[k] = (const char *)srcs[k] + head * sizeof(T);
            n -= (size_t)head;
        }
        using S = ShapeOp<OP, NSRC, T>;
        p.nvec = n / V;
        p.tail = (uint32_t)(n % V);
        auto k = combine_vec<OP, T, NSRC, S::unroll, S::policy>;
        const int bpc = !S::alu_heavy || S::blocks_per_cu < resident_blocks((const void *)k)
                            ? S::blocks_per_cu
                            : resident_blocks((const void *)k);
        const unsigned grid = grid_for((uint64_t)kBlock * S::unroll, p.nvec, bpc);
        return launch(k, dim3(grid), st, p, final);
    }
    const long sh = shift_head<T>(&ptrs[0], 1, &ptrs[1], NSRC, n);
    if constexpr (!std::is_same<T, x80>::value) {
        if (sh >= 0) {
            p.head = (uint32_t)sh;
            p.dst = (char *)dst + sh * sizeof(T);
            for (int k = 0; k < NSRC; ++k) p.src[k] = (const char *)srcs[k] + sh * sizeof(T);
            n -= (size_t)sh;
            using S = ShapeOp<OP, NSRC, T>;
            p.nvec = n / V;
            p.tail = (uint32_t)(n % V);
            auto k = combine_vec<OP, T, NSRC, S::unroll, S::policy, true>;
            const unsigned grid = grid_for((uint64_t)kBlock * S::unroll, p.nvec, S::blocks_per_cu);
            return launch(k, dim3(grid), st, p, final);
        }
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
    const void *outs[kMaxSrc];
    int nout = 0;
    for (int k = 0; k < NSRC; ++k) {
        p.src[k] = srcs[k];
        p.dst[k] = dsts[k];
        if (dsts[k] != nullptr) outs[nout++] = dsts[k];
    }
    constexpr int V = 16 / sizeof(T);
    const long head = vector_head<T>(outs, nout, srcs, NSRC, n);
    if (head >= 0) {
        if (head > 0) {
            p.head = (uint32_t)head;
            for (int k = 0; k < NSRC; ++k) {
                p.src[k] = (const char *)srcs[k] + head * sizeof(T);
                if (dsts[k] != nullptr) p.dst[k] = (char *)dsts[k] + head * sizeof(T);
            }
            n -= (size_t)head;
        }
        using S = OrdersShape<OP, NSRC, T>;
        p.nvec = n / V;
        p.tail = (uint32_t)(n % V);
        bool all = true;
        for (int k = 0; k < NSRC; ++k) all = all && dsts[k] != nullptr;
        auto k = all ? combine_orders_vec<OP, T, NSRC, S::unroll, S::policy, true>
                     : combine_orders_vec<OP, T, NSRC, S::unroll, S::policy, false>;
        int bpc = !S::alu_heavy || S::blocks_per_cu < resident_blocks((const void *)k)
                      ? S::blocks_per_cu
                      : resident_blocks((const void *)k);
        // the measured ALU-heavy folds -- x87 sum/product, float complex
        // product (profiles/r04/alu_grid/) -- one vector per lane, every
        // block queued at once, so the hardware hands out the last round's
        // work as slots free instead of a resident grid's fixed rounds
        if ((S::alu_heavy && (OP == MI355_OP_SUM || OP == MI355_OP_PROD)) ||
            (std::is_same<T, cplxf>::value && OP == MI355_OP_PROD))
            bpc = 1 << 20;
        const unsigned grid = grid_for((uint64_t)kBlock * S::unroll, p.nvec, bpc);
        return launch(k, dim3(grid), st, p);
    }
    const long sh = nout > 0 ? shift_head<T>(outs, nout, srcs, NSRC, n) : -1;
    if constexpr (!std::is_same<T, x80>::value) {
        if (sh >= 0) {
            p.head = (uint32_t)sh;
            for (int k = 0; k < NSRC; ++k) {
                p.src[k] = (const char *)srcs[k] + sh * sizeof(T);
                if (dsts[k] != nullptr) p.dst[k] = (char *)dsts[k] + sh * sizeof(T);
            }
            n -= (size_t)sh;
            using S = OrdersShape<OP, NSRC, T>;
            p.nvec = n / V;
            p.tail = (uint32_t)(n % V);
            const bool all = nout == NSRC;
            auto k = all ? combine_orders_vec<OP, T, NSRC, S::unroll, S::policy, true, true>
                         : combine_orders_vec<OP, T, NSRC, S::unroll, S::policy, false, true>;
            const unsigned grid = grid_for((uint64_t)kBlock * S::unroll, p.nvec, S::blocks_per_cu);
            return launch(k, dim3(grid), st, p);
        }
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

// One element type's entry points, defined by combine_t_<name>.hip
#define MI355_COMBINE_TYPE(T, NAME)                                                                  \
    namespace mi355k {                                                                               \
    int combine_##NAME(int op, void *dst, const void *const *srcs, int nsrc, size_t n, hipStream_t st) { \
        return dispatch_op<T>(op, dst, srcs, nsrc, n, st);                                           \
    }                                                                                                \
    int orders_##NAME(int op, void *const *dsts, const void *const *srcs, int nsrc, size_t n,       \
                      hipStream_t st) {                                                              \
        return dispatch_orders<T>(op, dsts, srcs, nsrc, n, st);                                      \
    }                                                                                                \
    }
#define MI355_COMBINE_DECL(NAME)                                                                     \
    int combine_##NAME(int op, void *dst, const void *const *srcs, int nsrc, size_t n, hipStream_t st); \
    int orders_##NAME(int op, void *const *dsts, const void *const *srcs, int nsrc, size_t n, hipStream_t st);
MI355_COMBINE_DECL(short)
MI355_COMBINE_DECL(int)
MI355_COMBINE_DECL(long)
MI355_COMBINE_DECL(float)
MI355_COMBINE_DECL(double)
MI355_COMBINE_DECL(longdouble)
MI355_COMBINE_DECL(complexf)
MI355_COMBINE_DECL(complexd)
#undef MI355_COMBINE_DECL

}  // namespace mi355k
