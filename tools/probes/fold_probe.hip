// fold_probe.hip -- what bounds the k-source fold (combine_vec, reduce-scatter
// kernel) on MI355X: source placement, store and load cache policy, launch
// shape, and the read-only ceiling of k concurrent streams (tuning tool, not
// part of the library). 256 MiB per source, double sum, HIP events, median of
// 7 launches.
//   build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/probes/fold_probe.hip -o tools/probes/fold_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
union P2 {
    u32x4 v;
    double e[2];
};

struct Srcs {
    const u32x4 *s[8];
};

enum { ST_NT_SC1 = 0, ST_NT = 1, ST_PLAIN = 2, ST_NONE = 3, ST_SC1 = 4, ST_BSC1 = 5 };

template <int ST>
__device__ __forceinline__ void store(u32x4 *p, u32x4 v) {
    if constexpr (ST == ST_NT_SC1)
        asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (ST == ST_SC1)
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (ST == ST_NT)
        __builtin_nontemporal_store(v, p);
    else if constexpr (ST == ST_PLAIN)
        *p = v;
    else if (v.x == 0x7ff80123u && v.y == 0x5u)  // never: keeps the loads alive
        *p = v;
}

// NT: 0 plain, 1 non-temporal, 2 system-coherent (two dwordx2 sc0 sc1, the
// fused kernel's loads of the members' buffers)
template <int NT>
__device__ __forceinline__ u32x4 load(const u32x4 *p) {
    if constexpr (NT == 2) {
        const unsigned long long *q = (const unsigned long long *)p;
        const unsigned long long lo = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const unsigned long long hi = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        u32x4 r;
        r.x = (unsigned)lo; r.y = (unsigned)(lo >> 32); r.z = (unsigned)hi; r.w = (unsigned)(hi >> 32);
        return r;
    } else if constexpr (NT) {
        return __builtin_nontemporal_load(p);
    } else {
        return *p;
    }
}

// grid-stride, U vectors per lane, all K*U loads before the adds (the library's combine_vec)
template <int K, int U, int ST, int NT>
__global__ __launch_bounds__(256) void fold_gs(Srcs in, u32x4 *d, size_t nvec) {
    const size_t step = (size_t)gridDim.x * 256 * U;
    for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < nvec; base += step) {
        P2 x[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * 256;
            if (i < nvec) {
#pragma unroll
                for (int k = 0; k < K; ++k) x[u][k].v = load<NT>(in.s[k] + i);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * 256;
            if (i < nvec) {
                P2 a = x[u][0];
#pragma unroll
                for (int k = 1; k < K; ++k) {
                    a.e[0] = a.e[0] + x[u][k].e[0];
                    a.e[1] = a.e[1] + x[u][k].e[1];
                }
                store<ST>(d + i, a.v);
            }
        }
    }
}

// Round 4: fold_gs with 16-byte loads issued as inline asm (global_load_dwordx4
// with the cache bits POL names), every load of a pass issued before the first
// wait. The compiler does not track an asm load's destination, so each loaded
// vector is tied to an explicit s_waitcnt through a "+v" operand: COUNTED = 0
// waits for vmcnt(0) once (the later waits are already satisfied); COUNTED = 1
// waits for each vector with vmcnt(loads issued after it), so the first
// sources' adds overlap the last loads (vmcnt retires in issue order on gfx9,
// and the previous pass's stores were issued before these loads). A partial
// last pass falls back to vmcnt(0).
enum { LD_SYS = 0, LD_NT = 1, LD_PLAIN = 2 };
template <int POL>
__device__ __forceinline__ u32x4 ld16_asm(const u32x4 *p) {
    u32x4 r;
    if constexpr (POL == LD_SYS)
        asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1" : "=v"(r) : "v"(p) : "memory");
    else if constexpr (POL == LD_NT)
        asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(r) : "v"(p) : "memory");
    else
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
    return r;
}
template <int N>
__device__ __forceinline__ void wait_vm(u32x4 &v) {
    asm volatile("s_waitcnt vmcnt(%1)" : "+v"(v) : "i"(N));
}
// group u's K vectors: load j = u*K + k has K*U-1-j loads and u stores (groups
// 0..u-1, stored since) issued after it
template <int K, int U, int UU, int KK>
__device__ __forceinline__ void wait_group(P2 (&x)[U][K]) {
    if constexpr (KK < K) {
        wait_vm<K * U - 1 - (UU * K + KK) + UU>(x[UU][KK].v);
        wait_group<K, U, UU, KK + 1>(x);
    }
}
template <int K, int U, int ST, int UU>
__device__ __forceinline__ void fold_counted(P2 (&x)[U][K], u32x4 *d, size_t base) {
    if constexpr (UU < U) {
        wait_group<K, U, UU, 0>(x);
        P2 a = x[UU][0];
#pragma unroll
        for (int k = 1; k < K; ++k) {
            a.e[0] = a.e[0] + x[UU][k].e[0];
            a.e[1] = a.e[1] + x[UU][k].e[1];
        }
        store<ST>(d + base + (size_t)UU * 256, a.v);
        fold_counted<K, U, ST, UU + 1>(x, d, base);
    }
}
template <int K, int U, int ST, int POL, int COUNTED>
__global__ __launch_bounds__(256) void fold_asm(Srcs in, u32x4 *d, size_t nvec) {
    const size_t step = (size_t)gridDim.x * 256 * U;
    for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < nvec; base += step) {
        P2 x[U][K];
        const bool full = base + (size_t)(U - 1) * 256 < nvec;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * 256;
            if (i < nvec) {
#pragma unroll
                for (int k = 0; k < K; ++k) x[u][k].v = ld16_asm<POL>(in.s[k] + i);
            }
        }
        if (COUNTED && full) {
            fold_counted<K, U, ST, 0>(x, d, base);
            continue;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < K; ++k) wait_vm<0>(x[u][k].v);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * 256;
            if (i < nvec) {
                P2 a = x[u][0];
#pragma unroll
                for (int k = 1; k < K; ++k) {
                    a.e[0] = a.e[0] + x[u][k].e[0];
                    a.e[1] = a.e[1] + x[u][k].e[1];
                }
                store<ST>(d + i, a.v);
            }
        }
    }
}

// as fold_gs, but full passes (all U vectors in range) run without per-vector
// range tests; only the last, partial pass is guarded
template <int K, int U, int ST, int NT>
__global__ __launch_bounds__(256) void fold_nog(Srcs in, u32x4 *d, size_t nvec) {
    const size_t step = (size_t)gridDim.x * 256 * U;
    size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    for (; base + (size_t)(U - 1) * 256 < nvec; base += step) {
        P2 x[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int k = 0; k < K; ++k) x[u][k].v = load<NT>(in.s[k] + base + (size_t)u * 256);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            P2 a = x[u][0];
#pragma unroll
            for (int k = 1; k < K; ++k) {
                a.e[0] = a.e[0] + x[u][k].e[0];
                a.e[1] = a.e[1] + x[u][k].e[1];
            }
            store<ST>(d + base + (size_t)u * 256, a.v);
        }
    }
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * 256;
        if (i < nvec) {
            P2 a;
            a.v = load<NT>(in.s[0] + i);
            for (int k = 1; k < K; ++k) {
                P2 b;
                b.v = load<NT>(in.s[k] + i);
                a.e[0] = a.e[0] + b.e[0];
                a.e[1] = a.e[1] + b.e[1];
            }
            store<ST>(d + i, a.v);
        }
    }
}

// as fold_gs, but the loads issued source-major: src0's U vectors, then src1's, ...
template <int K, int U, int ST, int NT>
__global__ __launch_bounds__(256) void fold_sm(Srcs in, u32x4 *d, size_t nvec) {
    const size_t step = (size_t)gridDim.x * 256 * U;
    for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < nvec; base += step) {
        P2 x[U][K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                size_t i = base + (size_t)u * 256;
                if (i < nvec) x[u][k].v = load<NT>(in.s[k] + i);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * 256;
            if (i < nvec) {
                P2 a = x[u][0];
#pragma unroll
                for (int k = 1; k < K; ++k) {
                    a.e[0] = a.e[0] + x[u][k].e[0];
                    a.e[1] = a.e[1] + x[u][k].e[1];
                }
                store<ST>(d + i, a.v);
            }
        }
    }
}

// each lane owns U CONSECUTIVE vectors (64 B per source per lane at U = 4): a wave covers 4 KiB per source
template <int K, int U, int ST, int NT>
__global__ __launch_bounds__(256) void fold_lane(Srcs in, u32x4 *d, size_t nvec) {
    const size_t step = (size_t)gridDim.x * 256 * U;
    for (size_t base = ((size_t)blockIdx.x * 256 + threadIdx.x) * U; base < nvec; base += step) {
        P2 x[U][K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (base + u < nvec) x[u][k].v = load<NT>(in.s[k] + base + u);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (base + u < nvec) {
                P2 a = x[u][0];
#pragma unroll
                for (int k = 1; k < K; ++k) {
                    a.e[0] = a.e[0] + x[u][k].e[0];
                    a.e[1] = a.e[1] + x[u][k].e[1];
                }
                store<ST>(d + base + u, a.v);
            }
        }
    }
}

// each block owns one contiguous range (chunk of `per` vectors), U vectors per lane per step
template <int K, int U, int ST, int NT>
__global__ __launch_bounds__(256) void fold_part(Srcs in, u32x4 *d, size_t nvec) {
    const size_t per = (nvec + gridDim.x - 1) / gridDim.x;
    const size_t lo = (size_t)blockIdx.x * per, hi = lo + per < nvec ? lo + per : nvec;
    for (size_t base = lo + threadIdx.x; base < hi; base += 256 * U) {
        P2 x[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * 256;
            if (i < hi) {
#pragma unroll
                for (int k = 0; k < K; ++k) x[u][k].v = load<NT>(in.s[k] + i);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * 256;
            if (i < hi) {
                P2 a = x[u][0];
#pragma unroll
                for (int k = 1; k < K; ++k) {
                    a.e[0] = a.e[0] + x[u][k].e[0];
                    a.e[1] = a.e[1] + x[u][k].e[1];
                }
                store<ST>(d + i, a.v);
            }
        }
    }
}

// software-pipelined: the next pass's K*U loads are issued BEFORE this pass's
// stores, so the wait for them (vmcnt counts loads and stores in issue order
// on gfx9) does not include the store acknowledgements
template <int K, int U, int ST, int NT>
__global__ __launch_bounds__(256) void fold_pipe(Srcs in, u32x4 *d, size_t nvec) {
    const size_t step = (size_t)gridDim.x * 256 * U;
    size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    if (base >= nvec) return;
    P2 x[U][K];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        size_t i = base + (size_t)u * 256;
        if (i < nvec) {
#pragma unroll
            for (int k = 0; k < K; ++k) x[u][k].v = load<NT>(in.s[k] + i);
        }
    }
    for (;;) {
        const size_t next = base + step;
        P2 y[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = next + (size_t)u * 256;
            if (i < nvec) {
#pragma unroll
                for (int k = 0; k < K; ++k) y[u][k].v = load<NT>(in.s[k] + i);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * 256;
            if (i < nvec) {
                P2 a = x[u][0];
#pragma unroll
                for (int k = 1; k < K; ++k) {
                    a.e[0] = a.e[0] + x[u][k].e[0];
                    a.e[1] = a.e[1] + x[u][k].e[1];
                }
                store<ST>(d + i, a.v);
            }
        }
        if (next >= nvec) break;
        base = next;
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < K; ++k) x[u][k] = y[u][k];
    }
}

// fold_pipe with block-uniform full passes: every load of a full pass is
// unconditional (no per-lane guards), the prefetch of pass i+1 is issued
// before the stores of pass i, and the last (partial) pass is guarded
template <int K, int U, int ST, int NT>
__device__ __forceinline__ void fold_store(const P2 (&x)[U][K], u32x4 *d, size_t base) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        P2 a = x[u][0];
#pragma unroll
        for (int k = 1; k < K; ++k) {
            a.e[0] = a.e[0] + x[u][k].e[0];
            a.e[1] = a.e[1] + x[u][k].e[1];
        }
        store<ST>(d + base + (size_t)u * 256, a.v);
    }
}
template <int K, int U, int ST, int NT>
__global__ __launch_bounds__(256) void fold_pipe2(Srcs in, u32x4 *d, size_t nvec) {
    const size_t step = (size_t)gridDim.x * 256 * U;
    size_t bb = (size_t)blockIdx.x * 256 * U;  // block-uniform
    const size_t t = threadIdx.x;
    if (bb + 256 * U <= nvec) {
        P2 x[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < K; ++k) x[u][k].v = load<NT>(in.s[k] + bb + t + (size_t)u * 256);
        while (bb + step + 256 * U <= nvec) {
            P2 y[U][K];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int k = 0; k < K; ++k) y[u][k].v = load<NT>(in.s[k] + bb + step + t + (size_t)u * 256);
            fold_store<K, U, ST, NT>(x, d, bb + t);
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int k = 0; k < K; ++k) x[u][k] = y[u][k];
            bb += step;
        }
        fold_store<K, U, ST, NT>(x, d, bb + t);
        bb += step;
    }
    // the partial pass (at most one per block)
    for (int u = 0; u < U; ++u) {
        const size_t i = bb + t + (size_t)u * 256;
        if (i < nvec) {
            P2 a;
            a.v = load<NT>(in.s[0] + i);
            for (int k = 1; k < K; ++k) {
                P2 b;
                b.v = load<NT>(in.s[k] + i);
                a.e[0] = a.e[0] + b.e[0];
                a.e[1] = a.e[1] + b.e[1];
            }
            store<ST>(d + i, a.v);
        }
    }
}

// ping-pong registers (no copies): prefetch pass i+1 into one set, then fold
// and store pass i from the other; the scheduling barrier keeps the prefetch
// ahead of the fold's waits. Every path into the loop header ends "loads of
// the held pass, then the previous pass's stores", so the compiler's vmcnt
// wait for the held pass leaves the stores (and the new prefetch) in flight.
template <int K, int U, int NT>
__device__ __forceinline__ void load_pass(P2 (&x)[U][K], const Srcs &in, size_t base) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int k = 0; k < K; ++k) x[u][k].v = load<NT>(in.s[k] + base + (size_t)u * 256);
    __builtin_amdgcn_sched_barrier(0);
}
template <int K, int U, int ST, int NT>
__global__ __launch_bounds__(256) void fold_pp(Srcs in, u32x4 *d, size_t nvec) {
    const size_t step = (size_t)gridDim.x * 256 * U;
    size_t bb = (size_t)blockIdx.x * 256 * U;
    const size_t t = threadIdx.x;
    auto full = [&](size_t b) { return b + 256 * U <= nvec; };
    if (full(bb)) {
        P2 x[U][K], y[U][K];
        load_pass<K, U, NT>(x, in, bb + t);
        if (full(bb + step)) {
            load_pass<K, U, NT>(y, in, bb + step + t);
            fold_store<K, U, ST, NT>(x, d, bb + t);
            bb += step;  // y holds bb
            for (;;) {
                if (!full(bb + step)) {
                    fold_store<K, U, ST, NT>(y, d, bb + t);
                    bb += step;
                    break;
                }
                load_pass<K, U, NT>(x, in, bb + step + t);
                fold_store<K, U, ST, NT>(y, d, bb + t);
                bb += step;  // x holds bb
                if (!full(bb + step)) {
                    fold_store<K, U, ST, NT>(x, d, bb + t);
                    bb += step;
                    break;
                }
                load_pass<K, U, NT>(y, in, bb + step + t);
                fold_store<K, U, ST, NT>(x, d, bb + t);
                bb += step;  // y holds bb
            }
        } else {
            fold_store<K, U, ST, NT>(x, d, bb + t);
            bb += step;
        }
    }
    for (int u = 0; u < U; ++u) {
        const size_t i = bb + t + (size_t)u * 256;
        if (i < nvec) {
            P2 a;
            a.v = load<NT>(in.s[0] + i);
            for (int k = 1; k < K; ++k) {
                P2 b;
                b.v = load<NT>(in.s[k] + i);
                a.e[0] = a.e[0] + b.e[0];
                a.e[1] = a.e[1] + b.e[1];
            }
            store<ST>(d + i, a.v);
        }
    }
}

// delayed stores: pass i's results stay in registers and are stored after
// pass i+1's loads are issued, so the wait for pass i+1's loads leaves them
// in flight (vmcnt retires loads and stores in issue order on gfx9: in
// fold_gs the wait for pass i+1 also waits for pass i's store
// acknowledgements). Full passes are block-uniform and unguarded.
template <int K, int U>
__device__ __forceinline__ void fold_regs(const P2 (&x)[U][K], P2 (&r)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        P2 a = x[u][0];
#pragma unroll
        for (int k = 1; k < K; ++k) {
            a.e[0] = a.e[0] + x[u][k].e[0];
            a.e[1] = a.e[1] + x[u][k].e[1];
        }
        r[u] = a;
    }
}
// two result sets used alternately (the loop unrolled by two): overwriting a
// result register that a store has not yet read would make the compiler wait
// for that store (vmcnt(0) per pass)
template <int K, int U, int ST, int NT>
__device__ __forceinline__ void ds_load(P2 (&x)[U][K], const Srcs &in, size_t base) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int k = 0; k < K; ++k) x[u][k].v = load<NT>(in.s[k] + base + (size_t)u * 256);
    __builtin_amdgcn_sched_barrier(0);
}
// ST_BSC1: `buffer_store_dwordx4 ... sc1` through the builtin (the compiler
// counts it in vmcnt; an inline-asm store it cannot see, so its waits for
// loads issued before such stores are vmcnt(0))
template <int U, int ST>
__device__ __forceinline__ void ds_store(const P2 (&r)[U], u32x4 *d, size_t base) {
    if constexpr (ST == ST_BSC1) {
        const size_t t = threadIdx.x;
        const size_t bbase = __builtin_amdgcn_readfirstlane((unsigned)((base - t) >> 8)) * (size_t)256;  // uniform
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(d + bbase, 0, (int)0xFFFFFFF0u, 0x00020000);
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(r[u].v, rs, (unsigned)((t + (size_t)u * 256) * 16), 0, 16);
        __builtin_amdgcn_sched_barrier(0);
    } else {
#pragma unroll
        for (int u = 0; u < U; ++u) store<ST>(d + base + (size_t)u * 256, r[u].v);
    }
}
template <int K, int U, int ST, int NT>
__global__ __launch_bounds__(256) void fold_ds(Srcs in, u32x4 *d, size_t nvec) {
    const size_t step = (size_t)gridDim.x * 256 * U;
    size_t bb = (size_t)blockIdx.x * 256 * U;
    const size_t t = threadIdx.x;
    auto full = [&](size_t b) { return b + 256 * U <= nvec; };
    if (full(bb)) {
        P2 x[U][K], r0[U], r1[U];
        ds_load<K, U, ST, NT>(x, in, bb + t);
        fold_regs<K, U>(x, r0);
        size_t rb = bb + t;
        bb += step;
        for (;;) {
            if (!full(bb)) { ds_store<U, ST>(r0, d, rb); break; }
            ds_load<K, U, ST, NT>(x, in, bb + t);
            ds_store<U, ST>(r0, d, rb);
            fold_regs<K, U>(x, r1);
            rb = bb + t;
            bb += step;
            if (!full(bb)) { ds_store<U, ST>(r1, d, rb); break; }
            ds_load<K, U, ST, NT>(x, in, bb + t);
            ds_store<U, ST>(r1, d, rb);
            fold_regs<K, U>(x, r0);
            rb = bb + t;
            bb += step;
        }
    }
    for (int u = 0; u < U; ++u) {
        const size_t i = bb + t + (size_t)u * 256;
        if (i < nvec) {
            P2 a;
            a.v = load<NT>(in.s[0] + i);
            for (int k = 1; k < K; ++k) {
                P2 b;
                b.v = load<NT>(in.s[k] + i);
                a.e[0] = a.e[0] + b.e[0];
                a.e[1] = a.e[1] + b.e[1];
            }
            store<ST == ST_BSC1 ? ST_SC1 : ST>(d + i, a.v);
        }
    }
}

template <typename F>
double time_us(F launch) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    launch();
    launch();
    CHECK(hipDeviceSynchronize());
    std::vector<double> ts;
    for (int r = 0; r < 7; ++r) {
        CHECK(hipEventRecord(a, 0));
        launch();
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms * 1e3);
    }
    std::sort(ts.begin(), ts.end());
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return ts[ts.size() / 2];
}

int main(int argc, char **argv) {
    const size_t bytes = 256ull << 20, nvec = bytes / 16;
    int cus = 256;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    // placement A: 8 separate allocations; B: one allocation, source k at k * (bytes + stagger)
    std::vector<void *> sep(8);
    for (int k = 0; k < 8; ++k) {
        CHECK(hipMalloc(&sep[k], bytes));
        CHECK(hipMemset(sep[k], 0x11 * (k + 1), bytes));
    }
    const size_t max_stagger = 8ull << 20;
    char *big;
    CHECK(hipMalloc(&big, 8 * (bytes + max_stagger)));
    CHECK(hipMemset(big, 0x22, 8 * (bytes + max_stagger)));
    u32x4 *d;
    CHECK(hipMalloc(&d, bytes + max_stagger));
    CHECK(hipMemset(d, 0, bytes + max_stagger));
    CHECK(hipDeviceSynchronize());
    printf("separate allocations at:");
    for (int k = 0; k < 8; ++k) printf(" %p", sep[k]);
    printf("\n");

    auto srcs_sep = [&]() { Srcs s{}; for (int k = 0; k < 8; ++k) s.s[k] = (const u32x4 *)sep[k]; return s; };
    auto srcs_stag = [&](size_t st) {
        Srcs s{};
        for (int k = 0; k < 8; ++k) s.s[k] = (const u32x4 *)(big + k * (bytes + st));
        return s;
    };
    auto rep = [&](const char *what, int k, double us) {
        printf("%-58s k=%d %8.2f us %6.0f GB/s (k+1)S  %6.0f GB/s reads\n", what, k, us,
               (k + 1.0) * bytes / us / 1e3, (double)k * bytes / us / 1e3);
        fflush(stdout);
    };
    char name[128];
#define RUN(KERNEL, K, U, ST, NT, BPC, SRCS, LABEL) do {                                            \
        Srcs s_ = (SRCS);                                                                           \
        snprintf(name, sizeof name, "%s<U%d,%s,%s> %d/CU %s", #KERNEL, U, #ST, NT == 2 ? "sys-ld" : NT ? "nt-ld" : "ld", \
                 BPC, LABEL);                                                                       \
        rep(name, K, time_us([&] { hipLaunchKernelGGL((KERNEL<K, U, ST, NT>), dim3(cus * BPC), dim3(256), 0, 0, \
                                                        s_, d, nvec); }));                          \
    } while (0)

    if (argc > 1 && argv[1][0] == 'p') {  // software-pipelined loads vs the library shape
        // correctness of the hand-scheduled kernel first: against fold_gs on distinct per-source data
        {
            Srcs s_ = srcs_sep();
            std::vector<double> h(nvec * 2);
            for (int k = 0; k < 8; ++k) {
                uint64_t z = 0x9E3779B97F4A7C15ull * (k + 1);
                for (auto &v : h) { z ^= z << 13; z ^= z >> 7; z ^= z << 17; v = (double)(int64_t)z * 0x1p-63; }
                CHECK(hipMemcpy(sep[k], h.data(), bytes, hipMemcpyHostToDevice));
            }
            u32x4 *d2;
            CHECK(hipMalloc(&d2, bytes));
            hipLaunchKernelGGL((fold_gs<8, 4, ST_SC1, 1>), dim3(cus * 8), dim3(256), 0, 0, s_, d, nvec);
            for (int bpc : {1, 2, 4, 8}) {
                CHECK(hipMemset(d2, 0xff, bytes));
                hipLaunchKernelGGL((fold_ds<8, 4, ST_BSC1, 1>), dim3(cus * bpc), dim3(256), 0, 0, s_, d2, nvec - 77);
                CHECK(hipDeviceSynchronize());
                std::vector<double> a(nvec * 2), b(nvec * 2);
                CHECK(hipMemcpy(a.data(), d, bytes, hipMemcpyDeviceToHost));
                CHECK(hipMemcpy(b.data(), d2, bytes, hipMemcpyDeviceToHost));
                size_t bad = 0;
                for (size_t i = 0; i < (nvec - 77) * 2; ++i) bad += memcmp(&a[i], &b[i], 8) != 0;
                printf("fold_ds<U4> %d/CU vs fold_gs: %zu mismatches of %zu\n", bpc, bad, (nvec - 77) * 2);
            }
            CHECK(hipFree(d2));
        }
        for (int r = 0; r < 3; ++r) {
            RUN(fold_gs, 8, 4, ST_SC1, 1, 8, srcs_sep(), "library shape");
            RUN(fold_ds, 8, 4, ST_SC1, 1, 8, srcs_sep(), "delayed stores (asm)");
            RUN(fold_ds, 8, 4, ST_BSC1, 1, 8, srcs_sep(), "delayed stores");
            RUN(fold_ds, 8, 4, ST_BSC1, 1, 4, srcs_sep(), "delayed stores");
            RUN(fold_ds, 8, 2, ST_BSC1, 1, 8, srcs_sep(), "delayed stores");
            RUN(fold_ds, 8, 2, ST_BSC1, 1, 4, srcs_sep(), "delayed stores");
            RUN(fold_ds, 8, 1, ST_BSC1, 1, 8, srcs_sep(), "delayed stores");
            RUN(fold_gs, 4, 1, ST_SC1, 1, 1, srcs_sep(), "library shape");
            RUN(fold_ds, 4, 1, ST_BSC1, 1, 1, srcs_sep(), "delayed stores");
            RUN(fold_ds, 4, 1, ST_BSC1, 1, 2, srcs_sep(), "delayed stores");
            RUN(fold_ds, 4, 2, ST_BSC1, 1, 2, srcs_sep(), "delayed stores");
            RUN(fold_gs, 2, 1, ST_SC1, 1, 2, srcs_sep(), "library shape");
            RUN(fold_ds, 2, 1, ST_BSC1, 1, 2, srcs_sep(), "delayed stores");
            RUN(fold_ds, 2, 2, ST_BSC1, 1, 2, srcs_sep(), "delayed stores");
            RUN(fold_ds, 2, 4, ST_BSC1, 1, 1, srcs_sep(), "delayed stores");
            RUN(fold_ds, 2, 1, ST_BSC1, 1, 4, srcs_sep(), "delayed stores");
            RUN(fold_gs, 1, 4, ST_NT_SC1, 0, 1, srcs_sep(), "copy, library-like");
            RUN(fold_ds, 1, 4, ST_BSC1, 0, 1, srcs_sep(), "copy, delayed stores");
            RUN(fold_ds, 1, 8, ST_BSC1, 0, 1, srcs_sep(), "copy, delayed stores");
            RUN(fold_ds, 1, 4, ST_BSC1, 0, 2, srcs_sep(), "copy, delayed stores");
            RUN(fold_pp, 8, 2, ST_SC1, 1, 8, srcs_sep(), "compiler-scheduled ping-pong");
            RUN(fold_pp, 8, 2, ST_SC1, 1, 4, srcs_sep(), "compiler-scheduled ping-pong");
            RUN(fold_gs, 8, 4, ST_NONE, 1, 8, srcs_sep(), "no store: read ceiling");
        }
        return 0;
    }
    if (argc > 1 && argv[1][0] == 's') {  // system-coherent loads (sc0 sc1) vs the library's load policies
        for (int r = 0; r < 3; ++r) {
            RUN(fold_gs, 8, 4, ST_SC1, 1, 8, srcs_sep(), "library shape k=8");
            RUN(fold_gs, 8, 4, ST_SC1, 2, 8, srcs_sep(), "k=8, system-coherent loads");
            RUN(fold_gs, 2, 1, ST_SC1, 1, 2, srcs_sep(), "library shape k=2");
            RUN(fold_gs, 2, 1, ST_SC1, 2, 2, srcs_sep(), "k=2, system-coherent loads");
            RUN(fold_gs, 2, 2, ST_SC1, 2, 2, srcs_sep(), "k=2, system-coherent loads");
            RUN(fold_gs, 1, 4, ST_NT_SC1, 0, 1, srcs_sep(), "copy, library-like");
            RUN(fold_gs, 1, 4, ST_NT_SC1, 2, 1, srcs_sep(), "copy, system-coherent loads");
            RUN(fold_gs, 1, 4, ST_NT_SC1, 2, 4, srcs_sep(), "copy, system-coherent loads");
        }
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'S') {  // round 4: 16-byte system-coherent loads (fold_asm) vs the library's
#define RUNA(K, U, ST, POL, C, BPC, LABEL) do {                                                     \
        Srcs s_ = srcs_sep();                                                                       \
        snprintf(name, sizeof name, "fold_asm<U%d,%s,%s,%s> %d/CU %s", U, #ST, #POL,                \
                 C ? "counted" : "vmcnt0", BPC, LABEL);                                             \
        rep(name, K, time_us([&] { hipLaunchKernelGGL((fold_asm<K, U, ST, POL, C>), dim3(cus * BPC), \
                                                        dim3(256), 0, 0, s_, d, nvec); }));         \
    } while (0)
        // correctness first: every asm variant against fold_gs (nt loads) on distinct per-source data,
        // over a length that leaves a partial last pass
        {
            Srcs s_ = srcs_sep();
            std::vector<double> h(nvec * 2);
            for (int k = 0; k < 8; ++k) {
                uint64_t z = 0x9E3779B97F4A7C15ull * (k + 3);
                for (auto &v : h) { z ^= z << 13; z ^= z >> 7; z ^= z << 17; v = (double)(int64_t)z * 0x1p-63; }
                CHECK(hipMemcpy(sep[k], h.data(), bytes, hipMemcpyHostToDevice));
            }
            u32x4 *d2;
            CHECK(hipMalloc(&d2, bytes));
            const size_t nv = nvec - 77;
            std::vector<double> a(nv * 2), b(nv * 2);
            auto check = [&](const char *what, auto launch_ref, auto launch) {
                CHECK(hipMemset(d, 0xff, bytes));
                CHECK(hipMemset(d2, 0xee, bytes));
                launch_ref();
                launch();
                CHECK(hipDeviceSynchronize());
                CHECK(hipMemcpy(a.data(), d, nv * 16, hipMemcpyDeviceToHost));
                CHECK(hipMemcpy(b.data(), d2, nv * 16, hipMemcpyDeviceToHost));
                size_t bad = 0;
                for (size_t i = 0; i < nv * 2; ++i) bad += memcmp(&a[i], &b[i], 8) != 0;
                printf("check %-40s vs fold_gs: %zu mismatches of %zu\n", what, bad, nv * 2);
                fflush(stdout);
            };
#define CHK(K, U, BPC, POL, C)                                                                                  \
            check(#K " " #U " " #POL " " #C,                                                                   \
                  [&] { hipLaunchKernelGGL((fold_gs<K, U, ST_SC1, 1>), dim3(cus * BPC), dim3(256), 0, 0, s_, d, nv); }, \
                  [&] { hipLaunchKernelGGL((fold_asm<K, U, ST_SC1, POL, C>), dim3(cus * BPC), dim3(256), 0, 0, s_, d2, nv); })
            CHK(8, 4, 8, LD_SYS, 0);
            CHK(8, 4, 8, LD_SYS, 1);
            CHK(2, 1, 2, LD_SYS, 0);
            CHK(2, 1, 2, LD_SYS, 1);
            CHK(2, 2, 2, LD_SYS, 1);
            CHK(1, 4, 1, LD_SYS, 1);
            CHK(8, 4, 8, LD_NT, 1);
            CHECK(hipFree(d2));
        }
        for (int r = 0; r < 3; ++r) {
            RUN(fold_gs, 8, 4, ST_SC1, 1, 8, srcs_sep(), "library shape k=8");
            RUNA(8, 4, ST_SC1, LD_NT, 0, 8, "k=8 asm nt loads");
            RUNA(8, 4, ST_SC1, LD_NT, 1, 8, "k=8 asm nt loads");
            RUNA(8, 4, ST_SC1, LD_SYS, 0, 8, "k=8 16-B system-coherent");
            RUNA(8, 4, ST_SC1, LD_SYS, 1, 8, "k=8 16-B system-coherent");
            RUNA(8, 2, ST_SC1, LD_SYS, 1, 8, "k=8 16-B system-coherent");
            RUN(fold_gs, 8, 4, ST_SC1, 2, 8, srcs_sep(), "k=8, 2x8-B system-coherent (r03)");
            RUN(fold_gs, 2, 1, ST_SC1, 1, 2, srcs_sep(), "library shape k=2");
            RUNA(2, 1, ST_SC1, LD_NT, 1, 2, "k=2 asm nt loads");
            RUNA(2, 1, ST_SC1, LD_SYS, 0, 2, "k=2 16-B system-coherent");
            RUNA(2, 1, ST_SC1, LD_SYS, 1, 2, "k=2 16-B system-coherent");
            RUNA(2, 2, ST_SC1, LD_SYS, 1, 2, "k=2 16-B system-coherent");
            RUN(fold_gs, 2, 1, ST_SC1, 2, 2, srcs_sep(), "k=2, 2x8-B system-coherent (r03)");
            RUN(fold_gs, 1, 4, ST_NT_SC1, 0, 1, srcs_sep(), "copy, library-like");
            RUNA(1, 4, ST_NT_SC1, LD_SYS, 1, 1, "copy 16-B system-coherent");
            RUNA(1, 4, ST_NT_SC1, LD_PLAIN, 1, 1, "copy asm plain loads");
        }
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'g') {  // unguarded full passes
        for (int r = 0; r < 2; ++r) {
            RUN(fold_gs, 8, 4, ST_SC1, 1, 8, srcs_sep(), "library shape");
            RUN(fold_nog, 8, 4, ST_SC1, 1, 8, srcs_sep(), "unguarded full passes");
            RUN(fold_nog, 8, 4, ST_SC1, 1, 4, srcs_sep(), "unguarded full passes");
            RUN(fold_nog, 8, 2, ST_SC1, 1, 8, srcs_sep(), "unguarded full passes");
            RUN(fold_gs, 3, 2, ST_SC1, 1, 1, srcs_sep(), "library shape");
            RUN(fold_nog, 3, 2, ST_SC1, 1, 1, srcs_sep(), "unguarded full passes");
            RUN(fold_nog, 3, 2, ST_SC1, 1, 2, srcs_sep(), "unguarded full passes");
            RUN(fold_gs, 2, 1, ST_SC1, 1, 2, srcs_sep(), "library shape");
            RUN(fold_nog, 2, 2, ST_SC1, 1, 2, srcs_sep(), "unguarded full passes");
            RUN(fold_nog, 2, 4, ST_SC1, 1, 1, srcs_sep(), "unguarded full passes");
            RUN(fold_nog, 2, 4, ST_SC1, 1, 2, srcs_sep(), "unguarded full passes");
            RUN(fold_gs, 1, 4, ST_NT_SC1, 0, 1, srcs_sep(), "copy, library-like");
            RUN(fold_nog, 1, 4, ST_NT_SC1, 0, 1, srcs_sep(), "copy, unguarded");
            RUN(fold_nog, 1, 4, ST_SC1, 1, 1, srcs_sep(), "copy, unguarded");
            RUN(fold_nog, 1, 8, ST_SC1, 1, 1, srcs_sep(), "copy, unguarded");
        }
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'o') {  // load order / lane layout at k = 8 and k = 2
        for (int r = 0; r < 2; ++r) {
            RUN(fold_gs, 8, 4, ST_SC1, 1, 8, srcs_sep(), "library shape");
            RUN(fold_sm, 8, 4, ST_SC1, 1, 8, srcs_sep(), "source-major loads");
            RUN(fold_sm, 8, 4, ST_SC1, 1, 4, srcs_sep(), "source-major loads");
            RUN(fold_sm, 8, 2, ST_SC1, 1, 8, srcs_sep(), "source-major loads");
            RUN(fold_lane, 8, 4, ST_SC1, 1, 4, srcs_sep(), "4 consecutive vectors per lane");
            RUN(fold_lane, 8, 2, ST_SC1, 1, 8, srcs_sep(), "2 consecutive vectors per lane");
            RUN(fold_lane, 8, 4, ST_SC1, 1, 8, srcs_sep(), "4 consecutive vectors per lane");
            RUN(fold_gs, 8, 4, ST_SC1, 1, 8, srcs_stag(0), "one arena");
            RUN(fold_sm, 8, 4, ST_SC1, 1, 8, srcs_stag(0), "one arena, source-major");
            RUN(fold_gs, 2, 1, ST_SC1, 1, 2, srcs_sep(), "library shape");
            RUN(fold_sm, 2, 2, ST_SC1, 1, 2, srcs_sep(), "source-major loads");
            RUN(fold_lane, 2, 2, ST_SC1, 1, 2, srcs_sep(), "2 consecutive vectors per lane");
            RUN(fold_lane, 2, 4, ST_SC1, 1, 1, srcs_sep(), "4 consecutive vectors per lane");
        }
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'c') {  // store policy of the copy and of the k = 2 / 4 / 8 folds
        for (int r = 0; r < 2; ++r) {
            RUN(fold_gs, 1, 4, ST_NT_SC1, 0, 1, srcs_sep(), "copy");
            RUN(fold_gs, 1, 4, ST_SC1, 0, 1, srcs_sep(), "copy");
            RUN(fold_gs, 1, 4, ST_NT, 0, 1, srcs_sep(), "copy");
            RUN(fold_gs, 1, 4, ST_SC1, 0, 2, srcs_sep(), "copy");
            RUN(fold_gs, 1, 4, ST_SC1, 1, 1, srcs_sep(), "copy");
            RUN(fold_gs, 2, 1, ST_SC1, 1, 2, srcs_sep(), "");
            RUN(fold_gs, 2, 2, ST_SC1, 1, 2, srcs_sep(), "");
            RUN(fold_gs, 2, 1, ST_SC1, 1, 4, srcs_sep(), "");
            RUN(fold_gs, 3, 2, ST_SC1, 1, 1, srcs_sep(), "");
            RUN(fold_gs, 3, 2, ST_NT_SC1, 1, 1, srcs_sep(), "");
            RUN(fold_gs, 4, 1, ST_SC1, 1, 1, srcs_sep(), "");
            RUN(fold_gs, 4, 1, ST_NT_SC1, 1, 1, srcs_sep(), "");
            RUN(fold_gs, 4, 2, ST_SC1, 1, 2, srcs_sep(), "");
            RUN(fold_gs, 8, 4, ST_SC1, 1, 8, srcs_sep(), "");
            RUN(fold_gs, 8, 4, ST_SC1, 1, 4, srcs_sep(), "");
        }
        return 0;
    }
    if (argc > 1) {  // placement/content study only
        std::vector<void *> sepg(8);
        for (int k = 0; k < 8; ++k) {
            CHECK(hipMalloc(&sepg[k], 1ull << 30));
            CHECK(hipMemset(sepg[k], 0x11 * (k + 1), 1ull << 30));
        }
        auto srcs_g = [&]() { Srcs s{}; for (int k = 0; k < 8; ++k) s.s[k] = (const u32x4 *)sepg[k]; return s; };
        auto srcs_stag_mixed = [&]() {
            Srcs s{};
            for (int k = 0; k < 8; ++k) {
                s.s[k] = (const u32x4 *)(big + k * bytes);
                CHECK(hipMemset(big + k * bytes, 0x11 * (k + 1), bytes));
            }
            return s;
        };
        for (int r = 0; r < 2; ++r) {
            RUN(fold_gs, 8, 4, ST_NT_SC1, 1, 8, srcs_sep(), "separate 256 MiB allocations");
            RUN(fold_gs, 8, 4, ST_NONE, 1, 8, srcs_sep(), "separate 256 MiB allocations (no store)");
            RUN(fold_gs, 8, 4, ST_NT_SC1, 1, 8, srcs_g(), "separate 1 GiB allocations");
            RUN(fold_gs, 8, 4, ST_NONE, 1, 8, srcs_g(), "separate 1 GiB allocations (no store)");
            RUN(fold_gs, 8, 4, ST_NT_SC1, 1, 8, srcs_stag_mixed(), "one allocation, per-source content");
            RUN(fold_gs, 8, 4, ST_NONE, 1, 8, srcs_stag_mixed(), "one allocation, per-source content (no store)");
            RUN(fold_gs, 8, 4, ST_SC1, 1, 8, srcs_stag_mixed(), "one allocation, per-source content");
            RUN(fold_gs, 8, 2, ST_SC1, 1, 8, srcs_stag_mixed(), "one allocation, per-source content");
            RUN(fold_gs, 8, 2, ST_SC1, 1, 4, srcs_stag_mixed(), "one allocation, per-source content");
            RUN(fold_gs, 8, 4, ST_SC1, 1, 4, srcs_stag_mixed(), "one allocation, per-source content");
            RUN(fold_gs, 8, 4, ST_NT_SC1, 0, 8, srcs_stag_mixed(), "one allocation, per-source content");
            RUN(fold_gs, 8, 4, ST_SC1, 0, 8, srcs_stag_mixed(), "one allocation, per-source content");
            RUN(fold_gs, 2, 1, ST_SC1, 1, 2, srcs_stag_mixed(), "one allocation, per-source content");
            RUN(fold_gs, 2, 1, ST_NT_SC1, 1, 2, srcs_stag_mixed(), "one allocation, per-source content");
            RUN(fold_gs, 2, 1, ST_NT, 1, 2, srcs_stag_mixed(), "one allocation, per-source content");
        }
        return 0;
    }
    for (int r = 0; r < 2; ++r) {
        printf("--- pass %d\n", r);
        // the library's k=8 shape on separate allocations, then read-only ceilings
        RUN(fold_gs, 8, 4, ST_NT_SC1, 1, 8, srcs_sep(), "separate");
        RUN(fold_gs, 8, 4, ST_NONE, 1, 8, srcs_sep(), "separate (no store: read ceiling)");
        RUN(fold_gs, 1, 4, ST_NONE, 1, 8, srcs_sep(), "separate (no store: read ceiling)");
        RUN(fold_gs, 2, 4, ST_NONE, 1, 8, srcs_sep(), "separate (no store: read ceiling)");
        RUN(fold_gs, 4, 4, ST_NONE, 1, 8, srcs_sep(), "separate (no store: read ceiling)");
        // placement
        for (size_t st : {(size_t)0, (size_t)4096, (size_t)(68 << 10), (size_t)(1 << 20) + 4096,
                          (size_t)(4 << 20) + 12288}) {
            char lab[64];
            snprintf(lab, sizeof lab, "stagger %zu B", st);
            RUN(fold_gs, 8, 4, ST_NT_SC1, 1, 8, srcs_stag(st), lab);
            RUN(fold_gs, 8, 4, ST_NONE, 1, 8, srcs_stag(st), lab);
        }
        // store policy
        RUN(fold_gs, 8, 4, ST_NT, 1, 8, srcs_sep(), "separate");
        RUN(fold_gs, 8, 4, ST_PLAIN, 1, 8, srcs_sep(), "separate");
        RUN(fold_gs, 8, 4, ST_SC1, 1, 8, srcs_sep(), "separate");
        // load policy
        RUN(fold_gs, 8, 4, ST_NT_SC1, 0, 8, srcs_sep(), "separate");
        // shapes
        RUN(fold_gs, 8, 2, ST_NT_SC1, 1, 4, srcs_sep(), "separate");
        RUN(fold_gs, 8, 2, ST_NT_SC1, 1, 8, srcs_sep(), "separate");
        RUN(fold_gs, 8, 1, ST_NT_SC1, 1, 8, srcs_sep(), "separate");
        RUN(fold_gs, 8, 1, ST_NT_SC1, 1, 4, srcs_sep(), "separate");
        RUN(fold_part, 8, 1, ST_NT_SC1, 1, 2, srcs_sep(), "separate");
        RUN(fold_part, 8, 2, ST_NT_SC1, 1, 2, srcs_sep(), "separate");
        RUN(fold_part, 8, 1, ST_NT_SC1, 1, 4, srcs_sep(), "separate");
        RUN(fold_part, 8, 2, ST_NT_SC1, 1, 4, srcs_sep(), "separate");
        RUN(fold_part, 8, 4, ST_NT_SC1, 1, 4, srcs_sep(), "separate");
        // k = 2 for reference
        RUN(fold_gs, 2, 1, ST_NT_SC1, 1, 2, srcs_sep(), "separate");
        RUN(fold_gs, 2, 1, ST_NT, 1, 2, srcs_sep(), "separate");
        RUN(fold_gs, 2, 1, ST_NONE, 1, 2, srcs_sep(), "separate (no store)");
        RUN(fold_part, 2, 2, ST_NT_SC1, 1, 2, srcs_sep(), "separate");
        RUN(fold_part, 2, 4, ST_NT_SC1, 1, 1, srcs_sep(), "separate");
    }
    return 0;
}
