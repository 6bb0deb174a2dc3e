// cold_probe.hip -- warm vs cold (rotating-footprint) rates of the reduction
// path's streaming kernels (tuning tool, not part of the library).
//
// Why: every earlier HBM probe ran at 256 MiB per buffer, the size of the
// Infinity Cache (MI355X_MICROARCH.md: a line stays resident only while the
// traffic between two uses of it fits in ~256 MiB), and FETCH_SIZE counts
// Infinity-Cache hits, so a warm figure alone cannot say "HBM".
//   warm    the same buffer set every launch (what a benchmark loop does)
//   rotate  R disjoint buffer sets taken in turn, R chosen so that the
//           footprint is >= 2 GiB (8x the Infinity Cache): between two uses
//           of a line, >= 1.75 GiB of other traffic went by
// Kernels: the library's own (through its C ABI: mi355_copy_segments,
// mi355_combine, mi355_combine_orders -- the product code objects) and, for
// the copy, variants of its loop compiled here (load / store policy, blocks
// per CU, vectors per lane).
//
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -I include -I osss-gasnet_amd/csrc tools/probes/cold_probe.hip \
//          -L osss-gasnet_amd/lib -lshmem_reduce -Wl,-rpath,$PWD/osss-gasnet_amd/lib -o tools/probes/cold_probe
// run:   tools/probes/cold_probe [lib|copy|all|copy2|orders]   (one JSON line per measurement)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#include "mi355_reduce.h"
#include "combine_kernels.h"   // the library's fold kernels, instantiated here at other launch shapes

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

static constexpr size_t MiB = 1ull << 20;
static constexpr size_t kFootprint = 2304 * MiB;   // >= 2 GiB + one set

// ---- copy variants (the library's copy_segments<4,1> loop, policies varied)
enum { LD_PLAIN = 0, LD_NT = 1 };
enum { ST_NT_SC1 = 0, ST_PLAIN = 1, ST_NT = 2, ST_SC1 = 3 };

template <int LD>
__device__ __forceinline__ u32x4 ld(const u32x4 *p) {
    if constexpr (LD == LD_NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <int ST>
__device__ __forceinline__ void st(u32x4 *p, u32x4 v) {
    if constexpr (ST == ST_NT_SC1) asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (ST == ST_SC1) asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (ST == ST_NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <int U, int LD, int ST>
__global__ __launch_bounds__(256) void copy_pipe(const u32x4 *s, u32x4 *d, uint64_t nvec) {
    const uint64_t step = (uint64_t)gridDim.x * 256 * U;
    uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x;
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t i = base + (uint64_t)u * 256;
        if (i < nvec) x[u] = ld<LD>(s + i);
    }
    while (base < nvec) {
        const uint64_t next = base + step;
        u32x4 y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = next + (uint64_t)u * 256;
            if (i < nvec) y[u] = ld<LD>(s + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = base + (uint64_t)u * 256;
            if (i < nvec) st<ST>(d + i, x[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = y[u];
        base = next;
    }
}

// each block copies one contiguous chunk of the buffer (the placement that
// keeps a block's DRAM pages together), same pipelined inner loop
template <int U, int LD, int ST>
__global__ __launch_bounds__(256) void copy_chunk(const u32x4 *s, u32x4 *d, uint64_t nvec) {
    const uint64_t per = (nvec + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = (uint64_t)blockIdx.x * per;
    const uint64_t hi = lo + per < nvec ? lo + per : nvec;
    for (uint64_t base = lo + threadIdx.x; base < hi; base += 256 * U) {
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = base + (uint64_t)u * 256;
            if (i < hi) x[u] = ld<LD>(s + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = base + (uint64_t)u * 256;
            if (i < hi) st<ST>(d + i, x[u]);
        }
    }
}

// ---- every-member fold variants (the library's combine_orders_vec for a
// double sum at 8 sources: member q's chain is src q, then the others in
// member order; 8 loads and 8 stores per vector)
template <int U, int LD, int ST>
__global__ __launch_bounds__(256) void orders8(const u32x4 *s0, const u32x4 *s1, const u32x4 *s2, const u32x4 *s3,
                                               const u32x4 *s4, const u32x4 *s5, const u32x4 *s6, const u32x4 *s7,
                                               u32x4 *d0, u32x4 *d1, u32x4 *d2, u32x4 *d3, u32x4 *d4, u32x4 *d5,
                                               u32x4 *d6, u32x4 *d7, uint64_t nvec) {
    const u32x4 *s[8] = {s0, s1, s2, s3, s4, s5, s6, s7};
    u32x4 *d[8] = {d0, d1, d2, d3, d4, d5, d6, d7};
    typedef double f64x2 __attribute__((ext_vector_type(2)));
    const uint64_t step = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; base < nvec; base += step) {
        u32x4 x[U][8];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = base + (uint64_t)u * 256;
            if (i < nvec)
#pragma unroll
                for (int k = 0; k < 8; ++k) x[u][k] = ld<LD>(s[k] + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = base + (uint64_t)u * 256;
            if (i >= nvec) continue;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                f64x2 acc = __builtin_bit_cast(f64x2, x[u][q]);
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if (k != q) acc += __builtin_bit_cast(f64x2, x[u][k]);
                st<ST>(d[q] + i, __builtin_bit_cast(u32x4, acc));
            }
        }
    }
}


// ---- realigning copy / fold prototypes (target 16-byte aligned, sources at
// another phase delta): output vector i = bytes [delta, delta + 16) of the
// source's aligned vectors A_i : A_(i+1). MODE 0: each lane loads both;
// MODE 1: A_(i+1) from the next lane (__shfl_down), lane 63 loads its own.
__device__ __forceinline__ u32x4 funnel(u32x4 a, u32x4 b, unsigned q, unsigned r) {
    unsigned w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    u32x4 o;
    // q uniform: selects, no register-array indexing
    unsigned lo0 = q == 0 ? w[0] : q == 1 ? w[1] : q == 2 ? w[2] : w[3];
    unsigned lo1 = q == 0 ? w[1] : q == 1 ? w[2] : q == 2 ? w[3] : w[4];
    unsigned lo2 = q == 0 ? w[2] : q == 1 ? w[3] : q == 2 ? w[4] : w[5];
    unsigned lo3 = q == 0 ? w[3] : q == 1 ? w[4] : q == 2 ? w[5] : w[6];
    unsigned lo4 = q == 0 ? w[4] : q == 1 ? w[5] : q == 2 ? w[6] : w[7];
    o.x = __builtin_amdgcn_alignbyte(lo1, lo0, r);
    o.y = __builtin_amdgcn_alignbyte(lo2, lo1, r);
    o.z = __builtin_amdgcn_alignbyte(lo3, lo2, r);
    o.w = __builtin_amdgcn_alignbyte(lo4, lo3, r);
    return o;
}
__device__ __forceinline__ u32x4 shfl_next(u32x4 v) {
    u32x4 o;
    o.x = __shfl_down((int)v.x, 1);
    o.y = __shfl_down((int)v.y, 1);
    o.z = __shfl_down((int)v.z, 1);
    o.w = __shfl_down((int)v.w, 1);
    return o;
}
// A_(i+1) from the next lane with a DPP wave shift (wave_shl:1: lane l reads
// lane l + 1; lane 63 keeps `old`, here its own load of A_(i+1))
__device__ __forceinline__ u32x4 dpp_next(u32x4 v, u32x4 old) {
    u32x4 o;
    o.x = (unsigned)__builtin_amdgcn_update_dpp((int)old.x, (int)v.x, 0x130, 0xF, 0xF, false);
    o.y = (unsigned)__builtin_amdgcn_update_dpp((int)old.y, (int)v.y, 0x130, 0xF, 0xF, false);
    o.z = (unsigned)__builtin_amdgcn_update_dpp((int)old.z, (int)v.z, 0x130, 0xF, 0xF, false);
    o.w = (unsigned)__builtin_amdgcn_update_dpp((int)old.w, (int)v.w, 0x130, 0xF, 0xF, false);
    return o;
}
template <int LD>
__global__ __launch_bounds__(256) void fold2_dpp(const u32x4 *sa0, const u32x4 *sa1, u32x4 *d, uint64_t nvec,
                                                 unsigned delta) {
    typedef double f64x2 __attribute__((ext_vector_type(2)));
    const unsigned q = delta >> 2, r = delta & 3;
    const bool last = (threadIdx.x & 63) == 63;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i - (threadIdx.x & 63) < nvec;
         i += (uint64_t)gridDim.x * 256) {
        const uint64_t ic = i < nvec ? i : nvec - 1;
        u32x4 a0 = ld<LD>(sa0 + ic), a1 = ld<LD>(sa1 + ic), o0 = {0, 0, 0, 0}, o1 = {0, 0, 0, 0};
        if (last) {
            o0 = ld<LD>(sa0 + ic + 1);
            o1 = ld<LD>(sa1 + ic + 1);
        }
        const u32x4 b0 = dpp_next(a0, o0), b1 = dpp_next(a1, o1);
        if (i < nvec) {
            f64x2 x = __builtin_bit_cast(f64x2, funnel(a0, b0, q, r)) + __builtin_bit_cast(f64x2, funnel(a1, b1, q, r));
            st<ST_SC1>(d + i, __builtin_bit_cast(u32x4, x));
        }
    }
}
template <int LD>
__global__ __launch_bounds__(256) void copy_dpp(const u32x4 *sa, u32x4 *d, uint64_t nvec, unsigned delta) {
    const unsigned q = delta >> 2, r = delta & 3;
    const bool last = (threadIdx.x & 63) == 63;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i - (threadIdx.x & 63) < nvec;
         i += (uint64_t)gridDim.x * 256) {
        const uint64_t ic = i < nvec ? i : nvec - 1;
        u32x4 a = ld<LD>(sa + ic), o = {0, 0, 0, 0};
        if (last) o = ld<LD>(sa + ic + 1);
        const u32x4 b = dpp_next(a, o);
        if (i < nvec) st<ST_NT_SC1>(d + i, funnel(a, b, q, r));
    }
}
// misaligned dwordx4: loads straight from a 4-byte-aligned (not 16) address,
// relying on the hardware's unaligned access mode
__global__ __launch_bounds__(256) void fold2_unal(const char *s0, const char *s1, u32x4 *d, uint64_t nvec) {
    typedef double f64x2 __attribute__((ext_vector_type(2)));
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (uint64_t)gridDim.x * 256) {
        const u32x4 a = __builtin_nontemporal_load((const u32x4 *)(s0 + 16 * i));
        const u32x4 b = __builtin_nontemporal_load((const u32x4 *)(s1 + 16 * i));
        f64x2 x = __builtin_bit_cast(f64x2, a) + __builtin_bit_cast(f64x2, b);
        st<ST_SC1>(d + i, __builtin_bit_cast(u32x4, x));
    }
}
__global__ __launch_bounds__(256) void copy_unal(const char *s, u32x4 *d, uint64_t nvec) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (uint64_t)gridDim.x * 256)
        st<ST_NT_SC1>(d + i, *(const u32x4 *)(s + 16 * i));
}
// copy_segments_shift's loop (pipelined, U vectors per lane) on unaligned sources
template <int U, bool PIPE>
__global__ __launch_bounds__(256) void copy_unal_u(const char *src, u32x4 *d, uint64_t nvec) {
    const mi355k::u32x4_any *s = (const mi355k::u32x4_any *)src;
    const uint64_t step = (uint64_t)gridDim.x * 256 * U;
    uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x;
    if constexpr (PIPE) {
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = base + (uint64_t)u * 256;
            if (i < nvec) x[u] = s[i];
        }
        while (base < nvec) {
            const uint64_t next = base + step;
            u32x4 y[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t i = next + (uint64_t)u * 256;
                if (i < nvec) y[u] = s[i];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t i = base + (uint64_t)u * 256;
                if (i < nvec) st<ST_NT_SC1>(d + i, x[u]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) x[u] = y[u];
            base = next;
        }
    } else {
        for (; base < nvec; base += step) {
            u32x4 x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t i = base + (uint64_t)u * 256;
                if (i < nvec) x[u] = s[i];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t i = base + (uint64_t)u * 256;
                if (i < nvec) st<ST_NT_SC1>(d + i, x[u]);
            }
        }
    }
}
// sa: the source's aligned base (source - delta); nvec output vectors; every
// lane of a wave active for the shuffle (lanes past the end load a clamped index)
template <int U, int MODE, int LD, int ST>
__global__ __launch_bounds__(256) void copy_shift(const u32x4 *sa, u32x4 *d, uint64_t nvec, unsigned delta) {
    const unsigned q = delta >> 2, r = delta & 3;
    const uint64_t step = (uint64_t)gridDim.x * 256 * U;
    const bool last = (threadIdx.x & 63) == 63;
    for (uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; base - (threadIdx.x & 63) < nvec; base += step) {
        u32x4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = base + (uint64_t)u * 256;
            const uint64_t ic = i < nvec ? i : nvec - 1;
            a[u] = ld<LD>(sa + ic);
            if (MODE == 0) b[u] = ld<LD>(sa + ic + 1);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (MODE == 1) {
                b[u] = shfl_next(a[u]);
                const uint64_t i = base + (uint64_t)u * 256;
                if (last && i < nvec) b[u] = ld<LD>(sa + i + 1);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = base + (uint64_t)u * 256;
            if (i < nvec) st<ST>(d + i, funnel(a[u], b[u], q, r));
        }
    }
}
template <int MODE, int LDA = LD_NT, int LDB = LD_NT, int U = 1>
__global__ __launch_bounds__(256) void fold2_shift(const u32x4 *sa0, const u32x4 *sa1, u32x4 *d, uint64_t nvec,
                                                   unsigned delta) {
    typedef double f64x2 __attribute__((ext_vector_type(2)));
    const unsigned q = delta >> 2, r = delta & 3;
    const bool last = (threadIdx.x & 63) == 63;
    const uint64_t step = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; base - (threadIdx.x & 63) < nvec; base += step) {
        u32x4 a0[U], a1[U], b0[U], b1[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = base + (uint64_t)u * 256;
            const uint64_t ic = i < nvec ? i : nvec - 1;
            a0[u] = ld<LDA>(sa0 + ic);
            a1[u] = ld<LDA>(sa1 + ic);
            if (MODE == 0) {
                b0[u] = ld<LDB>(sa0 + ic + 1);
                b1[u] = ld<LDB>(sa1 + ic + 1);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = base + (uint64_t)u * 256;
            if (MODE == 1) {
                b0[u] = shfl_next(a0[u]);
                b1[u] = shfl_next(a1[u]);
                if (last && i < nvec) {
                    b0[u] = ld<LDB>(sa0 + i + 1);
                    b1[u] = ld<LDB>(sa1 + i + 1);
                }
            }
            if (i < nvec) {
                f64x2 x = __builtin_bit_cast(f64x2, funnel(a0[u], b0[u], q, r)) +
                          __builtin_bit_cast(f64x2, funnel(a1[u], b1[u], q, r));
                st<ST_SC1>(d + i, __builtin_bit_cast(u32x4, x));
            }
        }
    }
}

// ---- timing
static hipEvent_t g_a, g_b;
static int g_cus = 256;

struct Stat { double med_us, mean_us; };

// launch(set) for set = 0..nsets-1 in turn; warm = always set 0
static Stat timed(const std::function<void(int)> &launch, int nsets, bool rotate, int reps) {
    for (int i = 0; i < (rotate ? nsets : 3); ++i) launch(rotate ? i % nsets : 0);
    CHECK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
        const int s = rotate ? r % nsets : 0;
        CHECK(hipEventRecord(g_a, 0));
        launch(s);
        CHECK(hipEventRecord(g_b, 0));
        CHECK(hipEventSynchronize(g_b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, g_a, g_b));
        t.push_back(ms * 1e3f);
    }
    std::vector<float> s = t;
    std::sort(s.begin(), s.end());
    double sum = 0;
    for (float x : t) sum += x;
    return {s[s.size() / 2], sum / t.size()};
}

// with the library's own event stamps (mi355_time_next_launch): the kernel's
// duration, no marker packets
static Stat timed_lib(const std::function<void(int)> &launch, int nsets, bool rotate, int reps) {
    for (int i = 0; i < (rotate ? nsets : 3); ++i) launch(rotate ? i % nsets : 0);
    CHECK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
        const int s = rotate ? r % nsets : 0;
        mi355_time_next_launch(g_a, g_b);
        launch(s);
        CHECK(hipEventSynchronize(g_b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, g_a, g_b));
        t.push_back(ms * 1e3f);
    }
    std::vector<float> s = t;
    std::sort(s.begin(), s.end());
    double sum = 0;
    for (float x : t) sum += x;
    return {s[s.size() / 2], sum / t.size()};
}

static char *g_pool;
static size_t g_pool_bytes;
static size_t g_skew;      // extra bytes between consecutive buffers (orders_skew)
static int g_skew_from;    // ... from buffer index g_skew_from on
static size_t g_dst_mis;   // bytes added to every output pointer (misaligned-target probe)
static size_t g_src_mis;   // ... to every source pointer (linepeel)

static void emit(const char *kernel, const char *variant, size_t alg, int nsets, Stat w, Stat c) {
    printf("{\"kernel\": \"%s\", \"variant\": \"%s\", \"alg_bytes\": %zu, \"sets\": %d, \"footprint_MiB\": %zu, "
           "\"warm_us\": %.2f, \"warm_mean_us\": %.2f, \"warm_TB_s\": %.3f, \"cold_us\": %.2f, \"cold_mean_us\": %.2f, "
           "\"cold_TB_s\": %.3f, \"cold_frac\": %.4f, \"warm_frac\": %.4f}\n",
           kernel, variant, alg, nsets, nsets * alg / MiB, w.med_us, w.mean_us, alg / (w.mean_us * 1e-6) / 1e12,
           c.med_us, c.mean_us, alg / (c.mean_us * 1e-6) / 1e12, alg / (c.mean_us * 1e-6) / 8e12,
           alg / (w.mean_us * 1e-6) / 8e12);
    fflush(stdout);
}

// sets of (nbuf buffers of `bytes`), carved from the pool
static int sets_for(size_t set_bytes) {
    int n = (int)((kFootprint + set_bytes - 1) / set_bytes);
    if (n < 4) n = 4;
    if ((size_t)n * set_bytes > g_pool_bytes) n = (int)(g_pool_bytes / set_bytes);
    return n;
}
static char *buf(int set, int k, int nbuf, size_t bytes) {
    const size_t j = (size_t)set * nbuf + k;
    const size_t sk = k >= g_skew_from ? (size_t)(k - g_skew_from + 1) * g_skew : 0;
    return g_pool + j * (bytes + (size_t)nbuf * g_skew) + sk;
}

template <typename K>
static void copy_variant(const char *name, K kern, int bpc, int u, size_t bytes, bool chunk = false) {
    const uint64_t nvec = bytes / 16;
    const int nsets = sets_for(2 * bytes);
    uint64_t want = (nvec + 256ull * u - 1) / (256ull * u);
    unsigned grid = (unsigned)std::min<uint64_t>(want, (uint64_t)g_cus * bpc);
    if (chunk) grid = g_cus * bpc;
    auto launch = [&](int s) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, (const u32x4 *)buf(s, 0, 2, bytes),
                           (u32x4 *)buf(s, 1, 2, bytes), nvec);
    };
    Stat w = timed(launch, nsets, false, 30);
    Stat c = timed(launch, nsets, true, 4 * nsets);
    char v[96];
    snprintf(v, sizeof v, "%s bpc=%d U=%d", name, bpc, u);
    emit("copy", v, 2 * bytes, nsets, w, c);
}

static void lib_copy(size_t bytes, const char *name = "copy_segments<4,1>") {
    const int nsets = sets_for(2 * bytes);
    auto launch = [&](int s) {
        void *d[1] = {buf(s, 1, 2, bytes) + g_dst_mis};
        const void *sr[1] = {buf(s, 0, 2, bytes) + g_src_mis};
        size_t nb[1] = {bytes - (g_dst_mis ? 16 : 0)};
        if (mi355_copy_segments(d, sr, nb, 1, nullptr) != 0) exit(2);
    };
    Stat w = timed_lib(launch, nsets, false, 30);
    Stat c = timed_lib(launch, nsets, true, 4 * nsets);
    emit(name, "library", 2 * bytes, nsets, w, c);
}

static void lib_fold(const char *name, int op, int dtype, int k, size_t bytes) {
    const int nbuf = k + 1;
    const int nsets = sets_for(nbuf * bytes);
    const size_t n = bytes / mi355_dtype_size(dtype);
    auto launch = [&](int s) {
        const void *sr[8];
        for (int j = 0; j < k; ++j) sr[j] = buf(s, j, nbuf, bytes) + g_src_mis;
        if (mi355_combine(op, dtype, buf(s, k, nbuf, bytes) + g_dst_mis, sr, k, n - (g_dst_mis ? 1 : 0), nullptr) != 0) exit(2);
    };
    Stat w = timed_lib(launch, nsets, false, 30);
    Stat c = timed_lib(launch, nsets, true, std::max(40, 2 * nsets));
    char v[64];
    snprintf(v, sizeof v, "library, %d x %zu MiB", k, bytes / MiB);
    emit(name, v, (size_t)nbuf * bytes, nsets, w, c);
}

static void lib_orders(const char *name, int op, int dtype, int k, size_t bytes) {
    const int nbuf = 2 * k;
    const int nsets = sets_for(nbuf * bytes);
    const size_t n = bytes / mi355_dtype_size(dtype);
    auto launch = [&](int s) {
        const void *sr[8];
        void *ds[8];
        for (int j = 0; j < k; ++j) {
            sr[j] = buf(s, j, nbuf, bytes) + g_src_mis;
            ds[j] = buf(s, k + j, nbuf, bytes) + g_dst_mis;
        }
        if (mi355_combine_orders(op, dtype, ds, sr, k, n - (g_dst_mis ? 1 : 0), nullptr) != 0) exit(2);
    };
    Stat w = timed_lib(launch, nsets, false, 30);
    Stat c = timed_lib(launch, nsets, true, std::max(40, 2 * nsets));
    char v[64];
    snprintf(v, sizeof v, "library, %d x %zu MiB", k, bytes / MiB);
    emit(name, v, (size_t)nbuf * bytes, nsets, w, c);
}

template <typename K>
static void orders_variant(const char *name, K kern, int bpc, int u, size_t bytes) {
    const uint64_t nvec = bytes / 16;
    const int nsets = sets_for(16 * bytes);
    uint64_t want = (nvec + 256ull * u - 1) / (256ull * u);
    const unsigned grid = (unsigned)std::min<uint64_t>(want, (uint64_t)g_cus * bpc);
    auto launch = [&](int st) {
        const u32x4 *sp[8];
        u32x4 *dp[8];
        for (int k = 0; k < 8; ++k) {
            sp[k] = (const u32x4 *)buf(st, k, 16, bytes);
            dp[k] = (u32x4 *)buf(st, 8 + k, 16, bytes);
        }
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, sp[0], sp[1], sp[2], sp[3], sp[4], sp[5], sp[6], sp[7],
                           dp[0], dp[1], dp[2], dp[3], dp[4], dp[5], dp[6], dp[7], nvec);
    };
    Stat w = timed(launch, nsets, false, 30);
    Stat c = timed(launch, nsets, true, std::max(40, 4 * nsets));
    char v[96];
    snprintf(v, sizeof v, "%s bpc=%d U=%d", name, bpc, u);
    emit("orders8<sum,double>", v, 16 * bytes, nsets, w, c);
}

// ---- the library's combine_vec at a chosen shape (k8shapes)
template <int OP, typename T, int U>
static void fold_shape(const char *name, size_t bytes, int bpc) {
    constexpr int NS = 8;
    const int nbuf = NS + 1;
    const int nsets = sets_for(nbuf * (bytes + g_skew));
    const uint64_t nvec = bytes / 16;
    const unsigned grid = (unsigned)std::min<uint64_t>((nvec + 256ull * U - 1) / (256ull * U), (uint64_t)g_cus * bpc);
    auto launch = [&](int st) {
        mi355k::CombineParams p{};
        p.dst = buf(st, NS, nbuf, bytes);
        for (int k = 0; k < NS; ++k) p.src[k] = buf(st, k, nbuf, bytes);
        p.nvec = nvec;
        hipLaunchKernelGGL((mi355k::combine_vec<OP, T, NS, U, mi355k::POL_NT_LOAD, false>), dim3(grid), dim3(256), 0, 0, p);
    };
    Stat w = timed(launch, nsets, false, 30);
    Stat c = timed(launch, nsets, true, std::max(40, 2 * nsets));
    char v[96];
    snprintf(v, sizeof v, "8 x %zu MiB U=%d bpc=%d", bytes / MiB, U, bpc);
    emit(name, v, (size_t)nbuf * bytes, nsets, w, c);
}
template <int OP, typename T>
static void fold_shapes(const char *name, size_t bytes) {
    for (int bpc : {2, 4, 8}) {
        fold_shape<OP, T, 1>(name, bytes, bpc);
        fold_shape<OP, T, 2>(name, bytes, bpc);
        fold_shape<OP, T, 4>(name, bytes, bpc);
    }
}

// ---- the library's combine_orders_vec at a chosen shape (o8shapes)
template <int OP, typename T, int U>
static void orders_shape(const char *name, size_t bytes, int bpc) {
    constexpr int NS = 8;
    const int nbuf = 2 * NS;
    const int nsets = sets_for(nbuf * (bytes + g_skew));
    const uint64_t nvec = bytes / 16;
    const unsigned grid = (unsigned)std::min<uint64_t>((nvec + 256ull * U - 1) / (256ull * U), (uint64_t)g_cus * bpc);
    auto launch = [&](int st) {
        mi355k::OrdersParams p{};
        for (int k = 0; k < NS; ++k) {
            p.src[k] = buf(st, k, nbuf, bytes);
            p.dst[k] = buf(st, NS + k, nbuf, bytes);
        }
        p.nvec = nvec;
        hipLaunchKernelGGL((mi355k::combine_orders_vec<OP, T, NS, U, mi355k::POL_NT_LOAD, true, false>), dim3(grid),
                           dim3(256), 0, 0, p);
    };
    Stat w = timed(launch, nsets, false, 30);
    Stat c = timed(launch, nsets, true, std::max(40, 2 * nsets));
    char v[96];
    snprintf(v, sizeof v, "8 x %zu MiB U=%d bpc=%d grid=%u", bytes / MiB, U, bpc, grid);
    emit(name, v, (size_t)nbuf * bytes, nsets, w, c);
}

int main(int argc, char **argv) {
    const std::string what = argc > 1 ? argv[1] : "all";
    CHECK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, 0));
    CHECK(hipEventCreate(&g_a));
    CHECK(hipEventCreate(&g_b));
    g_pool_bytes = kFootprint + 1024 * MiB;
    CHECK(hipMalloc(&g_pool, g_pool_bytes));
    // full-mantissa-ish bytes everywhere (doubles in [-1, 1), no NaN)
    {
        std::vector<double> h(64 * MiB / 8);
        uint64_t z = 0x9E3779B97F4A7C15ull;
        for (auto &x : h) {
            z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull; z ^= z >> 27; z *= 0x94D049BB133111EBull; z ^= z >> 31;
            x = (double)(z >> 11) * 0x1p-53 - 0.5;
        }
        for (size_t off = 0; off < g_pool_bytes; off += 64 * MiB)
            CHECK(hipMemcpy(g_pool + off, h.data(), std::min(64 * MiB, g_pool_bytes - off), hipMemcpyHostToDevice));
    }
    const size_t S = 256 * MiB;
    if (what == "lib" || what == "all") {
        lib_copy(S);                                                            // the N = 1 headline's kernel
        lib_fold("combine_vec<sum,double,2>", MI355_OP_SUM, MI355_DOUBLE, 2, S);
        lib_fold("combine_vec<sum,double,8>", MI355_OP_SUM, MI355_DOUBLE, 8, S);
        lib_fold("combine_vec<and,longlong,8>", MI355_OP_AND, MI355_LONGLONG, 8, 64 * MiB);
        lib_fold("combine_vec<and,longlong,8>", MI355_OP_AND, MI355_LONGLONG, 8, 8 * MiB);   // config 4 N = 8 shard
        lib_fold("combine_vec<max,float,8>", MI355_OP_MAX, MI355_FLOAT, 8, 64 * MiB);
        lib_orders("combine_orders_vec<sum,double,8>", MI355_OP_SUM, MI355_DOUBLE, 8, 32 * MiB);
        lib_orders("combine_orders_vec<max,float,8>", MI355_OP_MAX, MI355_FLOAT, 8, 8 * MiB);
    }
    if (what == "copy" || what == "all") {
        copy_variant("pipe ld=plain st=nt_sc1", copy_pipe<4, LD_PLAIN, ST_NT_SC1>, 1, 4, S);   // = library
        copy_variant("pipe ld=plain st=nt_sc1", copy_pipe<4, LD_PLAIN, ST_NT_SC1>, 2, 4, S);
        copy_variant("pipe ld=plain st=nt_sc1", copy_pipe<8, LD_PLAIN, ST_NT_SC1>, 1, 8, S);
        copy_variant("pipe ld=plain st=nt_sc1", copy_pipe<2, LD_PLAIN, ST_NT_SC1>, 2, 2, S);
        copy_variant("pipe ld=plain st=nt_sc1", copy_pipe<4, LD_PLAIN, ST_NT_SC1>, 4, 4, S);
        copy_variant("pipe ld=nt st=nt_sc1", copy_pipe<4, LD_NT, ST_NT_SC1>, 1, 4, S);
        copy_variant("pipe ld=nt st=nt_sc1", copy_pipe<4, LD_NT, ST_NT_SC1>, 2, 4, S);
        copy_variant("pipe ld=plain st=nt", copy_pipe<4, LD_PLAIN, ST_NT>, 1, 4, S);
        copy_variant("pipe ld=plain st=plain", copy_pipe<4, LD_PLAIN, ST_PLAIN>, 1, 4, S);
        copy_variant("pipe ld=plain st=sc1", copy_pipe<4, LD_PLAIN, ST_SC1>, 1, 4, S);
        copy_variant("pipe ld=nt st=sc1", copy_pipe<4, LD_NT, ST_SC1>, 1, 4, S);
        copy_variant("chunk ld=plain st=nt_sc1", copy_chunk<4, LD_PLAIN, ST_NT_SC1>, 1, 4, S, true);
        copy_variant("chunk ld=plain st=nt_sc1", copy_chunk<4, LD_PLAIN, ST_NT_SC1>, 2, 4, S, true);
        copy_variant("chunk ld=nt st=nt_sc1", copy_chunk<4, LD_NT, ST_NT_SC1>, 2, 4, S, true);
    }
    if (what == "copy2") {   // round 5: cold copy, more policies
        copy_variant("pipe ld=nt st=nt_sc1", copy_pipe<4, LD_NT, ST_NT_SC1>, 2, 4, S);
        copy_variant("pipe ld=nt st=nt_sc1", copy_pipe<2, LD_NT, ST_NT_SC1>, 4, 2, S);
        copy_variant("pipe ld=nt st=nt_sc1", copy_pipe<8, LD_NT, ST_NT_SC1>, 2, 8, S);
        copy_variant("pipe ld=nt st=nt_sc1", copy_pipe<4, LD_NT, ST_NT_SC1>, 4, 4, S);
        copy_variant("pipe ld=nt st=nt", copy_pipe<4, LD_NT, ST_NT>, 2, 4, S);
        copy_variant("pipe ld=nt st=plain", copy_pipe<4, LD_NT, ST_PLAIN>, 2, 4, S);
        copy_variant("pipe ld=plain st=nt_sc1", copy_pipe<4, LD_PLAIN, ST_NT_SC1>, 1, 4, S);
    }
    if (what == "orders") {   // round 5: the every-member fold, cold
        const size_t B = 32 * MiB;
        orders_variant("ld=nt st=sc1", orders8<4, LD_NT, ST_SC1>, 8, 4, B);   // = library (Shape<8>)
        orders_variant("ld=nt st=sc1", orders8<2, LD_NT, ST_SC1>, 8, 2, B);
        orders_variant("ld=nt st=sc1", orders8<1, LD_NT, ST_SC1>, 8, 1, B);
        orders_variant("ld=nt st=sc1", orders8<4, LD_NT, ST_SC1>, 2, 4, B);
        orders_variant("ld=nt st=sc1", orders8<2, LD_NT, ST_SC1>, 4, 2, B);
        orders_variant("ld=nt st=nt_sc1", orders8<4, LD_NT, ST_NT_SC1>, 8, 4, B);
        orders_variant("ld=nt st=nt_sc1", orders8<2, LD_NT, ST_NT_SC1>, 4, 2, B);
        orders_variant("ld=plain st=nt_sc1", orders8<4, LD_PLAIN, ST_NT_SC1>, 8, 4, B);
        orders_variant("ld=plain st=sc1", orders8<4, LD_PLAIN, ST_SC1>, 8, 4, B);
        orders_variant("ld=nt st=nt", orders8<4, LD_NT, ST_NT>, 8, 4, B);
        orders_variant("ld=nt st=plain", orders8<4, LD_NT, ST_PLAIN>, 8, 4, B);
    }
    if (what == "orders_skew") {   // round 5: do same-offset buffers (power-of-two stride) collide in DRAM?
        for (size_t sk : {(size_t)0, (size_t)256, (size_t)4096, (size_t)65536 + 256, (size_t)MiB + 4096,
                          (size_t)2 * MiB + 768}) {
            g_skew = sk;
            char nm[96];
            snprintf(nm, sizeof nm, "combine_orders_vec<sum,double,8> skew=%zu", sk);
            lib_orders(nm, MI355_OP_SUM, MI355_DOUBLE, 8, 32 * MiB);
            snprintf(nm, sizeof nm, "copy_segments<4,1> skew=%zu", sk);
            lib_copy(S, nm);
        }
        g_skew = 0;
    }
    if (what == "orders_skew2") {   // finer: which stride, and outputs only
        for (int from : {0, 8})
            for (size_t sk : {(size_t)1024, (size_t)2048, (size_t)4096, (size_t)8192, (size_t)12288, (size_t)16384,
                              (size_t)32768, (size_t)4096 + 256, (size_t)3 * 4096 + 512}) {
                g_skew = sk;
                g_skew_from = from;
                char nm[96];
                snprintf(nm, sizeof nm, "combine_orders_vec<sum,double,8> skew=%zu from=%d", sk, from);
                lib_orders(nm, MI355_OP_SUM, MI355_DOUBLE, 8, 32 * MiB);
            }
        for (size_t sk : {(size_t)0, (size_t)4096}) {
            g_skew = sk;
            g_skew_from = 0;
            char nm[96];
            snprintf(nm, sizeof nm, "combine_orders_vec<max,float,8> 8 MiB skew=%zu", sk);
            lib_orders(nm, MI355_OP_MAX, MI355_FLOAT, 8, 8 * MiB);
            snprintf(nm, sizeof nm, "combine_vec<sum,double,8> 32 MiB skew=%zu", sk);
            lib_fold(nm, MI355_OP_SUM, MI355_DOUBLE, 8, 32 * MiB);
            snprintf(nm, sizeof nm, "combine_vec<and,longlong,8> 8 MiB skew=%zu", sk);
            lib_fold(nm, MI355_OP_AND, MI355_LONGLONG, 8, 8 * MiB);
            snprintf(nm, sizeof nm, "combine_vec<sum,double,2> 256 MiB skew=%zu", sk);
            lib_fold(nm, MI355_OP_SUM, MI355_DOUBLE, 2, S);
        }
        g_skew = 0;
        g_skew_from = 0;
    }
    if (what == "segs") {   // round 5: the all-gather's shape (7 shards into one target at N = 8)
        const size_t B = 32 * MiB;
        for (int mode = 0; mode < 3; ++mode) {
            // 0: one 224 MiB segment; 1: 7 x 32 MiB, target contiguous (the gather's layout), sources
            // staggered 4352 B apart; 2: both sides staggered (what a decorrelated target would give)
            const size_t stag = 4352;
            const size_t set = 16 * (B + stag);
            const int nsets = sets_for(set);
            auto launch = [&](int st) {
                char *base = g_pool + (size_t)st * set;
                void *d[7];
                const void *sr[7];
                size_t nb[7];
                if (mode == 0) {
                    d[0] = base;
                    sr[0] = base + 8 * (B + stag);
                    nb[0] = 7 * B;
                    if (mi355_copy_segments(d, sr, nb, 1, nullptr) != 0) exit(2);
                    return;
                }
                for (int i = 0; i < 7; ++i) {
                    d[i] = mode == 1 ? base + (size_t)(i + 1) * B : base + (size_t)(i + 1) * (B + stag);
                    sr[i] = base + (size_t)(8 + i) * (B + stag);
                    nb[i] = B;
                }
                if (mi355_copy_segments(d, sr, nb, 7, nullptr) != 0) exit(2);
            };
            Stat w = timed_lib(launch, nsets, false, 30);
            Stat c = timed_lib(launch, nsets, true, std::max(40, 4 * nsets));
            static const char *nm[3] = {"1 x 224 MiB", "7 x 32 MiB, target contiguous", "7 x 32 MiB, both staggered"};
            emit("copy_segments", nm[mode], 14 * B, nsets, w, c);
        }
    }
    if (what == "k8shapes") {   // the eight-source fold's launch shape per type (library: U=4, 8 blocks/CU)
        g_skew = 4352;
        fold_shapes<MI355_OP_SUM, double>("combine_vec<sum,double,8>", 64 * MiB);
        fold_shapes<MI355_OP_MAX, float>("combine_vec<max,float,8>", 64 * MiB);
        fold_shapes<MI355_OP_AND, long long>("combine_vec<and,longlong,8>", 64 * MiB);
        fold_shapes<MI355_OP_SUM, double>("combine_vec<sum,double,8>", 8 * MiB);
        g_skew = 0;
    }
    if (what == "o8shapes") {   // the every-member fold's shape at shard sizes (library: float max U=1 bpc=8, double sum U=4 bpc=8)
        g_skew = 4352;
        for (int bpc : {2, 4, 8}) {
            orders_shape<MI355_OP_MAX, float, 1>("combine_orders_vec<max,float,8>", 8 * MiB, bpc);
            orders_shape<MI355_OP_MAX, float, 2>("combine_orders_vec<max,float,8>", 8 * MiB, bpc);
        }
        orders_shape<MI355_OP_MAX, float, 1>("combine_orders_vec<max,float,8>", 32 * MiB, 8);
        orders_shape<MI355_OP_MAX, float, 2>("combine_orders_vec<max,float,8>", 32 * MiB, 4);
        for (int bpc : {2, 4, 8}) {
            orders_shape<MI355_OP_SUM, double, 2>("combine_orders_vec<sum,double,8>", 8 * MiB, bpc);
            orders_shape<MI355_OP_SUM, double, 4>("combine_orders_vec<sum,double,8>", 8 * MiB, bpc);
        }
        orders_shape<MI355_OP_SUM, double, 4>("combine_orders_vec<sum,double,8>", 32 * MiB, 8);
        g_skew = 0;
    }
    if (what == "k2types") {   // the two-source fold per element type (Shape<2, T> tuning)
        g_skew = 4352;
        lib_fold("combine_vec<sum,short,2>", MI355_OP_SUM, MI355_SHORT, 2, S);
        lib_fold("combine_vec<sum,int,2>", MI355_OP_SUM, MI355_INT, 2, S);
        lib_fold("combine_vec<xor,long,2>", MI355_OP_XOR, MI355_LONG, 2, S);
        lib_fold("combine_vec<sum,float,2>", MI355_OP_SUM, MI355_FLOAT, 2, S);
        lib_fold("combine_vec<max,float,2>", MI355_OP_MAX, MI355_FLOAT, 2, S);
        lib_fold("combine_vec<sum,double,2>", MI355_OP_SUM, MI355_DOUBLE, 2, S);
        lib_fold("combine_vec<prod,double,2>", MI355_OP_PROD, MI355_DOUBLE, 2, S);
        lib_fold("combine_vec<sum,complexf,2>", MI355_OP_SUM, MI355_COMPLEXF, 2, S);
        lib_fold("combine_vec<prod,complexf,2>", MI355_OP_PROD, MI355_COMPLEXF, 2, S);
        lib_fold("combine_vec<sum,complexd,2>", MI355_OP_SUM, MI355_COMPLEXD, 2, S);
        lib_fold("combine_vec<prod,complexd,2>", MI355_OP_PROD, MI355_COMPLEXD, 2, S);
        g_skew = 0;
    }
    if (what == "misaligned") {   // target 8 bytes off the sources' 16-byte phase
        g_skew = 4352;
        for (size_t mis : {(size_t)0, (size_t)8, (size_t)4}) {
            g_dst_mis = mis;
            char nm[96];
            snprintf(nm, sizeof nm, "copy_segments dst+%zu", mis);
            lib_copy(S, nm);
            snprintf(nm, sizeof nm, "combine_vec<sum,double,2> dst+%zu", mis);
            if (mis % 8 == 0) lib_fold(nm, MI355_OP_SUM, MI355_DOUBLE, 2, S);
            snprintf(nm, sizeof nm, "combine_vec<sum,float,2> dst+%zu", mis);
            lib_fold(nm, MI355_OP_SUM, MI355_FLOAT, 2, S);
            snprintf(nm, sizeof nm, "combine_orders_vec<sum,double,8> dst+%zu", mis);
            if (mis % 8 == 0) lib_orders(nm, MI355_OP_SUM, MI355_DOUBLE, 8, 32 * MiB);
        }
        g_dst_mis = 0;
        g_skew = 0;
    }
    if (what == "linepeel") {   // targets off a 128-byte line: aligned (+16, +48) and shifted (+8, +72)
        g_skew = 4352;
        for (size_t mis : {(size_t)16, (size_t)48, (size_t)8, (size_t)72}) {
            g_dst_mis = mis;
            char nm[96];
            snprintf(nm, sizeof nm, "copy_segments dst+%zu", mis);
            lib_copy(S, nm);
            snprintf(nm, sizeof nm, "combine_vec<sum,double,2> dst+%zu", mis);
            lib_fold(nm, MI355_OP_SUM, MI355_DOUBLE, 2, S);
            snprintf(nm, sizeof nm, "combine_vec<sum,float,2> dst+%zu", mis);
            lib_fold(nm, MI355_OP_SUM, MI355_FLOAT, 2, S);
            snprintf(nm, sizeof nm, "combine_orders_vec<sum,double,8> dst+%zu", mis);
            lib_orders(nm, MI355_OP_SUM, MI355_DOUBLE, 8, 32 * MiB);
        }
        g_dst_mis = 0;
        // sources off their line, target on it; both 16 bytes off
        for (size_t dm : {(size_t)0, (size_t)16}) {
            g_src_mis = 16;
            g_dst_mis = dm;
            char nm[96];
            snprintf(nm, sizeof nm, "copy_segments src+16 dst+%zu", dm);
            lib_copy(S, nm);
            snprintf(nm, sizeof nm, "combine_vec<sum,double,2> src+16 dst+%zu", dm);
            lib_fold(nm, MI355_OP_SUM, MI355_DOUBLE, 2, S);
            snprintf(nm, sizeof nm, "combine_orders_vec<sum,double,8> src+16 dst+%zu", dm);
            lib_orders(nm, MI355_OP_SUM, MI355_DOUBLE, 8, 32 * MiB);
        }
        g_src_mis = 0;
        g_dst_mis = 0;
        g_skew = 0;
    }
    if (what == "unalcopy") {   // the shifted copy's loop shape
        const size_t B = S - 4096;
        const uint64_t nvec = B / 16;
        g_skew = 4352;
        const int nsets = sets_for(2 * (S + g_skew));
        struct V { const char *name; void (*k)(const char *, u32x4 *, uint64_t); int U; int bpc; };
        const V vs[] = {{"pipe U=4 bpc=1", copy_unal_u<4, true>, 4, 1}, {"pipe U=4 bpc=2", copy_unal_u<4, true>, 4, 2},
                        {"pipe U=2 bpc=2", copy_unal_u<2, true>, 2, 2}, {"pipe U=2 bpc=4", copy_unal_u<2, true>, 2, 4},
                        {"flat U=1 bpc=2", copy_unal_u<1, false>, 1, 2}, {"flat U=1 bpc=4", copy_unal_u<1, false>, 1, 4},
                        {"flat U=2 bpc=2", copy_unal_u<2, false>, 2, 2}, {"flat U=4 bpc=1", copy_unal_u<4, false>, 4, 1},
                        {"flat U=4 bpc=2", copy_unal_u<4, false>, 4, 2}};
        for (const V &v : vs) {
            const unsigned grid = (unsigned)std::min<uint64_t>((nvec + 256ull * v.U - 1) / (256ull * v.U), (uint64_t)g_cus * v.bpc);
            auto launch = [&](int st) {
                hipLaunchKernelGGL(v.k, dim3(grid), dim3(256), 0, 0, (const char *)buf(st, 0, 2, S) + 8,
                                   (u32x4 *)buf(st, 1, 2, S), nvec);
            };
            Stat w = timed(launch, nsets, false, 30);
            Stat c = timed(launch, nsets, true, std::max(40, 4 * nsets));
            emit("copy_unal", v.name, 2 * B, nsets, w, c);
        }
        g_skew = 0;
    }
    if (what == "unal") {   // misaligned 16-byte loads: correct? fast?
        const size_t B = S - 4096;
        const uint64_t nvec = B / 16;
        g_skew = 4352;
        {
            const char *a = buf(0, 0, 4, S), *b = buf(0, 1, 4, S);
            u32x4 *o1 = (u32x4 *)buf(0, 2, 4, S), *o2 = (u32x4 *)buf(0, 3, 4, S);
            const size_t cmpn = 4 * MiB;
            std::vector<char> h1(cmpn), h2(cmpn);
            int bad = 0;
            for (unsigned dl : {8u, 4u, 12u, 1u, 2u, 3u, 6u, 15u}) {
                hipLaunchKernelGGL((fold2_shift<0>), dim3(g_cus * 2), dim3(256), 0, 0, (const u32x4 *)a, (const u32x4 *)b, o1, nvec, dl);
                hipLaunchKernelGGL(fold2_unal, dim3(g_cus * 2), dim3(256), 0, 0, a + dl, b + dl, o2, nvec);
                CHECK(hipDeviceSynchronize());
                for (size_t off : {(size_t)0, B - cmpn}) {
                    CHECK(hipMemcpy(h1.data(), (char *)o1 + off, cmpn, hipMemcpyDeviceToHost));
                    CHECK(hipMemcpy(h2.data(), (char *)o2 + off, cmpn, hipMemcpyDeviceToHost));
                    if (memcmp(h1.data(), h2.data(), cmpn) != 0) { ++bad; printf("{\"fold_mismatch_delta\": %u, \"off\": %zu}\n", dl, off); }
                }
                hipLaunchKernelGGL(copy_unal, dim3(g_cus * 2), dim3(256), 0, 0, a + dl, o2, nvec);
                CHECK(hipDeviceSynchronize());
                std::vector<char> hs(cmpn + 16);
                CHECK(hipMemcpy(hs.data(), a, cmpn + 16, hipMemcpyDeviceToHost));
                CHECK(hipMemcpy(h2.data(), (char *)o2, cmpn, hipMemcpyDeviceToHost));
                if (memcmp(hs.data() + dl, h2.data(), cmpn) != 0) { ++bad; printf("{\"copy_mismatch_delta\": %u}\n", dl); }
            }
            printf("{\"unal_check_mismatches\": %d}\n", bad);
            fflush(stdout);
        }
        for (int v = 0; v < 8; ++v) {
            const int nbuf = v % 4 < 2 ? 2 : 3;
            const int nsets = sets_for(nbuf * (S + g_skew));
            const unsigned grid = (unsigned)g_cus * (v % 2 ? 4 : 2);
            const size_t mis = v < 4 ? 8 : 3;
            auto launch = [&](int st) {
                const char *a = buf(st, 0, nbuf, S) + mis, *b = buf(st, 1, nbuf, S) + mis;
                u32x4 *dd = (u32x4 *)buf(st, nbuf - 1, nbuf, S);
                if (v % 4 < 2) hipLaunchKernelGGL(copy_unal, dim3(grid), dim3(256), 0, 0, a, dd, nvec);
                else hipLaunchKernelGGL(fold2_unal, dim3(grid), dim3(256), 0, 0, a, b, dd, nvec);
            };
            Stat w = timed(launch, nsets, false, 30);
            Stat c = timed(launch, nsets, true, std::max(40, 4 * nsets));
            static const char *nm[8] = {"copy unal+8 bpc=2", "copy unal+8 bpc=4", "fold2 unal+8 bpc=2", "fold2 unal+8 bpc=4",
                                        "copy unal+3 bpc=2", "copy unal+3 bpc=4", "fold2 unal+3 bpc=2", "fold2 unal+3 bpc=4"};
            emit("shift", nm[v], (size_t)nbuf * B, nsets, w, c);
        }
        g_skew = 0;
    }
    if (what == "dpp") {   // DPP neighbour exchange: correctness against the two-load form, then rates
        const size_t B = S - 4096;
        const uint64_t nvec = B / 16;
        g_skew = 4352;
        {   // correctness: 3 buffers of set 0 (a, b, out) + a reference out
            const u32x4 *a = (const u32x4 *)buf(0, 0, 4, S), *b = (const u32x4 *)buf(0, 1, 4, S);
            u32x4 *o1 = (u32x4 *)buf(0, 2, 4, S), *o2 = (u32x4 *)buf(0, 3, 4, S);
            const size_t cmpn = 4 * MiB;
            std::vector<char> h1(cmpn), h2(cmpn);
            int bad = 0;
            for (unsigned dl : {4u, 8u, 12u, 2u, 6u, 1u, 15u}) {
                hipLaunchKernelGGL((fold2_shift<0>), dim3(g_cus * 2), dim3(256), 0, 0, a, b, o1, nvec, dl);
                hipLaunchKernelGGL((fold2_dpp<LD_NT>), dim3(g_cus * 2), dim3(256), 0, 0, a, b, o2, nvec, dl);
                CHECK(hipDeviceSynchronize());
                for (size_t off : {(size_t)0, B - cmpn}) {
                    CHECK(hipMemcpy(h1.data(), (char *)o1 + off, cmpn, hipMemcpyDeviceToHost));
                    CHECK(hipMemcpy(h2.data(), (char *)o2 + off, cmpn, hipMemcpyDeviceToHost));
                    bad += memcmp(h1.data(), h2.data(), cmpn) != 0;
                }
                hipLaunchKernelGGL((copy_shift<4, 0, LD_PLAIN, ST_NT_SC1>), dim3(g_cus * 2), dim3(256), 0, 0, a, o1, nvec, dl);
                hipLaunchKernelGGL((copy_dpp<LD_PLAIN>), dim3(g_cus * 2), dim3(256), 0, 0, a, o2, nvec, dl);
                CHECK(hipDeviceSynchronize());
                for (size_t off : {(size_t)0, B - cmpn}) {
                    CHECK(hipMemcpy(h1.data(), (char *)o1 + off, cmpn, hipMemcpyDeviceToHost));
                    CHECK(hipMemcpy(h2.data(), (char *)o2 + off, cmpn, hipMemcpyDeviceToHost));
                    bad += memcmp(h1.data(), h2.data(), cmpn) != 0;
                }
                // the copy against the host: out[j] = src bytes [dl + 16 j, ...)
                std::vector<char> hs(cmpn + 16);
                CHECK(hipMemcpy(hs.data(), (const char *)a, cmpn + 16, hipMemcpyDeviceToHost));
                CHECK(hipMemcpy(h2.data(), (char *)o2, cmpn, hipMemcpyDeviceToHost));
                bad += memcmp(hs.data() + dl, h2.data(), cmpn) != 0;
            }
            printf("{\"dpp_check_mismatches\": %d}\n", bad);
            if (bad) return 3;
        }
        for (int v = 0; v < 4; ++v) {
            const int nbuf = v < 2 ? 2 : 3;
            const int nsets = sets_for(nbuf * (S + g_skew));
            const unsigned grid = (unsigned)g_cus * 2;
            auto launch = [&](int st) {
                const u32x4 *a = (const u32x4 *)buf(st, 0, nbuf, S);
                u32x4 *dd = (u32x4 *)buf(st, nbuf - 1, nbuf, S);
                const u32x4 *b = (const u32x4 *)buf(st, 1, nbuf, S);
                if (v == 0) hipLaunchKernelGGL(copy_dpp<LD_PLAIN>, dim3(grid), dim3(256), 0, 0, a, dd, nvec, 8u);
                if (v == 1) hipLaunchKernelGGL(copy_dpp<LD_NT>, dim3(grid), dim3(256), 0, 0, a, dd, nvec, 8u);
                if (v == 2) hipLaunchKernelGGL(fold2_dpp<LD_NT>, dim3(grid), dim3(256), 0, 0, a, b, dd, nvec, 8u);
                if (v == 3) hipLaunchKernelGGL(fold2_dpp<LD_PLAIN>, dim3(grid), dim3(256), 0, 0, a, b, dd, nvec, 8u);
            };
            Stat w = timed(launch, nsets, false, 30);
            Stat c = timed(launch, nsets, true, std::max(40, 4 * nsets));
            static const char *nm[4] = {"copy dpp plain bpc=2", "copy dpp nt bpc=2", "fold2 dpp nt bpc=2", "fold2 dpp plain bpc=2"};
            emit("shift", nm[v], (size_t)nbuf * B, nsets, w, c);
        }
        g_skew = 0;
    }
    if (what == "shift") {   // realigning copy / k = 2 fold, target aligned, sources 8 bytes off
        const size_t B = S - 4096;
        const uint64_t nvec = B / 16;
        g_skew = 4352;
        for (int v = 0; v < 12; ++v) {
            const int nbuf = v < 4 ? 2 : 3;
            const int nsets = sets_for(nbuf * (S + g_skew));
            const unsigned grid = v < 4 ? (unsigned)g_cus * (v % 2 ? 2 : 1) : v >= 10 ? (unsigned)g_cus * 4 : (unsigned)g_cus * 2;
            auto launch = [&](int st) {
                const u32x4 *a = (const u32x4 *)buf(st, 0, nbuf, S);
                u32x4 *dd = (u32x4 *)buf(st, nbuf - 1, nbuf, S);
                if (v == 0) hipLaunchKernelGGL((copy_shift<4, 0, LD_PLAIN, ST_NT_SC1>), dim3(grid), dim3(256), 0, 0, a, dd, nvec, 8u);
                if (v == 1) hipLaunchKernelGGL((copy_shift<4, 0, LD_PLAIN, ST_NT_SC1>), dim3(grid), dim3(256), 0, 0, a, dd, nvec, 8u);
                if (v == 2) hipLaunchKernelGGL((copy_shift<4, 1, LD_PLAIN, ST_NT_SC1>), dim3(grid), dim3(256), 0, 0, a, dd, nvec, 8u);
                if (v == 3) hipLaunchKernelGGL((copy_shift<4, 1, LD_PLAIN, ST_NT_SC1>), dim3(grid), dim3(256), 0, 0, a, dd, nvec, 8u);
                const u32x4 *b = (const u32x4 *)buf(st, 1, nbuf, S);
                if (v == 4) hipLaunchKernelGGL(fold2_shift<0>, dim3(grid), dim3(256), 0, 0, a, b, dd, nvec, 8u);
                if (v == 5) hipLaunchKernelGGL(fold2_shift<1>, dim3(grid), dim3(256), 0, 0, a, b, dd, nvec, 8u);
                if (v == 6) hipLaunchKernelGGL((fold2_shift<0, LD_PLAIN, LD_PLAIN>), dim3(grid), dim3(256), 0, 0, a, b, dd, nvec, 8u);
                if (v == 7) hipLaunchKernelGGL((fold2_shift<0, LD_NT, LD_PLAIN>), dim3(grid), dim3(256), 0, 0, a, b, dd, nvec, 8u);
                if (v == 8) hipLaunchKernelGGL((fold2_shift<0, LD_PLAIN, LD_NT>), dim3(grid), dim3(256), 0, 0, a, b, dd, nvec, 8u);
                if (v == 9) hipLaunchKernelGGL((fold2_shift<0, LD_NT, LD_NT, 2>), dim3(grid), dim3(256), 0, 0, a, b, dd, nvec, 8u);
                if (v == 10) hipLaunchKernelGGL((fold2_shift<0, LD_NT, LD_NT>), dim3(grid), dim3(256), 0, 0, a, b, dd, nvec, 8u);
                if (v == 11) hipLaunchKernelGGL((fold2_shift<0, LD_PLAIN, LD_PLAIN>), dim3(grid), dim3(256), 0, 0, a, b, dd, nvec, 8u);
            };
            Stat w = timed(launch, nsets, false, 30);
            Stat c = timed(launch, nsets, true, std::max(40, 4 * nsets));
            static const char *nm[12] = {"copy two-load bpc=1", "copy two-load bpc=2", "copy shfl bpc=1", "copy shfl bpc=2",
                                        "fold2 double two-load bpc=2", "fold2 double shfl bpc=2",
                                        "fold2 two-load plain/plain bpc=2", "fold2 two-load nt/plain bpc=2",
                                        "fold2 two-load plain/nt bpc=2", "fold2 two-load nt/nt U=2 bpc=2",
                                        "fold2 two-load nt/nt bpc=4", "fold2 two-load plain/plain bpc=4"};
            emit("shift", nm[v], (size_t)nbuf * B, nsets, w, c);
        }
        g_skew = 0;
    }
    CHECK(hipFree(g_pool));
    return 0;
}
