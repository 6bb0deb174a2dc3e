// copy_tail.hip -- where the 1-PE identity copy's time goes across its blocks
// (round 6 probe). The library's copy loop (combine.hip copy_segments<4,1>:
// grid-stride, one block per CU, 4 vectors per lane software-pipelined, plain
// loads, `nt sc1` stores) with each block's start and end stamped with
// s_memrealtime (100 MHz), 256 MiB, warm (one pair) and cold (5 pairs in
// turn). If the last block ends well after the median one, a balanced
// distribution of the work (a work queue) would shorten the call.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/copy_tail.hip -o tools/probes/copy_tail
// run:   tools/probes/copy_tail      (one JSON line per configuration)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int kBlock = 256;

__device__ __forceinline__ void st16(u32x4 *p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

template <int UNROLL>
__global__ __launch_bounds__(kBlock) void copy_stamped(const u32x4 *s, u32x4 *d, uint64_t nvec, uint64_t *stamps,
                                                       unsigned remap = 0) {
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    const uint64_t step = (uint64_t)gridDim.x * kBlock * UNROLL;
    // remap (probe): block b copies block (b ^ remap)'s sub-chunks, the loop unchanged
    uint64_t base = (uint64_t)(blockIdx.x ^ remap) * kBlock * UNROLL + threadIdx.x;
    u32x4 x[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
        const uint64_t i = base + (uint64_t)u * kBlock;
        if (i < nvec) x[u] = s[i];
    }
    while (base < nvec) {
        const uint64_t next = base + step;
        u32x4 y[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = next + (uint64_t)u * kBlock;
            if (i < nvec) y[u] = s[i];
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
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = t_start;
        stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

// Rotated static loop: pass k of the grid-stride loop gives block b the
// sub-chunk (b + k) mod grid of stripe k instead of sub-chunk b, so every
// block meets every residue of the stripe (warm, the blocks with even
// blockIdx finished ~13 us before the odd ones: their fixed sub-chunks'
// source lines stayed in the Infinity Cache more often).
// (generalized: pass k gives block b the sub-chunk ((b + k * rot) mod grid) xor xr)
template <int UNROLL>
__global__ __launch_bounds__(kBlock) void copy_rot(const u32x4 *s, u32x4 *d, uint64_t nvec, uint64_t *stamps,
                                                   unsigned rot, unsigned xr) {
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    const uint64_t sub = (uint64_t)kBlock * UNROLL;              // vectors per sub-chunk
    const uint64_t step = (uint64_t)gridDim.x * sub;             // vectors per stripe (pass)
    unsigned jr = blockIdx.x;                                    // rotated index, before the xor
    unsigned j = jr ^ xr;                                        // this pass's sub-chunk
    uint64_t stripe = 0;
    uint64_t base = (uint64_t)j * sub + threadIdx.x;
    u32x4 x[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
        const uint64_t i = base + (uint64_t)u * kBlock;
        if (i < nvec) x[u] = s[i];
    }
    while (stripe < nvec) {
        const uint64_t nstripe = stripe + step;
        jr = (jr + rot) % gridDim.x;
        j = jr ^ xr;
        const uint64_t next = nstripe + (uint64_t)j * sub + threadIdx.x;
        u32x4 y[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = next + (uint64_t)u * kBlock;
            if (i < nvec) y[u] = s[i];
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = base + (uint64_t)u * kBlock;
            if (i < nvec) st16(d + i, x[u]);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) x[u] = y[u];
        base = next;
        stripe = nstripe;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = t_start;
        stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

// copy_rot without the division: the grid is a power of two, so the rotated
// index wraps with a mask (rmask = grid - 1); the stripe loop as copy_stamped.
template <int UNROLL>
__global__ __launch_bounds__(kBlock) void copy_rotm(const u32x4 *s, u32x4 *d, uint64_t nvec, uint64_t *stamps,
                                                    unsigned rot, unsigned rmask) {
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    const uint64_t sub = (uint64_t)kBlock * UNROLL;
    const uint64_t step = (uint64_t)gridDim.x * sub;
    unsigned j = blockIdx.x;
    uint64_t stripe = 0;
    uint64_t base = (uint64_t)j * sub + threadIdx.x;
    u32x4 x[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
        const uint64_t i = base + (uint64_t)u * kBlock;
        if (i < nvec) x[u] = s[i];
    }
    while (base < nvec) {
        stripe += step;
        j = (j + rot) & rmask;
        const uint64_t next = stripe + (uint64_t)j * sub + threadIdx.x;
        u32x4 y[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = next + (uint64_t)u * kBlock;
            if (i < nvec) y[u] = s[i];
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
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = t_start;
        stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

// Dynamic variant: each WAVE takes chunks of 64 x U vectors from one of 8
// per-XCD queues (queue q holds chunks q, q + 8, ...; an atomic head per
// queue), moving on to the next queue when its own is empty. The atomic for
// the chunk after next is issued before the next chunk's loads, so waiting
// for its value never waits for those loads (vmcnt counts in issue order):
// the queue costs no latency in the steady state. The last block to finish
// resets the heads for the next launch.
// the 8 heads 4 KiB apart: atomics on one line serialize (~88 per us, measured
// here with the heads in one 32-byte word group: 842 us per 256 MiB at U = 4)
constexpr size_t kHeadStride = 1024;

template <int U>
__global__ __launch_bounds__(kBlock) void copy_dyn(const u32x4 *s, u32x4 *d, uint64_t nvec, unsigned *heads,
                                                   unsigned *done_count, uint64_t *stamps) {
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    constexpr uint64_t CV = 64ull * U;
    const uint64_t nchunks = (nvec + CV - 1) / CV;
    const unsigned lane = threadIdx.x & 63;
    int q = blockIdx.x & 7, tried = 1;
    auto count_of = [&](int qq) -> uint64_t { return nchunks > (uint64_t)qq ? (nchunks - 1 - qq) / 8 + 1 : 0; };
    auto issue = [&](int qq) -> unsigned {
        unsigned k = 0;
        if (lane == 0) k = __hip_atomic_fetch_add(heads + (size_t)qq * kHeadStride, 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
        return k;
    };
    // chunk from a ticket of queue q, or the next queue's (blocking), or ~0
    auto resolve = [&](unsigned ticket) -> uint64_t {
        uint64_t k = __builtin_amdgcn_readfirstlane(ticket);
        while (k >= count_of(q)) {
            if (tried >= 8) return ~0ull;
            q = (q + 1) & 7;
            ++tried;
            k = __builtin_amdgcn_readfirstlane(issue(q));
        }
        return (uint64_t)q + 8 * k;
    };
    uint64_t c = resolve(issue(q));
    unsigned ticket = c != ~0ull ? issue(q) : 0u;
    u32x4 x[U];
    if (c != ~0ull) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = c * CV + (uint64_t)u * 64 + lane;
            if (i < nvec) x[u] = s[i];
        }
    }
    while (c != ~0ull) {
        const uint64_t n = resolve(ticket);           // waits for the ticket only
        if (n != ~0ull) ticket = issue(q);             // the chunk after n, before n's loads
        u32x4 y[U];
        if (n != ~0ull) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t i = n * CV + (uint64_t)u * 64 + lane;
                if (i < nvec) y[u] = s[i];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = c * CV + (uint64_t)u * 64 + lane;
            if (i < nvec) st16(d + i, x[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = y[u];
        c = n;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = t_start;
        stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
        const unsigned prev = __hip_atomic_fetch_add(done_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev + 1 == gridDim.x) {
            for (int i = 0; i < 8; ++i)
                __hip_atomic_store(heads + (size_t)i * kHeadStride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(done_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Hybrid: the library's static grid-stride loop over the first part of the
// vectors (whole passes, about 7/8), then every wave pulls chunks of the rest
// (64 x UD vectors) from the 8 per-XCD queues: blocks that finish their static
// share early take more of the tail. One grab per chunk, waited for at once
// (the compiler drains the wave's loads there: the tail part only).
template <int UD>
__global__ __launch_bounds__(kBlock) void copy_hyb(const u32x4 *s, u32x4 *d, uint64_t nvec, uint64_t nstatic,
                                                   unsigned *heads, unsigned *done_count, uint64_t *stamps) {
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    constexpr int UNROLL = 4;
    const uint64_t step = (uint64_t)gridDim.x * kBlock * UNROLL;
    uint64_t base = (uint64_t)blockIdx.x * kBlock * UNROLL + threadIdx.x;
    u32x4 x[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
        const uint64_t i = base + (uint64_t)u * kBlock;
        if (i < nstatic) x[u] = s[i];
    }
    while (base < nstatic) {
        const uint64_t next = base + step;
        u32x4 y[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = next + (uint64_t)u * kBlock;
            if (i < nstatic) y[u] = s[i];
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t i = base + (uint64_t)u * kBlock;
            if (i < nstatic) st16(d + i, x[u]);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) x[u] = y[u];
        base = next;
    }
    // the tail: chunks of CV vectors after nstatic, chunk g in queue g % 8
    constexpr uint64_t CV = 64ull * UD;
    const uint64_t nchunks = (nvec - nstatic + CV - 1) / CV;
    const unsigned lane = threadIdx.x & 63;
    auto count_of = [&](int qq) -> uint64_t { return nchunks > (uint64_t)qq ? (nchunks - 1 - qq) / 8 + 1 : 0; };
    int q = blockIdx.x & 7;
    for (int tried = 0; tried < 8;) {
        unsigned k = 0;
        if (lane == 0)
            k = __hip_atomic_fetch_add(heads + (size_t)q * kHeadStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        k = __builtin_amdgcn_readfirstlane(k);
        if (k >= count_of(q)) {
            q = (q + 1) & 7;
            ++tried;
            continue;
        }
        const uint64_t b = nstatic + ((uint64_t)q + 8ull * k) * CV + lane;
        u32x4 z[UD];
        if (b + (UD - 1) * 64ull < nvec) {
#pragma unroll
            for (int u = 0; u < UD; ++u) z[u] = s[b + (uint64_t)u * 64];
#pragma unroll
            for (int u = 0; u < UD; ++u) st16(d + b + (uint64_t)u * 64, z[u]);
        } else {
            for (int u = 0; u < UD; ++u)
                if (b + (uint64_t)u * 64 < nvec) st16(d + b + (uint64_t)u * 64, s[b + (uint64_t)u * 64]);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = t_start;
        stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
        const unsigned prev = __hip_atomic_fetch_add(done_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev + 1 == gridDim.x) {
            for (int i = 0; i < 8; ++i)
                __hip_atomic_store(heads + (size_t)i * kHeadStride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(done_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

__global__ void fill(unsigned *p, uint64_t n, unsigned seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = (unsigned)(i * 2654435761u) ^ seed;
}

int main() {
    const size_t S = 256ull << 20;
    const uint64_t nvec = S / 16;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int pairs = 5;
    std::vector<char *> bufs(2 * pairs);
    for (int i = 0; i < 2 * pairs; ++i) {
        CHECK(hipMalloc((void **)&bufs[i], S));
        fill<<<1024, 256>>>((unsigned *)bufs[i], S / 4, 977u * i);
    }
    unsigned *heads, *done;
    CHECK(hipMalloc((void **)&heads, 8 * kHeadStride * 4));
    CHECK(hipMalloc((void **)&done, 64));
    CHECK(hipMemset(heads, 0, 8 * kHeadStride * 4));
    CHECK(hipMemset(done, 0, 64));
    uint64_t *stamps;
    CHECK(hipMalloc((void **)&stamps, 2 * 4096 * sizeof(uint64_t)));
    CHECK(hipDeviceSynchronize());
    // kind 0 static<4>, 4/8/16 dyn<U>; 100 + t: hybrid, static share t/16, tail chunks of 64 x 8
    struct V { const char *name; int kind; int bpc; };
    const bool xcd_only = getenv("COPY_TAIL_XCD") != nullptr;   // per-XCD end times of the static loop only
    // kind 1000 + 16 * rot + xor: copy_rot with that rotation and xor
    const V all[] = {{"static U4", 0, 1}, {"static xor 1", 3001, 1}, {"static xor 2", 3002, 1}, {"static xor 4", 3004, 1},
                     {"static xor 8", 3008, 1}, {"mask rot 0", 2000, 1}, {"mask rot 8", 2008, 1}, {"mask rot 1", 2001, 1},
                     {"mask rot 32", 2032, 1}, {"mask rot 8", 2008, 2},
                     {"rot 0 xor 0", 1000, 1}, {"rot 0 xor 0", 1000, 2}, {"xor 1", 1001, 1}, {"xor 2", 1002, 1}, {"xor 4", 1004, 1},
                     {"xor 8", 1008, 1}, {"rot 8", 1000 + 16 * 8, 1}, {"rot 2", 1000 + 16 * 2, 1},
                     {"hybrid 15/16 UD8", 115, 1}, {"hybrid 14/16 UD8", 114, 1},
                     {"hybrid 12/16 UD8", 112, 1}, {"hybrid 14/16 UD4", 214, 1}, {"hybrid 14/16 UD8", 114, 2}};
    const std::vector<V> vs(all, all + (xcd_only ? 5 : sizeof all / sizeof all[0]));
    std::vector<unsigned> hs(S / 4), hd(S / 4);
    for (const V &v : vs) {
        const unsigned grid = (unsigned)cus * v.bpc;
        auto launch = [&](int p) {
            const u32x4 *src = (const u32x4 *)bufs[2 * p];
            u32x4 *dst = (u32x4 *)bufs[2 * p + 1];
            const uint64_t stp = (uint64_t)grid * kBlock * 4;
            const uint64_t nst = v.kind >= 100 ? nvec * (uint64_t)(v.kind % 100) / 16 / stp * stp : 0;
            switch (v.kind) {
            case 0: copy_stamped<4><<<grid, kBlock>>>(src, dst, nvec, stamps); break;
            case 1: copy_rot<4><<<grid, kBlock>>>(src, dst, nvec, stamps, 1u, 0u); break;
            case 112: case 114: case 115:
                copy_hyb<8><<<grid, kBlock>>>(src, dst, nvec, nst, heads, done, stamps); break;
            case 214: copy_hyb<4><<<grid, kBlock>>>(src, dst, nvec, nst, heads, done, stamps); break;
            default:
                if (v.kind >= 3000) {
                    copy_stamped<4><<<grid, kBlock>>>(src, dst, nvec, stamps, (unsigned)(v.kind - 3000));
                    break;
                }
                if (v.kind >= 2000) {
                    copy_rotm<4><<<grid, kBlock>>>(src, dst, nvec, stamps, (unsigned)(v.kind - 2000), grid - 1);
                    break;
                }
                if (v.kind >= 1000) {
                    copy_rot<4><<<grid, kBlock>>>(src, dst, nvec, stamps, (unsigned)(v.kind - 1000) / 16,
                                                  (unsigned)(v.kind - 1000) % 16);
                    break;
                }
            case 4: copy_dyn<4><<<grid, kBlock>>>(src, dst, nvec, heads, done, stamps); break;
            case 8: copy_dyn<8><<<grid, kBlock>>>(src, dst, nvec, heads, done, stamps); break;
            case 16: copy_dyn<16><<<grid, kBlock>>>(src, dst, nvec, heads, done, stamps); break;
            }
        };
        // correctness: pair 0 after a fresh fill of its target
        CHECK(hipMemset(bufs[1], 0, S));
        launch(0);
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(hs.data(), bufs[0], S, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(hd.data(), bufs[1], S, hipMemcpyDeviceToHost));
        const bool ok = hs == hd;
        hipEvent_t e0, e1;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        std::vector<uint64_t> h(2 * grid);
        for (int cold = 0; cold < 2; ++cold) {
            std::vector<double> med_end, last_end, first_end, kern;
            std::vector<double> xcd_end(8, 0.0), xcd_start(8, 0.0);   // mean end / start per blockIdx % 8
            for (int r = 0; r < 60; ++r) {
                const int p = cold ? r % pairs : 0;
                CHECK(hipEventRecord(e0, 0));
                launch(p);
                CHECK(hipEventRecord(e1, 0));
                CHECK(hipDeviceSynchronize());
                float ms = 0;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                if (r < 10) continue;
                CHECK(hipMemcpy(h.data(), stamps, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
                uint64_t t0 = UINT64_MAX;
                std::vector<uint64_t> ends(grid);
                for (unsigned b = 0; b < grid; ++b) {
                    t0 = std::min(t0, h[2 * b]);
                    ends[b] = h[2 * b + 1];
                }
                for (unsigned b = 0; b < grid; ++b) {
                    xcd_end[b % 8] += (h[2 * b + 1] - t0) * 0.01 / (grid / 8) / 50.0;
                    xcd_start[b % 8] += (h[2 * b] - t0) * 0.01 / (grid / 8) / 50.0;
                }
                for (auto &e : ends) e -= t0;
                std::sort(ends.begin(), ends.end());
                first_end.push_back(ends.front() * 0.01);
                med_end.push_back(ends[grid / 2] * 0.01);
                last_end.push_back(ends.back() * 0.01);
                kern.push_back(ms * 1e3);
            }
            auto mean = [](const std::vector<double> &x) {
                double t = 0;
                for (double y : x) t += y;
                return t / x.size();
            };
            printf("{\"variant\": \"%s\", \"blocks_per_cu\": %d, \"grid\": %u, \"cold\": %s, \"copy_ok\": %s, "
                   "\"kernel_event_us\": %.2f, \"first_block_end_us\": %.2f, \"median_block_end_us\": %.2f, "
                   "\"last_block_end_us\": %.2f, \"tail_us\": %.2f, \"frac_event\": %.4f}\n",
                   v.name, v.bpc, grid, cold ? "true" : "false", ok ? "true" : "false", mean(kern), mean(first_end),
                   mean(med_end), mean(last_end), mean(last_end) - mean(med_end), 2.0 * S / (mean(kern) * 1e-6) / 8e12);
            if (xcd_only) {
                printf("{\"variant\": \"%s\", \"cold\": %s, \"mean_end_us_by_blockIdx_mod_8\": [", v.name,
                       cold ? "true" : "false");
                for (int x = 0; x < 8; ++x) printf("%s%.2f", x ? ", " : "", xcd_end[x]);
                printf("], \"mean_start_us_by_blockIdx_mod_8\": [");
                for (int x = 0; x < 8; ++x) printf("%s%.2f", x ? ", " : "", xcd_start[x]);
                printf("]}\n");
            }
            fflush(stdout);
        }
    }
    for (auto b : bufs) CHECK(hipFree(b));
    return 0;
}
