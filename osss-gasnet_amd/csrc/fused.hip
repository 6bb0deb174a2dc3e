// fused.hip -- the whole P2P reduction of a small message in ONE launch.
//
// The multi-launch schedule (reduce.c) pays, per call, three host barriers and
// three launch/completion round trips (~6.5 us each on MI355X). For the
// many-small-bucket regime (BASELINE config 5: 4096 x 64 KiB on 8 GPUs) that
// fixed cost is the whole call. Here every cross-PE step is a device-side
// flag exchange instead, through each PE's signal region (uncached device
// memory, mapped into every peer over xGMI), and the host waits once:
//
//   arrive   lane q of block 0 stores this call's pair count into member q's
//            ARRIVE[my PE]; every block waits until ARRIVE[q] holds member
//            q's count for every member (its source is ready: the kernel runs
//            after the work queued before it on the same stream), then
//            acquires at system scope (invalidates this CU's stale lines)
//   reduce   fold shard `me` of every member's source, in active-set order
//            (the reference's PE_start order), into this PE's target shard,
//            with system-scope write-through stores -- or (ordered) in EVERY
//            member's reference order (own source first, reduce-op.c:226-264):
//            this PE's version into its target, member q's into slot q of
//            this PE's version area, from which q gathers it
//   rsdone   the last block of the grid publishes RSDONE[my PE] to every
//            member; every block waits for all members' RSDONE, acquires
//   gather   copy the other members' shards from their targets (ordered:
//            this PE's version of them from their version areas)
//   agdone   the last block publishes AGDONE, waits for every member's AGDONE
//            (nobody reads this PE's buffers any more) and stores the call's
//            epoch to the host-coherent flag
//
// Pair counts instead of a reset protocol: PE p's slot for PE q only ever
// grows by one per collective both take part in, so a member that runs ahead
// into the next call can never satisfy a wait of the current one too early
// (the same argument as the host barrier in runtime.c). The counts are kept
// on the device (CALLS[q] of this PE's region): every block reads them when it
// starts, and the last block advances them once all members are done -- by
// then every block has started, so none can read an advanced count. No host
// state is involved, which is what lets a captured HIP graph replay the call.
//
// All blocks of the grid must be co-resident (they wait on each other's last
// block), also beside the grids of other PEs sharing this GPU: the grid is
// capped by the kernel's occupancy and the number of such PEs
// (coresident_grid; at most MI355_FUSED_MAX_BLOCKS, one block per CU).
// Every wait is bounded by p.timeout_ticks of the 100 MHz real-time counter.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#include "ops.h"
#include "residency.h"

namespace {

using namespace mi355;

constexpr int kBlock = 256;
constexpr int kBatch = 8;  // members' vectors in flight per lane in the fold

// Probe build only (csrc/Makefile `probe`, tools/fused_phases.py): the real-time
// stamps of each call's phases, per call epoch in a ring of 64 -- [0] first
// block start, [1] last block start, [2] last block past the ARRIVE wait, [3]
// last block done folding, [4] last block past the RSDONE wait, [5] last block
// done gathering, [6] the grid's last block past the AGDONE wait.
#ifdef MI355_FUSED_PHASES
__device__ unsigned long long g_phase[64][8];
#define PHASE_MAX(c, k)                                                                             \
    do {                                                                                            \
        if (threadIdx.x == 0)                                                                       \
            atomicMax(&g_phase[(c).epoch & 63][k], (unsigned long long)__builtin_amdgcn_s_memrealtime()); \
    } while (0)
#define PHASE_MIN(c, k)                                                                             \
    do {                                                                                            \
        if (threadIdx.x == 0)                                                                       \
            atomicMin(&g_phase[(c).epoch & 63][k], (unsigned long long)__builtin_amdgcn_s_memrealtime()); \
    } while (0)
#define PHASE_RESET_NEXT(c)                                                                         \
    do {                                                                                            \
        if (threadIdx.x < 8) g_phase[((c).epoch + 1) & 63][threadIdx.x] = threadIdx.x == 0 ? ~0ull : 0ull; \
    } while (0)
#else
#define PHASE_MAX(c, k) ((void)0)
#define PHASE_MIN(c, k) ((void)0)
#define PHASE_RESET_NEXT(c) ((void)0)
#endif

// The protocol helpers below (counts, waits, block counting, publish, finish,
// staging copy, the server's mailbox) are inlined into every kernel: in the
// large complex-product instantiations the compiler had left them as calls,
// whose frames took 1,264 bytes of scratch per lane (round 4;
// tools/check_residency.py --no-scratch).
#define FUSED_HELPER __device__ __forceinline__

__device__ __forceinline__ void st_sys_u64(unsigned long long *p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned long long ld_sys_u64(const unsigned long long *p) {
    return __hip_atomic_load(const_cast<unsigned long long *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// 16-byte store, write-through to memory at system scope: a peer reads it
// over xGMI after the flag that follows it
__device__ __forceinline__ void st16_sys(u32x4 *p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

// Loads of the members' buffers (their sources, targets, version areas), at
// system scope: `global_load_dwordx2 ... sc0 sc1` never returns a stale L2 or
// L1 line -- a peer GPU's memory is cached without coherence (non-coherent
// MTYPE), and on one GPU the 8 XCD L2s are not coherent with each other -- so
// a block reads what the members wrote for THIS call without invalidating its
// caches first (MI355FusedArgs.no_acquire). Every such byte is read once per
// call, so bypassing the caches costs nothing.
__device__ __forceinline__ u32x4 ld16_sys(const void *p) {
    const unsigned long long *q = (const unsigned long long *)p;
    const unsigned long long lo = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned long long hi = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    u32x4 r;
    r.x = (unsigned)lo;
    r.y = (unsigned)(lo >> 32);
    r.z = (unsigned)hi;
    r.w = (unsigned)(hi >> 32);
    return r;
}
// The folds' form of the same load: one 16-byte `buffer_load_dwordx4 ...
// sc0 sc1` from a wave-uniform base (a member's buffer) at a per-lane byte
// offset, through the builtin so the compiler places the waits. Round 4
// (tools/probes/fold_probe S, profiles/r04/fold_probe_sysload16.txt): 16-byte
// system-coherent loads fold 2 sources in 134 us per 256 MiB against 143 us
// for ld16_sys's two 8-byte loads (8 sources: 441 vs 459 us); non-temporal
// loads take 116 / 381 us, so the multi-launch folds keep theirs.
// The offset must stay below 4 GiB: the fused path is capped at 1 GiB, and
// mi355_fused_allreduce / mi355_fused_server refuse a call whose bytes per
// member reach kMaxFusedBytes (an out-of-range buffer load returns 0 silently).
constexpr uint64_t kMaxFusedBytes = 1ull << 32;
__device__ __forceinline__ u32x4 ld16_sys_at(const char *base, uint32_t off) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(base), 0, (int)0xFFFFFFF0u, 0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 17);  // aux 17: sc0 | sc1
}
template <typename T>
__device__ __forceinline__ T ld_elem_sys(const T *p) {
    static_assert(sizeof(T) == 2 || sizeof(T) == 4 || sizeof(T) == 8 || sizeof(T) == 16, "element size");
    T v;
    if constexpr (sizeof(T) == 16) {
        const u32x4 w = ld16_sys(p);
        __builtin_memcpy(&v, &w, 16);
    } else if constexpr (sizeof(T) == 8) {
        const unsigned long long w =
            __hip_atomic_load((const unsigned long long *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_memcpy(&v, &w, 8);
    } else if constexpr (sizeof(T) == 4) {
        const unsigned w = __hip_atomic_load((const unsigned *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_memcpy(&v, &w, 4);
    } else {
        const unsigned short w =
            __hip_atomic_load((const unsigned short *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_memcpy(&v, &w, 2);
    }
    return v;
}

// This call's pair count with every member (lanes of wave 0, into LDS).
FUSED_HELPER void load_counts(const MI355FusedArgs &a, const unsigned long long *mine, unsigned long long *cnt) {
    if (threadIdx.x < a.nmembers) cnt[threadIdx.x] = ld_sys_u64(mine + MI355_SIG_CALLS + a.pe[threadIdx.x]) + 1;
    __syncthreads();
}

// Wait until slot `base + pe[i]` of this PE's signal region holds cnt[i]
// for every member i; lanes i < nmembers of wave 0 poll one member each.
// acquire = false only where every later read of the members' buffers is a
// system-coherent load (fused_body under no_acquire); fused_pull's copies
// read with plain loads and always acquire.
FUSED_HELPER bool wait_members(const MI355FusedArgs &a, const unsigned long long *mine, const unsigned long long *cnt,
                             int base, bool include_self, bool acquire = true) {
    bool ok = true;
    if (threadIdx.x < 64) {
        const int i = threadIdx.x;
        bool need = i < a.nmembers && (include_self || i != a.me);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        unsigned spins = 0;
        while (true) {
            bool done = !need || ld_sys_u64(mine + base + a.pe[i]) >= cnt[i];
            if (__all(done)) break;
            if ((++spins & 63u) == 0 && __builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (i == 0 && acquire) {
            // acquire at system scope: drop this CU's and XCD's stale copies of
            // peer data (redundant beside the system-coherent loads of the
            // members' buffers; kept unless the init test showed those fresh)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    return ok;
}

// Count this block in on a local counter; true for the grid's last block.
FUSED_HELPER bool last_block(unsigned long long *counter) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ int is_last;
    if (threadIdx.x == 0) {
        const uint64_t prev = __hip_atomic_fetch_add(counter, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        is_last = prev + 1 == gridDim.x;
        if (is_last) st_sys_u64(counter, 0);
    }
    __syncthreads();
    return is_last != 0;
}

FUSED_HELPER void publish(const MI355FusedArgs &a, const unsigned long long *cnt, int base) {
    // lanes of wave 0: one member each (this PE included)
    if (threadIdx.x < a.nmembers) st_sys_u64(a.sig[threadIdx.x] + base + a.pe[a.me], cnt[threadIdx.x]);
}

// Advance the pair counts (the call is over on every member), then report.
FUSED_HELPER void finish(const MI355FusedArgs &a, unsigned long long *mine, const unsigned long long *cnt, bool ok,
                       unsigned epoch) {
    if (ok && threadIdx.x < a.nmembers) st_sys_u64(mine + MI355_SIG_CALLS + a.pe[threadIdx.x], cnt[threadIdx.x]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        if (!ok) {
            st_sys_u64(mine + MI355_SIG_ERROR, 1);
            if (a.err_flag) __hip_atomic_store(a.err_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (a.host_flag)
            __hip_atomic_store(a.host_flag, ok ? epoch : (epoch | 0x80000000u), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Byte copy shared by `nblocks` blocks, this one being number `bi` of them:
// 16-byte vectors when both ends allow it, then the byte tail; stores
// write-through at system scope (the destination is read by peers or by the
// host next). A block that stored the byte tail (plain stores) releases at
// system scope.
// block_copy_issue only issues the stores (true if this thread stored a
// plain tail byte); block_drain waits for them and releases if needed.
__device__ bool block_copy_issue(void *dst, const void *src, uint64_t nbytes, unsigned bi, unsigned nblocks) {
    const bool vec = ((((uintptr_t)dst) | ((uintptr_t)src)) & 15) == 0;
    const uint64_t nv = vec ? nbytes / 16 : 0;
    for (uint64_t v = (uint64_t)bi * kBlock + threadIdx.x; v < nv; v += (uint64_t)nblocks * kBlock)
        st16_sys((u32x4 *)dst + v, ((const u32x4 *)src)[v]);
    bool plain = false;
    for (uint64_t b = nv * 16 + (uint64_t)bi * kBlock + threadIdx.x; b < nbytes;
         b += (uint64_t)nblocks * kBlock) {
        ((char *)dst)[b] = ((const char *)src)[b];
        plain = true;
    }
    return plain;
}

__device__ void block_drain(bool plain) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (__syncthreads_or(plain) && threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

FUSED_HELPER void block_copy(void *dst, const void *src, uint64_t nbytes, unsigned bi, unsigned nblocks) {
    block_drain(block_copy_issue(dst, src, nbytes, bi, nblocks));
}

// One call's parameters. The launched kernel's come from its arguments (the
// members' buffers in a.src/a.dst, offsets 0); a persistent server's
// (fused_server) from its mailbox, as symmetric-heap byte offsets added to
// the members' heap bases in a.src/a.dst.
struct Call {
    uint64_t soff, doff;  // byte offsets added to a.src[i] / a.dst[i]
    uint64_t n, shard;    // as MI355FusedArgs
    unsigned epoch;
    int oneshot;
};
__device__ __forceinline__ const char *src_of(const MI355FusedArgs &a, const Call &c, int i) {
    return (const char *)a.src[i] + c.soff;
}
__device__ __forceinline__ char *dst_of(const MI355FusedArgs &a, const Call &c, int i) {
    return (char *)a.dst[i] + c.doff;
}

// Member at position j of the fold order that starts with member `first`
// and continues with the others in member order (first = 0: member order;
// first = q: member q's reference order, reduce-op.c:226-264).
__device__ __forceinline__ int order_member(int j, int first) {
    return j == 0 ? first : (j - 1 < first ? j - 1 : j);
}

// Vector v of the shard starting at element lo, folded over every member in
// the order starting with `first`. kBatch members' vectors are loaded before
// any is folded, so their (xGMI) latencies overlap instead of adding up.
template <int OP, typename T>
__device__ __forceinline__ Pack<T> fold_vec(const MI355FusedArgs &a, const Call &c, uint64_t lo, uint64_t v, int first) {
    constexpr int V = 16 / sizeof(T);
    const int nm = a.nmembers;
    Pack<T> acc;
    for (int k0 = 0; k0 < nm; k0 += kBatch) {
        Pack<T> x[kBatch];
#pragma unroll
        for (int j = 0; j < kBatch; ++j)
            if (k0 + j < nm)
                x[j].v = ld16_sys_at(src_of(a, c, order_member(k0 + j, first)) + lo * sizeof(T), (uint32_t)(v * 16));
#pragma unroll
        for (int j = 0; j < kBatch; ++j) {
            if (k0 + j >= nm) break;
            if (k0 + j == 0) {
                acc = x[0];
            } else {
#pragma unroll
                for (int e = 0; e < V; ++e) acc.e[e] = apply<OP>(acc.e[e], x[j].e[e]);
            }
        }
    }
    return acc;
}

template <int OP, typename T>
__device__ __forceinline__ T fold_elem(const MI355FusedArgs &a, const Call &c, uint64_t i, int first) {
    const int nm = a.nmembers;
    T acc;
    for (int k0 = 0; k0 < nm; k0 += kBatch) {
        T x[kBatch];
#pragma unroll
        for (int j = 0; j < kBatch; ++j)
            if (k0 + j < nm) x[j] = ld_elem_sys((const T *)src_of(a, c, order_member(k0 + j, first)) + i);
#pragma unroll
        for (int j = 0; j < kBatch; ++j) {
            if (k0 + j >= nm) break;
            acc = k0 + j == 0 ? x[0] : apply<OP>(acc, x[j]);
        }
    }
    return acc;
}

// Where member q's version of element r of this PE's shard goes: its target
// shard for q == me, else slot (q < me ? q : q - 1) of this PE's version area.
template <typename T>
__device__ __forceinline__ T *version_elem(const MI355FusedArgs &a, const Call &c, int q, uint64_t r) {
    if (q == a.me) return (T *)dst_of(a, c, a.me) + (uint64_t)a.me * c.shard + r;
    return (T *)((char *)a.ver[a.me] + (uint64_t)(q < a.me ? q : q - 1) * c.shard * sizeof(T)) + r;
}

// Vector v of shard `me` in EVERY member's reference order. Up to kBatch
// members the sources are loaded once and all folds come from registers;
// beyond that (and for the software x87 type, whose fold is long code) one
// fold per member re-reads the vectors (cache hits after the first).
template <int OP, typename T>
__device__ __forceinline__ void versions_vec(const MI355FusedArgs &a, const Call &c, uint64_t lo, uint64_t v) {
    constexpr int V = 16 / sizeof(T);
    const int nm = a.nmembers;
    if constexpr (!std::is_same<T, x80>::value) {
        if (nm <= kBatch) {
            Pack<T> x[kBatch];
#pragma unroll
            for (int j = 0; j < kBatch; ++j)
                if (j < nm) x[j].v = ld16_sys_at(src_of(a, c, j) + lo * sizeof(T), (uint32_t)(v * 16));
#pragma unroll
            for (int q = 0; q < kBatch; ++q) {
                if (q >= nm) break;
                Pack<T> acc = x[q];
#pragma unroll
                for (int k = 0; k < kBatch; ++k) {
                    if (k >= nm) break;
                    if (k == q) continue;
#pragma unroll
                    for (int e = 0; e < V; ++e) acc.e[e] = apply<OP>(acc.e[e], x[k].e[e]);
                }
                st16_sys((u32x4 *)version_elem<T>(a, c, q, v * V), acc.v);
            }
            return;
        }
    }
    // this PE's own version last: in place (dst == src) it overwrites the
    // source vector the other folds still read
    for (int j = 0; j < nm; ++j) {
        const int q = j < a.me ? j : j + 1 < nm ? j + 1 : a.me;
        st16_sys((u32x4 *)version_elem<T>(a, c, q, v * V), fold_vec<OP, T>(a, c, lo, v, q).v);
    }
}

// The whole call, on every block of the grid (the launched kernel's and the
// server's). next_counts: this block ran the previous call of the same
// active set (a server's later calls), so every pair count is the one it
// held then plus one -- LDS keeps them, no read of CALLS.
template <int OP, typename T>
__device__ __forceinline__ void fused_body(const MI355FusedArgs &a, const Call &c, bool next_counts = false) {
    constexpr int V = 16 / sizeof(T);
    unsigned long long *mine = a.sig[a.me];
    __shared__ int ok_all;
    __shared__ unsigned long long cnt[MI355_FUSED_MAX_MEMBERS];
    if (threadIdx.x == 0) ok_all = 1;
    if (next_counts) {
        if (threadIdx.x < a.nmembers) ++cnt[threadIdx.x];
        __syncthreads();
    } else {
        load_counts(a, mine, cnt);
    }
    PHASE_MIN(c, 0);
    PHASE_MAX(c, 1);

    const bool staged = a.host_src != nullptr;
    if (staged) {
        // ---- stage in: this PE's host source -> its staging source (every
        // block; the host may have rewritten the source since the last call,
        // so drop stale cached copies first). The grid's last block then
        // announces arrival to every member, this PE included: the blocks
        // that read src[me] below wait for it like for the peers.
        if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        __syncthreads();
        block_copy((void *)src_of(a, c, a.me), a.host_src, c.n * sizeof(T), blockIdx.x, gridDim.x);
        if (last_block(mine + MI355_SIG_STAGE_COUNT)) {
            if (threadIdx.x < a.nmembers)
                st_sys_u64(a.sig[threadIdx.x] + MI355_SIG_ARRIVE + a.pe[a.me], cnt[threadIdx.x]);
        }
    } else if (blockIdx.x == 0) {
        // ---- arrive (the source was written before the kernel started)
        if (threadIdx.x < a.nmembers && threadIdx.x != a.me)
            st_sys_u64(a.sig[threadIdx.x] + MI355_SIG_ARRIVE + a.pe[a.me], cnt[threadIdx.x]);
    }
    __syncthreads();
    if (!wait_members(a, mine, cnt, MI355_SIG_ARRIVE, staged, !a.no_acquire)) ok_all = 0;
    __syncthreads();
    PHASE_MAX(c, 2);
    if (!ok_all) goto fail;

    {
        // ---- fold: one-shot = the whole array from every member's source
        // (no reduce-scatter/all-gather split, one flag exchange fewer);
        // otherwise shard `me` (the reduce-scatter leg). Ordered one-shot
        // folds in this PE's own reference order; ordered two-shot computes
        // every member's order of shard `me` (versions_vec).
        const bool oneshot = c.oneshot != 0;
        const bool versions = a.ordered != 0 && !oneshot;
        const int first = a.ordered != 0 && oneshot ? a.me : 0;
        bool tail_plain = false;
        const uint64_t lo = oneshot ? 0 : (uint64_t)a.me * c.shard;
        const uint64_t hi = oneshot ? c.n : (lo + c.shard < c.n ? lo + c.shard : c.n);
        // staged one-shot: nobody reads this PE's result but the caller, so
        // the fold writes it straight to the caller's target (host memory
        // over PCIe, or device memory) instead of to dst[me] and a stage-out
        // copy after this PE's AGDONE (round 6: BASELINE config 1's 4 KiB
        // call on shmem_malloc'd arrays)
        const bool direct_out = staged && oneshot && (((uintptr_t)a.host_dst) & 15) == 0;
        char *const out = direct_out ? (char *)a.host_dst : dst_of(a, c, a.me);
        if (hi > lo) {
            const uint64_t nv = (hi - lo) / V;
            u32x4 *d = (u32x4 *)(out + lo * sizeof(T));
            for (uint64_t v = (uint64_t)blockIdx.x * kBlock + threadIdx.x; v < nv;
                 v += (uint64_t)gridDim.x * kBlock) {
                if (versions) versions_vec<OP, T>(a, c, lo, v);
                else st16_sys(d + v, fold_vec<OP, T>(a, c, lo, v, first).v);
            }
            const uint64_t tail0 = lo + nv * V;
            if (tail0 < hi && blockIdx.x == 0 && threadIdx.x < hi - tail0) {
                const uint64_t i = tail0 + threadIdx.x;
                if (!versions) {
                    ((T *)out)[i] = fold_elem<OP, T>(a, c, i, first);
                } else {
                    for (int j = 0; j < a.nmembers; ++j) {  // own version last (in place, as versions_vec)
                        const int q = j < a.me ? j : j + 1 < a.nmembers ? j + 1 : a.me;
                        *version_elem<T>(a, c, q, i - lo) = fold_elem<OP, T>(a, c, i, q);
                    }
                }
            }
            if (tail0 < hi && blockIdx.x == 0) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // plain tail stores
            }
        }
        PHASE_MAX(c, 3);
        if (!oneshot) {
            if (last_block(mine + MI355_SIG_RS_COUNT)) publish(a, cnt, MI355_SIG_RSDONE);

            // ---- every shard is reduced
            if (!wait_members(a, mine, cnt, MI355_SIG_RSDONE, true, !a.no_acquire)) ok_all = 0;
            __syncthreads();
            PHASE_MAX(c, 4);
            if (!ok_all) goto fail;

            // ---- gather the other shards: one grid-stride loop over all of
            // them, from their owners' targets, or (ordered) from the slot of
            // this PE's version in the owners' version areas
            const uint64_t shard_v = c.shard / V;  // c.shard is a multiple of V
            const uint64_t total_v = shard_v * (uint64_t)a.nmembers;
            for (uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x; g < total_v;
                 g += (uint64_t)gridDim.x * kBlock) {
                const int j = (int)(g / shard_v);
                if (j == a.me) continue;
                const uint64_t r0 = (g - (uint64_t)j * shard_v) * V;  // element within shard j
                const uint64_t e0 = (uint64_t)j * c.shard + r0;
                if (e0 >= c.n) continue;
                const T *from = versions ? (const T *)((const char *)a.ver[j] +
                                                       (uint64_t)(a.me < j ? a.me : a.me - 1) * c.shard * sizeof(T)) - e0 + r0
                                         : (const T *)dst_of(a, c, j);
                if (e0 + V <= c.n) {
                    const u32x4 v = ld16_sys(from + e0);
                    st16_sys((u32x4 *)(dst_of(a, c, a.me) + e0 * sizeof(T)), v);
                } else {
                    for (uint64_t e = e0; e < c.n; ++e) ((T *)dst_of(a, c, a.me))[e] = ld_elem_sys(from + e);
                    tail_plain = true;
                }
            }
        }
        // one-shot: AGDONE below means "this PE has finished reading the
        // members' sources" -- every member waits for all of them before it
        // returns, as after the gather
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (__syncthreads_or(tail_plain) && threadIdx.x == 0)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // the element tail went through L2
        PHASE_MAX(c, 5);
        if (last_block(mine + MI355_SIG_AG_COUNT)) {
            publish(a, cnt, MI355_SIG_AGDONE);
            if (!staged || direct_out) {
                __syncthreads();
                if (!wait_members(a, mine, cnt, MI355_SIG_AGDONE, true, !a.no_acquire)) ok_all = 0;
                __syncthreads();
                PHASE_MAX(c, 6);
                PHASE_RESET_NEXT(c);
                finish(a, mine, cnt, ok_all != 0, c.epoch);
                return;
            }
        }
        if (!staged || direct_out) return;
        // ---- stage out (every block): dst[me] is complete once this PE's own
        // AGDONE slot shows this call (published above by the gather's last
        // block, after every block's write-through stores drained); acquire,
        // copy this block's part to the host target, count the blocks out;
        // the last one waits for every member's AGDONE and reports
        if (threadIdx.x == 0) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (ld_sys_u64(mine + MI355_SIG_AGDONE + a.pe[a.me]) < cnt[a.me]) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
                    ok_all = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        }
        __syncthreads();
        if (ok_all) block_copy(a.host_dst, dst_of(a, c, a.me), c.n * sizeof(T), blockIdx.x, gridDim.x);
        if (last_block(mine + MI355_SIG_STAGE_COUNT)) {
            if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            __syncthreads();
            if (!wait_members(a, mine, cnt, MI355_SIG_AGDONE, true, !a.no_acquire)) ok_all = 0;
            __syncthreads();
            finish(a, mine, cnt, ok_all != 0, c.epoch);
        }
        return;
    }
fail:
    finish(a, mine, cnt, false, c.epoch);
}

template <int OP, typename T>
__global__ __launch_bounds__(kBlock) void fused_allreduce(MI355FusedArgs a) {
    fused_body<OP, T>(a, Call{0, 0, a.n, a.shard, a.epoch, a.oneshot});
}

// ---------------------------------------------------------------------------
// persistent server (mi355_reduce.h, mi355_fused_server)
// ---------------------------------------------------------------------------
__device__ __forceinline__ unsigned ld_sys_u32(const unsigned *p) {
    return __hip_atomic_load(const_cast<unsigned *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys_u32(unsigned *p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Block 0 takes the next call from the host mailbox (or QUIT: on the host's
// command, or after idle_ticks without a call) and broadcasts it in the
// signal region; every other block waits for the broadcast. Both lines are
// read whole by lanes 0-15 of wave 0 (one 64-byte request) and count when
// their head and tail words both hold the awaited seq (written last) and the
// check word (dword 12) matches the call's dwords 1-11 (mi355_mailbox_check):
// a snapshot torn between an old and a new call is read again. Every block
// then holds the call in f[] (LDS). A broadcast seq only advances after the
// host saw the previous call complete, which needs every block, so no block
// can miss one.
__device__ __forceinline__ bool line_has(const unsigned *line, unsigned seq, unsigned &v) {
    const unsigned lane = threadIdx.x & 15;
    v = ld_sys_u32(line + lane);
    unsigned x = lane >= 1 && lane <= 11 ? v : 0u;
    x ^= __shfl_xor(x, 8, 16);
    x ^= __shfl_xor(x, 4, 16);
    x ^= __shfl_xor(x, 2, 16);
    x ^= __shfl_xor(x, 1, 16);
    const unsigned head = __shfl(v, 0), tail = __shfl(v, 15), check = __shfl(v, 12);
    return head == seq && tail == seq && check == (__shfl(x, 0) ^ (seq * 0x9E3779B1u));
}

FUSED_HELPER void server_next(const MI355FusedArgs &a, MI355ServerMailbox *mb, unsigned seq,
                            unsigned long long idle_ticks, unsigned *f) {
    unsigned *slot = (unsigned *)(a.sig[a.me] + MI355_SIG_SERVER);
    if (threadIdx.x < 64) {
        const unsigned lane = threadIdx.x;
        unsigned v = 0;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        if (blockIdx.x == 0) {
            const unsigned *box = (const unsigned *)mb;
            bool idle = false;
            while (!line_has(box, seq, v)) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) {
                    // final look: a call rung before this point is served;
                    // after it, the host sees EXITED and launches instead
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
                    if (line_has(box, seq, v)) break;
                    idle = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            if (idle && lane == 1) v = MI355_SERVER_QUIT;  // dword 1: cmd
            if (idle) {  // the broadcast's check word covers the QUIT (every lane shuffles: uniform)
                unsigned x = lane >= 1 && lane <= 11 ? v : 0u;
                x ^= __shfl_xor(x, 8, 16);
                x ^= __shfl_xor(x, 4, 16);
                x ^= __shfl_xor(x, 2, 16);
                x ^= __shfl_xor(x, 1, 16);
                const unsigned check = __shfl(x, 0) ^ (seq * 0x9E3779B1u);
                if (lane == 12) v = check;
            }
            // broadcast: the call (dwords 1-14), then head and tail
            if (lane >= 1 && lane < 15) st_sys_u32(slot + lane, v);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            if (lane == 0 || lane == 15) st_sys_u32(slot + lane, seq);
            if (lane < 16) f[lane] = v;
            const unsigned cmd = __shfl(v, 1);
            if (cmd != MI355_SERVER_RUN && lane == 0) {
                // every other block has its QUIT once it reads the broadcast;
                // tell the host which seq was not served
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                st_sys_u32(&mb->state_seq, idle ? seq : seq + 1);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                st_sys_u32(&mb->state, MI355_SERVER_EXITED);
            }
        } else {
            unsigned spins = 0;
            bool got = true;
            while (!line_has(slot, seq, v)) {
                // block 0 broadcasts a call or QUIT within idle_ticks (plus a
                // call's duration); this bound is only a safety net
                if ((++spins & 63u) == 0 && __builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks + idle_ticks) {
                    got = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            if (lane < 16) f[lane] = got ? v : (lane == 1 ? MI355_SERVER_QUIT : 0u);
        }
    }
    __syncthreads();
}

template <int OP, typename T>
__global__ __launch_bounds__(kBlock) void fused_server(MI355FusedArgs a, MI355ServerMailbox *mb, unsigned first_seq,
                                                       unsigned long long idle_ticks) {
    __shared__ unsigned f[16];  // the mailbox line (MI355ServerMailbox's first 16 dwords)
    for (unsigned seq = first_seq;; ++seq) {
        server_next(a, mb, seq, idle_ticks, f);
        if (f[1] != MI355_SERVER_RUN) return;
        auto u64 = [&](int w) { return (uint64_t)f[w] | ((uint64_t)f[w + 1] << 32); };
        const Call c{u64(2), u64(4), u64(6), u64(8), f[10], (int)f[11]};
        if (a.nmembers == 1) {
            // the 1-PE identity: nobody to wait for -- copy, count the
            // blocks out, the last one reports. The caller may have rewritten
            // the source since the last call (other XCDs' kernels, DMA): drop
            // this CU's and XCD's copies of it first
            if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            __syncthreads();
            block_copy(dst_of(a, c, 0), src_of(a, c, 0), c.n * sizeof(T), blockIdx.x, gridDim.x);
            if (last_block(a.sig[0] + MI355_SIG_AG_COUNT) && threadIdx.x == 0)
                __hip_atomic_store(a.host_flag, c.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        } else {
            fused_body<OP, T>(a, c, seq != first_seq);
        }
        __syncthreads();  // f[] is rewritten by the next server_next
    }
}

// One-launch pull collective: arrive, copy this member's segments (sources
// are peers' mapped buffers, read after the acquire in wait_members), then
// "done reading" (AGDONE) from every member before the call completes.
__global__ __launch_bounds__(kBlock) void fused_pull(MI355PullArgs p) {
    const MI355FusedArgs &a = p.m;
    unsigned long long *mine = a.sig[a.me];
    __shared__ int ok_all;
    __shared__ unsigned long long cnt[MI355_FUSED_MAX_MEMBERS];
    if (threadIdx.x == 0) ok_all = 1;
    load_counts(a, mine, cnt);
    if (blockIdx.x == 0 && threadIdx.x < a.nmembers && threadIdx.x != a.me)
        st_sys_u64(a.sig[threadIdx.x] + MI355_SIG_ARRIVE + a.pe[a.me], cnt[threadIdx.x]);
    __syncthreads();
    if (!wait_members(a, mine, cnt, MI355_SIG_ARRIVE, false)) ok_all = 0;
    __syncthreads();
    if (!ok_all) {  // this block timed out: report it (the host aborts the job)
        finish(a, mine, cnt, false, a.epoch);
        return;
    }
    {
        // every segment's loads in flight together (one segment per peer:
        // all links busy at once), one drain at the end
        bool plain = false;
        for (int k = 0; k < p.nseg; ++k) plain |= block_copy_issue(p.dst[k], p.src[k], p.nbytes[k], blockIdx.x, gridDim.x);
        block_drain(plain);
    }
    if (last_block(mine + MI355_SIG_AG_COUNT)) {
        publish(a, cnt, MI355_SIG_AGDONE);
        __syncthreads();
        if (!wait_members(a, mine, cnt, MI355_SIG_AGDONE, true)) ok_all = 0;
        __syncthreads();
        finish(a, mine, cnt, ok_all != 0, a.epoch);
    }
}

// Device barrier: one block; lanes of wave 0 handle one member each.
__global__ __launch_bounds__(64) void device_barrier(MI355FusedArgs a) {
    unsigned long long *mine = a.sig[a.me];
    __shared__ unsigned long long cnt[MI355_FUSED_MAX_MEMBERS];
    load_counts(a, mine, cnt);
    // the work queued before this kernel completed (kernel boundary); make
    // it visible at system scope before peers are told
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    if (threadIdx.x < a.nmembers && threadIdx.x != a.me)
        st_sys_u64(a.sig[threadIdx.x] + MI355_SIG_ARRIVE + a.pe[a.me], cnt[threadIdx.x]);
    const bool ok = wait_members(a, mine, cnt, MI355_SIG_ARRIVE, false);
    finish(a, mine, cnt, ok, a.epoch);
}

extern "C" void mi355i_take_launch_events(void **start_event, void **stop_event);  // combine.hip
extern "C" void mi355i_note_launch(const void *kernel);                           // combine.hip

// Launch, carrying the event pair armed by mi355_time_next_launch (if any)
// as hipExtLaunchKernel stamps: no marker packets on the stream.
template <typename K, typename P>
void launch_stamped(K kernel, unsigned grid, unsigned block, hipStream_t st, const P &p) {
    void *e0 = nullptr, *e1 = nullptr;
    mi355i_take_launch_events(&e0, &e1);
    mi355i_note_launch((const void *)kernel);
    if (e0 != nullptr || e1 != nullptr)
        hipExtLaunchKernelGGL(kernel, dim3(grid), dim3(block), 0, st, (hipEvent_t)e0, (hipEvent_t)e1, 0, p);
    else
        hipLaunchKernelGGL(kernel, dim3(grid), dim3(block), 0, st, p);
}

// Co-residency: every block of these grids waits for the grid's last block
// and for the other members, so all blocks of every such grid running on this
// GPU at once must be resident together. A launch is capped at the kernel's
// resident blocks per CU x CUs, divided among the `share` processes that may
// run such grids here at the same time. Resident blocks per CU: the occupancy
// query, but at most MI355_FUSED_RESIDENT_PER_CU (residency.h) -- 256-thread
// blocks are admitted per CU up to floor(800 / (ceil(sgpr / 16) * 16 + 16))
// (MI355X_MICROARCH.md "Residency"), which the query ignores (at 103-106
// SGPRs: 6 per CU where the query says 8; 9 PEs x 174 blocks on one GPU never
// all started) -- and one fewer as a margin. The build checks every such
// kernel's SGPR/VGPR/LDS use against the constant (tools/check_residency.py).
struct OccEntry {
    const void *fn;
    int blocks_per_cu;
};
OccEntry g_occ[256];
int g_nocc = 0;
int g_cus = 0;

unsigned coresident_grid(const void *fn, uint64_t want, int share) {
    if (g_cus == 0) {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        g_cus = cus;
    }
    int per_cu = -1;
    for (int i = 0; i < g_nocc; ++i)
        if (g_occ[i].fn == fn) per_cu = g_occ[i].blocks_per_cu;
    if (per_cu < 0) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, kBlock, 0) != hipSuccess || n < 1) n = 1;
        (void)hipGetLastError();
        if (n > MI355_FUSED_RESIDENT_PER_CU) n = MI355_FUSED_RESIDENT_PER_CU;
        per_cu = n > 1 ? n - 1 : 1;
        if (g_nocc < 256) g_occ[g_nocc++] = OccEntry{fn, per_cu};
    }
    uint64_t cap = (uint64_t)per_cu * (uint64_t)g_cus / (uint64_t)(share > 1 ? share : 1);
    if (cap < 1) cap = 1;
    if (want > cap) want = cap;
    return (unsigned)(want < 1 ? 1 : want);
}

template <typename T>
int launch_op(const MI355FusedArgs &a, unsigned grid, hipStream_t st) {
    switch (a.op) {
#define CASE(O)                                                                        \
    case O:                                                                            \
        if constexpr (valid_pair<O, T>()) {                                           \
            auto k = fused_allreduce<O, T>;                                            \
            launch_stamped(k, coresident_grid((const void *)k, grid, a.share), kBlock, st, a); \
            break;                                                                     \
        } else {                                                                       \
            return MI355_E_UNSUP;                                                      \
        }
        CASE(MI355_OP_SUM)
        CASE(MI355_OP_PROD)
        CASE(MI355_OP_AND)
        CASE(MI355_OP_OR)
        CASE(MI355_OP_XOR)
        CASE(MI355_OP_MIN)
        CASE(MI355_OP_MAX)
#undef CASE
    default: return MI355_E_INVAL;
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

template <typename T>
int launch_server(const MI355FusedArgs &a, MI355ServerMailbox *mb, unsigned first_seq, unsigned long long idle_ticks,
                  unsigned grid, hipStream_t st) {
    switch (a.op) {
#define CASE(O)                                                                                          \
    case O:                                                                                              \
        if constexpr (valid_pair<O, T>()) {                                                             \
            auto k = fused_server<O, T>;                                                                 \
            mi355i_note_launch((const void *)k);                                                         \
            hipLaunchKernelGGL(k, dim3(coresident_grid((const void *)k, grid, a.share)), dim3(kBlock), 0, st, a, mb, \
                               first_seq, idle_ticks);                                                   \
            break;                                                                                       \
        } else {                                                                                         \
            return MI355_E_UNSUP;                                                                        \
        }
        CASE(MI355_OP_SUM)
        CASE(MI355_OP_PROD)
        CASE(MI355_OP_AND)
        CASE(MI355_OP_OR)
        CASE(MI355_OP_XOR)
        CASE(MI355_OP_MIN)
        CASE(MI355_OP_MAX)
#undef CASE
    default: return MI355_E_INVAL;
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

constexpr int kMaxPoke = 1024;
struct PokeParams {
    unsigned long long *ptr[kMaxPoke];
    unsigned long long value;
    unsigned long long *out;
    int n;
};

__global__ __launch_bounds__(kBlock) void poke_kernel(PokeParams p) {
    for (int i = threadIdx.x; i < p.n; i += kBlock) st_sys_u64(p.ptr[i], p.value);
}

__global__ __launch_bounds__(kBlock) void peek_kernel(PokeParams p) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    for (int i = threadIdx.x; i < p.n; i += kBlock) p.out[i] = ld_sys_u64(p.ptr[i]);
}

// Plain (cached) loads, as the folds and gathers read peers' buffers: no
// fence, no scope bits, so a line another agent rewrote can come from this
// XCD's L2. Every block reads every word (blocks are dealt over the XCDs).
__global__ __launch_bounds__(kBlock) void peek_cached_kernel(PokeParams p) {
    for (int i = threadIdx.x; i < p.n; i += kBlock) p.out[(size_t)blockIdx.x * p.n + i] = *p.ptr[i];
}

// System-coherent loads, no fence: what the fused kernel's reads of the
// members' buffers see without an acquire (the init coherence test).
__global__ __launch_bounds__(kBlock) void peek_sysload_kernel(PokeParams p) {
    for (int i = threadIdx.x; i < p.n; i += kBlock) p.out[(size_t)blockIdx.x * p.n + i] = ld_sys_u64(p.ptr[i]);
}

// ---- the caller's producer path (runtime.c producer_test, round 4) ----
// A caller writes its source with plain stores in its own kernel, then calls;
// the peers then read it. mark_plain_kernel is that caller kernel: block b
// stores value + b into dst[b] with a plain (write-back, L2-cached) store,
// the blocks dealt over the XCDs.
__global__ __launch_bounds__(64) void mark_plain_kernel(unsigned long long *dst, int words, unsigned long long value) {
    if (threadIdx.x == 0 && (int)blockIdx.x < words) dst[blockIdx.x] = value + blockIdx.x;
}

constexpr int kProducerMaxPes = 64;
struct ProducerReadParams {
    const unsigned long long *src[kProducerMaxPes];
    const unsigned long long *flag;  // this PE's flag words [np], or null: no wait
    unsigned long long token, timeout_ticks;
    unsigned long long *out;         // [3][nblocks][np * words] + 1 timeout word
    int np, words;
};

// The peers' side: (optionally) wait on this PE's signal words for every
// member's token -- the fused kernel's ARRIVE wait -- then read every
// member's marker words three ways: plain loads without an acquire (as a
// multi-launch fold would without mi355_acquire_system), 16-byte system-
// coherent loads (the fused kernel's folds, ld16_sys_at), and plain loads
// after a system-scope acquire (the multi-launch schedules' protocol).
__global__ __launch_bounds__(kBlock) void producer_read_kernel(ProducerReadParams p) {
    __shared__ int timed_out;
    if (threadIdx.x == 0) timed_out = 0;
    __syncthreads();
    if (p.flag != nullptr && threadIdx.x < 64) {
        const int q = threadIdx.x;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        unsigned spins = 0;
        while (true) {
            const bool done = q >= p.np || ld_sys_u64(p.flag + q) == p.token;
            if (__all(done)) break;
            if ((++spins & 63u) == 0 && __builtin_amdgcn_s_memrealtime() - t0 > p.timeout_ticks) {
                if (q == 0) timed_out = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
    const int per = p.np * p.words;
    unsigned long long *plain = p.out + (size_t)blockIdx.x * per;
    unsigned long long *sys = p.out + ((size_t)gridDim.x + blockIdx.x) * per;
    unsigned long long *acq = p.out + ((size_t)2 * gridDim.x + blockIdx.x) * per;
    for (int i = threadIdx.x; i < per; i += kBlock) plain[i] = p.src[i / p.words][i % p.words];
    for (int i = 2 * threadIdx.x; i < per; i += 2 * kBlock) {  // words even: pairs never straddle members
        const int q = i / p.words, w = i % p.words;
        const u32x4 v = ld16_sys_at((const char *)p.src[q], (uint32_t)(w * 8));
        sys[i] = (unsigned long long)v.x | ((unsigned long long)v.y << 32);
        sys[i + 1] = (unsigned long long)v.z | ((unsigned long long)v.w << 32);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: this CU's L1, its XCD's L2
    __syncthreads();
    for (int i = threadIdx.x; i < per; i += kBlock) acq[i] = p.src[i / p.words][i % p.words];
    if (threadIdx.x == 0 && timed_out) p.out[(size_t)3 * gridDim.x * per] = 1;
}

}  // namespace

extern "C" int mi355_mark_plain(unsigned long long *dst, int words, unsigned long long value, void *stream) {
    if (dst == nullptr || words < 1 || words > 1024) return MI355_E_INVAL;
    hipLaunchKernelGGL(mark_plain_kernel, dim3(words), dim3(64), 0, (hipStream_t)stream, dst, words, value);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

extern "C" int mi355_producer_read(const unsigned long long *const *src, int np, int words,
                                   const unsigned long long *flag, unsigned long long token,
                                   unsigned long long timeout_ticks, unsigned long long *out, int nblocks,
                                   void *stream) {
    if (src == nullptr || out == nullptr || np < 1 || np > kProducerMaxPes || words < 2 || (words & 1) != 0 ||
        nblocks < 1 || nblocks > 256)
        return MI355_E_INVAL;
    ProducerReadParams p{};
    for (int q = 0; q < np; ++q) p.src[q] = src[q];
    p.flag = flag;
    p.token = token;
    p.timeout_ticks = timeout_ticks;
    p.out = out;
    p.np = np;
    p.words = words;
    hipLaunchKernelGGL(producer_read_kernel, dim3(nblocks), dim3(kBlock), 0, (hipStream_t)stream, p);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

extern "C" int mi355_poke(unsigned long long *const *dst, int n, unsigned long long value, void *stream) {
    if (n < 0 || n > kMaxPoke || (n > 0 && dst == nullptr)) return MI355_E_INVAL;
    if (n == 0) return 0;
    PokeParams p{};
    for (int i = 0; i < n; ++i) p.ptr[i] = dst[i];
    p.value = value;
    p.n = n;
    hipLaunchKernelGGL(poke_kernel, dim3(1), dim3(kBlock), 0, (hipStream_t)stream, p);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

extern "C" int mi355_peek(const unsigned long long *const *src, int n, unsigned long long *out, void *stream) {
    if (n < 0 || n > kMaxPoke || (n > 0 && (src == nullptr || out == nullptr))) return MI355_E_INVAL;
    if (n == 0) return 0;
    PokeParams p{};
    for (int i = 0; i < n; ++i) p.ptr[i] = const_cast<unsigned long long *>(src[i]);
    p.out = out;
    p.n = n;
    hipLaunchKernelGGL(peek_kernel, dim3(1), dim3(kBlock), 0, (hipStream_t)stream, p);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

extern "C" int mi355_peek_cached(const unsigned long long *const *src, int n, unsigned long long *out, int nblocks,
                                 void *stream) {
    if (n < 0 || n > kMaxPoke || nblocks < 1 || nblocks > 256 || (n > 0 && (src == nullptr || out == nullptr)))
        return MI355_E_INVAL;
    if (n == 0) return 0;
    PokeParams p{};
    for (int i = 0; i < n; ++i) p.ptr[i] = const_cast<unsigned long long *>(src[i]);
    p.out = out;
    p.n = n;
    hipLaunchKernelGGL(peek_cached_kernel, dim3(nblocks), dim3(kBlock), 0, (hipStream_t)stream, p);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

extern "C" int mi355_peek_sysload(const unsigned long long *const *src, int n, unsigned long long *out, int nblocks,
                                  void *stream) {
    if (n < 0 || n > kMaxPoke || nblocks < 1 || nblocks > 256 || (n > 0 && (src == nullptr || out == nullptr)))
        return MI355_E_INVAL;
    if (n == 0) return 0;
    PokeParams p{};
    for (int i = 0; i < n; ++i) p.ptr[i] = const_cast<unsigned long long *>(src[i]);
    p.out = out;
    p.n = n;
    hipLaunchKernelGGL(peek_sysload_kernel, dim3(nblocks), dim3(kBlock), 0, (hipStream_t)stream, p);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

extern "C" int mi355_fused_allreduce(const MI355FusedArgs *a, void *stream) {
    if (a == nullptr || !mi355_op_supported(a->op, a->dtype)) return MI355_E_UNSUP;
    if (a->nmembers < 2 || a->nmembers > MI355_FUSED_MAX_MEMBERS || a->me < 0 || a->me >= a->nmembers)
        return MI355_E_INVAL;
    const size_t es = mi355_dtype_size(a->dtype);
    if (a->shard == 0 || (a->shard * es) % 16 != 0) return MI355_E_INVAL;
    // the folds address a member's buffer with 32-bit buffer offsets (ld16_sys_at)
    if (a->n * es >= kMaxFusedBytes || (uint64_t)a->shard * es * (uint64_t)a->nmembers >= kMaxFusedBytes)
        return MI355_E_INVAL;
    for (int i = 0; i < a->nmembers; ++i)
        if (a->src[i] == nullptr || a->dst[i] == nullptr || a->sig[i] == nullptr ||
            (((uintptr_t)a->src[i] | (uintptr_t)a->dst[i]) & 15) != 0 || a->pe[i] < 0 ||
            a->pe[i] >= MI355_SIG_RSDONE)
            return MI355_E_INVAL;
    if (a->oneshot && a->src[a->me] == a->dst[a->me]) return MI355_E_INVAL;  // it overwrites dst while peers read src
    if (a->ordered && !a->oneshot)
        for (int i = 0; i < a->nmembers; ++i)
            if (a->ver[i] == nullptr || ((uintptr_t)a->ver[i] & 15) != 0) return MI355_E_INVAL;
    // enough blocks for the larger of the two legs (one-shot: the whole
    // array), all of them co-resident
    const uint64_t vecs = a->oneshot ? (a->n * es + 15) / 16 : (a->shard * es / 16) * (uint64_t)(a->nmembers - 1);
    uint64_t grid = (vecs + kBlock - 1) / kBlock;
    if (grid < 1) grid = 1;
    if (grid > MI355_FUSED_MAX_BLOCKS) grid = MI355_FUSED_MAX_BLOCKS;
    hipStream_t st = (hipStream_t)stream;
    switch (a->dtype) {
    case MI355_SHORT: return launch_op<int16_t>(*a, (unsigned)grid, st);
    case MI355_INT: return launch_op<int32_t>(*a, (unsigned)grid, st);
    case MI355_LONG:
    case MI355_LONGLONG: return launch_op<int64_t>(*a, (unsigned)grid, st);
    case MI355_FLOAT: return launch_op<float>(*a, (unsigned)grid, st);
    case MI355_DOUBLE: return launch_op<double>(*a, (unsigned)grid, st);
    case MI355_LONGDOUBLE: return launch_op<x80>(*a, (unsigned)grid, st);
    case MI355_COMPLEXF: return launch_op<cplxf>(*a, (unsigned)grid, st);
    case MI355_COMPLEXD: return launch_op<cplxd>(*a, (unsigned)grid, st);
    default: return MI355_E_INVAL;
    }
}

extern "C" int mi355_fused_pull(const MI355PullArgs *p, void *stream) {
    if (p == nullptr || p->nseg < 0 || p->nseg > MI355_PULL_MAX_SEGS) return MI355_E_INVAL;
    const MI355FusedArgs *a = &p->m;
    if (a->nmembers < 2 || a->nmembers > MI355_FUSED_MAX_MEMBERS || a->me < 0 || a->me >= a->nmembers)
        return MI355_E_INVAL;
    uint64_t total = 0;
    for (int k = 0; k < p->nseg; ++k) {
        if (p->nbytes[k] != 0 && (p->dst[k] == nullptr || p->src[k] == nullptr)) return MI355_E_INVAL;
        total += p->nbytes[k];
    }
    for (int i = 0; i < a->nmembers; ++i)
        if (a->sig[i] == nullptr || a->pe[i] < 0 || a->pe[i] >= MI355_SIG_RSDONE) return MI355_E_INVAL;
    uint64_t grid = (total + 16 * kBlock - 1) / (16 * kBlock);
    if (grid < 1) grid = 1;
    if (grid > MI355_FUSED_MAX_BLOCKS) grid = MI355_FUSED_MAX_BLOCKS;
    launch_stamped(fused_pull, coresident_grid((const void *)fused_pull, grid, a->share), kBlock, (hipStream_t)stream,
                   *p);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

extern "C" int mi355_device_barrier(const MI355FusedArgs *a, void *stream) {
    if (a == nullptr || a->nmembers < 1 || a->nmembers > MI355_FUSED_MAX_MEMBERS || a->me < 0 ||
        a->me >= a->nmembers)
        return MI355_E_INVAL;
    for (int i = 0; i < a->nmembers; ++i)
        if (a->sig[i] == nullptr || a->pe[i] < 0 || a->pe[i] >= MI355_SIG_RSDONE) return MI355_E_INVAL;
    hipLaunchKernelGGL(device_barrier, dim3(1), dim3(64), 0, (hipStream_t)stream, *a);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

extern "C" int mi355_fused_server(const MI355FusedArgs *a, MI355ServerMailbox *mbox, unsigned first_seq,
                                  unsigned long long idle_ticks, unsigned long long grid_vecs, void *stream) {
    if (a == nullptr || mbox == nullptr || !mi355_op_supported(a->op, a->dtype)) return MI355_E_UNSUP;
    // one member: the 1-PE identity (one-shot copy of the caller's source)
    if (a->nmembers < 1 || a->nmembers > MI355_FUSED_MAX_MEMBERS || a->me < 0 || a->me >= a->nmembers)
        return MI355_E_INVAL;
    if (a->host_src != nullptr || a->host_dst != nullptr || a->host_flag == nullptr) return MI355_E_INVAL;
    if (grid_vecs * 16 >= kMaxFusedBytes) return MI355_E_INVAL;   // 32-bit buffer offsets (ld16_sys_at)
    for (int i = 0; i < a->nmembers; ++i)
        if (a->src[i] == nullptr || a->dst[i] == nullptr || a->sig[i] == nullptr ||
            (((uintptr_t)a->src[i] | (uintptr_t)a->dst[i]) & 15) != 0 || a->pe[i] < 0 ||
            a->pe[i] >= MI355_SIG_RSDONE)
            return MI355_E_INVAL;
    if (a->ordered)
        for (int i = 0; i < a->nmembers; ++i)
            if (a->ver[i] == nullptr || ((uintptr_t)a->ver[i] & 15) != 0) return MI355_E_INVAL;
    // the grid a launched call moving grid_vecs 16-byte vectors per PE gets
    uint64_t grid = (grid_vecs + kBlock - 1) / kBlock;
    if (grid < 1) grid = 1;
    if (grid > MI355_FUSED_MAX_BLOCKS) grid = MI355_FUSED_MAX_BLOCKS;
    hipStream_t st = (hipStream_t)stream;
    switch (a->dtype) {
    case MI355_SHORT: return launch_server<int16_t>(*a, mbox, first_seq, idle_ticks, (unsigned)grid, st);
    case MI355_INT: return launch_server<int32_t>(*a, mbox, first_seq, idle_ticks, (unsigned)grid, st);
    case MI355_LONG:
    case MI355_LONGLONG: return launch_server<int64_t>(*a, mbox, first_seq, idle_ticks, (unsigned)grid, st);
    case MI355_FLOAT: return launch_server<float>(*a, mbox, first_seq, idle_ticks, (unsigned)grid, st);
    case MI355_DOUBLE: return launch_server<double>(*a, mbox, first_seq, idle_ticks, (unsigned)grid, st);
    case MI355_LONGDOUBLE: return launch_server<x80>(*a, mbox, first_seq, idle_ticks, (unsigned)grid, st);
    case MI355_COMPLEXF: return launch_server<cplxf>(*a, mbox, first_seq, idle_ticks, (unsigned)grid, st);
    case MI355_COMPLEXD: return launch_server<cplxd>(*a, mbox, first_seq, idle_ticks, (unsigned)grid, st);
    default: return MI355_E_INVAL;
    }
}

#ifdef MI355_FUSED_PHASES
// probe build: copy the phase ring out (64 calls x 8 stamps)
extern "C" int mi355_fused_phases(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), sizeof(g_phase)) == hipSuccess ? 0 : -1;
}
extern "C" int mi355_fused_phases_reset(void) {
    unsigned long long h[64][8];
    for (int i = 0; i < 64; ++i)
        for (int k = 0; k < 8; ++k) h[i][k] = k == 0 ? ~0ull : 0ull;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_phase), h, sizeof(h)) == hipSuccess ? 0 : -1;
}
#endif
