// x80_lane_probe.hip -- why did per-lane divergence between x80.h's fast and
// general paths give nondeterministic one-ulp errors (ADVICE
// round 2)? Folds three operand arrays, acc = (a op b) op c, op = x87 add or
// multiply, with three kernels:
//   general  every lane takes the general (branchy, soft-float) path
//   vote     the library's form: fast path when every lane of the wave can
//   lane     per-lane choice: fast where possible, general elsewhere (diverges)
//   lane_asm lane, storing through the library's inline-asm write-through
//            store (combine_kernels.h st16_fold: global_store_dwordx4 sc1 +
//            s_nop 1), as the fold kernels store
// and compares each against the host's x87 (long double (a op b) op c) on
// every element, several repeats. Prints mismatch counts per repeat and the
// first mismatches' bits. (Round 3: the branchy general path of round 2 gave
// ~0.7 % wrong products here, varying per run; the vote and lane kernels
// matched the host.)
//
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I osss-gasnet_amd/csrc \
//          tools/x80_lane_probe.hip -o tools/x80_lane_probe
// run:   tools/x80_lane_probe [n] [reps]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "x80.h"

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));            \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

enum { K_GENERAL = 0, K_VOTE = 1, K_LANE = 2, K_LANE_ASM = 3 };
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

template <int OP, int K>
__device__ __forceinline__ x80 op2(const x80 &a, const x80 &b) {
    if constexpr (K == K_VOTE) {
        return x80_op<OP>(a, b);
    } else if constexpr (K == K_GENERAL) {
        return OP == 0 ? x80d::add_general(a, b) : x80d::mul_general(a, b);
    } else {
        x80 r = a;
        const bool ok = OP == 0 ? x80d::add_fast(a, b, r) : x80d::mul_fast(a, b, r);
        if (!ok) r = OP == 0 ? x80d::add_general(a, b) : x80d::mul_general(a, b);
        return r;
    }
}

template <int OP, int K>
__global__ __launch_bounds__(256) void fold3(const x80 *a, const x80 *b, const x80 *c, x80 *out, uint64_t n) {
    constexpr int KK = K == K_LANE_ASM ? K_LANE : K;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const x80 r = op2<OP, KK>(op2<OP, KK>(a[i], b[i]), c[i]);
        if constexpr (K == K_LANE_ASM) {
            u32x4v v;
            __builtin_memcpy(&v, &r, 16);
            asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(out + i), "v"(v) : "memory");
        } else {
            out[i] = r;
        }
    }
}

static uint64_t sm_state;
static uint64_t splitmix() {
    uint64_t z = (sm_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <int OP, int K>
static void run(const x80 *a, const x80 *b, const x80 *c, x80 *out, uint64_t n) {
    hipLaunchKernelGGL((fold3<OP, K>), dim3(2048), dim3(256), 0, 0, a, b, c, out, n);
    CK(hipGetLastError());
}

static void hexx(const x80 &v, char *buf) { snprintf(buf, 32, "%04x:%016llx", v.se, (unsigned long long)v.m); }

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 200000;
    const int reps = argc > 2 ? atoi(argv[2]) : 6;
    x80 *h[3];
    sm_state = 99;
    for (int k = 0; k < 3; ++k) {
        h[k] = (x80 *)calloc(n, sizeof(x80));
        for (uint64_t i = 0; i < n; ++i) {
            uint64_t m = splitmix();
            uint16_t se = (uint16_t)splitmix();
            if (splitmix() & 1) {  // half near 1.0: the fast path's domain
                se = (uint16_t)((se & 0x8000) | (16383 + (int)(splitmix() % 140) - 70));
                m |= 1ull << 63;
            }
            h[k][i].m = m;
            h[k][i].se = se;
        }
    }
    x80 *d[3], *o[4];
    for (int k = 0; k < 3; ++k) {
        CK(hipMalloc(&d[k], n * sizeof(x80)));
        CK(hipMemcpy(d[k], h[k], n * sizeof(x80), hipMemcpyHostToDevice));
    }
    for (int k = 0; k < 4; ++k) CK(hipMalloc(&o[k], n * sizeof(x80)));
    x80 *t = (x80 *)calloc(n, sizeof(x80));
    x80 *truth[2];
    for (int op = 0; op < 2; ++op) {  // the host x87
        truth[op] = (x80 *)calloc(n, sizeof(x80));
        for (uint64_t i = 0; i < n; ++i) {
            long double v[3];
            for (int k = 0; k < 3; ++k) {
                memset(&v[k], 0, sizeof v[k]);
                memcpy(&v[k], &h[k][i], 10);
            }
            volatile long double r = op == 0 ? (v[0] + v[1]) + v[2] : (v[0] * v[1]) * v[2];
            long double rr = r;
            memcpy(&truth[op][i], &rr, 10);
        }
    }
    const char *kn[4] = {"general", "vote", "lane", "lane_asm"};
    long total_bad[2][4] = {{0}};  // [op][kernel]
    for (int op = 0; op < 2; ++op) {
        for (int rep = 0; rep < reps; ++rep) {
            if (op == 0) {
                run<0, K_GENERAL>(d[0], d[1], d[2], o[0], n);
                run<0, K_VOTE>(d[0], d[1], d[2], o[1], n);
                run<0, K_LANE>(d[0], d[1], d[2], o[2], n);
                run<0, K_LANE_ASM>(d[0], d[1], d[2], o[3], n);
            } else {
                run<1, K_GENERAL>(d[0], d[1], d[2], o[0], n);
                run<1, K_VOTE>(d[0], d[1], d[2], o[1], n);
                run<1, K_LANE>(d[0], d[1], d[2], o[2], n);
                run<1, K_LANE_ASM>(d[0], d[1], d[2], o[3], n);
            }
            CK(hipDeviceSynchronize());
            const x80 *g = truth[op];
            for (int k = 0; k < 4; ++k) {
                CK(hipMemcpy(t, o[k], n * sizeof(x80), hipMemcpyDeviceToHost));
                long bad = 0;
                for (uint64_t i = 0; i < n; ++i) {
                    if (g[i].m == t[i].m && g[i].se == t[i].se) continue;
                    if (bad < 3) {
                        char s0[32], s1[32], s2[32], sg[32], st[32];
                        hexx(h[0][i], s0), hexx(h[1][i], s1), hexx(h[2][i], s2), hexx(g[i], sg), hexx(t[i], st);
                        printf("  %s %s rep %d i %llu ops %s %s %s host %s %s %s\n", op ? "mul" : "add", kn[k], rep,
                               (unsigned long long)i, s0, s1, s2, sg, kn[k], st);
                    }
                    ++bad;
                }
                total_bad[op][k] += bad;
                printf("%s rep %d %s vs host x87: %ld mismatches of %llu\n", op ? "mul" : "add", rep, kn[k], bad,
                       (unsigned long long)n);
            }
        }
    }
    printf("SUMMARY vs host x87, add: general %ld vote %ld lane %ld lane_asm %ld; mul: general %ld vote %ld lane %ld "
           "lane_asm %ld (over %d reps x %llu)\n", total_bad[0][0], total_bad[0][1], total_bad[0][2], total_bad[0][3],
           total_bad[1][0], total_bad[1][1], total_bad[1][2], total_bad[1][3], reps, (unsigned long long)n);
    return 0;
}
