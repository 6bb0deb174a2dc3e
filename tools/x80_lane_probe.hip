// x80_lane_probe.hip -- the mechanism behind round 2's nondeterministic x87
// errors. Folds three operand arrays,
// acc = (a op b) op c, op = x87 add or multiply, with these kernels:
//   general  every lane takes the general path
//   vote     the library's form: fast path when every lane of the wave can
//   lane     per-lane choice: fast where possible, general elsewhere (diverges)
//   lane_asm lane, storing through the library's inline-asm write-through
//            store (combine_kernels.h st16_fold: global_store_dwordx4 sc1 +
//            s_nop 1), as the fold kernels store
//   hwid     general, also recording each element's HW_ID (wave slot, SIMD,
//            CU) and XCC_ID, to place the mismatches on the hardware
// and compares each against the host's x87 (long double (a op b) op c) on
// every element, several repeats. Per repeat: mismatch count, split by the
// element's block (< 256: the grid's first block on each CU; >= 256: the
// rest), and the first mismatches' bits.
//
// Round 4 adds the experiment that names the mechanism: before every kernel,
// optionally run `regscrub` (x80_regscrub.h), which fills every VGPR and AGPR
// of every SIMD with a fixed pattern. A kernel that reads a register it never
// wrote returns whatever the register's previous occupant left there, which
// differs per run (which wave of which earlier kernel last held those
// physical registers); scrubbing makes that value the pattern, the same on
// every run and every slot. A kernel that reads only what it wrote is not
// affected by the scrub.
//
// build (round-2 header, the "before"; or -I osss-gasnet_amd/csrc for today's):
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I tools/x80_round2 -I tools \
//         tools/x80_lane_probe.hip -o tools/x80_lane_probe_r2
// run:   x80_lane_probe [n] [reps] [grid] [scrub: none|zero|ones|a5] [kernels: gvlah] [code object]
// With a code object (tools/x80_isa_variants.py: this program's own device
// assembly, reassembled, optionally with s_nop inserted at chosen sites), the
// `general` kernels come from it instead of this binary (hipModuleLaunchKernel);
// "-" for none. [lds]: dynamic LDS bytes per block of the general and hwid
// kernels -- above half the CU's 160 KiB only one block fits per CU, so every
// wave runs alone on its SIMD and the later blocks wait for the earlier ones.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "x80.h"
#include "x80_regscrub.h"

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));            \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

enum { K_GENERAL = 0, K_VOTE = 1, K_LANE = 2, K_LANE_ASM = 3, K_HWID = 4, NK = 5 };
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
__global__ __launch_bounds__(256) void fold3(const x80 *a, const x80 *b, const x80 *c, x80 *out, uint32_t *hw,
                                             uint64_t n) {
    constexpr int KK = K == K_LANE_ASM ? K_LANE : K == K_HWID ? K_GENERAL : K;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const x80 r = op2<OP, KK>(op2<OP, KK>(a[i], b[i]), c[i]);
        if constexpr (K == K_LANE_ASM) {
            u32x4v v;
            __builtin_memcpy(&v, &r, 16);
            asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(out + i), "v"(v) : "memory");
        } else {
            out[i] = r;
        }
        if constexpr (K == K_HWID) {
            uint32_t id, xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            hw[2 * i] = id;
            hw[2 * i + 1] = xcc;
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

static int g_grid = 2048;
static unsigned g_lds = 0;  // dynamic LDS per block of the general kernels: > 80 KiB admits one block per CU
static hipFunction_t g_ext[2] = {nullptr, nullptr};  // general add / mul from an external code object
static int g_scrub = -1;  // -1: none, else the pattern's index
static const uint32_t kPatterns[3] = {0x00000000u, 0xFFFFFFFFu, 0xA5A5A5A5u};

template <int OP, int K>
static void run(const x80 *a, const x80 *b, const x80 *c, x80 *out, uint32_t *hw, uint64_t n) {
    if (g_scrub >= 0) {
        hipLaunchKernelGGL(regscrub, dim3(4096), dim3(256), 0, 0, kPatterns[g_scrub]);
        CK(hipGetLastError());
    }
    if (K == K_GENERAL && g_ext[OP] != nullptr) {
        void *args[] = {(void *)&a, (void *)&b, (void *)&c, (void *)&out, (void *)&hw, (void *)&n};
        CK(hipModuleLaunchKernel(g_ext[OP], g_grid, 1, 1, 256, 1, 1, g_lds, 0, args, nullptr));
        return;
    }
    hipLaunchKernelGGL((fold3<OP, K>), dim3(g_grid), dim3(256), K == K_GENERAL || K == K_HWID ? g_lds : 0, 0, a, b, c,
                       out, hw, n);
    CK(hipGetLastError());
}

static void hexx(const x80 &v, char *buf) { snprintf(buf, 32, "%04x:%016llx", v.se, (unsigned long long)v.m); }

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 200000;
    const int reps = argc > 2 ? atoi(argv[2]) : 6;
    g_grid = argc > 3 ? atoi(argv[3]) : 2048;
    const char *scrub = argc > 4 ? argv[4] : "none";
    const char *which = argc > 5 ? argv[5] : "gvlah";
    g_scrub = !strcmp(scrub, "zero") ? 0 : !strcmp(scrub, "ones") ? 1 : !strcmp(scrub, "a5") ? 2 : -1;
    bool want[NK] = {strchr(which, 'g') != 0, strchr(which, 'v') != 0, strchr(which, 'l') != 0,
                     strchr(which, 'a') != 0, strchr(which, 'h') != 0};
    const char *co = argc > 6 && strcmp(argv[6], "-") != 0 ? argv[6] : nullptr;
    g_lds = argc > 7 ? (unsigned)atoi(argv[7]) : 0;
    if (co != nullptr) {
        hipModule_t mod;
        CK(hipModuleLoad(&mod, co));
        CK(hipModuleGetFunction(&g_ext[0], mod, "_Z5fold3ILi0ELi0EEvPK3x80S2_S2_PS0_Pjm"));
        CK(hipModuleGetFunction(&g_ext[1], mod, "_Z5fold3ILi1ELi0EEvPK3x80S2_S2_PS0_Pjm"));
    }
    printf("CONFIG n %llu reps %d grid %d scrub %s kernels %s code object %s dynamic LDS %u\n", (unsigned long long)n,
           reps, g_grid, scrub, which, co ? co : "(built in)", g_lds);
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
    x80 *d[3], *o[NK];
    uint32_t *dhw;
    for (int k = 0; k < 3; ++k) {
        CK(hipMalloc(&d[k], n * sizeof(x80)));
        CK(hipMemcpy(d[k], h[k], n * sizeof(x80), hipMemcpyHostToDevice));
    }
    for (int k = 0; k < NK; ++k) CK(hipMalloc(&o[k], n * sizeof(x80)));
    CK(hipMalloc(&dhw, n * 8));
    uint32_t *hhw = (uint32_t *)calloc(n, 8);
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
    const char *kn[NK] = {"general", "vote", "lane", "lane_asm", "hwid"};
    long total_bad[2][NK] = {{0}};  // [op][kernel]
    long total_first[2][NK] = {{0}};  // mismatches in blocks < 256 (grid's first block per CU)
    long wave_hist[2][16] = {{0}};  // hwid kernel: mismatches by HW_ID.WAVE_ID (slot in the SIMD)
    long wave_all[16] = {0};        // hwid kernel: elements by WAVE_ID
    for (int op = 0; op < 2; ++op) {
        for (int rep = 0; rep < reps; ++rep) {
            for (int k = 0; k < NK; ++k) {
                if (!want[k]) continue;
                CK(hipMemset(o[k], 0, n * sizeof(x80)));
            }
#define RUN_ALL(OP)                                                                       \
    do {                                                                                  \
        if (want[0]) run<OP, K_GENERAL>(d[0], d[1], d[2], o[0], dhw, n);                  \
        if (want[1]) run<OP, K_VOTE>(d[0], d[1], d[2], o[1], dhw, n);                     \
        if (want[2]) run<OP, K_LANE>(d[0], d[1], d[2], o[2], dhw, n);                     \
        if (want[3]) run<OP, K_LANE_ASM>(d[0], d[1], d[2], o[3], dhw, n);                 \
        if (want[4]) run<OP, K_HWID>(d[0], d[1], d[2], o[4], dhw, n);                     \
    } while (0)
            if (op == 0) RUN_ALL(0);
            else RUN_ALL(1);
            CK(hipDeviceSynchronize());
            if (want[4]) CK(hipMemcpy(hhw, dhw, n * 8, hipMemcpyDeviceToHost));
            const x80 *g = truth[op];
            for (int k = 0; k < NK; ++k) {
                if (!want[k]) continue;
                CK(hipMemcpy(t, o[k], n * sizeof(x80), hipMemcpyDeviceToHost));
                long bad = 0, first = 0;
                for (uint64_t i = 0; i < n; ++i) {
                    if (k == K_HWID && op == 0 && rep == 0) ++wave_all[hhw[2 * i] & 15];
                    if (g[i].m == t[i].m && g[i].se == t[i].se) continue;
                    const uint64_t blk = (i / 256) % (uint64_t)g_grid;
                    if (blk < 256) ++first;
                    if (k == K_HWID) ++wave_hist[op][hhw[2 * i] & 15];
                    if (bad < 3) {
                        char s0[32], s1[32], s2[32], sg[32], st[32];
                        hexx(h[0][i], s0), hexx(h[1][i], s1), hexx(h[2][i], s2), hexx(g[i], sg), hexx(t[i], st);
                        printf("  %s %s rep %d i %llu block %llu ops %s %s %s host %s %s %s", op ? "mul" : "add",
                               kn[k], rep, (unsigned long long)i, (unsigned long long)blk, s0, s1, s2, sg, kn[k], st);
                        if (k == K_HWID)
                            printf(" hw_id %08x (wave %u simd %u cu %u se %u) xcc %u", hhw[2 * i], hhw[2 * i] & 15,
                                   (hhw[2 * i] >> 4) & 3, (hhw[2 * i] >> 8) & 15, (hhw[2 * i] >> 13) & 7,
                                   hhw[2 * i + 1] & 15);
                        printf("\n");
                    }
                    ++bad;
                }
                total_bad[op][k] += bad;
                total_first[op][k] += first;
                printf("%s rep %d %s vs host x87: %ld mismatches of %llu (%ld in blocks < 256)\n", op ? "mul" : "add",
                       rep, kn[k], bad, (unsigned long long)n, first);
            }
        }
    }
    printf("SUMMARY grid %d scrub %s vs host x87 (mismatches / of them in blocks < 256), over %d reps x %llu:\n", g_grid,
           scrub, reps, (unsigned long long)n);
    for (int op = 0; op < 2; ++op) {
        printf("  %s:", op ? "mul" : "add");
        for (int k = 0; k < NK; ++k)
            if (want[k]) printf(" %s %ld/%ld", kn[k], total_bad[op][k], total_first[op][k]);
        printf("\n");
    }
    if (want[4]) {
        printf("  hwid kernel, by WAVE_ID (slot of the wave in its SIMD): elements / add mismatches / mul mismatches:");
        for (int w = 0; w < 16; ++w)
            if (wave_all[w] || wave_hist[0][w] || wave_hist[1][w])
                printf(" [%d] %ld/%ld/%ld", w, wave_all[w], wave_hist[0][w], wave_hist[1][w]);
        printf("\n");
    }
    return 0;
}
