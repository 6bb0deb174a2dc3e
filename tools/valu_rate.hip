// valu_rate.hip -- issue cost of the integer VALU instruction kinds the x87
// software arithmetic is made of (x80.h), on MI355X: cycles per wave64
// instruction per SIMD with W waves per SIMD, from s_memtime (shader clock
// ticks) around a loop of 8 independent chains, plus the wall-clock rate. Gives
// the VALU roofline the long double every-member fold is held against
// (DESIGN.md section 4). Measurement tool.
//   build: hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o tools/valu_rate
//   run:   tools/valu_rate [waves_per_simd ...]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                     \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

constexpr int kIters = 2048;
constexpr int kPerIter = 16;  // instructions per loop iteration (8 chains x 2)

enum Kind { ADD32, XOR32, SHL64, ADDC, CNDMASK, CMP64, MIX, MAD64, MULLO, MULHI, MOV, ADD32_E64, XOR32_E64,
            CNDMASK_VCC, CMP32, CNDMASK_VCC_STATIC, NKIND };
static const char *kNames[NKIND] = {"v_add_u32", "v_xor_b32", "v_lshlrev_b64", "v_add_co+v_addc_co",
                                    "v_cndmask_b32(sgpr mask)", "v_cmp_gt_u64(sgpr)", "x87-add mix",
                                    "v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mov_b32",
                                    "v_add_u32_e64", "v_xor_b32_e64", "v_cndmask_b32_e32(vcc)", "v_cmp_gt_u32(sgpr)",
                                    "v_cndmask_b32_e32(vcc set before the loop)"};

template <int K>
__global__ __launch_bounds__(256) void rate(uint64_t *out, uint64_t *cyc, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13,
             a6 = a0 * 17, a7 = a0 * 19;
    uint64_t b0 = a0, b1 = a1, b2 = a2, b3 = a3, b4 = a4, b5 = a5, b6 = a6, b7 = a7;
    const uint32_t k = seed | 1;
    if constexpr (K == CNDMASK_VCC_STATIC)
        asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\ts_nop 4" : : "v"(a0), "v"(k) : "vcc");
    uint64_t t0;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0));
    for (int it = 0; it < kIters; ++it) {
        if constexpr (K == ADD32) {
#define OP2(x) asm volatile("v_add_u32 %0, %0, %1\n\tv_add_u32 %0, %0, %1" : "+v"(x) : "v"(k))
            OP2(a0); OP2(a1); OP2(a2); OP2(a3); OP2(a4); OP2(a5); OP2(a6); OP2(a7);
#undef OP2
        } else if constexpr (K == XOR32) {
#define OP2(x) asm volatile("v_xor_b32 %0, %0, %1\n\tv_xor_b32 %0, %0, %1" : "+v"(x) : "v"(k))
            OP2(a0); OP2(a1); OP2(a2); OP2(a3); OP2(a4); OP2(a5); OP2(a6); OP2(a7);
#undef OP2
        } else if constexpr (K == SHL64) {
#define OP2(x) asm volatile("v_lshlrev_b64 %0, 1, %0\n\tv_lshlrev_b64 %0, 1, %0" : "+v"(x))
            OP2(b0); OP2(b1); OP2(b2); OP2(b3); OP2(b4); OP2(b5); OP2(b6); OP2(b7);
#undef OP2
        } else if constexpr (K == ADDC) {
            // 4 independent 64-bit adds, each a carry pair (VCC between them)
#define OP2(x, y)                                                                               \
    asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %2, vcc" : "+v"(x), "+v"(y) \
                 : "v"(k) : "vcc")
            OP2(a0, a1); OP2(a2, a3); OP2(a4, a5); OP2(a6, a7);
            OP2(a0, a1); OP2(a2, a3); OP2(a4, a5); OP2(a6, a7);
#undef OP2
        } else if constexpr (K == CNDMASK) {
            uint64_t m;
            asm volatile("v_cmp_gt_u32 %0, %1, %2" : "=s"(m) : "v"(a0), "v"(k));
#define OP2(x) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2\n\tv_cndmask_b32_e64 %0, %1, %0, %2" \
                            : "+v"(x) : "v"(k), "s"(m))
            OP2(a1); OP2(a2); OP2(a3); OP2(a4); OP2(a5); OP2(a6); OP2(a7); OP2(a0);
#undef OP2
        } else if constexpr (K == CMP64) {
            uint64_t m0, m1;
#define OP2(x, y) asm volatile("v_cmp_gt_u64 %0, %2, %3\n\tv_cmp_gt_u64 %1, %3, %2" : "=s"(m0), "=s"(m1) \
                               : "v"(x), "v"(y))
            OP2(b0, b1); OP2(b2, b3); OP2(b4, b5); OP2(b6, b7);
            OP2(b1, b2); OP2(b3, b4); OP2(b5, b6); OP2(b7, b0);
#undef OP2
            a0 ^= (uint32_t)m0;
            a1 ^= (uint32_t)m1;
        } else if constexpr (K == MAD64) {
#define OP2(x) asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0\n\tv_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(x) \
                            : "v"(k) : "vcc")
            OP2(b0); OP2(b1); OP2(b2); OP2(b3); OP2(b4); OP2(b5); OP2(b6); OP2(b7);
#undef OP2
        } else if constexpr (K == MULLO) {
#define OP2(x) asm volatile("v_mul_lo_u32 %0, %0, %1\n\tv_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(k))
            OP2(a0); OP2(a1); OP2(a2); OP2(a3); OP2(a4); OP2(a5); OP2(a6); OP2(a7);
#undef OP2
        } else if constexpr (K == MULHI) {
#define OP2(x) asm volatile("v_mul_hi_u32 %0, %0, %1\n\tv_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(k))
            OP2(a0); OP2(a1); OP2(a2); OP2(a3); OP2(a4); OP2(a5); OP2(a6); OP2(a7);
#undef OP2
        } else if constexpr (K == ADD32_E64) {
            // the same operation as ADD32 in the 8-byte (VOP3) encoding
#define OP2(x) asm volatile("v_add_u32_e64 %0, %0, %1\n\tv_add_u32_e64 %0, %0, %1" : "+v"(x) : "v"(k))
            OP2(a0); OP2(a1); OP2(a2); OP2(a3); OP2(a4); OP2(a5); OP2(a6); OP2(a7);
#undef OP2
        } else if constexpr (K == XOR32_E64) {
#define OP2(x) asm volatile("v_xor_b32_e64 %0, %0, %1\n\tv_xor_b32_e64 %0, %0, %1" : "+v"(x) : "v"(k))
            OP2(a0); OP2(a1); OP2(a2); OP2(a3); OP2(a4); OP2(a5); OP2(a6); OP2(a7);
#undef OP2
        } else if constexpr (K == CNDMASK_VCC) {
            // the VOP2 form: the lane mask in VCC, written once per iteration
            asm volatile("v_cmp_gt_u32 vcc, %0, %1" : : "v"(a0), "v"(k) : "vcc");
#define OP2(x) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc\n\tv_cndmask_b32_e32 %0, %1, %0, vcc" \
                            : "+v"(x) : "v"(k) : "vcc")
            OP2(a1); OP2(a2); OP2(a3); OP2(a4); OP2(a5); OP2(a6); OP2(a7); OP2(a0);
#undef OP2
        } else if constexpr (K == CNDMASK_VCC_STATIC) {
            // VCC read only, written once before the timed loop
#define OP2(x) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc\n\tv_cndmask_b32_e32 %0, %1, %0, vcc" \
                            : "+v"(x) : "v"(k))
            OP2(a1); OP2(a2); OP2(a3); OP2(a4); OP2(a5); OP2(a6); OP2(a7); OP2(a0);
#undef OP2
        } else if constexpr (K == CMP32) {
            uint64_t m0, m1;
#define OP2(x, y) asm volatile("v_cmp_gt_u32 %0, %2, %3\n\tv_cmp_gt_u32 %1, %3, %2" : "=s"(m0), "=s"(m1) \
                               : "v"(x), "v"(y))
            OP2(a0, a1); OP2(a2, a3); OP2(a4, a5); OP2(a6, a7);
            OP2(a1, a2); OP2(a3, a4); OP2(a5, a6); OP2(a7, a0);
#undef OP2
            a0 ^= (uint32_t)m0;
            a1 ^= (uint32_t)m1;
        } else if constexpr (K == MOV) {
#define OP2(x, y) asm volatile("v_mov_b32 %0, %1\n\tv_mov_b32 %1, %0" : "+v"(x), "+v"(y))
            OP2(a0, a1); OP2(a2, a3); OP2(a4, a5); OP2(a6, a7);
            OP2(a1, a2); OP2(a3, a4); OP2(a5, a6); OP2(a7, a0);
#undef OP2
        } else {
            // the x87 fast add's mix per 16: 2 addc-pairs, 2 xor, 2 cndmask,
            // 2 sub, 2 64-bit shifts, 1 or, 1 ffbh, 1 cmp64, 1 max, 1 and
            uint64_t m;
            asm volatile(
                "v_add_co_u32 %0, vcc, %0, %10\n\tv_addc_co_u32 %1, vcc, %1, %10, vcc\n\t"
                "v_xor_b32 %2, %2, %10\n\tv_xor_b32 %3, %3, %10\n\t"
                "v_cmp_gt_u64 %9, %8, %7\n\t"
                "v_sub_u32 %4, %4, %10\n\tv_sub_u32 %5, %5, %10\n\t"
                "v_lshlrev_b64 %7, 1, %7\n\tv_lshrrev_b64 %8, 1, %8\n\t"
                "v_or_b32 %6, %6, %10\n\tv_ffbh_u32 %2, %3\n\t"
                "v_cndmask_b32_e64 %4, %4, %5, %9\n\tv_cndmask_b32_e64 %5, %6, %5, %9\n\t"
                "v_add_co_u32 %2, vcc, %2, %10\n\tv_addc_co_u32 %3, vcc, %3, %10, vcc\n\t"
                "v_max_i32 %6, %6, %4"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(b0), "+v"(b1),
                  "=&s"(m)
                : "v"(k)
                : "vcc");
        }
    }
    uint64_t t1;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1));
    const uint64_t r = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) ^ b0 ^ b1 ^ b2 ^ b3 ^ b4 ^ b5 ^ b6 ^ b7;
    const unsigned gw = (blockIdx.x * blockDim.x + threadIdx.x) / 64;
    if ((threadIdx.x & 63) == 0) cyc[gw] = t1 - t0;
    if (r == 0x12345) out[0] = r;  // keeps the chains live
}

template <int K>
static void run(int waves_per_simd, int cus) {
    const int blocks = cus * waves_per_simd;  // 256 threads = one wave per SIMD per block
    const int nw = blocks * 4;
    uint64_t *out, *cyc;
    CHECK(hipMalloc(&out, 8));
    CHECK(hipMalloc(&cyc, nw * 8));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    rate<K><<<blocks, 256>>>(out, cyc, 7);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    rate<K><<<blocks, 256>>>(out, cyc, 9);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    uint64_t *h = (uint64_t *)malloc(nw * 8);
    CHECK(hipMemcpy(h, cyc, nw * 8, hipMemcpyDeviceToHost));
    double mean = 0;
    for (int i = 0; i < nw; ++i) mean += (double)h[i];
    mean /= nw;
    const double insts = (double)kIters * kPerIter;  // per wave
    // each SIMD ran waves_per_simd waves concurrently: SIMD cycles per instruction
    const double cpi_simd = mean / (insts * waves_per_simd);
    const double wall_rate = (double)nw * insts / (ms * 1e-3);  // wave-instructions / s, whole chip
    printf("{\"kind\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_inst_per_simd\": %.3f, "
           "\"wave_cycles_per_inst\": %.2f, \"chip_wave_insts_per_s\": %.4g, \"ms\": %.3f}\n",
           kNames[K], waves_per_simd, cpi_simd, mean / insts, wall_rate, ms);
    free(h);
    CHECK(hipFree(out));
    CHECK(hipFree(cyc));
}

template <int K>
static void sweep(int argc, char **argv, int cus) {
    for (int i = 1; i < argc; ++i) run<K>(atoi(argv[i]), cus);
}

int main(int argc, char **argv) {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const char *defs[] = {"", "1", "2", "4", "8"};
    if (argc < 2) {
        argc = 5;
        argv = (char **)defs;
    }
    sweep<ADD32>(argc, argv, cus);
    sweep<XOR32>(argc, argv, cus);
    sweep<SHL64>(argc, argv, cus);
    sweep<ADDC>(argc, argv, cus);
    sweep<CNDMASK>(argc, argv, cus);
    sweep<CMP64>(argc, argv, cus);
    sweep<MIX>(argc, argv, cus);
    sweep<MAD64>(argc, argv, cus);
    sweep<MULLO>(argc, argv, cus);
    sweep<MULHI>(argc, argv, cus);
    sweep<MOV>(argc, argv, cus);
    sweep<ADD32_E64>(argc, argv, cus);
    sweep<XOR32_E64>(argc, argv, cus);
    sweep<CNDMASK_VCC>(argc, argv, cus);
    sweep<CMP32>(argc, argv, cus);
    sweep<CNDMASK_VCC_STATIC>(argc, argv, cus);
    return 0;
}
