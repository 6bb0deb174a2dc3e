// Residency probe for tests/test_residency.py: two kernels named like the
// library's spin-waiting grids, one with a normal SGPR budget and one whose
// inline asm clobbers s0-s101 (about the 106 SGPRs of fused_allreduce, which
// admits 6 blocks of 256 threads per CU). tools/check_residency.py must pass
// both at MI355_FUSED_RESIDENT_PER_CU = 6 and fail the heavy one at 7.
#include <hip/hip_runtime.h>

__global__ __launch_bounds__(256) void fused_allreduce_light(int *p) {
    if (p) p[threadIdx.x] = (int)threadIdx.x;
}

__global__ __launch_bounds__(256) void fused_allreduce_heavy(int *p) {
    asm volatile("" ::: "s0", "s1", "s2", "s3", "s4", "s5", "s6", "s7", "s8", "s9", "s10", "s11", "s12", "s13", "s14", "s15", "s16", "s17", "s18", "s19", "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28", "s29", "s30", "s31", "s32", "s33", "s34", "s35", "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95", "s96", "s97", "s98", "s99", "s100", "s101", "memory");
    if (p) p[threadIdx.x] = (int)threadIdx.x;
}
