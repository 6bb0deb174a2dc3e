/* bench_loop.c -- the timed loop of bench.py, in C.
 *
 * Not part of libshmem_reduce.so: a separate libshmem_bench.so that calls the
 * public entry point exactly as an OpenSHMEM C program does (the reference's
 * callers are C programs), so the per-call time bench.py reports is the
 * library's entry-to-return time with no Python/ctypes marshalling in it
 * (~2 us per call through ctypes, profiles/r01/overhead*.txt).
 *
 * The caller (bench.py) still brackets the loop with shmem_barrier_all and a
 * device synchronize on both sides and takes its own wall clock around it.
 */
#define _POSIX_C_SOURCE 199309L /* clock_gettime under -std=c11 */
#include <stddef.h>
#include <time.h>

#include <shmem.h>

/* K back-to-back shmem_double_sum_to_all calls with identical arguments;
 * pWrk/pSync as a conforming caller passes them. */
void shmemb_double_sum_loop (double *target, double *source, int nreduce, int PE_start, int logPE_stride,
                             int PE_size, double *pWrk, long *pSync, int iters)
{
    for (int i = 0; i < iters; ++i)
        shmem_double_sum_to_all (target, source, nreduce, PE_start, logPE_stride, PE_size, pWrk, pSync);
}

/* K calls taking npairs disjoint (target, source) pairs in turn: call i
 * reduces sources[i % npairs] into targets[i % npairs]. With npairs x 2 S
 * well beyond the 256 MiB Infinity Cache, every call streams its buffers from
 * HBM (bench.py's headline_rotating leg); otherwise the same call. */
void shmemb_double_sum_rotating (double **targets, double **sources, int npairs, int nreduce, int PE_start,
                                 int logPE_stride, int PE_size, double *pWrk, long *pSync, int iters)
{
    for (int i = 0; i < iters; ++i)
        shmem_double_sum_to_all (targets[i % npairs], sources[i % npairs], nreduce, PE_start, logPE_stride,
                                 PE_size, pWrk, pSync);
}

/* The same calls, each timed on its own (CLOCK_MONOTONIC, entry to return):
 * us[i] = call i's duration in microseconds. For the distribution (median,
 * tails) beside the bracketed mean of the loop above (median over
 * the timed reps); a separate run, so the clock reads stay out of the
 * headline's timed region. */
void shmemb_double_sum_times (double *target, double *source, int nreduce, int PE_start, int logPE_stride,
                              int PE_size, double *pWrk, long *pSync, int iters, double *us)
{
    struct timespec t0, t1;
    for (int i = 0; i < iters; ++i) {
        clock_gettime (CLOCK_MONOTONIC, &t0);
        shmem_double_sum_to_all (target, source, nreduce, PE_start, logPE_stride, PE_size, pWrk, pSync);
        clock_gettime (CLOCK_MONOTONIC, &t1);
        us[i] = (double) (t1.tv_sec - t0.tv_sec) * 1e6 + (double) (t1.tv_nsec - t0.tv_nsec) * 1e-3;
    }
}

/* BASELINE config 4's op-coverage pair, same shape of loop */
void shmemb_float_max_loop (float *target, float *source, int nreduce, int PE_start, int logPE_stride,
                            int PE_size, float *pWrk, long *pSync, int iters)
{
    for (int i = 0; i < iters; ++i)
        shmem_float_max_to_all (target, source, nreduce, PE_start, logPE_stride, PE_size, pWrk, pSync);
}

void shmemb_longlong_and_loop (long long *target, long long *source, int nreduce, int PE_start, int logPE_stride,
                               int PE_size, long long *pWrk, long *pSync, int iters)
{
    for (int i = 0; i < iters; ++i)
        shmem_longlong_and_to_all (target, source, nreduce, PE_start, logPE_stride, PE_size, pWrk, pSync);
}

/* BASELINE config 1's call: shmem_int_sum_to_all (4 KiB at 2 PEs) */
void shmemb_int_sum_loop (int *target, int *source, int nreduce, int PE_start, int logPE_stride, int PE_size,
                          int *pWrk, long *pSync, int iters)
{
    for (int i = 0; i < iters; ++i)
        shmem_int_sum_to_all (target, source, nreduce, PE_start, logPE_stride, PE_size, pWrk, pSync);
}
