/*
 * pshmem.h -- profiling (PSHMEM) names of the reduction surface.
 *
 * The reference exports every reduction as a strong pshmem_ symbol with the
 * shmem_ name as a weak alias (src/reduce/reduce-op.c:291-380; declarations
 * src/pshmem.h:545-735). libshmem_reduce.so does the same, so a tool can
 * interpose shmem_* and forward to pshmem_*.
 */
#ifndef _PSHMEM_H
#define _PSHMEM_H 1

#include <shmem.h>

#ifdef __cplusplus
extern "C" {
#endif

void pstart_pes (int npes);
void pshmem_init (void);
void pshmem_finalize (void);
void pshmem_global_exit (int status);
int pshmem_my_pe (void);
int pshmem_n_pes (void);
void *pshmem_malloc (size_t size);
void pshmem_free (void *ptr);
void pshmem_barrier_all (void);
void pshmem_barrier (int PE_start, int logPE_stride, int PE_size, long *pSync);
void pshmem_quiet (void);

void pshmem_putmem (void *dest, const void *src, size_t nelems, int pe);
void pshmem_getmem (void *dest, const void *src, size_t nelems, int pe);
void pshmem_put32 (void *dest, const void *src, size_t nelems, int pe);
void pshmem_put64 (void *dest, const void *src, size_t nelems, int pe);
void pshmem_put128 (void *dest, const void *src, size_t nelems, int pe);
void pshmem_get32 (void *dest, const void *src, size_t nelems, int pe);
void pshmem_get64 (void *dest, const void *src, size_t nelems, int pe);
void pshmem_get128 (void *dest, const void *src, size_t nelems, int pe);
void pshmem_char_put (char *dest, const char *src, size_t nelems, int pe);
void pshmem_short_put (short *dest, const short *src, size_t nelems, int pe);
void pshmem_int_put (int *dest, const int *src, size_t nelems, int pe);
void pshmem_long_put (long *dest, const long *src, size_t nelems, int pe);
void pshmem_longlong_put (long long *dest, const long long *src, size_t nelems, int pe);
void pshmem_longdouble_put (long double *dest, const long double *src, size_t nelems, int pe);
void pshmem_double_put (double *dest, const double *src, size_t nelems, int pe);
void pshmem_float_put (float *dest, const float *src, size_t nelems, int pe);
void pshmem_char_get (char *dest, const char *src, size_t nelems, int pe);
void pshmem_short_get (short *dest, const short *src, size_t nelems, int pe);
void pshmem_int_get (int *dest, const int *src, size_t nelems, int pe);
void pshmem_long_get (long *dest, const long *src, size_t nelems, int pe);
void pshmem_longlong_get (long long *dest, const long long *src, size_t nelems, int pe);
void pshmem_longdouble_get (long double *dest, const long double *src, size_t nelems, int pe);
void pshmem_double_get (double *dest, const double *src, size_t nelems, int pe);
void pshmem_float_get (float *dest, const float *src, size_t nelems, int pe);
void pshmem_broadcast64 (void *target, const void *source, size_t nelems, int PE_root, int PE_start,
                         int logPE_stride, int PE_size, long *pSync);
void pshmem_broadcast32 (void *target, const void *source, size_t nelems, int PE_root, int PE_start,
                         int logPE_stride, int PE_size, long *pSync);
void pshmem_fcollect64 (void *target, const void *source, size_t nelems, int PE_start, int logPE_stride,
                        int PE_size, long *pSync);
void pshmem_fcollect32 (void *target, const void *source, size_t nelems, int PE_start, int logPE_stride,
                        int PE_size, long *pSync);
void pshmem_collect64 (void *target, const void *source, size_t nelems, int PE_start, int logPE_stride,
                       int PE_size, long *pSync);
void pshmem_collect32 (void *target, const void *source, size_t nelems, int PE_start, int logPE_stride,
                       int PE_size, long *pSync);

    void pshmem_short_sum_to_all (short *target, short *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            short *pWrk, long *pSync);
    void pshmem_int_sum_to_all (int *target, int *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            int *pWrk, long *pSync);
    void pshmem_long_sum_to_all (long *target, long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long *pWrk, long *pSync);
    void pshmem_longlong_sum_to_all (long long *target, long long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long long *pWrk, long *pSync);
    void pshmem_float_sum_to_all (float *target, float *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            float *pWrk, long *pSync);
    void pshmem_double_sum_to_all (double *target, double *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            double *pWrk, long *pSync);
    void pshmem_longdouble_sum_to_all (long double *target, long double *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long double *pWrk, long *pSync);
    void pshmem_complexf_sum_to_all (COMPLEXIFY (float) *target, COMPLEXIFY (float) *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            COMPLEXIFY (float) *pWrk, long *pSync);
    void pshmem_complexd_sum_to_all (COMPLEXIFY (double) *target, COMPLEXIFY (double) *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            COMPLEXIFY (double) *pWrk, long *pSync);
    void pshmem_short_prod_to_all (short *target, short *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            short *pWrk, long *pSync);
    void pshmem_int_prod_to_all (int *target, int *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            int *pWrk, long *pSync);
    void pshmem_long_prod_to_all (long *target, long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long *pWrk, long *pSync);
    void pshmem_longlong_prod_to_all (long long *target, long long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long long *pWrk, long *pSync);
    void pshmem_float_prod_to_all (float *target, float *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            float *pWrk, long *pSync);
    void pshmem_double_prod_to_all (double *target, double *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            double *pWrk, long *pSync);
    void pshmem_longdouble_prod_to_all (long double *target, long double *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long double *pWrk, long *pSync);
    void pshmem_complexf_prod_to_all (COMPLEXIFY (float) *target, COMPLEXIFY (float) *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            COMPLEXIFY (float) *pWrk, long *pSync);
    void pshmem_complexd_prod_to_all (COMPLEXIFY (double) *target, COMPLEXIFY (double) *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            COMPLEXIFY (double) *pWrk, long *pSync);
    void pshmem_short_and_to_all (short *target, short *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            short *pWrk, long *pSync);
    void pshmem_int_and_to_all (int *target, int *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            int *pWrk, long *pSync);
    void pshmem_long_and_to_all (long *target, long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long *pWrk, long *pSync);
    void pshmem_longlong_and_to_all (long long *target, long long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long long *pWrk, long *pSync);
    void pshmem_short_or_to_all (short *target, short *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            short *pWrk, long *pSync);
    void pshmem_int_or_to_all (int *target, int *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            int *pWrk, long *pSync);
    void pshmem_long_or_to_all (long *target, long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long *pWrk, long *pSync);
    void pshmem_longlong_or_to_all (long long *target, long long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long long *pWrk, long *pSync);
    void pshmem_short_xor_to_all (short *target, short *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            short *pWrk, long *pSync);
    void pshmem_int_xor_to_all (int *target, int *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            int *pWrk, long *pSync);
    void pshmem_long_xor_to_all (long *target, long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long *pWrk, long *pSync);
    void pshmem_longlong_xor_to_all (long long *target, long long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long long *pWrk, long *pSync);
    void pshmem_short_max_to_all (short *target, short *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            short *pWrk, long *pSync);
    void pshmem_int_max_to_all (int *target, int *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            int *pWrk, long *pSync);
    void pshmem_long_max_to_all (long *target, long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long *pWrk, long *pSync);
    void pshmem_longlong_max_to_all (long long *target, long long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long long *pWrk, long *pSync);
    void pshmem_float_max_to_all (float *target, float *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            float *pWrk, long *pSync);
    void pshmem_double_max_to_all (double *target, double *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            double *pWrk, long *pSync);
    void pshmem_longdouble_max_to_all (long double *target, long double *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long double *pWrk, long *pSync);
    void pshmem_short_min_to_all (short *target, short *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            short *pWrk, long *pSync);
    void pshmem_int_min_to_all (int *target, int *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            int *pWrk, long *pSync);
    void pshmem_long_min_to_all (long *target, long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long *pWrk, long *pSync);
    void pshmem_longlong_min_to_all (long long *target, long long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long long *pWrk, long *pSync);
    void pshmem_float_min_to_all (float *target, float *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            float *pWrk, long *pSync);
    void pshmem_double_min_to_all (double *target, double *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            double *pWrk, long *pSync);
    void pshmem_longdouble_min_to_all (long double *target, long double *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long double *pWrk, long *pSync);

#ifdef __cplusplus
}
#endif

#endif /* _PSHMEM_H */
