/*
 * shmem.h -- OpenSHMEM 1.3 reduction surface of the MI355X reduction path.
 *
 * Drop-in for the reduction subset of the reference header
 * (openshmem-org/osss-gasnet src/shmem.h):
 *   - constants           src/shmem.h:1495-1505 (values identical, LP64)
 *   - 44 *_to_all          src/shmem.h:1507-1743 (signatures identical)
 *   - _SHMEM_* aliases    src/shmem.h:2210-2218
 *   - the minimal runtime  src/shmem.h:156-328 (start_pes/init/finalize/
 *     my_pe/n_pes), :692-797 (barrier_all, barrier, quiet), :974-993
 *     (shmem_malloc/shmem_free)
 *
 * Everything here is implemented in libshmem_reduce.so. The element-wise
 * combine runs as HIP kernels on the PE's GPU (gfx950); see DESIGN.md.
 */
#ifndef _SHMEM_H
#define _SHMEM_H 1

#include <sys/types.h>
#include <stddef.h>

/* C and C++ spell complex numbers differently (reference src/shmem.h:74-80) */
#ifdef __cplusplus
# include <complex>
# define COMPLEXIFY(T) std::complex<T>
#else
# include <complex.h>
# define COMPLEXIFY(T) T _Complex
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define SHMEM_MAJOR_VERSION 1
#define SHMEM_MINOR_VERSION 3
#define SHMEM_MAX_NAME_LEN 64
#define SHMEM_VENDOR_STRING "MI355X OpenSHMEM reduction path"

/* Fortran values are multiples of these (reference src/shmem.h:1495) */
#define SHMEM_INTERNAL_F2C_SCALE        ( sizeof (long) / sizeof (int) )
#define SHMEM_BCAST_SYNC_SIZE           (128L / SHMEM_INTERNAL_F2C_SCALE)
#define SHMEM_BARRIER_SYNC_SIZE         (128L / SHMEM_INTERNAL_F2C_SCALE)
#define SHMEM_REDUCE_SYNC_SIZE          (256L / SHMEM_INTERNAL_F2C_SCALE)
#define SHMEM_REDUCE_MIN_WRKDATA_SIZE   (128L / SHMEM_INTERNAL_F2C_SCALE)

/* pSync arrays must hold this value on entry (reference src/shmem.h:1505) */
#define SHMEM_SYNC_VALUE (-1L)

/* deprecated spellings (reference src/shmem.h:2210-2218) */
#define _SHMEM_MAJOR_VERSION            SHMEM_MAJOR_VERSION
#define _SHMEM_MINOR_VERSION            SHMEM_MINOR_VERSION
#define _SHMEM_MAX_NAME_LEN             SHMEM_MAX_NAME_LEN
#define _SHMEM_VENDOR_STRING            SHMEM_VENDOR_STRING
#define _SHMEM_BCAST_SYNC_SIZE          SHMEM_BCAST_SYNC_SIZE
#define _SHMEM_BARRIER_SYNC_SIZE        SHMEM_BARRIER_SYNC_SIZE
#define _SHMEM_REDUCE_SYNC_SIZE         SHMEM_REDUCE_SYNC_SIZE
#define _SHMEM_REDUCE_MIN_WRKDATA_SIZE  SHMEM_REDUCE_MIN_WRKDATA_SIZE
#define _SHMEM_SYNC_VALUE               SHMEM_SYNC_VALUE

/* ---- minimal runtime (the reduction path needs PEs, a heap, barriers) ---- */
void start_pes (int npes);
void shmem_init (void);
void shmem_finalize (void);
void shmem_global_exit (int status);
int shmem_my_pe (void);
int shmem_n_pes (void);
int _my_pe (void);
int _num_pes (void);
void *shmem_malloc (size_t size);
void shmem_free (void *ptr);
void shmem_barrier_all (void);
void shmem_barrier (int PE_start, int logPE_stride, int PE_size, long *pSync);
void shmem_quiet (void);

/* ---- one-sided put/get (reference src/shmem.h:395-470); the remote
 *      address must be in the device symmetric heap (shmemx_malloc_device) ---- */
void shmem_putmem (void *dest, const void *src, size_t nelems, int pe);
void shmem_getmem (void *dest, const void *src, size_t nelems, int pe);
void shmem_put32 (void *dest, const void *src, size_t nelems, int pe);
void shmem_put64 (void *dest, const void *src, size_t nelems, int pe);
void shmem_put128 (void *dest, const void *src, size_t nelems, int pe);
void shmem_get32 (void *dest, const void *src, size_t nelems, int pe);
void shmem_get64 (void *dest, const void *src, size_t nelems, int pe);
void shmem_get128 (void *dest, const void *src, size_t nelems, int pe);
void shmem_char_put (char *dest, const char *src, size_t nelems, int pe);
void shmem_short_put (short *dest, const short *src, size_t nelems, int pe);
void shmem_int_put (int *dest, const int *src, size_t nelems, int pe);
void shmem_long_put (long *dest, const long *src, size_t nelems, int pe);
void shmem_longlong_put (long long *dest, const long long *src, size_t nelems, int pe);
void shmem_longdouble_put (long double *dest, const long double *src, size_t nelems, int pe);
void shmem_double_put (double *dest, const double *src, size_t nelems, int pe);
void shmem_float_put (float *dest, const float *src, size_t nelems, int pe);
void shmem_char_get (char *dest, const char *src, size_t nelems, int pe);
void shmem_short_get (short *dest, const short *src, size_t nelems, int pe);
void shmem_int_get (int *dest, const int *src, size_t nelems, int pe);
void shmem_long_get (long *dest, const long *src, size_t nelems, int pe);
void shmem_longlong_get (long long *dest, const long long *src, size_t nelems, int pe);
void shmem_longdouble_get (long double *dest, const long double *src, size_t nelems, int pe);
void shmem_double_get (double *dest, const double *src, size_t nelems, int pe);
void shmem_float_get (float *dest, const float *src, size_t nelems, int pe);

/* ---- broadcast / collect (reference src/shmem.h:1746-1779); sources in the
 *      device symmetric heap ---- */
#define SHMEM_COLLECT_SYNC_SIZE (128L / SHMEM_INTERNAL_F2C_SCALE)
#define _SHMEM_COLLECT_SYNC_SIZE SHMEM_COLLECT_SYNC_SIZE
void shmem_broadcast64 (void *target, const void *source, size_t nelems, int PE_root, int PE_start,
                        int logPE_stride, int PE_size, long *pSync);
void shmem_broadcast32 (void *target, const void *source, size_t nelems, int PE_root, int PE_start,
                        int logPE_stride, int PE_size, long *pSync);
void shmem_fcollect64 (void *target, const void *source, size_t nelems, int PE_start, int logPE_stride,
                       int PE_size, long *pSync);
void shmem_fcollect32 (void *target, const void *source, size_t nelems, int PE_start, int logPE_stride,
                       int PE_size, long *pSync);
void shmem_collect64 (void *target, const void *source, size_t nelems, int PE_start, int logPE_stride,
                      int PE_size, long *pSync);
void shmem_collect32 (void *target, const void *source, size_t nelems, int PE_start, int logPE_stride,
                      int PE_size, long *pSync);

/* ---- reductions: target = op-fold over the active set of source ---- */
    void shmem_short_sum_to_all (short *target, short *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            short *pWrk, long *pSync);
    void shmem_int_sum_to_all (int *target, int *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            int *pWrk, long *pSync);
    void shmem_long_sum_to_all (long *target, long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long *pWrk, long *pSync);
    void shmem_longlong_sum_to_all (long long *target, long long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long long *pWrk, long *pSync);
    void shmem_float_sum_to_all (float *target, float *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            float *pWrk, long *pSync);
    void shmem_double_sum_to_all (double *target, double *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            double *pWrk, long *pSync);
    void shmem_longdouble_sum_to_all (long double *target, long double *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long double *pWrk, long *pSync);
    void shmem_complexf_sum_to_all (COMPLEXIFY (float) *target, COMPLEXIFY (float) *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            COMPLEXIFY (float) *pWrk, long *pSync);
    void shmem_complexd_sum_to_all (COMPLEXIFY (double) *target, COMPLEXIFY (double) *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            COMPLEXIFY (double) *pWrk, long *pSync);
    void shmem_short_prod_to_all (short *target, short *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            short *pWrk, long *pSync);
    void shmem_int_prod_to_all (int *target, int *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            int *pWrk, long *pSync);
    void shmem_long_prod_to_all (long *target, long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long *pWrk, long *pSync);
    void shmem_longlong_prod_to_all (long long *target, long long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long long *pWrk, long *pSync);
    void shmem_float_prod_to_all (float *target, float *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            float *pWrk, long *pSync);
    void shmem_double_prod_to_all (double *target, double *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            double *pWrk, long *pSync);
    void shmem_longdouble_prod_to_all (long double *target, long double *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long double *pWrk, long *pSync);
    void shmem_complexf_prod_to_all (COMPLEXIFY (float) *target, COMPLEXIFY (float) *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            COMPLEXIFY (float) *pWrk, long *pSync);
    void shmem_complexd_prod_to_all (COMPLEXIFY (double) *target, COMPLEXIFY (double) *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            COMPLEXIFY (double) *pWrk, long *pSync);
    void shmem_short_and_to_all (short *target, short *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            short *pWrk, long *pSync);
    void shmem_int_and_to_all (int *target, int *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            int *pWrk, long *pSync);
    void shmem_long_and_to_all (long *target, long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long *pWrk, long *pSync);
    void shmem_longlong_and_to_all (long long *target, long long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long long *pWrk, long *pSync);
    void shmem_short_or_to_all (short *target, short *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            short *pWrk, long *pSync);
    void shmem_int_or_to_all (int *target, int *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            int *pWrk, long *pSync);
    void shmem_long_or_to_all (long *target, long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long *pWrk, long *pSync);
    void shmem_longlong_or_to_all (long long *target, long long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long long *pWrk, long *pSync);
    void shmem_short_xor_to_all (short *target, short *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            short *pWrk, long *pSync);
    void shmem_int_xor_to_all (int *target, int *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            int *pWrk, long *pSync);
    void shmem_long_xor_to_all (long *target, long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long *pWrk, long *pSync);
    void shmem_longlong_xor_to_all (long long *target, long long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long long *pWrk, long *pSync);
    void shmem_short_max_to_all (short *target, short *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            short *pWrk, long *pSync);
    void shmem_int_max_to_all (int *target, int *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            int *pWrk, long *pSync);
    void shmem_long_max_to_all (long *target, long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long *pWrk, long *pSync);
    void shmem_longlong_max_to_all (long long *target, long long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long long *pWrk, long *pSync);
    void shmem_float_max_to_all (float *target, float *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            float *pWrk, long *pSync);
    void shmem_double_max_to_all (double *target, double *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            double *pWrk, long *pSync);
    void shmem_longdouble_max_to_all (long double *target, long double *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long double *pWrk, long *pSync);
    void shmem_short_min_to_all (short *target, short *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            short *pWrk, long *pSync);
    void shmem_int_min_to_all (int *target, int *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            int *pWrk, long *pSync);
    void shmem_long_min_to_all (long *target, long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long *pWrk, long *pSync);
    void shmem_longlong_min_to_all (long long *target, long long *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long long *pWrk, long *pSync);
    void shmem_float_min_to_all (float *target, float *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            float *pWrk, long *pSync);
    void shmem_double_min_to_all (double *target, double *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            double *pWrk, long *pSync);
    void shmem_longdouble_min_to_all (long double *target, long double *source,
            int nreduce, int PE_start, int logPE_stride, int PE_size,
            long double *pWrk, long *pSync);

#ifdef __cplusplus
}
#endif

#endif /* _SHMEM_H */
