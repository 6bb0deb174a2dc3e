/*
 * shmem_fortran.h -- C prototypes of the Fortran-callable names exported by
 * libshmem_reduce.so (osss-gasnet_amd/csrc/fortran.c). Fortran programs do not
 * include this; it documents the ABI (every argument by reference, single
 * trailing underscore, INTEGER pSync) for C/ctypes callers and the ABI test.
 *
 * Reference interface: src/fortran/fortran.c:1218-1256 (the 37 REDUCIFY
 * reductions), :95-134 (init and PE queries), :636-645 (barriers, quiet).
 * Each shmem_*_ name is a weak alias of the strong pshmem_*_ name
 * (reference: the #pragma weak block at fortran.c:1108-1216).
 */
#ifndef SHMEM_FORTRAN_H
#define SHMEM_FORTRAN_H 1

#ifdef __cplusplus
# include <complex>
# define SHMEM_F_COMPLEX(T) std::complex<T>
extern "C" {
#else
# include <complex.h>
# define SHMEM_F_COMPLEX(T) T _Complex
#endif

/* weak names */
void start_pes_ (int *npes);
void shmem_init_ (void);
void shmem_finalize_ (void);
void shmem_global_exit_ (int *status);
int my_pe_ (void);
int num_pes_ (void);
int shmem_my_pe_ (void);
int shmem_n_pes_ (void);
void shmem_barrier_all_ (void);
void shmem_quiet_ (void);
void shmem_barrier_ (int *PE_start, int *logPE_stride, int *PE_size, int *pSync);
void shmem_int2_sum_to_all_ (short *target, short *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, short *pWrk, int *pSync);
void shmem_int4_sum_to_all_ (int *target, int *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, int *pWrk, int *pSync);
void shmem_int8_sum_to_all_ (long *target, long *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long *pWrk, int *pSync);
void shmem_real4_sum_to_all_ (float *target, float *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, float *pWrk, int *pSync);
void shmem_real8_sum_to_all_ (double *target, double *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, double *pWrk, int *pSync);
void shmem_real16_sum_to_all_ (long double *target, long double *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long double *pWrk, int *pSync);
void shmem_int2_prod_to_all_ (short *target, short *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, short *pWrk, int *pSync);
void shmem_int4_prod_to_all_ (int *target, int *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, int *pWrk, int *pSync);
void shmem_int8_prod_to_all_ (long *target, long *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long *pWrk, int *pSync);
void shmem_real4_prod_to_all_ (float *target, float *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, float *pWrk, int *pSync);
void shmem_real8_prod_to_all_ (double *target, double *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, double *pWrk, int *pSync);
void shmem_real16_prod_to_all_ (long double *target, long double *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long double *pWrk, int *pSync);
void shmem_int2_max_to_all_ (short *target, short *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, short *pWrk, int *pSync);
void shmem_int4_max_to_all_ (int *target, int *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, int *pWrk, int *pSync);
void shmem_int8_max_to_all_ (long *target, long *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long *pWrk, int *pSync);
void shmem_real4_max_to_all_ (float *target, float *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, float *pWrk, int *pSync);
void shmem_real8_max_to_all_ (double *target, double *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, double *pWrk, int *pSync);
void shmem_real16_max_to_all_ (long double *target, long double *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long double *pWrk, int *pSync);
void shmem_int2_min_to_all_ (short *target, short *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, short *pWrk, int *pSync);
void shmem_int4_min_to_all_ (int *target, int *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, int *pWrk, int *pSync);
void shmem_int8_min_to_all_ (long *target, long *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long *pWrk, int *pSync);
void shmem_real4_min_to_all_ (float *target, float *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, float *pWrk, int *pSync);
void shmem_real8_min_to_all_ (double *target, double *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, double *pWrk, int *pSync);
void shmem_real16_min_to_all_ (long double *target, long double *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long double *pWrk, int *pSync);
void shmem_int2_and_to_all_ (short *target, short *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, short *pWrk, int *pSync);
void shmem_int4_and_to_all_ (int *target, int *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, int *pWrk, int *pSync);
void shmem_int8_and_to_all_ (long *target, long *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long *pWrk, int *pSync);
void shmem_int2_or_to_all_ (short *target, short *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, short *pWrk, int *pSync);
void shmem_int4_or_to_all_ (int *target, int *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, int *pWrk, int *pSync);
void shmem_int8_or_to_all_ (long *target, long *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long *pWrk, int *pSync);
void shmem_int2_xor_to_all_ (short *target, short *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, short *pWrk, int *pSync);
void shmem_int4_xor_to_all_ (int *target, int *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, int *pWrk, int *pSync);
void shmem_int8_xor_to_all_ (long *target, long *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long *pWrk, int *pSync);
void shmem_comp4_sum_to_all_ (SHMEM_F_COMPLEX (float) *target, SHMEM_F_COMPLEX (float) *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, SHMEM_F_COMPLEX (float) *pWrk, int *pSync);
void shmem_comp8_sum_to_all_ (SHMEM_F_COMPLEX (double) *target, SHMEM_F_COMPLEX (double) *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, SHMEM_F_COMPLEX (double) *pWrk, int *pSync);
void shmem_comp4_prod_to_all_ (SHMEM_F_COMPLEX (float) *target, SHMEM_F_COMPLEX (float) *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, SHMEM_F_COMPLEX (float) *pWrk, int *pSync);
void shmem_comp8_prod_to_all_ (SHMEM_F_COMPLEX (double) *target, SHMEM_F_COMPLEX (double) *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, SHMEM_F_COMPLEX (double) *pWrk, int *pSync);

/* strong (PSHMEM) names */
void pstart_pes_ (int *npes);
void pshmem_init_ (void);
void pshmem_finalize_ (void);
void pshmem_global_exit_ (int *status);
int pmy_pe_ (void);
int pnum_pes_ (void);
int pshmem_my_pe_ (void);
int pshmem_n_pes_ (void);
void pshmem_barrier_all_ (void);
void pshmem_quiet_ (void);
void pshmem_barrier_ (int *PE_start, int *logPE_stride, int *PE_size, int *pSync);
void pshmem_int2_sum_to_all_ (short *target, short *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, short *pWrk, int *pSync);
void pshmem_int4_sum_to_all_ (int *target, int *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, int *pWrk, int *pSync);
void pshmem_int8_sum_to_all_ (long *target, long *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long *pWrk, int *pSync);
void pshmem_real4_sum_to_all_ (float *target, float *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, float *pWrk, int *pSync);
void pshmem_real8_sum_to_all_ (double *target, double *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, double *pWrk, int *pSync);
void pshmem_real16_sum_to_all_ (long double *target, long double *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long double *pWrk, int *pSync);
void pshmem_int2_prod_to_all_ (short *target, short *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, short *pWrk, int *pSync);
void pshmem_int4_prod_to_all_ (int *target, int *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, int *pWrk, int *pSync);
void pshmem_int8_prod_to_all_ (long *target, long *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long *pWrk, int *pSync);
void pshmem_real4_prod_to_all_ (float *target, float *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, float *pWrk, int *pSync);
void pshmem_real8_prod_to_all_ (double *target, double *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, double *pWrk, int *pSync);
void pshmem_real16_prod_to_all_ (long double *target, long double *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long double *pWrk, int *pSync);
void pshmem_int2_max_to_all_ (short *target, short *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, short *pWrk, int *pSync);
void pshmem_int4_max_to_all_ (int *target, int *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, int *pWrk, int *pSync);
void pshmem_int8_max_to_all_ (long *target, long *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long *pWrk, int *pSync);
void pshmem_real4_max_to_all_ (float *target, float *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, float *pWrk, int *pSync);
void pshmem_real8_max_to_all_ (double *target, double *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, double *pWrk, int *pSync);
void pshmem_real16_max_to_all_ (long double *target, long double *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long double *pWrk, int *pSync);
void pshmem_int2_min_to_all_ (short *target, short *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, short *pWrk, int *pSync);
void pshmem_int4_min_to_all_ (int *target, int *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, int *pWrk, int *pSync);
void pshmem_int8_min_to_all_ (long *target, long *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long *pWrk, int *pSync);
void pshmem_real4_min_to_all_ (float *target, float *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, float *pWrk, int *pSync);
void pshmem_real8_min_to_all_ (double *target, double *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, double *pWrk, int *pSync);
void pshmem_real16_min_to_all_ (long double *target, long double *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long double *pWrk, int *pSync);
void pshmem_int2_and_to_all_ (short *target, short *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, short *pWrk, int *pSync);
void pshmem_int4_and_to_all_ (int *target, int *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, int *pWrk, int *pSync);
void pshmem_int8_and_to_all_ (long *target, long *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long *pWrk, int *pSync);
void pshmem_int2_or_to_all_ (short *target, short *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, short *pWrk, int *pSync);
void pshmem_int4_or_to_all_ (int *target, int *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, int *pWrk, int *pSync);
void pshmem_int8_or_to_all_ (long *target, long *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long *pWrk, int *pSync);
void pshmem_int2_xor_to_all_ (short *target, short *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, short *pWrk, int *pSync);
void pshmem_int4_xor_to_all_ (int *target, int *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, int *pWrk, int *pSync);
void pshmem_int8_xor_to_all_ (long *target, long *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, long *pWrk, int *pSync);
void pshmem_comp4_sum_to_all_ (SHMEM_F_COMPLEX (float) *target, SHMEM_F_COMPLEX (float) *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, SHMEM_F_COMPLEX (float) *pWrk, int *pSync);
void pshmem_comp8_sum_to_all_ (SHMEM_F_COMPLEX (double) *target, SHMEM_F_COMPLEX (double) *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, SHMEM_F_COMPLEX (double) *pWrk, int *pSync);
void pshmem_comp4_prod_to_all_ (SHMEM_F_COMPLEX (float) *target, SHMEM_F_COMPLEX (float) *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, SHMEM_F_COMPLEX (float) *pWrk, int *pSync);
void pshmem_comp8_prod_to_all_ (SHMEM_F_COMPLEX (double) *target, SHMEM_F_COMPLEX (double) *source, int *nreduce,
        int *PE_start, int *logPE_stride, int *PE_size, SHMEM_F_COMPLEX (double) *pWrk, int *pSync);

#ifdef __cplusplus
}
#endif

#endif /* SHMEM_FORTRAN_H */
