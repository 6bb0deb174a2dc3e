/*
 * fortran.c -- the Fortran-callable reduction surface (callers of the path,
 * SURVEY.md 8b): every argument by reference, names with gfortran's single
 * trailing underscore, pshmem_*_ strong and shmem_*_ weak like the C names.
 *
 * Reference interface replaced: src/fortran/fortran.c:1218-1256 (REDUCIFY:
 * 37 <op>_to_all wrappers over the Fortran kinds int2/int4/int8, real4/8/16,
 * comp4/8), :95-134 (start_pes, shmem_init/finalize/global_exit, my_pe,
 * num_pes, shmem_my_pe, shmem_n_pes) and :636-645 (shmem_barrier,
 * shmem_barrier_all, shmem_quiet). As in the reference, a Fortran pSync is an
 * INTEGER array handed on as `long *` (the C side keeps pSync's contract: it
 * is read, never written, by this build).
 *
 * Kind -> C type (fortran.c:1238-1256): int2 short, int4 int, int8 long,
 * real4 float, real8 double, real16 long double, comp4 float complex,
 * comp8 double complex.
 */
#include <complex.h>

#include <pshmem.h>
#include <shmem.h>

#include "shmem_fortran.h"

#define WEAK_F(name) __attribute__ ((weak, alias ("p" #name)))

/* ---- runtime calls a Fortran reduction caller needs ------------------- */

void pstart_pes_ (int *npes) { (void) npes; pshmem_init (); }
void pshmem_init_ (void) { pshmem_init (); }
void pshmem_finalize_ (void) { pshmem_finalize (); }
void pshmem_global_exit_ (int *status) { pshmem_global_exit (*status); }
int pmy_pe_ (void) { return pshmem_my_pe (); }
int pnum_pes_ (void) { return pshmem_n_pes (); }
int pshmem_my_pe_ (void) { return pshmem_my_pe (); }
int pshmem_n_pes_ (void) { return pshmem_n_pes (); }
void pshmem_barrier_all_ (void) { pshmem_barrier_all (); }
void pshmem_quiet_ (void) { pshmem_quiet (); }
void pshmem_barrier_ (int *PE_start, int *logPE_stride, int *PE_size, int *pSync)
{
    pshmem_barrier (*PE_start, *logPE_stride, *PE_size, (long *) pSync);
}

void start_pes_ (int *npes) WEAK_F (start_pes_);
void shmem_init_ (void) WEAK_F (shmem_init_);
void shmem_finalize_ (void) WEAK_F (shmem_finalize_);
void shmem_global_exit_ (int *status) WEAK_F (shmem_global_exit_);
int my_pe_ (void) WEAK_F (my_pe_);
int num_pes_ (void) WEAK_F (num_pes_);
int shmem_my_pe_ (void) WEAK_F (shmem_my_pe_);
int shmem_n_pes_ (void) WEAK_F (shmem_n_pes_);
void shmem_barrier_all_ (void) WEAK_F (shmem_barrier_all_);
void shmem_quiet_ (void) WEAK_F (shmem_quiet_);
void shmem_barrier_ (int *PE_start, int *logPE_stride, int *PE_size, int *pSync) WEAK_F (shmem_barrier_);

/* ---- the 37 reductions ------------------------------------------------- */

/* (Fortran kind, C entry type name, C type) per op, in the reference's order */
#define F_ARITH(X, Op)                                                                                      \
    X (Op, int2, short, short)                                                                              \
    X (Op, int4, int, int)                                                                                  \
    X (Op, int8, long, long)                                                                                \
    X (Op, real4, float, float)                                                                             \
    X (Op, real8, double, double)                                                                           \
    X (Op, real16, longdouble, long double)
#define F_LOGIC(X, Op)                                                                                      \
    X (Op, int2, short, short)                                                                              \
    X (Op, int4, int, int)                                                                                  \
    X (Op, int8, long, long)
#define F_COMPLEX(X, Op)                                                                                    \
    X (Op, comp4, complexf, float _Complex)                                                                 \
    X (Op, comp8, complexd, double _Complex)

#define F_REDUCTION(Op, Kind, Cname, Ctype)                                                                 \
    void pshmem_##Kind##_##Op##_to_all_ (Ctype *target, Ctype *source, int *nreduce, int *PE_start,         \
                                         int *logPE_stride, int *PE_size, Ctype *pWrk, int *pSync)          \
    {                                                                                                       \
        pshmem_##Cname##_##Op##_to_all (target, source, *nreduce, *PE_start, *logPE_stride, *PE_size, pWrk, \
                                        (long *) pSync);                                                    \
    }                                                                                                       \
    void shmem_##Kind##_##Op##_to_all_ (Ctype *target, Ctype *source, int *nreduce, int *PE_start,          \
                                        int *logPE_stride, int *PE_size, Ctype *pWrk, int *pSync)           \
        WEAK_F (shmem_##Kind##_##Op##_to_all_);

F_ARITH (F_REDUCTION, sum)
F_ARITH (F_REDUCTION, prod)
F_ARITH (F_REDUCTION, max)
F_ARITH (F_REDUCTION, min)
F_LOGIC (F_REDUCTION, and)
F_LOGIC (F_REDUCTION, or)
F_LOGIC (F_REDUCTION, xor)
F_COMPLEX (F_REDUCTION, sum)
F_COMPLEX (F_REDUCTION, prod)
