/*
 * ref_ops.c -- exposes the REFERENCE's own operator functions, for pinning
 * the oracle. TEST INFRASTRUCTURE ONLY (built into oracle/_ref/, which is not
 * committed and is never loaded by the product).
 *
 * This translation unit #includes the reference source file where it lies
 * (REF_SRC = /root/reference/src/reduce/reduce-op.c, passed by the Makefile),
 * compiled unmodified with the reference's own headers. Its static operator
 * functions `<op>_<type>_func` (reduce-op.c:79-158) are reachable from here
 * and are wrapped below in one fold loop per operator:
 *     acc[i] = (*the_op) (acc[i], src[i]),   the_op = <op>_<type>_func
 * -- exactly the call `write_to[ti] = (*the_op)(write_to[ti], pWrk[j])` of
 * reduce-op.c:247-248, through a pointer gcc cannot see through (volatile),
 * so the operator runs as the reference's own build runs it: the out-of-line
 * function, called indirectly. (Inlined into the loop instead, gcc gives the
 * double complex add its operands in the other order -- same values, another
 * NaN payload -- so an inlined wrapper would not pin NaN payloads.)
 *
 * What is NOT taken from the reference: its schedule shmemi_udr_*_to_all
 * (:179-276) needs shmem_getmem/shmem_barrier over GASNet, which this image
 * lacks; the GASNet header is kept out with -D_COMMS_H (the include guard of
 * src/comms/comms.h) and the schedule functions are hidden and discarded by
 * --gc-sections, so no stand-in transport is written or linked.
 */
#include REF_SRC

#define EXPORT __attribute__ ((visibility ("default")))

#define REF_FOLD(OpCall, Name, Type)                                              \
    EXPORT void ref_##OpCall##_##Name (Type *acc, const Type *src, long n)         \
    {                                                                             \
        Type (*volatile the_op) (Type, Type) = OpCall##_##Name##_func;           \
        for (long i = 0; i < n; ++i)                                              \
            acc[i] = (*the_op) (acc[i], src[i]);                                  \
    }

#define REF_ARITH(Name, Type) REF_FOLD (sum, Name, Type) REF_FOLD (prod, Name, Type)
#define REF_LOGIC(Name, Type) REF_FOLD (and, Name, Type) REF_FOLD (or, Name, Type) REF_FOLD (xor, Name, Type)
#define REF_MINMAX(Name, Type) REF_FOLD (min, Name, Type) REF_FOLD (max, Name, Type)

REF_ARITH (short, short)
REF_ARITH (int, int)
REF_ARITH (long, long)
REF_ARITH (longlong, long long)
REF_ARITH (float, float)
REF_ARITH (double, double)
REF_ARITH (longdouble, long double)
REF_ARITH (complexf, float complex)
REF_ARITH (complexd, double complex)
REF_LOGIC (short, short)
REF_LOGIC (int, int)
REF_LOGIC (long, long)
REF_LOGIC (longlong, long long)
REF_MINMAX (short, short)
REF_MINMAX (int, int)
REF_MINMAX (long, long)
REF_MINMAX (longlong, long long)
REF_MINMAX (float, float)
REF_MINMAX (double, double)
REF_MINMAX (longdouble, long double)
