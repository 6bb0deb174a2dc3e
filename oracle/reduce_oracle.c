/*
 * reduce_oracle.c -- CPU restatement of the reference reduction, TEST
 * INFRASTRUCTURE ONLY.
 *
 * This file is the checker, never the product: only tests/, the smoke test in
 * __graft_entry__.py and the cpu_baseline leg of bench.py load liboracle.so.
 * libshmem_reduce.so does not link, load or call it (the product fails loudly
 * without a GPU).
 *
 * Pinning: the element operators below are checked bit-for-bit against the
 * reference's own compiled operator functions (src/reduce/reduce-op.c:79-158,
 * built by oracle/Makefile into oracle/_ref/libref_ops.so) through the golden
 * fixtures in tests/golden/ (tests/test_oracle_golden.py). The schedule
 * (fold order) is restated from reduce-op.c:179-276 and is NOT executed from
 * the reference: its transport (GASNet get + barrier) does not exist in this
 * image, so the fold order is "parity unpinned" by execution.
 *
 * Restated semantics:
 *   - operators (reduce-op.c:79-158): sum/prod `a+b`, `a*b`; and/or/xor bitwise;
 *     min/max `a<b?a:b`, `a>b?a:b`; the accumulator is always the LEFT operand;
 *     complex `a*b` is gcc's call to __muldc3/__mulsc3 (Annex G), long double
 *     is x87 extended (gcc on x86-64) -- both by compiling the same C here.
 *   - schedule (reduce-op.c:226-264): PE p starts from its own source, then
 *     folds in the other active-set members in ascending PE order, skipping
 *     itself, in chunks of SHMEM_REDUCE_MIN_WRKDATA_SIZE = 64 elements fetched
 *     into pWrk (the chunking does not change any result).
 */
#define _GNU_SOURCE
#include <complex.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

enum { OP_SUM, OP_PROD, OP_AND, OP_OR, OP_XOR, OP_MIN, OP_MAX };
enum { T_SHORT, T_INT, T_LONG, T_LONGLONG, T_FLOAT, T_DOUBLE, T_LONGDOUBLE, T_COMPLEXF, T_COMPLEXD };

#define CHUNK 64 /* SHMEM_REDUCE_MIN_WRKDATA_SIZE, reference src/shmem.h:1500 */

/* ---- operators ---------------------------------------------------------- */
#define ARITH(N, T)                                                     \
    static T o_sum_##N (T a, T b) { return a + b; }                     \
    static T o_prod_##N (T a, T b) { return a * b; }
#define LOGIC(N, T)                                                     \
    static T o_and_##N (T a, T b) { return a & b; }                     \
    static T o_or_##N (T a, T b) { return a | b; }                      \
    static T o_xor_##N (T a, T b) { return a ^ b; }
#define MINMAX(N, T)                                                    \
    static T o_min_##N (T a, T b) { return a < b ? a : b; }             \
    static T o_max_##N (T a, T b) { return a > b ? a : b; }

/* integer sum/prod: signed overflow wraps as in gcc's code for the
 * reference; spelled through unsigned so this file has no UB */
static short o_sum_short (short a, short b) { return (short) (unsigned short) ((unsigned) a + (unsigned) b); }
static short o_prod_short (short a, short b) { return (short) (unsigned short) ((unsigned) a * (unsigned) b); }
static int o_sum_int (int a, int b) { return (int) ((unsigned) a + (unsigned) b); }
static int o_prod_int (int a, int b) { return (int) ((unsigned) a * (unsigned) b); }
static long o_sum_long (long a, long b) { return (long) ((unsigned long) a + (unsigned long) b); }
static long o_prod_long (long a, long b) { return (long) ((unsigned long) a * (unsigned long) b); }
static long long o_sum_longlong (long long a, long long b) { return (long long) ((unsigned long long) a + (unsigned long long) b); }
static long long o_prod_longlong (long long a, long long b) { return (long long) ((unsigned long long) a * (unsigned long long) b); }
ARITH (float, float)
ARITH (double, double)
ARITH (longdouble, long double)
ARITH (complexf, float complex)
ARITH (complexd, double complex)
LOGIC (short, short)
LOGIC (int, int)
LOGIC (long, long)
LOGIC (longlong, long long)
MINMAX (short, short)
MINMAX (int, int)
MINMAX (long, long)
MINMAX (longlong, long long)
MINMAX (float, float)
MINMAX (double, double)
MINMAX (longdouble, long double)

/* ---- generic fold over typed arrays ------------------------------------- */
#define FOLD_FN(N, T)                                                                       \
    static void fold_##N (T (*op) (T, T), T *acc, const T *src, size_t n)                   \
    {                                                                                       \
        T wrk[CHUNK];                                                                       \
        size_t i = 0;                                                                       \
        for (; i + CHUNK <= n; i += CHUNK) {                                                \
            memcpy (wrk, src + i, sizeof wrk); /* the shmem_getmem into pWrk */            \
            for (size_t j = 0; j < CHUNK; ++j)                                              \
                acc[i + j] = (*op) (acc[i + j], wrk[j]);                                    \
        }                                                                                   \
        memcpy (wrk, src + i, (n - i) * sizeof (T));                                        \
        for (size_t j = 0; i + j < n; ++j)                                                  \
            acc[i + j] = (*op) (acc[i + j], wrk[j]);                                        \
    }
FOLD_FN (short, short)
FOLD_FN (int, int)
FOLD_FN (long, long)
FOLD_FN (longlong, long long)
FOLD_FN (float, float)
FOLD_FN (double, double)
FOLD_FN (longdouble, long double)
FOLD_FN (complexf, float complex)
FOLD_FN (complexd, double complex)

static size_t esize (int t)
{
    switch (t) {
    case T_SHORT: return sizeof (short);
    case T_INT: return sizeof (int);
    case T_LONG: return sizeof (long);
    case T_LONGLONG: return sizeof (long long);
    case T_FLOAT: return sizeof (float);
    case T_DOUBLE: return sizeof (double);
    case T_LONGDOUBLE: return sizeof (long double);
    case T_COMPLEXF: return sizeof (float complex);
    case T_COMPLEXD: return sizeof (double complex);
    default: return 0;
    }
}

/* acc[i] = acc[i] op src[i] for i < n; returns -1 for an undefined pair */
int oracle_fold (int op, int t, void *acc, const void *src, size_t n)
{
#define CASE_A(N)                                                                  \
    switch (op) {                                                                  \
    case OP_SUM: fold_##N (o_sum_##N, acc, src, n); return 0;                      \
    case OP_PROD: fold_##N (o_prod_##N, acc, src, n); return 0;                    \
    default: break;                                                                \
    }
#define CASE_L(N)                                                                  \
    switch (op) {                                                                  \
    case OP_AND: fold_##N (o_and_##N, acc, src, n); return 0;                      \
    case OP_OR: fold_##N (o_or_##N, acc, src, n); return 0;                        \
    case OP_XOR: fold_##N (o_xor_##N, acc, src, n); return 0;                      \
    default: break;                                                                \
    }
#define CASE_M(N)                                                                  \
    switch (op) {                                                                  \
    case OP_MIN: fold_##N (o_min_##N, acc, src, n); return 0;                      \
    case OP_MAX: fold_##N (o_max_##N, acc, src, n); return 0;                      \
    default: break;                                                                \
    }
    switch (t) {
    case T_SHORT: CASE_A (short) CASE_L (short) CASE_M (short) break;
    case T_INT: CASE_A (int) CASE_L (int) CASE_M (int) break;
    case T_LONG: CASE_A (long) CASE_L (long) CASE_M (long) break;
    case T_LONGLONG: CASE_A (longlong) CASE_L (longlong) CASE_M (longlong) break;
    case T_FLOAT: CASE_A (float) CASE_M (float) break;
    case T_DOUBLE: CASE_A (double) CASE_M (double) break;
    case T_LONGDOUBLE: CASE_A (longdouble) CASE_M (longdouble) break;
    case T_COMPLEXF: CASE_A (complexf) break;
    case T_COMPLEXD: CASE_A (complexd) break;
    default: break;
    }
    return -1;
}

/* The result the reference computes on active-set member `me` of `npes`
 * members whose sources are srcs[0..npes-1] in active-set (ascending PE)
 * order: own source first, then every other member ascending
 * (reduce-op.c:226-264). */
int oracle_reduce_pe (int op, int t, int npes, int me, const void *const *srcs, void *out, size_t n)
{
    const size_t es = esize (t);
    if (es == 0 || me < 0 || me >= npes)
        return -1;
    memmove (out, srcs[me], n * es);
    for (int i = 0; i < npes; ++i) {
        if (i == me)
            continue;
        if (oracle_fold (op, t, out, srcs[i], n) != 0)
            return -1;
    }
    return 0;
}

/* ---- CPU baseline: the reference algorithm timed with one process per PE -- */
/* Shared-memory transport: shmem_getmem = memcpy from the peer's source in a
 * MAP_SHARED region (the 64-element pWrk copies inside the fold),
 * shmem_barrier = process-shared pthread barrier. Each call is
 * reduce-op.c:226-266: the copy loop, a barrier, the chunked fold of every
 * other PE's source in ascending order (one indirect operator call per
 * element), a barrier. Returns the median seconds per call over `reps` timed
 * calls after `warm` untimed ones, max over PEs, or -1 on error. */
struct bench_shared {
    pthread_barrier_t bar;
    double t[1024];
    int cpu[1024];
};

static double mono (void)
{
    struct timespec ts;
    clock_gettime (CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

static int cmp_d (const void *a, const void *b)
{
    double x = *(const double *) a, y = *(const double *) b;
    return x < y ? -1 : x > y;
}

static void fill_double (double *p, size_t n, unsigned seed)
{
    uint64_t s = 0x9e3779b97f4a7c15ull ^ seed;
    for (size_t i = 0; i < n; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        p[i] = (double) (int64_t) s * 0x1p-63;
    }
}

/* SURVEY.md 8(d) inputs: config 1's ints src_p[i] = i*7 + p*1000003 (wrapping);
 * full-mantissa doubles otherwise */
static void fill_src (int t, void *p, size_t n, int pe)
{
    if (t == T_INT) {
        int *q = (int *) p;
        for (size_t i = 0; i < n; ++i)
            q[i] = (int) ((unsigned) i * 7u + (unsigned) pe * 1000003u);
    } else {
        fill_double ((double *) p, n, 1234u + (unsigned) pe);
    }
}

/* The `k`-th CPU of this process's affinity mask (wrapping), or -1. */
static int nth_allowed_cpu (int k)
{
    cpu_set_t set;
    if (sched_getaffinity (0, sizeof set, &set) != 0)
        return -1;
    const int cnt = CPU_COUNT (&set);
    if (cnt <= 0)
        return -1;
    k %= cnt;
    for (int c = 0; c < CPU_SETSIZE; ++c)
        if (CPU_ISSET (c, &set) && k-- == 0)
            return c;
    return -1;
}

/* op/t: OP_SUM with T_INT (config 1) or T_DOUBLE (configs 2, 3, 5). pin: PE p
 * runs pinned to the (p+2)-th CPU of the caller's affinity mask (the p-th when
 * fewer than npes + 2 are allowed); cpus_out (npes entries, or NULL) receives
 * the CPU each PE ran on. */
double oracle_cpu_baseline (int op, int t, int npes, size_t n, int warm, int reps, int pin, int *cpus_out)
{
    if (npes < 1 || npes > 1024 || reps < 1 || reps > 1000000 || (t != T_INT && t != T_DOUBLE))
        return -1.0;
    const size_t es = esize (t);
    const size_t bytes = n * es;
    const size_t slot = (bytes + 4095) / 4096 * 4096;
    size_t total = 4096 * ((sizeof (struct bench_shared) + 4095) / 4096) + 2 * (size_t) npes * slot;
    char *mem = mmap (NULL, total, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    if (mem == MAP_FAILED)
        return -1.0;
    struct bench_shared *sh = (struct bench_shared *) mem;
    pthread_barrierattr_t a;
    pthread_barrierattr_init (&a);
    pthread_barrierattr_setpshared (&a, PTHREAD_PROCESS_SHARED);
    pthread_barrier_init (&sh->bar, &a, (unsigned) npes);
    char *src = mem + 4096 * ((sizeof (struct bench_shared) + 4095) / 4096);
    char *tgt = src + (size_t) npes * slot;
    double *times = (double *) malloc (sizeof (double) * (size_t) reps);
    if (times == NULL)
        return -1.0;
    cpu_set_t saved; /* the caller's mask, restored when PE 0 returns */
    const int have_saved = sched_getaffinity (0, sizeof saved, &saved) == 0;
    pid_t kids[1024];
    int me = 0;
    for (int p = 1; p < npes; ++p) {
        pid_t k = fork ();
        if (k == 0) {
            me = p;
            break;
        }
        kids[p] = k;
    }
    sh->cpu[me] = -1;
    if (pin) {
        /* skip the first two allowed CPUs when there are spare ones: CPU 0
         * takes most of the host's interrupts */
        cpu_set_t set;
        const int skip = sched_getaffinity (0, sizeof set, &set) == 0 && CPU_COUNT (&set) >= npes + 2 ? 2 : 0;
        const int c = nth_allowed_cpu (me + skip);
        if (c >= 0) {
            cpu_set_t one;
            CPU_ZERO (&one);
            CPU_SET (c, &one);
            if (sched_setaffinity (0, sizeof one, &one) == 0)
                sh->cpu[me] = c;
        }
    }
    char *mysrc = src + (size_t) me * slot, *mytgt = tgt + (size_t) me * slot;
    fill_src (t, mysrc, n, me);
    for (int r = 0; r < warm + reps; ++r) {
        pthread_barrier_wait (&sh->bar);
        double t0 = mono ();
        /* reduce-op.c:226-266 with the shared-memory transport */
        if (t == T_INT) {
            for (size_t j = 0; j < n; ++j)
                ((int *) mytgt)[j] = ((const int *) mysrc)[j];
        } else {
            for (size_t j = 0; j < n; ++j)
                ((double *) mytgt)[j] = ((const double *) mysrc)[j];
        }
        pthread_barrier_wait (&sh->bar);
        for (int i = 0; i < npes; ++i)
            if (i != me)
                oracle_fold (op, t, mytgt, src + (size_t) i * slot, n);
        pthread_barrier_wait (&sh->bar);
        if (r >= warm)
            times[r - warm] = mono () - t0;
    }
    qsort (times, (size_t) reps, sizeof (double), cmp_d);
    sh->t[me] = times[reps / 2];
    free (times);
    if (me != 0)
        _exit (0);
    for (int p = 1; p < npes; ++p)
        waitpid (kids[p], NULL, 0);
    double worst = 0.0;
    for (int p = 0; p < npes; ++p) {
        if (sh->t[p] > worst)
            worst = sh->t[p];
        if (cpus_out != NULL)
            cpus_out[p] = sh->cpu[p];
    }
    pthread_barrier_destroy (&sh->bar);
    munmap (mem, total);
    if (pin && have_saved)
        sched_setaffinity (0, sizeof saved, &saved);
    return worst;
}

/* double sum, unpinned (tools/cpu_baseline.py, round 1) */
double oracle_cpu_baseline_double_sum (int npes, size_t n, int warm, int reps)
{
    return oracle_cpu_baseline (OP_SUM, T_DOUBLE, npes, n, warm, reps, 0, NULL);
}
