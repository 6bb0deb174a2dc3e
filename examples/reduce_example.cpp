/*
 * reduce_example.cpp -- a C++ OpenSHMEM caller: the complex reductions take
 * std::complex<T> (shmem.h's COMPLEXIFY, reference src/shmem.h:74-88) and
 * every prototype has C linkage, so a C++ program links the same symbols.
 *
 *   g++ -std=c++17 -Iinclude examples/reduce_example.cpp \
 *       -Losss-gasnet_amd/lib -lshmem_reduce -Wl,-rpath,$PWD/osss-gasnet_amd/lib -o reduce_example_cpp
 *   tools/oshrun -np 3 ./reduce_example_cpp
 *
 * Checks (values chosen so every partial result is exact in binary, so any
 * fold order gives the same bits):
 *   shmem_complexd_prod_to_all   prod over PEs of (1 + i*(p+1)/8) * 2^k
 *   shmem_complexf_sum_to_all    device-resident, sum of small integers
 *   shmem_longdouble_sum_to_all  64-bit significand sums beyond double's 53
 */
#include <complex>
#include <cstdio>
#include <vector>

#include <shmem.h>
#include <shmemx.h>

static long pSync[SHMEM_REDUCE_SYNC_SIZE];

int main ()
{
    for (long &v : pSync)
        v = SHMEM_SYNC_VALUE;
    shmem_init ();
    const int me = shmem_my_pe (), npes = shmem_n_pes ();
    const int n = 777;
    int bad = 0;

    using cd = std::complex<double>;
    auto *cs = static_cast<cd *> (shmem_malloc (n * sizeof (cd)));
    auto *ct = static_cast<cd *> (shmem_malloc (n * sizeof (cd)));
    for (int i = 0; i < n; ++i)
        cs[i] = cd (1.0, (me + 1) / 8.0) * double (1 << (i % 5));
    shmem_barrier_all ();
    shmem_complexd_prod_to_all (ct, cs, n, 0, 0, npes, nullptr, pSync);
    for (int i = 0; i < n; ++i) {
        cd want (1.0, 0.0);
        for (int p = 0; p < npes; ++p)
            want *= cd (1.0, (p + 1) / 8.0) * double (1 << (i % 5));
        bad += ct[i] != want;
    }
    shmem_barrier_all ();

    using cf = std::complex<float>;
    auto *ds = static_cast<cf *> (shmemx_malloc_device (n * sizeof (cf)));
    auto *dt = static_cast<cf *> (shmemx_malloc_device (n * sizeof (cf)));
    std::vector<cf> h (n);
    for (int i = 0; i < n; ++i)
        h[i] = cf (float (i + me), float (-i * me));
    shmemx_memcpy (ds, h.data (), n * sizeof (cf));
    shmem_complexf_sum_to_all (dt, ds, n, 0, 0, npes, nullptr, pSync);
    shmemx_memcpy (h.data (), dt, n * sizeof (cf));
    const int tri = npes * (npes - 1) / 2;
    for (int i = 0; i < n; ++i)
        bad += h[i] != cf (float (npes * i + tri), float (-i * tri));
    shmem_barrier_all ();

    auto *ls = static_cast<long double *> (shmem_malloc (n * sizeof (long double)));
    auto *lt = static_cast<long double *> (shmem_malloc (n * sizeof (long double)));
    const long double big = 1.0L * (1LL << 62); /* 2^62 + small: exact in 64 bits, not in 53 */
    for (int i = 0; i < n; ++i)
        ls[i] = big + (long double) (i + me);
    shmem_barrier_all ();
    shmem_longdouble_sum_to_all (lt, ls, n, 0, 0, npes, nullptr, pSync);
    for (int i = 0; i < n; ++i) {
        long double want = 0.0L;
        for (int p = 0; p < npes; ++p)
            want += big + (long double) (i + p);
        bad += lt[i] != want;
    }

    std::printf ("PE %d of %d: %s\n", me, npes, bad ? "FAILED" : "ok");
    shmem_free (lt);
    shmem_free (ls);
    shmemx_free_device (dt);
    shmemx_free_device (ds);
    shmem_free (ct);
    shmem_free (cs);
    shmem_finalize ();
    return bad != 0;
}
