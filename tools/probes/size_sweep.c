/* size_sweep.c -- per-call time and GiB/s reduced of shmem_double_sum_to_all
 * over message sizes 8 B .. 256 MiB per PE (OSU-style latency/bandwidth
 * sweep; tuning tool, not part of the library). Device-resident buffers,
 * calls back to back from C, median of `reps` timed blocks, PE 0 prints one
 * JSON line per size (time = max over PEs via shmem_double_max_to_all).
 *   gcc -O2 -Iinclude tools/probes/size_sweep.c -Losss-gasnet_amd/lib -lshmem_reduce \
 *       -Wl,-rpath,$PWD/osss-gasnet_amd/lib -o tools/probes/size_sweep
 *   tools/oshrun -np 4 --same-device tools/probes/size_sweep      (or run directly: 1 PE)
 *   tools/probes/size_sweep host [max_bytes]    source/target from shmem_malloc (host memory, staged)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <shmem.h>
#include <shmemx.h>

static long psync[SHMEM_REDUCE_SYNC_SIZE];

static int cmp (const void *a, const void *b)
{
    const double x = *(const double *) a, y = *(const double *) b;
    return x < y ? -1 : x > y;
}

int main (int argc, char **argv)
{
    const int host = argc > 1 && strcmp (argv[1], "host") == 0;
    const size_t max_bytes = argc > 2 ? (size_t) strtoull (argv[2], NULL, 10) : ((size_t) 1 << 28);
    for (int i = 0; i < SHMEM_REDUCE_SYNC_SIZE; ++i)
        psync[i] = SHMEM_SYNC_VALUE;
    shmem_init ();
    const int me = shmem_my_pe (), npes = shmem_n_pes ();
    const size_t nmax = max_bytes / sizeof (double); /* default 256 MiB of doubles */
    double *src = (double *) (host ? shmem_malloc (nmax * sizeof (double))
                                   : shmemx_malloc_device (nmax * sizeof (double)));
    double *dst = (double *) (host ? shmem_malloc (nmax * sizeof (double))
                                   : shmemx_malloc_device (nmax * sizeof (double)));
    double *h = (double *) malloc (nmax * sizeof (double));
    for (size_t i = 0; i < nmax; ++i)
        h[i] = (double) (i % 1000) * 0.5 + me;
    shmemx_memcpy (src, h, nmax * sizeof (double));
    free (h);
    static double tl[1], tm[1];
    for (size_t n = 1; n <= nmax; n = n == nmax / 2 ? nmax : n * 4) {
        const size_t bytes = n * sizeof (double);
        const int calls = bytes <= (1 << 20) ? 500 : bytes <= (16 << 20) ? 50 : 10;
        const int reps = 7;
        double t[7];
        for (int w = 0; w < 5; ++w)
            shmem_double_sum_to_all (dst, src, (int) n, 0, 0, npes, NULL, psync);
        for (int r = 0; r < reps; ++r) {
            shmem_barrier_all ();
            const double t0 = shmemx_wtime ();
            for (int c = 0; c < calls; ++c)
                shmem_double_sum_to_all (dst, src, (int) n, 0, 0, npes, NULL, psync);
            tl[0] = (shmemx_wtime () - t0) / calls;
            shmem_barrier_all ();
            shmem_double_max_to_all (tm, tl, 1, 0, 0, npes, NULL, psync);
            t[r] = tm[0];
        }
        qsort (t, reps, sizeof t[0], cmp);
        if (me == 0)
            printf ("{\"npes\": %d, \"memory\": \"%s\", \"bytes_per_pe\": %zu, \"us_per_call\": %.2f, "
                    "\"gib_s_reduced_per_pe\": %.2f}\n", npes, host ? "host" : "device", bytes, t[reps / 2] * 1e6,
                    (double) bytes / t[reps / 2] / (double) (1 << 30));
        fflush (stdout);
    }
    if (host) {
        shmem_free (dst);
        shmem_free (src);
    } else {
        shmemx_free_device (dst);
        shmemx_free_device (src);
    }
    shmem_finalize ();
    return 0;
}
