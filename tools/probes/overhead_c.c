/* overhead_c.c -- per-call cost of a 1-PE device-resident shmem_double_sum_to_all
 * from C (no Python in the loop). Tuning tool.
 *   gcc -O2 -Iinclude tools/probes/overhead_c.c -Losss-gasnet_amd/lib -lshmem_reduce \
 *       -Wl,-rpath,$PWD/osss-gasnet_amd/lib -o tools/probes/overhead_c */
#include <stdio.h>
#include <stdlib.h>
#include <shmem.h>
#include <shmemx.h>

static long psync[SHMEM_REDUCE_SYNC_SIZE];

int main (void)
{
    for (int i = 0; i < SHMEM_REDUCE_SYNC_SIZE; ++i) psync[i] = SHMEM_SYNC_VALUE;
    shmem_init ();
    size_t sizes[] = {1, 8192, (size_t) 1 << 25};
    for (int k = 0; k < 3; ++k) {
        size_t n = sizes[k];
        double *a = shmemx_malloc_device (n * 8), *b = shmemx_malloc_device (n * 8);
        double *h = malloc (n * 8);
        for (size_t i = 0; i < n; ++i) h[i] = (double) i;
        shmemx_memcpy (a, h, n * 8);
        int reps = n > 100000 ? 200 : 5000;
        for (int r = 0; r < 20; ++r) shmem_double_sum_to_all (b, a, (int) n, 0, 0, 1, NULL, psync);
        double t0 = shmemx_wtime ();
        for (int r = 0; r < reps; ++r) shmem_double_sum_to_all (b, a, (int) n, 0, 0, 1, NULL, psync);
        double t = (shmemx_wtime () - t0) / reps;
        printf ("n=%zu: %.2f us per call\n", n, t * 1e6);
        free (h);
        shmemx_free_device (b);
        shmemx_free_device (a);
    }
    shmem_finalize ();
    return 0;
}
