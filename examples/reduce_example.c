/*
 * reduce_example.c -- an unmodified-style OpenSHMEM 1.3 program using the
 * reduction collectives, built against this library instead of the reference:
 *
 *   gcc -std=c99 -Iinclude examples/reduce_example.c \
 *       -Losss-gasnet_amd/lib -lshmem_reduce -Wl,-rpath,$PWD/osss-gasnet_amd/lib -o reduce_example
 *   tools/oshrun -np 4 ./reduce_example
 *
 * It follows the reference's calling convention exactly (pWrk/pSync sized by
 * the SHMEM_REDUCE_* constants, pSync initialised to SHMEM_SYNC_VALUE, a
 * barrier before reusing pSync), reduces host arrays from shmem_malloc, and
 * also a device-resident array from the MI355X extension shmemx_malloc_device.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <shmem.h>
#include <shmemx.h>

#define N 1000

static long pSync[SHMEM_REDUCE_SYNC_SIZE];
static int pWrk[N / 2 + 1 > SHMEM_REDUCE_MIN_WRKDATA_SIZE ? N / 2 + 1 : SHMEM_REDUCE_MIN_WRKDATA_SIZE];

int main (void)
{
    for (int i = 0; i < SHMEM_REDUCE_SYNC_SIZE; ++i)
        pSync[i] = SHMEM_SYNC_VALUE;
    shmem_init ();
    const int me = shmem_my_pe (), npes = shmem_n_pes ();

    int *src = (int *) shmem_malloc (N * sizeof (int));
    int *dst = (int *) shmem_malloc (N * sizeof (int));
    for (int i = 0; i < N; ++i)
        src[i] = i * 7 + me * 1000003;
    shmem_barrier_all ();
    shmem_int_sum_to_all (dst, src, N, 0, 0, npes, pWrk, pSync);
    int bad = 0;
    for (int i = 0; i < N; ++i) {
        unsigned want = 0;
        for (int p = 0; p < npes; ++p)
            want += (unsigned) (i * 7 + p * 1000003);
        bad += dst[i] != (int) want;
    }
    shmem_barrier_all (); /* pSync may be reused after a barrier */

    /* device-resident: the array never leaves HBM */
    double *dsrc = (double *) shmemx_malloc_device (N * sizeof (double));
    double *ddst = (double *) shmemx_malloc_device (N * sizeof (double));
    double host[N];
    for (int i = 0; i < N; ++i)
        host[i] = 0.5 * i + me;
    shmemx_memcpy (dsrc, host, sizeof host);
    shmem_double_max_to_all (ddst, dsrc, N, 0, 0, npes, (double *) pWrk, pSync);
    shmemx_memcpy (host, ddst, sizeof host);
    for (int i = 0; i < N; ++i)
        bad += host[i] != 0.5 * i + (npes - 1);

    printf ("PE %d of %d: %s\n", me, npes, bad ? "FAILED" : "ok");
    shmemx_free_device (ddst);
    shmemx_free_device (dsrc);
    shmem_free (dst);
    shmem_free (src);
    shmem_finalize ();
    return bad != 0;
}
