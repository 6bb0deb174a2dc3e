/*
 * stream_example.c -- the stream-ordered reductions from C: a chain of
 * shmemx_long_sum_to_all_on_stream calls queued on a HIP stream with no host
 * wait, then the same chain captured once into a HIP graph and replayed.
 *
 *   gcc -std=c99 -D__HIP_PLATFORM_AMD__ -Iinclude -I/opt/rocm/include examples/stream_example.c \
 *       -Losss-gasnet_amd/lib -lshmem_reduce -L/opt/rocm/lib -lamdhip64 \
 *       -Wl,-rpath,$PWD/osss-gasnet_amd/lib -Wl,-rpath,/opt/rocm/lib -o stream_example
 *   tools/oshrun -np 4 ./stream_example
 *
 * PE p's source holds x[i] = i + p. After one sum over N PEs every element is
 * N*i + N(N-1)/2; each further link of the chain multiplies by N.
 */
#include <stdio.h>
#include <stdlib.h>

#include <hip/hip_runtime_api.h>
#include <shmem.h>
#include <shmemx.h>

#define N 4099 /* not a multiple of the shard alignment */
#define CHAIN 3

static long pSync[SHMEM_REDUCE_SYNC_SIZE];
static long pWrk[N / 2 + 1];

#define HIP_OK(call)                                                               \
    do {                                                                           \
        hipError_t e_ = (call);                                                    \
        if (e_ != hipSuccess) {                                                    \
            fprintf (stderr, "%s failed: %s\n", #call, hipGetErrorString (e_));    \
            return 1;                                                              \
        }                                                                          \
    } while (0)

static long expect (long i, int npes, int links)
{
    long v = (long) npes * i + (long) npes * (npes - 1) / 2;
    for (int k = 1; k < links; ++k)
        v *= npes;
    return v;
}

static int check (const long *got, int npes, int links, const char *what, int me)
{
    for (long i = 0; i < N; ++i)
        if (got[i] != expect (i, npes, links)) {
            printf ("PE %d %s: element %ld = %ld, want %ld\n", me, what, i, got[i], expect (i, npes, links));
            return 1;
        }
    return 0;
}

static void enqueue_chain (long **buf, int npes, hipStream_t st)
{
    for (int k = 0; k < CHAIN; ++k)
        shmemx_long_sum_to_all_on_stream (buf[k + 1], buf[k], N, 0, 0, npes, pWrk, pSync, (void *) st);
}

int main (void)
{
    for (int i = 0; i < SHMEM_REDUCE_SYNC_SIZE; ++i)
        pSync[i] = SHMEM_SYNC_VALUE;
    shmem_init ();
    const int me = shmem_my_pe (), npes = shmem_n_pes ();
    long *buf[CHAIN + 1];
    for (int k = 0; k <= CHAIN; ++k)
        buf[k] = (long *) shmemx_malloc_device (N * sizeof (long));
    long *x = (long *) malloc (N * sizeof (long));
    for (long i = 0; i < N; ++i)
        x[i] = i + me;
    HIP_OK (hipMemcpy (buf[0], x, N * sizeof (long), hipMemcpyHostToDevice));

    hipStream_t st;
    HIP_OK (hipStreamCreate (&st));
    int bad = 0;

    /* 1. queued back to back, one synchronize */
    enqueue_chain (buf, npes, st);
    HIP_OK (hipStreamSynchronize (st));
    for (int k = 1; k <= CHAIN; ++k) {
        HIP_OK (hipMemcpy (x, buf[k], N * sizeof (long), hipMemcpyDeviceToHost));
        bad |= check (x, npes, k, "stream chain", me);
    }

    /* 2. captured once, replayed three times */
    hipGraph_t g;
    hipGraphExec_t ge;
    HIP_OK (hipStreamBeginCapture (st, hipStreamCaptureModeRelaxed));
    enqueue_chain (buf, npes, st);
    HIP_OK (hipStreamEndCapture (st, &g));
    HIP_OK (hipGraphInstantiate (&ge, g, NULL, NULL, 0));
    for (int r = 0; r < 3; ++r) {
        HIP_OK (hipMemset (buf[CHAIN], 0, N * sizeof (long)));
        HIP_OK (hipDeviceSynchronize ());
        HIP_OK (hipGraphLaunch (ge, st));
        HIP_OK (hipStreamSynchronize (st));
        HIP_OK (hipMemcpy (x, buf[CHAIN], N * sizeof (long), hipMemcpyDeviceToHost));
        bad |= check (x, npes, CHAIN, "graph replay", me);
    }
    HIP_OK (hipGraphExecDestroy (ge));
    HIP_OK (hipGraphDestroy (g));
    HIP_OK (hipStreamDestroy (st));

    printf ("PE %d of %d: %s\n", me, npes, bad ? "MISMATCH" : "ok");
    free (x);
    for (int k = CHAIN; k >= 0; --k)
        shmemx_free_device (buf[k]);
    shmem_finalize ();
    return bad;
}
