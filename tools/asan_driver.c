/*
 * asan_driver.c -- walks the library's host code paths for the host-side
 * AddressSanitizer/UBSan build (tools/asan_check.sh): reductions on
 * shmem_malloc host arrays (staged), device symmetric arrays (fused and
 * multi-launch), in place, overlapping, on plain hipMalloc memory (staged
 * device), the stream-ordered variant, n = 0, a strided active set, and the
 * data-movement calls. Integer inputs, so every expected value is exact.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>
#include <shmem.h>
#include <shmemx.h>

static long pSync[SHMEM_REDUCE_SYNC_SIZE];
static long pWrk[SHMEM_REDUCE_MIN_WRKDATA_SIZE];
static int me, npes, bad;

#define HIP_OK(call)                                                                           \
    do {                                                                                       \
        hipError_t e_ = (call);                                                                \
        if (e_ != hipSuccess) {                                                                \
            fprintf (stderr, "PE %d: %s failed: %s\n", me, #call, hipGetErrorString (e_));     \
            exit (1);                                                                          \
        }                                                                                      \
    } while (0)

static long src_val (long i, int pe) { return 3 * i + pe; }

/* sum over the members {start + k*stride} of src_val */
static long want_sum (long i, int start, int stride, int size)
{
    long v = 0;
    for (int k = 0; k < size; ++k)
        v += src_val (i, start + k * stride);
    return v;
}

static void check (const char *what, const long *got, long n, long shift, int start, int stride, int size)
{
    for (long i = 0; i < n; ++i)
        if (got[i] != want_sum (i + shift, start, stride, size)) {
            printf ("PE %d %s: element %ld = %ld, want %ld\n", me, what, i, got[i],
                    want_sum (i + shift, start, stride, size));
            bad = 1;
            return;
        }
}

static void fill_host (long *p, long n, long shift)
{
    for (long i = 0; i < n; ++i)
        p[i] = src_val (i + shift, me);
}

static void fill_dev (long *d, long n, long shift, long *tmp)
{
    fill_host (tmp, n, shift);
    HIP_OK (hipMemcpy (d, tmp, n * sizeof (long), hipMemcpyHostToDevice));
}

static void read_dev (long *h, const long *d, long n)
{
    HIP_OK (hipMemcpy (h, d, n * sizeof (long), hipMemcpyDeviceToHost));
}

int main (void)
{
    for (int i = 0; i < SHMEM_REDUCE_SYNC_SIZE; ++i)
        pSync[i] = SHMEM_SYNC_VALUE;
    shmem_init ();
    me = shmem_my_pe ();
    npes = shmem_n_pes ();
    const long sizes[] = {0, 1, 1000, 300000};
    const long NMAX = 300000 + 16;
    long *tmp = (long *) malloc (NMAX * sizeof (long));
    long *hs = (long *) shmem_malloc (NMAX * sizeof (long));
    long *ht = (long *) shmem_malloc (NMAX * sizeof (long));
    long *ds = (long *) shmemx_malloc_device (NMAX * sizeof (long));
    long *dt = (long *) shmemx_malloc_device (NMAX * sizeof (long));
    long *priv = NULL;
    HIP_OK (hipMalloc ((void **) &priv, NMAX * sizeof (long)));
    hipStream_t st;
    HIP_OK (hipStreamCreate (&st));

    for (size_t z = 0; z < sizeof sizes / sizeof sizes[0]; ++z) {
        const long n = sizes[z];
        char what[64];
        /* host arrays: staged through the GPU */
        fill_host (hs, n, 0);
        shmem_long_sum_to_all (ht, hs, (int) n, 0, 0, npes, pWrk, pSync);
        snprintf (what, sizeof what, "host n=%ld", n);
        check (what, ht, n, 0, 0, 1, npes);
        shmem_barrier_all ();
        /* device symmetric arrays */
        fill_dev (ds, n, 0, tmp);
        shmem_long_sum_to_all (dt, ds, (int) n, 0, 0, npes, pWrk, pSync);
        read_dev (tmp, dt, n);
        snprintf (what, sizeof what, "device n=%ld", n);
        check (what, tmp, n, 0, 0, 1, npes);
        shmem_barrier_all ();
        /* in place */
        fill_dev (ds, n, 0, tmp);
        shmem_long_sum_to_all (ds, ds, (int) n, 0, 0, npes, pWrk, pSync);
        read_dev (tmp, ds, n);
        snprintf (what, sizeof what, "in-place n=%ld", n);
        check (what, tmp, n, 0, 0, 1, npes);
        shmem_barrier_all ();
        /* overlapping: target 5 elements above source */
        fill_dev (ds, n, 0, tmp);
        shmem_long_sum_to_all (ds + 5, ds, (int) n, 0, 0, npes, pWrk, pSync);
        read_dev (tmp, ds + 5, n);
        snprintf (what, sizeof what, "overlap n=%ld", n);
        check (what, tmp, n, 0, 0, 1, npes);
        shmem_barrier_all ();
        /* plain hipMalloc source (not symmetric): staged on the device */
        fill_dev (priv, n, 0, tmp);
        shmem_long_sum_to_all (dt, priv, (int) n, 0, 0, npes, pWrk, pSync);
        read_dev (tmp, dt, n);
        snprintf (what, sizeof what, "hipMalloc source n=%ld", n);
        check (what, tmp, n, 0, 0, 1, npes);
        shmem_barrier_all ();
        /* stream-ordered */
        fill_dev (ds, n, 0, tmp);
        shmemx_long_sum_to_all_on_stream (dt, ds, (int) n, 0, 0, npes, pWrk, pSync, (void *) st);
        HIP_OK (hipStreamSynchronize (st));
        read_dev (tmp, dt, n);
        snprintf (what, sizeof what, "stream n=%ld", n);
        check (what, tmp, n, 0, 0, 1, npes);
        shmem_barrier_all ();
    }

    /* strided set: even PEs and odd PEs separately (logPE_stride 1) */
    if (npes >= 2) {
        const int start = me % 2, size = (npes - start + 1) / 2;
        fill_dev (ds, 4099, 0, tmp);
        shmem_long_sum_to_all (dt, ds, 4099, start, 1, size, pWrk, pSync);
        read_dev (tmp, dt, 4099);
        check ("strided", tmp, 4099, 0, start, 2, size);
        shmem_barrier_all ();
    }

    /* data movement: broadcast from PE 0, fcollect, collect, put/get ring */
    {
        const long m = 777;
        fill_dev (ds, m, 0, tmp);
        HIP_OK (hipMemset (dt, 0, npes * m * sizeof (long)));
        shmem_broadcast64 (dt, ds, m, 0, 0, 0, npes, pSync);
        read_dev (tmp, dt, m);
        if (me != 0)
            for (long i = 0; i < m; ++i)
                if (tmp[i] != src_val (i, 0)) {
                    printf ("PE %d broadcast: element %ld = %ld\n", me, i, tmp[i]);
                    bad = 1;
                    break;
                }
        shmem_barrier_all ();
        shmem_fcollect64 (dt, ds, m, 0, 0, npes, pSync);
        read_dev (tmp, dt, npes * m);
        for (int p = 0; p < npes; ++p)
            for (long i = 0; i < m; ++i)
                if (tmp[p * m + i] != src_val (i, p)) {
                    printf ("PE %d fcollect: PE %d element %ld = %ld\n", me, p, i, tmp[p * m + i]);
                    bad = 1;
                    p = npes;
                    break;
                }
        shmem_barrier_all ();
        shmem_collect64 (dt, ds, (size_t) (me + 1), 0, 0, npes, pSync);
        read_dev (tmp, dt, (long) npes * (npes + 1) / 2);
        long off = 0;
        for (int p = 0; p < npes; ++p)
            for (long i = 0; i <= p; ++i, ++off)
                if (tmp[off] != src_val (i, p)) {
                    printf ("PE %d collect: PE %d element %ld = %ld\n", me, p, i, tmp[off]);
                    bad = 1;
                }
        shmem_barrier_all ();
        const int next = (me + 1) % npes, prev = (me + npes - 1) % npes;
        shmem_long_put (dt, hs, 100, next); /* hs still holds src_val(i, me) */
        shmem_barrier_all ();
        read_dev (tmp, dt, 100);
        for (long i = 0; i < 100; ++i)
            if (tmp[i] != src_val (i, prev)) {
                printf ("PE %d put: element %ld = %ld\n", me, i, tmp[i]);
                bad = 1;
                break;
            }
        shmem_barrier_all ();
        shmem_long_get (ht, ds, 100, next);
        for (long i = 0; i < 100; ++i)
            if (ht[i] != src_val (i, next)) {
                printf ("PE %d get: element %ld = %ld\n", me, i, ht[i]);
                bad = 1;
                break;
            }
        shmem_barrier_all ();
    }

    HIP_OK (hipStreamDestroy (st));
    HIP_OK (hipFree (priv));
    shmemx_free_device (dt);
    shmemx_free_device (ds);
    shmem_free (ht);
    shmem_free (hs);
    free (tmp);
    printf ("PE %d of %d: %s\n", me, npes, bad ? "MISMATCH" : "ok");
    shmem_finalize ();
    return bad;
}
