/*
 * rccl.c -- optional RCCL (ncclAllReduce over xGMI) schedule.
 *
 * Used when SHMEM_REDUCE_ALGORITHM=rccl, the active set is the whole job and
 * RCCL has the operator/type (rccl.h: ncclRedOp_t has sum/prod/max/min only,
 * no 16-bit integer, no complex multiply). RCCL's reduction order differs
 * from the reference's, so floating-point results on this path are within
 * the tolerance stated in DESIGN.md, not bit-exact.
 */
#define _DEFAULT_SOURCE
#include <stdio.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <rccl/rccl.h>

#include "mi355_reduce.h"
#include "shmemi.h"

int shmemi_rccl_supported (int op, int dtype)
{
    if (op == MI355_OP_AND || op == MI355_OP_OR || op == MI355_OP_XOR)
        return 0;
    switch (dtype) {
    case MI355_SHORT: /* widened to int32 through scratch C */
    case MI355_INT:
    case MI355_LONG:
    case MI355_LONGLONG:
    case MI355_FLOAT:
    case MI355_DOUBLE:
        return 1;
    case MI355_COMPLEXF:
    case MI355_COMPLEXD:
        return op == MI355_OP_SUM; /* component-wise */
    default:
        return 0;
    }
}

static double mono_s (void)
{
    struct timespec ts;
    clock_gettime (CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

/* Wait for a non-blocking communicator's pending work (init or an enqueue)
 * with a deadline; ncclSuccess, an error, or ncclInProgress on timeout. */
static ncclResult_t rccl_settle (ncclComm_t c, ncclResult_t r, double timeout_s)
{
    const double t0 = mono_s ();
    while (r == ncclInProgress) {
        if (mono_s () - t0 > timeout_s)
            return ncclInProgress;
        usleep (50);
        if (ncclCommGetAsyncError (c, &r) != ncclSuccess)
            return ncclSystemError;
    }
    return r;
}

/* The whole job's communicator, created non-blocking so a peer that never
 * arrives cannot hang this PE: 0, or -1 (nothing kept) when RCCL did not come
 * up within timeout_s. The unique id travels through the bootstrap segment. */
static int rccl_comm_create (double timeout_s, char *why, size_t why_len)
{
    ncclUniqueId id;
    _Static_assert (sizeof id <= sizeof shmemi.seg->rccl_id, "ncclUniqueId too large");
    memset (&id, 0, sizeof id);
    const int id_failed = shmemi.mype == 0 && ncclGetUniqueId (&id) != ncclSuccess;
    if (id_failed)
        memset (&id, 0, sizeof id); /* published as all zero: every PE gives up */
    if (shmemi.seg != NULL) { /* one PE has no bootstrap segment */
        if (shmemi.mype == 0)
            memcpy (shmemi.seg->rccl_id, &id, sizeof id);
        shmemi_barrier_set (0, 1, shmemi.npes);
        memcpy (&id, shmemi.seg->rccl_id, sizeof id);
    }
    static const ncclUniqueId zero_id;
    if (id_failed || memcmp (&id, &zero_id, sizeof id) == 0) {
        snprintf (why, why_len, "ncclGetUniqueId failed on PE 0");
        return -1;
    }
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclComm_t c = NULL;
    ncclResult_t r = ncclCommInitRankConfig (&c, shmemi.npes, id, shmemi.mype, &cfg);
    if (c != NULL)
        r = rccl_settle (c, r, timeout_s);
    if (r != ncclSuccess) {
        snprintf (why, why_len, "ncclCommInitRankConfig: %s",
                  r == ncclInProgress ? "timed out" : ncclGetErrorString (r));
        if (c != NULL)
            ncclCommAbort (c);
        return -1;
    }
    shmemi.rccl_comm = (void *) c;
    return 0;
}

int shmemi_rccl_comm (void **comm)
{
    if (shmemi.rccl_comm == NULL) {
        char why[160] = "";
        if (rccl_comm_create (shmemi.barrier_timeout, why, sizeof why) != 0)
            shmemi_fatal ("RCCL communicator: %s", why);
        shmemi_barrier_set (0, 1, shmemi.npes);
    }
    *comm = shmemi.rccl_comm;
    return 0;
}

/* Bring RCCL up without aborting the job when it cannot: 0 when the
 * communicator exists on this PE, -1 otherwise (callers agree among
 * themselves before relying on it, e.g. with a min reduction). */
int shmemx_rccl_init (double timeout_s)
{
    shmemi_init_check ("shmemx_rccl_init");
    if (shmemi.heap != NULL)
        shmemi_server_stop ();
    if (shmemi.rccl_comm != NULL)
        return 0;
    char why[160] = "";
    const int rc = rccl_comm_create (timeout_s, why, sizeof why);
    if (rc != 0)
        fprintf (stderr, "[shmem PE %d] RCCL unavailable: %s\n", shmemi.mype, why);
    return rc;
}

void shmemi_rccl_destroy (void)
{
    if (shmemi.rccl_comm != NULL) {
        ncclCommDestroy ((ncclComm_t) shmemi.rccl_comm);
        shmemi.rccl_comm = NULL;
    }
}

static int rccl_allreduce_short (int op, const void *src, void *dst, size_t n);

int shmemi_rccl_allreduce (int op, int dtype, const void *src, void *dst, size_t n)
{
    shmemi_server_stop (); /* RCCL's kernels wait on the peers too */
    if (dtype == MI355_SHORT)
        return rccl_allreduce_short (op, src, dst, n);
    ncclDataType_t t;
    size_t count = n;
    switch (dtype) {
    case MI355_INT: t = ncclInt32; break;
    case MI355_LONG:
    case MI355_LONGLONG: t = ncclInt64; break;
    case MI355_FLOAT: t = ncclFloat32; break;
    case MI355_DOUBLE: t = ncclFloat64; break;
    case MI355_COMPLEXF: t = ncclFloat32; count = 2 * n; break;
    case MI355_COMPLEXD: t = ncclFloat64; count = 2 * n; break;
    default: return -1;
    }
    ncclRedOp_t o;
    switch (op) {
    case MI355_OP_SUM: o = ncclSum; break;
    case MI355_OP_PROD: o = ncclProd; break;
    case MI355_OP_MIN: o = ncclMin; break;
    case MI355_OP_MAX: o = ncclMax; break;
    default: return -1;
    }
    void *comm = NULL;
    shmemi_rccl_comm (&comm);
    shmemi_timed_marker (0);
    ncclResult_t r = ncclAllReduce (src, dst, count, t, o, (ncclComm_t) comm, shmemi.stream);
    shmemi_timed_marker (1);
    r = rccl_settle ((ncclComm_t) comm, r, shmemi.barrier_timeout); /* non-blocking communicator */
    if (r == ncclSuccess) {
        /* the collective runs on the library stream: wait for it with the same
         * deadline (a peer whose enqueue failed never joins it) */
        const double t0 = mono_s ();
        hipError_t e;
        while ((e = hipStreamQuery (shmemi.stream)) == hipErrorNotReady) {
            if (mono_s () - t0 > shmemi.barrier_timeout) {
                r = ncclInProgress;
                break;
            }
            usleep (20);
        }
        if (r == ncclSuccess && e != hipSuccess)
            shmemi_hip_check (e, "hipStreamQuery after ncclAllReduce");
    }
    if (r != ncclSuccess) {
        /* drop the communicator: its queued work must not write dst later */
        ncclCommAbort ((ncclComm_t) comm);
        shmemi.rccl_comm = NULL;
        return -1;
    }
    return 0;
}

/* short: widen a chunk into the first half of scratch C, ncclAllReduce int32
 * into the second half, truncate into dst. Scratch C is free here: the
 * callers' sources/targets are user buffers or scratch A/B (staged()). */
static int rccl_allreduce_short (int op, const void *src, void *dst, size_t n)
{
    const size_t half = shmemi.scratch_chunk / 2 / 256 * 256;
    const size_t per = half / sizeof (int32_t);
    char *win = shmemi.heap + shmemi.scratch_off + 2 * shmemi.scratch_chunk, *wout = win + half;
    for (size_t b = 0; b < n; b += per) {
        const size_t cn = n - b < per ? n - b : per;
        if (mi355_convert_short (1, (const short *) src + b, win, cn, shmemi.stream) != 0)
            return -1;
        if (shmemi_rccl_allreduce (op, MI355_INT, win, wout, cn) != 0) /* synchronizes the stream */
            return -1;
        if (mi355_convert_short (0, wout, (short *) dst + b, cn, shmemi.stream) != 0)
            return -1;
    }
    SHMEMI_HIP (hipStreamSynchronize (shmemi.stream));
    return 0;
}
