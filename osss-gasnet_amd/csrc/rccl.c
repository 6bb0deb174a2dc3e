/*
 * rccl.c -- optional RCCL (ncclAllReduce over xGMI) schedule.
 *
 * Used when SHMEM_REDUCE_ALGORITHM=rccl, the active set is the whole job and
 * RCCL has the operator/type (rccl.h: ncclRedOp_t has sum/prod/max/min only,
 * no 16-bit integer, no complex multiply). RCCL's reduction order differs
 * from the reference's, so floating-point results on this path are within
 * the tolerance stated in DESIGN.md, not bit-exact.
 */
#include <string.h>

#include <rccl/rccl.h>

#include "mi355_reduce.h"
#include "shmemi.h"

int shmemi_rccl_supported (int op, int dtype)
{
    if (op == MI355_OP_AND || op == MI355_OP_OR || op == MI355_OP_XOR)
        return 0;
    switch (dtype) {
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

int shmemi_rccl_comm (void **comm)
{
    if (shmemi.rccl_comm == NULL) {
        ncclUniqueId id;
        _Static_assert (sizeof id <= sizeof shmemi.seg->rccl_id, "ncclUniqueId too large");
        if (shmemi.mype == 0 && ncclGetUniqueId (&id) != ncclSuccess)
            shmemi_fatal ("ncclGetUniqueId failed");
        if (shmemi.seg != NULL) { /* one PE has no bootstrap segment */
            if (shmemi.mype == 0)
                memcpy (shmemi.seg->rccl_id, &id, sizeof id);
            shmemi_barrier_set (0, 1, shmemi.npes);
            memcpy (&id, shmemi.seg->rccl_id, sizeof id);
        }
        ncclComm_t c;
        ncclResult_t r = ncclCommInitRank (&c, shmemi.npes, id, shmemi.mype);
        if (r != ncclSuccess)
            shmemi_fatal ("ncclCommInitRank: %s", ncclGetErrorString (r));
        shmemi.rccl_comm = (void *) c;
        shmemi_barrier_set (0, 1, shmemi.npes);
    }
    *comm = shmemi.rccl_comm;
    return 0;
}

void shmemi_rccl_destroy (void)
{
    if (shmemi.rccl_comm != NULL) {
        ncclCommDestroy ((ncclComm_t) shmemi.rccl_comm);
        shmemi.rccl_comm = NULL;
    }
}

int shmemi_rccl_allreduce (int op, int dtype, const void *src, void *dst, size_t n)
{
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
    if (r != ncclSuccess)
        return -1;
    SHMEMI_HIP (hipStreamSynchronize (shmemi.stream));
    return 0;
}
