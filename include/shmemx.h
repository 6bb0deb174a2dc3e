/*
 * shmemx.h -- MI355X extensions around the reduction path.
 *
 * Not part of the reference API (its experimental header src/shmemx.h holds
 * nb put/get and wtime, none of which this build provides except wtime).
 * These entry points let a caller keep reduction buffers device-resident in
 * the GPU symmetric heap and let the bench observe
 * kernel time on the library's own stream.
 */
#ifndef _SHMEMX_H
#define _SHMEMX_H 1

#include <stddef.h>
#include <shmem.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Device symmetric heap: memory in this PE's HBM, at the same offset from
 * the heap base on every PE, mapped into every peer GPU over xGMI.
 * Collective (all PEs call with the same size, like shmem_malloc). */
void *shmemx_malloc_device (size_t size);
void shmemx_free_device (void *ptr);
/* 1 if ptr lies in this PE's device symmetric heap. */
int shmemx_is_device_symmetric (const void *ptr);

/* Cross-PE schedule for *_to_all (env SHMEM_REDUCE_ALGORITHM sets the
 * default at init):
 *   SHMEMX_REDUCE_AUTO  = P2P shard schedule (below)
 *   SHMEMX_REDUCE_P2P   = each PE reduces 1/N of the elements from every
 *                         PE's source over xGMI, then gathers the other
 *                         shards; every PE receives identical bits, equal to
 *                         the reference's result on PE_start
 *   SHMEMX_REDUCE_EXACT = each PE folds all N sources in the reference order
 *                         (own first, then ascending); bit-identical to the
 *                         reference on every PE
 *   SHMEMX_REDUCE_RCCL  = ncclAllReduce where RCCL has the op/type, P2P
 *                         otherwise (FP results within the stated tolerance)
 */
enum shmemx_reduce_algorithm {
    SHMEMX_REDUCE_AUTO = 0,
    SHMEMX_REDUCE_P2P = 1,
    SHMEMX_REDUCE_EXACT = 2,
    SHMEMX_REDUCE_RCCL = 3
};
int shmemx_set_reduce_algorithm (int algorithm); /* returns the previous one */
int shmemx_get_reduce_algorithm (void);

/* Device and timing helpers (used by bench.py and the tests). */
int shmemx_device_id (void);                 /* HIP ordinal of this PE's GPU */
void shmemx_device_synchronize (void);        /* hipDeviceSynchronize, checked */
/* hipMemcpy (kind inferred from the pointers), checked; blocking. */
void shmemx_memcpy (void *dst, const void *src, size_t nbytes);
double shmemx_wtime (void);                   /* seconds, monotonic */

/* Kernel timing: while enabled, every dominant kernel the reduction path
 * launches is bracketed by HIP events on the library's stream. */
void shmemx_kernel_timing (int enable);        /* enable resets the counters */
/* Number of timed launches, total and per-launch average duration (ms) of the
 * launches timed since the last enable. Synchronizes the stream. */
void shmemx_kernel_timing_stats (long *launches, double *total_ms, double *avg_ms);

#ifdef __cplusplus
}
#endif

#endif /* _SHMEMX_H */
