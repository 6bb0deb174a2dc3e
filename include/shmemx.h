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
/* PE pe's copy of the device-heap object at ptr as an address kernels on this
 * PE's GPU can load from and store to (an IPC mapping of pe's heap; xGMI
 * traffic when pe is on another GPU); NULL if ptr is not in the device heap or
 * pe's heap is not mapped. Not dereferenceable by the host. */
void *shmemx_peer_device_ptr (const void *ptr, int pe);

/* Device buffers outside the heap (hipMalloc, a framework's tensors) as
 * *_to_all target/source with PE_size > 1: the members export the
 * allocations holding them (IPC), map each other's for the call and reduce
 * in place of staging them through scratch -- one host barrier per call for
 * the exchange, no copies. Applies when every member passes device memory
 * of the same kinds (heap / not heap) for target and for source, 16-byte
 * aligned, target == source or disjoint, and every allocation can be
 * exported (hipMalloc yes, virtual-memory hipMemCreate no); otherwise every
 * member stages, as with SHMEM_EXTERNAL_MAP=0. Mapped allocations stay open
 * for later calls (at most SHMEM_EXTERNAL_MAP_CACHE, default 64; they keep
 * the peer's memory alive after it frees it): flush closes them all on this
 * PE; stats = allocations mapped now, opened and closed since init. */
void shmemx_external_map_flush (void);
void shmemx_external_map_stats (long *mapped, long *opened, long *closed);
/* Calls on mapped buffers that staged instead because a member could not open
 * a peer's buffer (its export is re-made for the next call). */
long shmemx_external_map_fallbacks (void);

/* Cross-PE schedule for *_to_all (env SHMEM_REDUCE_ALGORITHM sets the
 * default at init):
 *   SHMEMX_REDUCE_AUTO  = P2P shard schedule (below)
 *   SHMEMX_REDUCE_P2P   = each PE reduces 1/N of the elements from every
 *                         PE's source over xGMI, then gathers the other
 *                         shards; every PE receives the reference's result
 *                         for itself (or PE_start's, see the result order)
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
/* The schedule thresholds at run time (defaults: SHMEM_FUSED_MAX_BYTES = 2 MiB,
 * SHMEM_ONESHOT_MAX_BYTES = 64 KiB): messages up to fused_max bytes per PE
 * take the one-launch fused kernel (capped at 1 GiB; 0 = never), those up to
 * oneshot_max of them its one-shot fold. Collective settings like the
 * algorithm: every PE sets the same value between calls (SHMEM_DEBUG=1
 * checks both per call). Return the previous value. A fused path that the
 * init self-test turned off stays off. */
size_t shmemx_set_fused_max_bytes (size_t bytes);
size_t shmemx_set_oneshot_max_bytes (size_t bytes);
size_t shmemx_get_fused_max_bytes (void);
size_t shmemx_get_oneshot_max_bytes (void);
/* Whether init set the two thresholds above from measurement (PE_size > 1,
 * SHMEM_FUSED_MAX_BYTES / SHMEM_ONESHOT_MAX_BYTES not given,
 * SHMEM_THRESHOLD_CALIBRATE not 0): 1 if it did. us[0..21] (n entries
 * filled): the job-wide median call times in microseconds of the measured
 * double sums -- fused then multi-launch at 64K, 256K, 512K, 1M, 2M, 4M
 * bytes, one-shot then two-shot at 16K, 32K, 64K, 128K, 256K (0: size not
 * measured, larger than the scratch buffers). Each threshold is the largest
 * size of the prefix of sizes where the fused (one-shot) call was no slower. */
int shmemx_threshold_calibration (double *us, int n);

/* Whose result the P2P schedules (and the stream-ordered calls) deliver
 * (env SHMEM_REDUCE_ORDER=reference|pe_start sets the default at init):
 *   SHMEMX_ORDER_REFERENCE (default) = every PE receives the result the
 *       reference computes on THAT PE: its own source first, then the others
 *       in ascending active-set order (reduce-op.c:226-264). Where the order
 *       matters (floating-point sum/prod from 3 PEs, floating-point min/max
 *       from 2: rounding, NaN and +-0 selects) the owner of each shard folds it
 *       in every member's order in one pass over the sources and each PE
 *       gathers its own version: the same xGMI traffic as the shard schedule,
 *       plus (N-1)/N of the message written to local HBM.
 *   SHMEMX_ORDER_PE_START = every PE receives PE_start's result (identical bits
 *       on all PEs, the plain shard schedule).
 * Integer and bitwise reductions are order-independent: both give the same. */
enum shmemx_reduce_order {
    SHMEMX_ORDER_REFERENCE = 0,
    SHMEMX_ORDER_PE_START = 1
};
int shmemx_set_reduce_order (int order); /* returns the previous one */
int shmemx_get_reduce_order (void);
/* The schedule and the result order are per-PE settings, but they decide
 * what the members do together: every member of an active set must use the
 * same algorithm, order and SHMEM_DEVICE_ORDER_SIZE when it calls, or one PE
 * may take the fused path while another takes the multi-launch one (a hang),
 * or gather version areas its peers never wrote. Init aborts when the PEs'
 * environment settings differ; SHMEM_DEBUG=1 also checks every call (below).
 * With 2 PEs, floating-point sum and product are computed once (a + b is
 * b + a) and both PEs get the same bits; for float and double (and their
 * complex types), where both operands are NaNs with different payloads, the
 * reference's PE 1 would keep its own operand's payload (x86 SSE returns the
 * first operand's), so the payload -- not the NaN-ness -- may differ from the
 * reference's there (tests/_compare.py compares those NaNs whatever the
 * payload). Long double is exact, payloads included: the x87 picks between
 * two NaNs by their kind and significand, not by operand position.
 *
 * SHMEM_DEBUG=1: every *_to_all call (host API and stream-ordered) first
 * exchanges its arguments with the other members of its active set -- op,
 * type, nreduce, PE_start, logPE_stride, PE_size, the target/source memory
 * kinds and their symmetric-heap offsets, the algorithm and order settings --
 * and aborts every PE with a message naming the first field that differs
 * (the reference's debug build checks init and symmetry,
 * src/reduce/reduce-op.c:395-398, src/utils/utils.h:74-129). Costs two host
 * barriers per call. The exchange runs on the host when the call is issued,
 * so a stream-ordered call captured into a HIP graph is checked once, at
 * capture time: its replays repeat the captured arguments and are not
 * checked again. */

/* Persistent fused server (opt-in; env SHMEM_PERSISTENT=1 sets it at init,
 * SHMEM_PERSISTENT_IDLE_US = how long it stays without a call, default 1000):
 * back-to-back blocking reductions of one (type, op, active set) that take
 * the one-launch fused schedule (up to SHMEM_FUSED_MAX_BYTES, device-resident
 * symmetric buffers) are served by a fused kernel left resident between
 * calls, fed through a host-coherent mailbox: no launch per call. Results are
 * those of the launched kernel. Caveats, hence opt-in: a served call is not
 * ordered after GPU work the caller queued -- complete it first (the caller's
 * writes to the source must be done); and while the server is resident, HIP
 * calls that wait on the null stream or the whole device (hipDeviceSynchronize,
 * hipStreamSynchronize(0), hipMemcpy) return only once it idles out -- on this
 * HIP the null stream waits for the server's non-blocking stream too.
 * shmemx_device_synchronize and every other GPU operation of this library
 * stop it first. */
int shmemx_set_persistent (int enable); /* returns the previous setting */
/* since init: calls served by a resident server, servers launched */
void shmemx_persistent_stats (long *served, long *launched);

/* Device and timing helpers (used by bench.py and the tests). */
int shmemx_device_id (void);                 /* HIP ordinal of this PE's GPU */
/* Link from this PE's GPU to PE pe's: type (hsa_amd_link_info_type_t: 4 =
 * xGMI, 2 = PCIe) and hop count; -1 if pe shares this GPU or is not visible. */
int shmemx_peer_link (int pe, int *link_type, int *hops);
/* 1 if PE pe's GPU is this PE's GPU (same PCI bus id), else 0. */
int shmemx_pe_same_device (int pe);
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
/* the same for one phase: 0 = each call's dominant kernel (the fold, or a 1-PE call's copy; what
 * shmemx_kernel_timing_stats reports), 1 = the all-gather copy of the P2P schedule */
void shmemx_kernel_timing_phase_stats (int phase, long *launches, double *total_ms, double *avg_ms);

/* What this PE's last *_to_all call ran (host API and stream-ordered calls):
 * the schedule, the dominant kernel -- the reduce-scatter fold of the P2P
 * schedules, the copy of a 1-PE call, the fused kernel -- and the bytes that
 * kernel streams, computed from the schedule the library chose, not assumed
 * by the caller. Returns 0, or -1 before the first call. */
typedef struct shmemx_call_info {
    char schedule[64];      /* "p2p", "p2p-rounds", "fused-oneshot", "fused-twoshot", "persistent",
                             * "identity", "exact", "rccl", "staged", "barrier-only" */
    char kernel[256];       /* demangled dominant kernel, as rocprofv3 names it ("" for rccl) */
    int ordered;            /* 1: every member's reference order (version areas written) */
    int sources, outputs;   /* buffers the dominant kernel reads / writes */
    int peer_sources;       /* of its sources, how many lie in other PEs' heaps */
    int launches;           /* dominant-kernel launches in the call (rounds) */
    unsigned long long bytes_per_buffer;  /* bytes of each source and output, per launch */
    unsigned long long alg_bytes;         /* (sources + outputs) x bytes_per_buffer, + the fused
                                           * two-shot's gather (2 (N-1) shards) */
    unsigned long long peer_bytes;        /* of alg_bytes, read from other PEs' heaps */
} shmemx_call_info;
int shmemx_last_call_info (shmemx_call_info *info);

/* The init-time coherence self-test of peer-heap reads (PE_size > 1 jobs):
 * every PE reads every peer's marker through its L2 (a cached load), each
 * peer rewrites its marker with a write-through store, and after a barrier
 * the reader re-reads it once without and once after mi355_acquire_system.
 * ran: the test ran (peer heaps mapped); passed: the re-read after the
 * acquire saw every new value on every PE (else the job runs the RCCL
 * schedule, like a failed mapping); stale_without_acquire: some PE's re-read
 * WITHOUT the acquire returned an old value (evidence that the acquire the
 * P2P schedules queue before reading peers' buffers is needed). All three
 * are the job's (OR / AND over the PEs). */
void shmemx_coherence_selftest (int *ran, int *passed, int *stale_without_acquire);
/* The same test's check of system-coherent loads (sc0 sc1, the fused kernel's
 * reads of the members' buffers), made before any acquire: sysload_fresh =
 * every block of every PE saw every peer's new value; acquires_skipped = the
 * fused kernel therefore runs without its per-block system-scope acquires
 * (SHMEM_FUSED_ACQUIRE=1 keeps them). */
void shmemx_coherence_sysload (int *sysload_fresh, int *acquires_skipped);
/* The init test of the CALLER's producer path (round 4): every PE wrote 32
 * words with plain stores from a kernel on the null stream, as a caller
 * writes its source, and every peer re-read them (after caching the old
 * values) in the fused kernel's ordering (same-stream flag, device wait) and
 * in the multi-launch schedules' (signal kernel, host wait, host barrier).
 * fresh[6] (1 = every block of every PE saw every new word), in order:
 * fused ordering plain loads / 16-byte system-coherent loads / plain loads
 * after a system-scope acquire, then the same three after the host-wait
 * ordering. The fused kernel skips its acquires only when fresh[1] (and
 * sysload_fresh) hold; it is not used when neither fresh[1] nor fresh[2];
 * the job runs RCCL when fresh[5] fails. ran = 0 above 64 PEs. */
void shmemx_coherence_producer (int *ran, int *fresh);
/* The init timing of device-side waits (PE_size > 1 jobs with signal regions):
 * us = the job's slowest PE's time per device barrier over all PEs; slow = 1
 * when that passed 1 ms (the hardware time-slices the PEs' queues: more PEs
 * on one GPU than it schedules together), and then the job runs host barriers
 * and no fused kernel. */
void shmemx_device_wait_report (int *slow, double *us);

/* Bring up the RCCL communicator of the whole job (what SHMEM_REDUCE_ALGORITHM=rccl uses) without
 * aborting when RCCL cannot come up within timeout_s seconds: 0 = ready on this PE, -1 = not. Every PE
 * must call it; agree on the outcome (e.g. a min reduction) before selecting the RCCL schedule. */
int shmemx_rccl_init (double timeout_s);

/* Stream-ordered collectives. Enqueued on `stream` (a hipStream_t; NULL =
 * the null stream) and return at once: the reduction runs after the work
 * queued on that stream before it, and the work queued after it sees the
 * result. Cross-PE ordering is device-side (a one-launch fused kernel for
 * messages up to SHMEM_FUSED_MAX_BYTES, else fold and gather kernels between
 * one-block device barriers), so a call can be captured into a HIP graph and
 * replayed; every replay is one more collective for all members.
 *   - target and source lie in the device symmetric heap, equal or disjoint
 *   - PE_size <= 32; P2P schedule whatever the reduce algorithm setting,
 *     delivering the result order set by shmemx_set_reduce_order
 *   - every member issues the same sequence of collectives, host-side and
 *     stream-ordered interleaved in the same order; one PE's stream-ordered
 *     calls run one at a time: one stream, or streams the caller orders
 *     (host-side calls use separate device flags and may overlap them)
 *   - a device-side wait that times out (SHMEM_BARRIER_TIMEOUT) is reported
 *     by the next shmem_barrier_all / shmem_quiet / stream-ordered call
 * pWrk and pSync are accepted for symmetry with shmem_*_to_all and unused. */
void shmemx_barrier_on_stream (int PE_start, int logPE_stride, int PE_size, void *stream);
void shmemx_short_sum_to_all_on_stream (short *target, short *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        short *pWrk, long *pSync, void *stream);
void shmemx_int_sum_to_all_on_stream (int *target, int *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        int *pWrk, long *pSync, void *stream);
void shmemx_long_sum_to_all_on_stream (long *target, long *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        long *pWrk, long *pSync, void *stream);
void shmemx_longlong_sum_to_all_on_stream (long long *target, long long *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        long long *pWrk, long *pSync, void *stream);
void shmemx_float_sum_to_all_on_stream (float *target, float *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        float *pWrk, long *pSync, void *stream);
void shmemx_double_sum_to_all_on_stream (double *target, double *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        double *pWrk, long *pSync, void *stream);
void shmemx_longdouble_sum_to_all_on_stream (long double *target, long double *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        long double *pWrk, long *pSync, void *stream);
void shmemx_complexf_sum_to_all_on_stream (COMPLEXIFY (float) *target, COMPLEXIFY (float) *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        COMPLEXIFY (float) *pWrk, long *pSync, void *stream);
void shmemx_complexd_sum_to_all_on_stream (COMPLEXIFY (double) *target, COMPLEXIFY (double) *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        COMPLEXIFY (double) *pWrk, long *pSync, void *stream);
void shmemx_short_prod_to_all_on_stream (short *target, short *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        short *pWrk, long *pSync, void *stream);
void shmemx_int_prod_to_all_on_stream (int *target, int *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        int *pWrk, long *pSync, void *stream);
void shmemx_long_prod_to_all_on_stream (long *target, long *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        long *pWrk, long *pSync, void *stream);
void shmemx_longlong_prod_to_all_on_stream (long long *target, long long *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        long long *pWrk, long *pSync, void *stream);
void shmemx_float_prod_to_all_on_stream (float *target, float *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        float *pWrk, long *pSync, void *stream);
void shmemx_double_prod_to_all_on_stream (double *target, double *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        double *pWrk, long *pSync, void *stream);
void shmemx_longdouble_prod_to_all_on_stream (long double *target, long double *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        long double *pWrk, long *pSync, void *stream);
void shmemx_complexf_prod_to_all_on_stream (COMPLEXIFY (float) *target, COMPLEXIFY (float) *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        COMPLEXIFY (float) *pWrk, long *pSync, void *stream);
void shmemx_complexd_prod_to_all_on_stream (COMPLEXIFY (double) *target, COMPLEXIFY (double) *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        COMPLEXIFY (double) *pWrk, long *pSync, void *stream);
void shmemx_short_and_to_all_on_stream (short *target, short *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        short *pWrk, long *pSync, void *stream);
void shmemx_int_and_to_all_on_stream (int *target, int *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        int *pWrk, long *pSync, void *stream);
void shmemx_long_and_to_all_on_stream (long *target, long *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        long *pWrk, long *pSync, void *stream);
void shmemx_longlong_and_to_all_on_stream (long long *target, long long *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        long long *pWrk, long *pSync, void *stream);
void shmemx_short_or_to_all_on_stream (short *target, short *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        short *pWrk, long *pSync, void *stream);
void shmemx_int_or_to_all_on_stream (int *target, int *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        int *pWrk, long *pSync, void *stream);
void shmemx_long_or_to_all_on_stream (long *target, long *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        long *pWrk, long *pSync, void *stream);
void shmemx_longlong_or_to_all_on_stream (long long *target, long long *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        long long *pWrk, long *pSync, void *stream);
void shmemx_short_xor_to_all_on_stream (short *target, short *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        short *pWrk, long *pSync, void *stream);
void shmemx_int_xor_to_all_on_stream (int *target, int *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        int *pWrk, long *pSync, void *stream);
void shmemx_long_xor_to_all_on_stream (long *target, long *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        long *pWrk, long *pSync, void *stream);
void shmemx_longlong_xor_to_all_on_stream (long long *target, long long *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        long long *pWrk, long *pSync, void *stream);
void shmemx_short_max_to_all_on_stream (short *target, short *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        short *pWrk, long *pSync, void *stream);
void shmemx_int_max_to_all_on_stream (int *target, int *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        int *pWrk, long *pSync, void *stream);
void shmemx_long_max_to_all_on_stream (long *target, long *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        long *pWrk, long *pSync, void *stream);
void shmemx_longlong_max_to_all_on_stream (long long *target, long long *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        long long *pWrk, long *pSync, void *stream);
void shmemx_float_max_to_all_on_stream (float *target, float *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        float *pWrk, long *pSync, void *stream);
void shmemx_double_max_to_all_on_stream (double *target, double *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        double *pWrk, long *pSync, void *stream);
void shmemx_longdouble_max_to_all_on_stream (long double *target, long double *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        long double *pWrk, long *pSync, void *stream);
void shmemx_short_min_to_all_on_stream (short *target, short *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        short *pWrk, long *pSync, void *stream);
void shmemx_int_min_to_all_on_stream (int *target, int *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        int *pWrk, long *pSync, void *stream);
void shmemx_long_min_to_all_on_stream (long *target, long *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        long *pWrk, long *pSync, void *stream);
void shmemx_longlong_min_to_all_on_stream (long long *target, long long *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        long long *pWrk, long *pSync, void *stream);
void shmemx_float_min_to_all_on_stream (float *target, float *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        float *pWrk, long *pSync, void *stream);
void shmemx_double_min_to_all_on_stream (double *target, double *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        double *pWrk, long *pSync, void *stream);
void shmemx_longdouble_min_to_all_on_stream (long double *target, long double *source,
        int nreduce, int PE_start, int logPE_stride, int PE_size,
        long double *pWrk, long *pSync, void *stream);


#ifdef __cplusplus
}
#endif

#endif /* _SHMEMX_H */
