/*
 * shmemi.h -- internal state of the MI355X reduction runtime (host C).
 *
 * Counterpart of the reference's per-PE state (src/utils/state.h:83-109)
 * cut down to what the reduction path needs, plus the GPU side: the HIP
 * device, the library stream, the device symmetric heap and the peer
 * mappings of every other PE's heap (xGMI).
 */
#ifndef SHMEMI_H
#define SHMEMI_H 1

#include <stddef.h>
#include <stdint.h>
#include <stdatomic.h>

#ifndef __HIP_PLATFORM_AMD__
#define __HIP_PLATFORM_AMD__ 1
#endif
#include <hip/hip_runtime_api.h>

#define SHMEMI_MAX_PES 1024
#define SHMEMI_ALIGN 256

/* ---- bootstrap segment (POSIX shm, one per job, node-local) ---- */

/* SHMEM_DEBUG=1: one collective's arguments as this PE passed them
 * (debug_check, reduce.c; shmemi_debug_exchange, runtime.c). Written under a
 * seqlock (seq odd while being written). */
struct shmemi_dbg_rec {
    _Atomic uint32_t seq;
    int32_t pad0;
    int32_t op, dtype, nreduce, pe_start, log_stride, pe_size;
    int32_t tkind, skind;       /* 0 host, 1 device heap, 2 other device memory */
    int32_t algorithm, order, persistent;
    int32_t overlap;            /* target vs source: 0 disjoint, 1 same, 2 overlapping above, 3 below */
    uint64_t toff, soff;        /* heap offsets (device heap kinds), else 0 */
    uint64_t fused_max, oneshot_max; /* the schedule thresholds (shmemx_set_fused_max_bytes / _oneshot_) */
    char fn[48];
};

/* Settings every PE of a job must share (compared at init). */
struct shmemi_settings {
    int32_t algorithm, order, debug, persistent, ext_map, calibrate;
    uint64_t order_chunk, fused_max, oneshot_max, scratch_chunk, user_size, hheap_size;
};

/* One *_to_all call's device buffers outside the symmetric heap, as this PE
 * passed them (extmap.c): the IPC export of the allocation holding each and
 * the offset in it, or the heap offset of a symmetric one. */
struct shmemi_ext_rec {
    int32_t ok;                 /* both buffers can be shared with the peers */
    int32_t same;               /* target == source */
    int32_t tkind, skind;       /* 1 device heap, 2 other device memory */
    hipIpcMemHandle_t th, sh;
    uint64_t toff, soff;
    int32_t open_ok;            /* second round: this member opened every peer's buffer */
    int32_t pad;
};

/* init-time threshold calibration (reduce.c): fused vs multi-launch at
 * SHMEMI_CALIB_NF sizes, one-shot vs two-shot at SHMEMI_CALIB_NO sizes */
#define SHMEMI_CALIB_NF 6
#define SHMEMI_CALIB_NO 5
#define SHMEMI_CALIB_SLOTS (2 * SHMEMI_CALIB_NF + 2 * SHMEMI_CALIB_NO)

struct shmemi_pe_info {
    int32_t pid;
    int32_t device;
    char pci_bus_id[32];
    hipIpcMemHandle_t heap_handle;
    hipIpcMemHandle_t sig_handle;
    uint64_t heap_size;
    int32_t published;
    int32_t selftest;           /* bit 0: signal region stores seen, bit 1: heap reads ok,
                                   bit 2: coherence test ran, bit 3: it passed, bit 4: stale without acquire,
                                   bit 5: system-coherent loads fresh without an acquire (write-through marker),
                                   bit 6: producer-path test ran, bits 7-12: its six outcomes (1 = fresh) in
                                   shmemi.prod[] order: fused ordering plain / sysload / acquire, then the
                                   host-wait ordering plain / sysload / acquire */
    uint64_t collect_bytes;     /* this PE's contribution to the current shmem_collect */
    uint64_t barrier_ns;        /* init: this PE's time per device barrier over the job (device_wait_test) */
    uint64_t calib_ns[SHMEMI_CALIB_SLOTS]; /* init: this PE's median call times (shmemi_calibrate_thresholds) */
    struct shmemi_settings settings;
    struct shmemi_dbg_rec dbg;
    struct shmemi_ext_rec ext;
};

struct shmemi_seg {
    _Atomic uint64_t magic;     /* written last by the creator */
    int32_t version;
    int32_t npes;
    _Atomic int32_t attached;
    _Atomic int32_t abort_flag;
    int32_t abort_pe;
    int32_t abort_status;
    char abort_msg[256];
    _Atomic int32_t rccl_id_ready;
    int32_t pad0;
    char rccl_id[128];          /* ncclUniqueId from PE 0 */
    uint64_t info_off;          /* -> struct shmemi_pe_info[npes] */
    uint64_t flags_off;         /* -> _Atomic uint64_t flags[npes][row] */
    uint64_t flags_row;         /* words per row (padded) */
    uint64_t dbg_off;           /* -> _Atomic uint64_t dbgcnt[npes][row]: SHMEM_DEBUG checks entered, per pair */
    uint64_t total_size;
};

/* ---- device heap allocator block ---- */
struct shmemi_block {
    size_t off, size;
    int used;
    struct shmemi_block *next;
};

struct shmemi_state {
    int initialized;
    int mype, npes;
    int device;
    hipStream_t stream;
    hipStream_t stream_in, stream_out;  /* staging copies (blocking streams) */
    hipEvent_t ev_in[2], ev_out[2];
    int algorithm;              /* enum shmemx_reduce_algorithm */
    int order;                  /* enum shmemx_reduce_order */
    double barrier_timeout;     /* seconds */
    int debug;
    int entry_sync;             /* SHMEM_ENTRY_SYNC: hipDeviceSynchronize on entry */
    int p2p_broken;             /* init self-test: peer heap reads failed */
    int peer_acquire;           /* queue mi355_acquire_system before reads of peers' buffers */
    int local_pes;              /* PEs on this GPU (this one included): co-residency share of the fused grids */
    int ext_map;                /* SHMEM_EXTERNAL_MAP: peers map device buffers outside the heap (extmap.c) */

    /* bootstrap */
    struct shmemi_seg *seg;
    size_t seg_size;
    char seg_name[128];
    int seg_unlinked;
    uint64_t *bar_count;        /* [npes]: barriers done with each peer */
    uint64_t *dbg_count;        /* [npes]: SHMEM_DEBUG collective checks entered with each peer */

    /* device symmetric heap: [user | scratch] */
    char *heap;                 /* this PE's base */
    char *heap_arena;           /* its hipMalloc'd arena (the heap starts heap_skew(mype) bytes in) */
    size_t heap_size;           /* total */
    size_t user_size;           /* user part */
    size_t scratch_off;         /* = user_size */
    size_t scratch_chunk;       /* bytes per staging buffer (3 buffers) */
    size_t order_off;           /* version areas of the per-PE-order schedule: 2 channels after scratch */
    size_t order_chunk;         /* bytes per channel */
    char **peer_heap;           /* [npes]: mapped base of every PE's heap */
    struct shmemi_block *blocks;

    /* symmetric host heap (hostheap.c): shmem_malloc's blocks */
    char *hheap;                /* this PE's segment */
    size_t hheap_size;          /* SHMEM_SYMMETRIC_HEAP_SIZE, page-rounded */
    int hheap_fd;               /* the shared-memory object (PE_size > 1), else -1 */
    int hheap_named;            /* its name not yet dropped */
    char **peer_hheap;          /* [npes]: every PE's segment, mapped here */
    struct shmemi_hostblk *host_blocks;

    /* [channel * npes + PE]: two-member float/double P2P calls with each PE
     * (reduce.c nan_pair: the parity picks the NaN word of the call) */
    uint64_t *pair_calls;

    /* RCCL */
    void *rccl_comm;            /* ncclComm_t of the whole world, lazily */

    /* signal region for the fused kernel: uncached device memory, mapped by peers */
    unsigned long long *sigmem;
    unsigned long long **peer_sig;  /* [npes] */
    size_t fused_max;           /* SHMEM_FUSED_MAX_BYTES: largest message on the fused path */
    size_t oneshot_max;         /* SHMEM_ONESHOT_MAX_BYTES: largest fused message folded one-shot */
    int fused_off;              /* a failed self-test disabled the fused path: the setters keep it off */
    int calib_want;             /* init-time calibration: bit 0 fused_max, bit 1 oneshot_max (not set by env) */
    int calib_ran;              /* the thresholds above came from the init-time calibration */
    double calib_us[SHMEMI_CALIB_SLOTS]; /* its job-wide (max over PEs) median call times */
    int sig_broken;             /* peers' signal-region stores failed the init self-test */
    int dev_wait_slow;          /* device-side waits across PEs time-sliced (init timing): host barriers, no fused kernel */
    double dev_barrier_us;      /* that timing: the job's slowest PE, microseconds per device barrier */

    /* completion signal: host-coherent word the last block of a kernel writes */
    unsigned *sig_flag;         /* hipHostMalloc coherent+mapped, same address on both sides */
    unsigned *sig_count;        /* device word, 0 between launches */
    unsigned sig_epoch;

    /* stream-ordered collectives (shmemx_*_on_stream, streamops.c) */
    unsigned *stream_err;       /* host-coherent: a device-side wait timed out */

    /* persistent fused server (opt-in, SHMEM_PERSISTENT; reduce.c) */
    struct {
        int enabled;            /* SHMEM_PERSISTENT / shmemx_set_persistent */
        double idle_s;          /* SHMEM_PERSISTENT_IDLE_US: the server exits after this long without a call */
        int running;
        int op, dtype, start, stride, size;  /* the calls it serves */
        int ordered;            /* the result order it was started with (ordered_pair) */
        const void *kernel;     /* its kernel stub (shmemx_last_call_info) */
        unsigned long long grid_elems;       /* the grid it was sized for */
        unsigned seq;           /* next mailbox seq */
        struct MI355ServerMailbox *mb;       /* host-coherent, device-accessible */
        hipStream_t st;         /* non-blocking stream of its own */
        double last_end;        /* when the last fused call returned (burst detection) */
        long served, launched;  /* statistics */
    } srv;

    /* the init-time coherence test of peer-heap reads (job-wide results) */
    int coh_ran, coh_passed, coh_stale;
    /* ... and whether system-coherent loads (the fused kernel's reads of the
     * members' buffers) saw the rewritten data with no acquire at all, on
     * every PE: then the fused kernel skips its per-block acquires
     * (fused_no_acquire; SHMEM_FUSED_ACQUIRE=1 keeps them) */
    int coh_sysload, fused_no_acquire;
    /* the caller's producer path (producer_test, job-wide ANDs): sources
     * written by plain stores in a kernel on the null stream, then read by
     * the peers after the fused kernel's ordering (same-stream flag, device
     * wait: prod[0..2]) and after the multi-launch schedules' ordering (signal
     * kernel, host wait, host barrier: prod[3..5]), each read three ways:
     * plain loads without an acquire, 16-byte system-coherent loads, plain
     * loads after a system-scope acquire (MI355_PROD_* indices) */
    int prod_ran, prod[6];
#define MI355_PROD_F_PLAIN 0
#define MI355_PROD_F_SYS 1
#define MI355_PROD_F_ACQ 2
#define MI355_PROD_H_PLAIN 3
#define MI355_PROD_H_SYS 4
#define MI355_PROD_H_ACQ 5

    /* what the last *_to_all call ran (shmemx_last_call_info); the kernel
     * stub is resolved to its name only on request */
    struct {
        int valid;
        const char *schedule;
        const void *kernel;
        int ordered, sources, outputs, peer_sources, launches;
        unsigned long long bytes_per_buffer, alg_bytes, peer_bytes;
    } last;

    /* kernel timing */
    int timing;
    int ntimed;
    int timed_cap;
    hipEvent_t *ev;             /* 2 per timed launch */
    int *timed_phase;           /* per timed launch: 0 dominant kernel, 1 all-gather copy */
};

extern struct shmemi_state shmemi;

/* runtime.c */
void shmemi_fatal (const char *fmt, ...) __attribute__ ((noreturn, format (printf, 1, 2)));
void shmemi_init_check (const char *fn);
void shmemi_hip_check (hipError_t e, const char *what);
void shmemi_barrier_set (int PE_start, int stride, int PE_size);
void shmemi_barrier_arrive (int PE_start, int stride, int PE_size);
int shmemi_in_device_heap (const void *p, size_t nbytes);
size_t shmemi_heap_offset (const void *p);
void *shmemi_peer_ptr (int pe, size_t off);
int shmemi_pe_same_device (int pe);
void shmemi_order_after_caller (int host_wait);
void shmemi_check_stream_err (const char *fn);
void shmemi_peer_acquire (hipStream_t st);
double shmemi_now (void);

/* hostheap.c: shmem_malloc's symmetric heap in host memory, mapped by every PE */
void shmemi_hheap_create (size_t size);
void shmemi_hheap_attach (void);
void shmemi_hheap_unlink (void);
void shmemi_hheap_finalize (void);
void *shmemi_host_malloc (size_t size);
int shmemi_host_free (void *p);
int shmemi_in_host_heap (const void *p, size_t nbytes);
void *shmemi_host_peer_ptr (int pe, const void *p);
void *shmemi_host_dev_ptr (const void *p, size_t nbytes);

/* reduce.c: the persistent fused server; every GPU operation that could wait
 * on it (another spin-waiting grid, a device-wide synchronization, freeing
 * memory) stops it first */
void shmemi_lazy_stream (hipStream_t *st, unsigned flags);
void shmemi_server_stop (void);

/* reduce.c: device-flag barrier on the library stream (host channel) */
int shmemi_dev_barrier_ok (int PE_start, int stride, int PE_size);
void shmemi_dev_barrier (int PE_start, int stride, int PE_size, int me, int last);
struct MI355FusedArgs;
void shmemi_member_args (struct MI355FusedArgs *a, int PE_start, int stride, int PE_size, int me);
void shmemi_calibrate_thresholds (int fused, int oneshot);
void shmemi_arm_signal (void);
void shmemi_wait_signal (void);
unsigned shmemi_next_epoch (void);
unsigned shmemi_wait_flag (unsigned epoch);
void shmemi_timed_begin (void);
void shmemi_timed_begin_phase (int phase);
void shmemi_timed_end (void);
void shmemi_timed_marker (int end);
int shmemi_rccl_comm (void **comm);
void shmemi_publish_count (size_t nbytes);
size_t shmemi_peer_count (int pe);
/* runtime.c: SHMEM_DEBUG's collective argument exchange over an active set */
void shmemi_debug_exchange (const struct shmemi_dbg_rec *mine, int PE_start, int stride, int PE_size);
struct shmemi_pe_info *shmemi_seg_info (int pe);

/* extmap.c: device buffers outside the symmetric heap reached by the peers
 * through IPC mappings of their allocations. A call that maps them addresses
 * them with the virtual offsets SHMEMI_EXT_TARGET / SHMEMI_EXT_SOURCE (plus
 * the byte offset into the buffer), which shmemi_peer_ptr resolves per PE. */
#define SHMEMI_EXT_TARGET ((size_t) 1 << 60)
#define SHMEMI_EXT_SOURCE ((size_t) 3 << 59)
enum { SHMEMI_PK_HOST = 0, SHMEMI_PK_DEV_SYM = 1, SHMEMI_PK_DEV_OTHER = 2 };
int shmemi_ext_begin (const char *fn, void *target, const void *source, size_t nbytes, int kt, int ks, int PE_start,
                      int stride, int PE_size, size_t *toff, size_t *soff);
void shmemi_ext_end (void);
void *shmemi_ext_ptr (int pe, size_t off);
void shmemi_ext_finalize (void);

#define SHMEMI_HIP(call) shmemi_hip_check ((call), #call)

/* trace.c: env-gated trace lines (SHMEM_LOG_LEVELS, SHMEM_LOG_FILE);
 * levels follow the reference's enum (src/utils/trace.h:59-83) */
enum shmemi_log_level {
    SHMEMI_LOG_DEBUG = 1, SHMEMI_LOG_INFO, SHMEMI_LOG_VERSION, SHMEMI_LOG_INIT, SHMEMI_LOG_FINALIZE,
    SHMEMI_LOG_BARRIER, SHMEMI_LOG_BROADCAST, SHMEMI_LOG_REDUCTION, SHMEMI_LOG_COLLECT, SHMEMI_LOG_QUIET,
    SHMEMI_LOG_MEMORY, SHMEMI_LOG_NOTICE, SHMEMI_LOG_NLEVELS
};
#define SHMEMX_VERSION_STRING "osss-gasnet MI355X reduction path (OpenSHMEM 1.3 API, gfx950)"
extern unsigned shmemi_trace_mask;
void shmemi_trace_init (void);
void shmemi_trace_fini (void);
void shmemi_trace_show_info (void);
void shmemi_trace_show_levels (void);
void shmemi_trace_emit (int level, const char *fmt, ...) __attribute__ ((format (printf, 2, 3)));
#define SHMEMI_TRACE(level, ...)                                                                            \
    do {                                                                                                    \
        if (__builtin_expect (shmemi_trace_mask & (1u << (level)), 0))                                      \
            shmemi_trace_emit ((level), __VA_ARGS__);                                                       \
    } while (0)

#endif /* SHMEMI_H */
