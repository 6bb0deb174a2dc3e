/*
 * mi355_reduce.h -- C ABI of the HIP combine layer (gfx950).
 *
 * This is the thin layer the host C runtime drives. It replaces the scalar
 * combine loops of the reference schedule:
 *   - the element functions    src/reduce/reduce-op.c:79-158
 *     (sum/prod, and/or/xor, min/max; called through `the_op`)
 *   - the per-PE combine loops src/reduce/reduce-op.c:241-261
 *     (`write_to[ti] = (*the_op)(write_to[ti], pWrk[j])`)
 *   - the initial copy         src/reduce/reduce-op.c:226-229
 * with streaming HIP kernels. Plain pointers and sizes only; `stream` is a
 * hipStream_t passed as void* (NULL = the null stream).
 *
 * Every function is asynchronous on `stream` and returns 0 on success, a
 * negative MI355_E* code for a rejected argument, or a positive hipError_t
 * from the launch.
 */
#ifndef MI355_REDUCE_H
#define MI355_REDUCE_H 1

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* reduce-op.c:79-158 operator families */
enum mi355_op {
    MI355_OP_SUM = 0,
    MI355_OP_PROD = 1,
    MI355_OP_AND = 2,
    MI355_OP_OR = 3,
    MI355_OP_XOR = 4,
    MI355_OP_MIN = 5,
    MI355_OP_MAX = 6,
    MI355_NUM_OPS = 7
};

/* reduce-op.c:278-286 element types (LP64 host ABI layouts) */
enum mi355_dtype {
    MI355_SHORT = 0,      /* int16                                        */
    MI355_INT = 1,        /* int32                                        */
    MI355_LONG = 2,       /* int64                                        */
    MI355_LONGLONG = 3,   /* int64                                        */
    MI355_FLOAT = 4,      /* binary32                                     */
    MI355_DOUBLE = 5,     /* binary64                                     */
    MI355_LONGDOUBLE = 6, /* x87 80-bit extended in a 16-byte slot        */
    MI355_COMPLEXF = 7,   /* {float re, im}                               */
    MI355_COMPLEXD = 8,   /* {double re, im}                              */
    MI355_NUM_DTYPES = 9
};

#define MI355_E_INVAL  (-1)   /* bad op/dtype/pointer/count        */
#define MI355_E_UNSUP  (-2)   /* op not defined for dtype          */

/* Bytes per element of a dtype (0 for an unknown dtype). */
size_t mi355_dtype_size (int dtype);

/* 1 if (op, dtype) is one of the 44 reference reductions. */
int mi355_op_supported (int op, int dtype);

/* dst[i] = (((srcs[0][i] op srcs[1][i]) op srcs[2][i]) ... op srcs[nsrc-1][i])
 * for i < n: a left fold with the accumulator on the left, exactly the
 * operand order of reduce-op.c:247-248. Sources may be peer (xGMI) pointers.
 * dst may alias srcs[0] exactly; other overlaps are undefined. nsrc >= 1
 * (nsrc == 1 is a copy). Any element-aligned pointers: 16-byte vectors, the
 * target peeled to its 128-byte line (the head folded element by element),
 * the sources read aligned when they share the target's 16-byte phase and
 * with unaligned loads at any other phases. Element by element: a 16-byte
 * element type (complex double, long double) whose target is not 16-byte
 * aligned, and long double sources off the target's phase. The same holds for mi355_combine_orders while its
 * outputs share one 16-byte phase (element by element otherwise) and, per
 * segment, for mi355_copy_segments at byte granularity. */
int mi355_combine (int op, int dtype, void *dst, const void *const *srcs,
                   int nsrc, size_t n, void *stream);

/* Every member's reference result at once: for each q < nsrc with dsts[q] != NULL,
 *   dsts[q][i] = (((srcs[q][i] op srcs[0][i]) op srcs[1][i]) ... op srcs[nsrc-1][i])
 * with srcs[q] itself skipped after the first operand: member q's OWN source
 * first, then the others in active-set order -- the order the reference folds
 * in on member q (reduce-op.c:226-264, the self-skip at :235). The P2P
 * schedule's owner of a shard computes every member's version of it from one
 * pass over the sources (the sources are read once, whatever nsrc). dsts[q]
 * may alias srcs[q] exactly (in place); other overlaps are undefined, and above
 * 8 sources at most one fold may be in place. 1 <= nsrc <= 32. */
#define MI355_ORDERS_MAX_SOURCES 32
int mi355_combine_orders (int op, int dtype, void *const *dsts, const void *const *srcs,
                          int nsrc, size_t n, void *stream);

/* nseg independent byte copies dsts[i] <- srcs[i] of nbytes[i] bytes in ONE
 * launch (the all-gather leg of the shard schedule). nseg <= 64. */
int mi355_copy_segments (void *const *dsts, const void *const *srcs,
                         const size_t *nbytes, int nseg, void *stream);

/* The two-member all-gather of a float/double sum or product: dst[i] =
 * own[i] quieted where own[i] is a NaN, else peer[i] (the other member's shard,
 * folded in its order: the same bits as this member's order except where
 * both operands are NaNs, where SSE keeps the first). own may alias dst.
 * nan_flag (may be NULL): the other member's word set by its fold when a NaN
 * came out (mi355_nan_flag_next_launch); while it reads 0 no result is NaN,
 * so the kernel copies peer[] and does not read own[]. */
int mi355_nan_patch_copy (int dtype, void *dst, const void *peer, const void *own, size_t n,
                          const unsigned long long *nan_flag, void *stream);

/* The NEXT fold this layer launches from the calling thread (mi355_combine,
 * float/double sum or product) stores 1 to *set (system scope) if any of its
 * results is a NaN, and 0 to *clear first (either may be NULL). */
void mi355_nan_flag_next_launch (unsigned long long *set, unsigned long long *clear);

/* Attach a pair of HIP events (hipEvent_t, created by the caller with timing
 * enabled) to the NEXT kernel this layer launches from the calling thread:
 * the runtime stamps that kernel's own start and end (hipExtLaunchKernel),
 * adding no marker packet to the stream. NULL, NULL cancels. */
void mi355_time_next_launch (void *start_event, void *stop_event);

/* Attach a completion signal to the NEXT kernel this layer launches from the
 * calling thread: when every block of it has finished and its stores are
 * written back to memory, one lane stores `epoch` to *flag (system scope).
 * `count` is a 4-byte device word holding 0 (the kernel leaves it at 0);
 * `flag` a device-visible pointer to host-coherent memory (hipHostMalloc
 * coherent + mapped). The host spins on *flag instead of synchronizing the
 * stream. Pass NULL flag to cancel. */
void mi355_signal_next_launch (unsigned *count, unsigned *flag, unsigned epoch);

/* Host stub of the kernel this layer launched last from the calling thread
 * (NULL before the first launch), and its demangled name as rocprofv3
 * prints it ("void mi355k::copy_segments<4, 1>(mi355k::SegParams<1>)") --
 * the runtime records which kernel carried a call (shmemx_last_call_info). */
const void *mi355_last_kernel (void);
int mi355_kernel_name (const void *kernel, char *buf, size_t len);

/* Launch a one-block kernel whose only job is to carry the armed signal:
 * the host learns that everything queued on `stream` before it is done. */
int mi355_signal_launch (void *stream);

/* Queue a system-scope acquire on every XCD of the current GPU (one small
 * kernel): afterwards kernels on `stream` do not see L2 copies of peer-GPU
 * memory older than this point. The P2P schedules queue it after each barrier
 * that precedes reads of other PEs' buffers. */
int mi355_acquire_system (void *stream);

/* n elements short -> int32 (widen != 0) or int32 -> short (truncating), on
 * `stream`: the RCCL schedule's 16-bit integer support (RCCL has no 16-bit
 * integer type). */
int mi355_convert_short (int widen, const void *src, void *dst, size_t n, void *stream);

/* ---- one-launch P2P reduction for small messages (fused.hip) ----
 * Signal region: per PE, MI355_SIG_WORDS 8-byte words of uncached device
 * memory mapped into every peer; all zero before first use. It holds
 * MI355_SIG_CHANNELS independent channels -- 0 for host-launched calls, 1 for
 * stream-ordered ones -- so the two kinds never share pair counts and may be
 * in flight at the same time. Offsets below are within a channel; the caller
 * passes sig[] pointers already offset to the channel's base. */
#define MI355_FUSED_MAX_MEMBERS 32
#define MI355_FUSED_MAX_BLOCKS 256
#define MI355_SIG_ARRIVE 0       /* [PE]: pair count of the last call the PE arrived at */
#define MI355_SIG_RSDONE 1024    /* [PE]: ... whose shard the PE has reduced           */
#define MI355_SIG_AGDONE 2048    /* [PE]: ... whose gather the PE has finished         */
#define MI355_SIG_CALLS 3072     /* [PE]: this PE's pair count of calls with the PE    */
#define MI355_SIG_RS_COUNT 4096  /* local block counters (own 128-byte lines)          */
#define MI355_SIG_AG_COUNT 4112
#define MI355_SIG_ERROR 4128
#define MI355_SIG_STAGE_COUNT 4144
#define MI355_SIG_SERVER 4160    /* persistent server's call broadcast (own line, 8 words) */
#define MI355_SIG_CHANNEL_WORDS 4176
#define MI355_SIG_CHANNELS 2
#define MI355_SIG_SELFTEST (MI355_SIG_CHANNELS * MI355_SIG_CHANNEL_WORDS) /* [PE]: init-time check */
#define MI355_SIG_SELFTEST2 (MI355_SIG_SELFTEST + 1024) /* [PE]: init-time producer-path check */
/* [channel][parity][partner PE]: "a NaN came out of this PE's two-member fold
 * of this parity's call with that partner" (mi355_nan_flag_next_launch) */
#define MI355_SIG_NANFLAG (MI355_SIG_SELFTEST2 + 1024)
#define MI355_SIG_NANFLAG_AT(chan, parity, pe) (MI355_SIG_NANFLAG + ((chan) * 2 + (parity)) * 1024 + (pe))
#define MI355_SIG_WORDS (MI355_SIG_NANFLAG + MI355_SIG_CHANNELS * 2 * 1024)

typedef struct MI355FusedArgs {
    int op, dtype;
    int nmembers, me;                 /* active-set size, this PE's index in it   */
    unsigned long long n;             /* elements                                 */
    unsigned long long shard;         /* elements per shard; shard*esize % 16 == 0 */
    const void *src[MI355_FUSED_MAX_MEMBERS];        /* members' sources (mapped) */
    void *dst[MI355_FUSED_MAX_MEMBERS];              /* members' targets (mapped) */
    unsigned long long *sig[MI355_FUSED_MAX_MEMBERS];/* members' signal regions   */
    int pe[MI355_FUSED_MAX_MEMBERS];  /* members' PE numbers (signal slot index)  */
    unsigned *host_flag;              /* host-coherent completion word, or NULL   */
    unsigned epoch;                   /* stored there when done (| 1u<<31: timeout) */
    unsigned *err_flag;               /* host-coherent; set to 1 on a timeout, or NULL */
    unsigned long long timeout_ticks; /* bound on every wait, 100 MHz ticks       */
    /* Host-staged form (or NULL): device-accessible pointers to this PE's page-locked HOST source and
     * target. The kernel first copies host_src into src[me], and at the end dst[me] into host_dst, so
     * a small reduction of host arrays is one launch (src/dst are then this PE's staging scratch). */
    const void *host_src;
    void *host_dst;
    /* 1: one-shot -- every member folds the whole array from all members' sources (one flag exchange
     * fewer than reduce-scatter + all-gather; for small messages). Needs dst != src. */
    int oneshot;
    /* 0: every member receives member 0's result (the fold in member order).
     * 1: every member receives the reference's result for ITSELF: its own source first, then the
     *    others in member order (reduce-op.c:226-264). One-shot folds in that order directly; the
     *    two-shot owner of shard j folds it in every member's order, keeps its own version in dst[j]
     *    and member q's in its version area, ver[j] + s * shard * esize with s = q < j ? q : q - 1
     *    (nmembers - 1 slots), and each member gathers its own version of the other shards there. */
    int ordered;
    void *ver[MI355_FUSED_MAX_MEMBERS];              /* members' version areas (mapped), if ordered */
    /* Processes that may run these spin-waiting kernels on this GPU at the same time (>= 1; 0 = 1):
     * the grid is capped at the kernel's resident blocks per CU (one fewer, as a margin) x CUs / share,
     * so every such grid can be resident at once and no spinning block keeps a peer's from starting. */
    int share;
    /* Every read of the members' buffers is a system-coherent load (sc0 sc1: never served from a
     * stale cache line), so the waits need no cache invalidation. 0: each block also runs a
     * system-scope acquire (buffer_inv sc0 sc1) after each wait -- one per block, which queue up
     * at every XCD's L2 on large grids. 1: it skips them; set only when the init coherence test
     * showed system-coherent loads of peers' rewritten memory fresh without any acquire. */
    int no_acquire;
} MI355FusedArgs;

/* Reduce-scatter + all-gather of n elements over the members in ONE launch:
 * every member ends with the fold of all members' sources -- in member order
 * (the reference's result on the first member), or with `ordered` in its own
 * reference order (the reference's result on that member). Every member must make the
 * matching call; buffers 16-byte aligned; dst == src or disjoint.
 *
 * Pair counts live on the device (MI355_SIG_CALLS): the kernel reads them at
 * its start and advances them when every member is done, so the call needs
 * no host state and replays correctly from a captured HIP graph. The
 * collectives of one PE on one channel (this and mi355_device_barrier) must
 * run one at a time, in the same order on every member. */
int mi355_fused_allreduce (const MI355FusedArgs *args, void *stream);

/* One-launch pull collective (small broadcast / fcollect): after every
 * member has arrived (its sources are ready), each member copies nseg byte
 * ranges -- typically out of peers' mapped sources -- into its own device
 * memory; the members then exchange "done reading" and the call completes
 * (m.host_flag / m.epoch as for mi355_fused_allreduce). m.op/dtype/n/shard/
 * src/dst are unused. */
#define MI355_PULL_MAX_SEGS 64
typedef struct MI355PullArgs {
    MI355FusedArgs m;
    int nseg;
    void *dst[MI355_PULL_MAX_SEGS];
    const void *src[MI355_PULL_MAX_SEGS];
    unsigned long long nbytes[MI355_PULL_MAX_SEGS];
} MI355PullArgs;
int mi355_fused_pull (const MI355PullArgs *args, void *stream);

/* ---- persistent fused server (opt-in; reduce.c, SHMEM_PERSISTENT) ----
 * A grid of the fused kernel that stays resident and serves back-to-back
 * calls of one (op, dtype, active set) from a mailbox in host-coherent
 * memory instead of one launch per call: the host writes the call and its
 * seq; block 0 of the server polls it, broadcasts the call to the other
 * blocks through this PE's signal region (MI355_SIG_SERVER, same layout) and every
 * block runs the fused kernel's body on the members' heap bases (args->src /
 * args->dst at offset 0) plus the call's byte offsets. The call completes
 * as a launched one does (args->host_flag = the call's epoch).
 * The server exits on cmd QUIT, or when no call came for idle_ticks (100 MHz
 * ticks): it then stores state = EXITED, state_seq = the first seq it did not
 * serve, and never serves again -- a host that rang that seq falls back to a
 * launch. Host-staged calls (host_src/host_dst) are not served. */
#define MI355_SERVER_RUN 1
#define MI355_SERVER_QUIT 2
#define MI355_SERVER_RUNNING 1
#define MI355_SERVER_EXITED 2
typedef struct MI355ServerMailbox {
    /* host -> device, one 64-byte line the server reads with one load: the
     * call and its check word, then seq_head and seq_tail (release, in that
     * order); a snapshot counts only when both hold the seq it waits for AND
     * its check word matches dwords 1-11 (a torn read of the line -- not
     * expected from one 64-byte aligned read over PCIe, but not guaranteed
     * either -- is then retried, not served) */
    unsigned seq_head;                   /* the server serves seq first_seq, first_seq + 1, ... */
    unsigned cmd;                        /* MI355_SERVER_RUN / _QUIT */
    unsigned long long src_off, dst_off; /* byte offsets into every member's symmetric heap */
    unsigned long long n, shard;         /* as MI355FusedArgs */
    unsigned epoch;
    int oneshot;
    unsigned check;                      /* mi355_mailbox_check of the line, written with the call */
    unsigned pad0[2];
    unsigned seq_tail;
    /* device -> host (own line) */
    unsigned state;                      /* MI355_SERVER_RUNNING (set by the host before the launch) / _EXITED */
    unsigned state_seq;                  /* EXITED: the first seq not served */
    unsigned pad1[14];
} MI355ServerMailbox;

/* The check word: dwords 1-11 of the line (cmd .. oneshot) xor-folded, mixed
 * with the seq. The server recomputes it from the snapshot it read. */
static inline unsigned mi355_mailbox_check (const MI355ServerMailbox *mb, unsigned seq)
{
    const unsigned *w = (const unsigned *) mb;
    unsigned x = 0;
    for (int i = 1; i <= 11; ++i)
        x ^= w[i];
    return x ^ (seq * 0x9E3779B1u);
}

/* Launch the server on `stream` (a stream of its own: it does not finish
 * until QUIT or idle). args: as for mi355_fused_allreduce with src/dst the
 * members' heap bases, n/shard/oneshot/epoch unused; grid_vecs sizes the
 * grid as a launch of the calls it is expected to serve (16-byte vectors
 * folded or gathered per PE: the one-shot array, or the gathered shards). mbox: device-accessible
 * host-coherent memory. One member (nmembers = 1) serves the 1-PE identity:
 * one-shot calls copy the source to the target. */
int mi355_fused_server (const MI355FusedArgs *args, MI355ServerMailbox *mbox, unsigned first_seq,
                        unsigned long long idle_ticks, unsigned long long grid_vecs, void *stream);

/* Device-side barrier over the members (one 64-lane block): ordered on
 * `stream` after the work queued before it, and the work queued after it
 * runs once every member has reached its matching barrier. Uses
 * nmembers/me/sig/pe/err_flag/host_flag/epoch/timeout_ticks of args. */
int mi355_device_barrier (const MI355FusedArgs *args, void *stream);

/* One-block kernels for the init-time interconnect check: store `value` to
 * each of n (peer-mapped) words at system scope; load n words at system scope
 * into out[] (device memory). n <= 1024. */
int mi355_poke (unsigned long long *const *dst, int n, unsigned long long value, void *stream);
int mi355_peek (const unsigned long long *const *src, int n, unsigned long long *out, void *stream);
/* The coherence check: nblocks blocks (<= 256, dealt over the XCDs) each load
 * the n words with plain, L2-cached loads -- as the folds read peers' buffers
 * -- into out[b * n + i]. */
int mi355_peek_cached (const unsigned long long *const *src, int n, unsigned long long *out, int nblocks,
                       void *stream);
/* The same with system-coherent loads (sc0 sc1, as the fused kernel reads the members' buffers) and
 * no fence: out[b * n + i]. */
int mi355_peek_sysload (const unsigned long long *const *src, int n, unsigned long long *out, int nblocks,
                        void *stream);

/* The init-time check of the CALLER's producer path (runtime.c producer_test):
 * mi355_mark_plain is a caller's kernel writing its source -- `words` blocks
 * (dealt over the XCDs), block b storing value + b into dst[b] with a plain
 * write-back store; words <= 1024. mi355_producer_read, nblocks blocks
 * (<= 256): when flag != NULL wave 0 first waits until flag[q] == token for
 * every q < np (bounded by timeout_ticks of s_memrealtime; a timeout sets
 * out[3 * nblocks * np * words] = 1), then every block reads the np x words
 * words of src[q] three ways into out: plain loads (third 0), 16-byte
 * system-coherent loads as the fused kernel's folds (third 1), plain loads
 * after a system-scope acquire (third 2); each third is [nblocks][np * words].
 * np <= 64, words even (16-byte aligned pairs). */
int mi355_mark_plain (unsigned long long *dst, int words, unsigned long long value, void *stream);
int mi355_producer_read (const unsigned long long *const *src, int np, int words, const unsigned long long *flag,
                         unsigned long long token, unsigned long long timeout_ticks, unsigned long long *out,
                         int nblocks, void *stream);

/* Shard i of nshards for n elements of elem_size bytes: the P2P schedule's
 * partition (contiguous, shard starts 256-byte aligned, trailing shards may
 * be empty). Host-only arithmetic, callable without a GPU. */
void mi355_shard_bounds (size_t n, size_t elem_size, int nshards, int i, size_t *lo, size_t *hi);

#ifdef __cplusplus
}
#endif

#endif /* MI355_REDUCE_H */
