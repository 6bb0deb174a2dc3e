/*
 * runtime.c -- minimal OpenSHMEM runtime for the MI355X reduction path.
 *
 * The reference brings PEs up through GASNet (src/updown/updown.c:126-184 ->
 * shmemi_comms_init, src/comms/gasnet/comms-inline.h:2893-2960). GASNet does
 * not exist here and the reduction path only needs: PE identity, one GPU per
 * PE, a symmetric heap, an active-set barrier, and the peer mappings that let
 * one GPU read another's heap over xGMI. This file provides exactly that:
 *
 *   identity   SHMEM_PE/SHMEM_NPES, else RANK/WORLD_SIZE (torchrun), else
 *              OMPI_COMM_WORLD_*, PMI_*; device = SHMEM_DEVICE, LOCAL_RANK or
 *              the PE number, modulo the visible GPUs
 *   bootstrap  one POSIX shared-memory segment per job (node-local): PE 0
 *              creates it, every PE publishes pid/GPU/IPC handle there
 *   heaps      device symmetric heap = one hipMalloc arena per PE, exported
 *              with hipIpcGetMemHandle and mapped by every peer; a
 *              deterministic first-fit allocator keeps offsets symmetric
 *              (reference: dlmalloc mspace, src/memory/memalloc.c:71-154)
 *   barrier    pairwise monotonic arrival counters in the segment: PE p
 *              passes once every q of the active set has signalled p as many
 *              times as p has met q in a barrier. This is the pSync contract
 *              of src/barrier/barrier-linear.c:57-85 without touching pSync.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <stdarg.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "pshmem.h"
#include "mi355_reduce.h"
#include "shmem.h"
#include "shmemx.h"
#include "shmemi.h"

struct shmemi_state shmemi;

#define SEG_MAGIC 0x4d49333535534d45ull /* "MI355SME" */
#define SEG_VERSION 8

static double now_s (void)
{
    struct timespec ts;
    clock_gettime (CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

double shmemx_wtime (void) { return now_s (); }
double shmemi_now (void) { return now_s (); }

/* Ask a running persistent server to exit without waiting for it (fatal
 * paths; it also leaves on its own after SHMEM_PERSISTENT_IDLE_US). */
static void server_quit_nowait (void)
{
    if (shmemi.srv.running && shmemi.srv.mb != NULL) {
        shmemi.srv.mb->cmd = MI355_SERVER_QUIT;
        shmemi.srv.mb->check = mi355_mailbox_check (shmemi.srv.mb, shmemi.srv.seq);
        __atomic_store_n (&shmemi.srv.mb->seq_head, shmemi.srv.seq, __ATOMIC_RELEASE);
        __atomic_store_n (&shmemi.srv.mb->seq_tail, shmemi.srv.seq, __ATOMIC_RELEASE);
        shmemi.srv.running = 0;
    }
}

void shmemi_fatal (const char *fmt, ...)
{
    char msg[256];
    va_list ap;
    va_start (ap, fmt);
    vsnprintf (msg, sizeof msg, fmt, ap);
    va_end (ap);
    fprintf (stderr, "[shmem PE %d/%d] FATAL: %s\n", shmemi.mype, shmemi.npes, msg);
    fflush (stderr);
    server_quit_nowait ();
    if (shmemi.seg != NULL) {
        int zero = 0;
        if (atomic_compare_exchange_strong (&shmemi.seg->abort_flag, &zero, 1)) {
            shmemi.seg->abort_pe = shmemi.mype;
            shmemi.seg->abort_status = 1;
            snprintf (shmemi.seg->abort_msg, sizeof shmemi.seg->abort_msg, "%s", msg);
        }
    }
    _exit (1);
}

void shmemi_hip_check (hipError_t e, const char *what)
{
    if (e != hipSuccess)
        shmemi_fatal ("%s failed: %s (%d)", what, hipGetErrorString (e), (int) e);
}

void shmemi_init_check (const char *fn)
{
    if (!shmemi.initialized)
        shmemi_fatal ("%s called before shmem_init()", fn);
}

/* ---------------------------------------------------------------------- */
/* environment                                                             */
/* ---------------------------------------------------------------------- */
static const char *env_first (const char *const *names)
{
    for (; *names != NULL; ++names) {
        const char *v = getenv (*names);
        if (v != NULL && *v != '\0')
            return v;
    }
    return NULL;
}

static long env_long (const char *const *names, long dflt)
{
    const char *v = env_first (names);
    if (v == NULL)
        return dflt;
    char *end = NULL;
    long x = strtol (v, &end, 10);
    if (end == v)
        return dflt;
    return x;
}

/* "512M", "2G", "4096" (reference unit parser: src/utils/unitparse.c:74-142) */
static size_t env_size (const char *name, size_t dflt)
{
    const char *v = getenv (name);
    if (v == NULL || *v == '\0')
        return dflt;
    char *end = NULL;
    double x = strtod (v, &end);
    if (end == v || x < 0)
        shmemi_fatal ("cannot parse %s=\"%s\"", name, v);
    switch (*end) {
    case 'k': case 'K': x *= 1024.0; break;
    case 'm': case 'M': x *= 1024.0 * 1024.0; break;
    case 'g': case 'G': x *= 1024.0 * 1024.0 * 1024.0; break;
    case 't': case 'T': x *= 1024.0 * 1024.0 * 1024.0 * 1024.0; break;
    default: break;
    }
    return (size_t) x;
}

static size_t round_up (size_t x, size_t a) { return (x + a - 1) / a * a; }

static int parse_order (const char *v)
{
    if (v == NULL || strcasecmp (v, "reference") == 0 || strcasecmp (v, "pe") == 0) return SHMEMX_ORDER_REFERENCE;
    if (strcasecmp (v, "pe_start") == 0 || strcasecmp (v, "uniform") == 0) return SHMEMX_ORDER_PE_START;
    shmemi_fatal ("unknown SHMEM_REDUCE_ORDER=\"%s\" (reference|pe_start)", v);
}

static int parse_algorithm (const char *v)
{
    if (v == NULL || strcasecmp (v, "auto") == 0) return SHMEMX_REDUCE_AUTO;
    if (strcasecmp (v, "p2p") == 0) return SHMEMX_REDUCE_P2P;
    if (strcasecmp (v, "exact") == 0) return SHMEMX_REDUCE_EXACT;
    if (strcasecmp (v, "rccl") == 0) return SHMEMX_REDUCE_RCCL;
    shmemi_fatal ("unknown SHMEM_REDUCE_ALGORITHM=\"%s\" (auto|p2p|exact|rccl)", v);
}

/* ---------------------------------------------------------------------- */
/* bootstrap segment                                                       */
/* ---------------------------------------------------------------------- */
static struct shmemi_pe_info *seg_info (int pe)
{
    return (struct shmemi_pe_info *) ((char *) shmemi.seg + shmemi.seg->info_off) + pe;
}

struct shmemi_pe_info *shmemi_seg_info (int pe) { return seg_info (pe); }

static _Atomic uint64_t *seg_flag (int row_pe, int from_pe)
{
    _Atomic uint64_t *base = (_Atomic uint64_t *) ((char *) shmemi.seg + shmemi.seg->flags_off);
    return base + (size_t) row_pe * shmemi.seg->flags_row + (size_t) from_pe;
}

static void seg_name (char *out, size_t len)
{
    const char *job = getenv ("SHMEM_JOB_ID");
    if (job != NULL && *job != '\0') {
        snprintf (out, len, "/mi355shmem-%u-%s", (unsigned) getuid (), job);
        return;
    }
    /* every PE launched by one torchrun agent / one launcher shares a parent */
    const char *port = getenv ("MASTER_PORT");
    snprintf (out, len, "/mi355shmem-%u-p%d-%s", (unsigned) getuid (), (int) getppid (),
              port != NULL ? port : "0");
}

static void check_abort (void)
{
    if (shmemi.seg != NULL && atomic_load (&shmemi.seg->abort_flag)) {
        fprintf (stderr, "[shmem PE %d/%d] aborting: PE %d failed: %s\n", shmemi.mype,
                 shmemi.npes, shmemi.seg->abort_pe, shmemi.seg->abort_msg);
        fflush (stderr);
        _exit (shmemi.seg->abort_status ? shmemi.seg->abort_status : 1);
    }
}

static void bootstrap_attach (void)
{
    const int npes = shmemi.npes;
    const size_t hdr = round_up (sizeof (struct shmemi_seg), 4096);
    const size_t info = round_up (sizeof (struct shmemi_pe_info) * (size_t) npes, 4096);
    const size_t row = round_up ((size_t) npes, 8);
    const size_t flags = round_up (row * (size_t) npes * sizeof (uint64_t), 4096);
    const size_t total = hdr + info + 2 * flags; /* barrier counts, SHMEM_DEBUG check counts */
    seg_name (shmemi.seg_name, sizeof shmemi.seg_name);

    /* SHMEM_BOOTSTRAP_TIMEOUT: how long a PE waits for PE 0 to create the
     * segment (a launcher may start PE 0 late; default: the barrier timeout) */
    static const char *bt_env[] = {"SHMEM_BOOTSTRAP_TIMEOUT", NULL};
    const double deadline = now_s () + (double) env_long (bt_env, (long) shmemi.barrier_timeout);
    if (shmemi.mype == 0) {
        shm_unlink (shmemi.seg_name); /* stale leftover of a crashed job */
        int fd = shm_open (shmemi.seg_name, O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0)
            shmemi_fatal ("shm_open(%s): %s", shmemi.seg_name, strerror (errno));
        if (ftruncate (fd, (off_t) total) != 0)
            shmemi_fatal ("ftruncate(%s, %zu): %s", shmemi.seg_name, total, strerror (errno));
        void *p = mmap (NULL, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close (fd);
        if (p == MAP_FAILED)
            shmemi_fatal ("mmap bootstrap segment: %s", strerror (errno));
        shmemi.seg = (struct shmemi_seg *) p;
        shmemi.seg->version = SEG_VERSION;
        shmemi.seg->npes = npes;
        shmemi.seg->info_off = hdr;
        shmemi.seg->flags_off = hdr + info;
        shmemi.seg->flags_row = row;
        shmemi.seg->dbg_off = hdr + info + flags;
        shmemi.seg->total_size = total;
        atomic_store (&shmemi.seg->magic, SEG_MAGIC);
    } else {
        for (;;) {
            if (now_s () > deadline)
                shmemi_fatal ("timed out waiting for PE 0 to create %s", shmemi.seg_name);
            int fd = shm_open (shmemi.seg_name, O_RDWR, 0600);
            if (fd < 0) {
                usleep (1000);
                continue;
            }
            struct stat st;
            if (fstat (fd, &st) != 0 || (size_t) st.st_size < total) {
                close (fd);
                usleep (1000);
                continue;
            }
            void *p = mmap (NULL, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            close (fd);
            if (p == MAP_FAILED)
                shmemi_fatal ("mmap bootstrap segment: %s", strerror (errno));
            struct shmemi_seg *s = (struct shmemi_seg *) p;
            if (atomic_load (&s->magic) != SEG_MAGIC) {
                munmap (p, total);
                usleep (1000);
                continue;
            }
            if (s->npes != npes || s->total_size != total)
                shmemi_fatal ("bootstrap segment %s belongs to a job of %d PEs, not %d",
                              shmemi.seg_name, s->npes, npes);
            shmemi.seg = s;
            break;
        }
    }
    shmemi.seg_size = total;
    atomic_fetch_add (&shmemi.seg->attached, 1);
    shmemi.bar_count = (uint64_t *) calloc ((size_t) npes, sizeof (uint64_t));
    shmemi.dbg_count = (uint64_t *) calloc ((size_t) npes, sizeof (uint64_t));
    if (shmemi.bar_count == NULL || shmemi.dbg_count == NULL)
        shmemi_fatal ("out of host memory");
}

/* Active-set barrier {PE_start + i*stride : i < PE_size}. Each PE adds one
 * arrival to every other member's row, then waits until it has seen, from each
 * member q, as many arrivals as barriers it has shared with q. A member that
 * races ahead to the next barrier only raises a count that is already due, so
 * no reset round (the reference's second pSync word) is needed. */
static void barrier_watch (int PE_start, int stride, int PE_size, void (*watch) (int q))
{
    if (PE_size <= 1 || shmemi.npes <= 1)
        return;
    const int me = shmemi.mype;
    for (int i = 0; i < PE_size; ++i) {
        const int q = PE_start + i * stride;
        if (q != me)
            atomic_fetch_add_explicit (seg_flag (q, me), 1, memory_order_release);
    }
    const double t0 = now_s ();
    for (int i = 0; i < PE_size; ++i) {
        const int q = PE_start + i * stride;
        if (q == me)
            continue;
        const uint64_t want = ++shmemi.bar_count[q];
        unsigned spins = 0;
        while (atomic_load_explicit (seg_flag (me, q), memory_order_acquire) < want) {
            if ((++spins & 1023u) == 0) {
                check_abort ();
                if (watch != NULL)
                    watch (q);
                if (now_s () - t0 > shmemi.barrier_timeout)
                    shmemi_fatal ("barrier timed out after %.0f s waiting for PE %d",
                                  shmemi.barrier_timeout, q);
                if (spins > 65536u)
                    sched_yield ();
            } else {
                __builtin_ia32_pause ();
            }
        }
    }
}

void shmemi_barrier_set (int PE_start, int stride, int PE_size)
{
    barrier_watch (PE_start, stride, PE_size, NULL);
}

/* This PE's arrival at a barrier of the set without the wait: the members
 * that wait see it (extmap.c: a PE that will stage anyway publishes its
 * record and goes on). Keeps the pair counts as a full barrier does. */
void shmemi_barrier_arrive (int PE_start, int stride, int PE_size)
{
    if (PE_size <= 1 || shmemi.npes <= 1)
        return;
    for (int i = 0; i < PE_size; ++i) {
        const int q = PE_start + i * stride;
        if (q != shmemi.mype) {
            atomic_fetch_add_explicit (seg_flag (q, shmemi.mype), 1, memory_order_release);
            ++shmemi.bar_count[q];
        }
    }
}

/* ---------------------------------------------------------------------- */
/* SHMEM_DEBUG=1: collective argument check                                 */
/* ---------------------------------------------------------------------- */
/* The reference's debug build checks that the library is initialised and
 * that target/source are symmetric (src/reduce/reduce-op.c:395-398 ->
 * src/utils/utils.h:74-129); a member passing a different nreduce, op or
 * active set is not caught and reads wrong peer offsets or hangs. Here every
 * member publishes its arguments in the bootstrap segment and counts, per
 * peer of its active set, the checks it has entered with that peer
 * (dbgcnt[me][q], like the barrier's pair counts). Members that see the
 * same count for each other are in the same collective (OpenSHMEM orders the
 * collectives of overlapping sets), so their records must agree: a member
 * compares them while it waits in the check's barrier -- which catches a
 * differing PE_start / stride / size without waiting out the barrier timeout
 * -- and again once it is through. A closing barrier keeps every record in
 * place until all members have compared. A mismatch aborts every PE with the
 * field. */
static struct shmemi_dbg_rec dbg_mine;

static _Atomic uint64_t *dbg_cnt (int row_pe, int peer)
{
    _Atomic uint64_t *base = (_Atomic uint64_t *) ((char *) shmemi.seg + shmemi.seg->dbg_off);
    return base + (size_t) row_pe * shmemi.seg->flags_row + (size_t) peer;
}

static void dbg_read (int pe, struct shmemi_dbg_rec *out)
{
    struct shmemi_dbg_rec *r = &seg_info (pe)->dbg;
    for (;;) {
        const uint32_t s0 = atomic_load_explicit (&r->seq, memory_order_acquire);
        if (s0 & 1u) {
            __builtin_ia32_pause ();
            continue;
        }
        memcpy ((char *) out + offsetof (struct shmemi_dbg_rec, op), (const char *) r + offsetof (struct shmemi_dbg_rec, op),
                sizeof *out - offsetof (struct shmemi_dbg_rec, op));
        atomic_thread_fence (memory_order_acquire);
        if (atomic_load_explicit (&r->seq, memory_order_relaxed) == s0)
            return;
    }
}

/* the first field in which b differs from a, or NULL */
static const char *dbg_diff (const struct shmemi_dbg_rec *a, const struct shmemi_dbg_rec *b, long *va, long *vb)
{
#define F(field, name)                                                                                          \
    if (a->field != b->field) {                                                                                 \
        *va = (long) a->field;                                                                                  \
        *vb = (long) b->field;                                                                                  \
        return name;                                                                                            \
    }
    F (pe_start, "PE_start")
    F (log_stride, "logPE_stride")
    F (pe_size, "PE_size")
    F (op, "reduction operator (enum mi355_op)")
    F (dtype, "element type (enum mi355_dtype)")
    F (nreduce, "nreduce")
    F (tkind, "target memory kind (0 host, 1 device symmetric heap, 2 other device memory)")
    F (skind, "source memory kind (0 host, 1 device symmetric heap, 2 other device memory)")
    F (toff, "target offset in the device symmetric heap")
    F (soff, "source offset in the device symmetric heap")
    F (algorithm, "reduce algorithm (shmemx_set_reduce_algorithm)")
    F (order, "result order (shmemx_set_reduce_order)")
    F (overlap, "target/source relation (0 disjoint, 1 the same buffer, 2 target overlapping above source, 3 below)")
    F (fused_max, "fused-kernel threshold in bytes (SHMEM_FUSED_MAX_BYTES / shmemx_set_fused_max_bytes)")
    F (oneshot_max, "one-shot threshold in bytes (SHMEM_ONESHOT_MAX_BYTES / shmemx_set_oneshot_max_bytes)")
#undef F
    if (strcmp (a->fn, b->fn) != 0) {
        *va = *vb = 0;
        return "collective";
    }
    return NULL;
}

/* q's record, if q is inside the check of the same collective as this PE
 * (the same pair count), compared with this PE's; 1 if compared */
static int dbg_compare (int q)
{
    if (atomic_load_explicit (dbg_cnt (q, shmemi.mype), memory_order_acquire) != shmemi.dbg_count[q])
        return 0;
    struct shmemi_dbg_rec theirs;
    dbg_read (q, &theirs);
    long va = 0, vb = 0;
    const char *f = dbg_diff (&dbg_mine, &theirs, &va, &vb);
    if (f != NULL && strcmp (f, "collective") == 0)
        shmemi_fatal ("SHMEM_DEBUG: collective mismatch: PE %d called %s, PE %d called %s", shmemi.mype,
                      dbg_mine.fn, q, theirs.fn);
    if (f != NULL)
        shmemi_fatal ("SHMEM_DEBUG: %s: %s is %ld on PE %d but %ld on PE %d (every member of the active set must "
                      "pass the same arguments)", dbg_mine.fn, f, va, shmemi.mype, vb, q);
    return 1;
}

static void dbg_watch (int q) { (void) dbg_compare (q); }

void shmemi_debug_exchange (const struct shmemi_dbg_rec *mine, int PE_start, int stride, int PE_size)
{
    if (shmemi.seg == NULL || PE_size < 2)
        return;
    struct shmemi_dbg_rec *r = &seg_info (shmemi.mype)->dbg;
    dbg_mine = *mine;
    const uint32_t s = atomic_load_explicit (&r->seq, memory_order_relaxed);
    atomic_store_explicit (&r->seq, s + 1, memory_order_relaxed);
    atomic_thread_fence (memory_order_release);
    memcpy ((char *) r + offsetof (struct shmemi_dbg_rec, op), (const char *) mine + offsetof (struct shmemi_dbg_rec, op),
            sizeof *r - offsetof (struct shmemi_dbg_rec, op));
    atomic_store_explicit (&r->seq, s + 2, memory_order_release);
    /* the record first, then the pair counts that make it current for each peer */
    for (int i = 0; i < PE_size; ++i) {
        const int q = PE_start + i * stride;
        if (q != shmemi.mype)
            atomic_store_explicit (dbg_cnt (shmemi.mype, q), ++shmemi.dbg_count[q], memory_order_release);
    }

    barrier_watch (PE_start, stride, PE_size, dbg_watch);
    for (int i = 0; i < PE_size; ++i) {
        const int q = PE_start + i * stride;
        if (q != shmemi.mype && !dbg_compare (q))
            shmemi_fatal ("SHMEM_DEBUG: %s: PE %d passed this call's synchronization from another call (a barrier "
                          "or a collective over other PEs): the members disagree on the active set (PE_start %d, "
                          "logPE_stride %d, PE_size %d here)", dbg_mine.fn, q, dbg_mine.pe_start,
                          dbg_mine.log_stride, dbg_mine.pe_size);
    }
    shmemi_barrier_set (PE_start, stride, PE_size); /* every member has compared: records may change */
}

/* ---------------------------------------------------------------------- */
/* device symmetric heap                                                   */
/* ---------------------------------------------------------------------- */
int shmemi_in_device_heap (const void *p, size_t nbytes)
{
    if (shmemi.heap == NULL || p == NULL)
        return 0;
    const char *c = (const char *) p;
    return c >= shmemi.heap && c + nbytes <= shmemi.heap + shmemi.user_size;
}

size_t shmemi_heap_offset (const void *p) { return (size_t) ((const char *) p - shmemi.heap); }

void *shmemi_peer_ptr (int pe, size_t off)
{
    if (__builtin_expect (off >= SHMEMI_EXT_TARGET, 0))
        return shmemi_ext_ptr (pe, off); /* a device buffer outside the heap, mapped for this call (extmap.c) */
    if (__builtin_expect (shmemi.peer_heap[pe] == NULL, 0))
        shmemi_fatal ("PE %d's device heap is not mapped here (IPC mapping failed at init): only the RCCL "
                      "schedule can reach it", pe);
    return shmemi.peer_heap[pe] + off;
}

/* Where PE `pe`'s heap starts in its hipMalloc'd arena. PEs that share a
 * GPU (the test layout) would otherwise have their symmetric objects at
 * offsets a large power of two apart in one HBM, so a fold reading the
 * members' sources at one element offset sends every stream to the same
 * channels (the version slots are staggered the same
 * way in reduce.c). 4,352 B = 17 x 256: the heap base stays 256-aligned. */
#define HEAP_STAGGER 4352
#define HEAP_STAGGER_SPAN (16 * HEAP_STAGGER)
static size_t heap_skew (int pe) { return (size_t) (pe % 16) * HEAP_STAGGER; }

static void heap_init (void)
{
    shmemi.user_size = round_up (env_size ("SHMEM_DEVICE_HEAP_SIZE", (size_t) 2 << 30), SHMEMI_ALIGN);
    size_t scratch = round_up (env_size ("SHMEM_DEVICE_SCRATCH_SIZE", (size_t) 768 << 20),
                               3 * SHMEMI_ALIGN);
    if (scratch < 3 * 65536)
        scratch = 3 * 65536;
    shmemi.scratch_off = shmemi.user_size;
    shmemi.scratch_chunk = scratch / 3 / SHMEMI_ALIGN * SHMEMI_ALIGN;
    /* version areas of the per-PE-order P2P schedule (reduce.c), one per
     * signal-region channel (host-launched / stream-ordered calls) */
    size_t order = round_up (env_size ("SHMEM_DEVICE_ORDER_SIZE", (size_t) 512 << 20), 2 * SHMEMI_ALIGN);
    if (order < 2 * 65536)
        order = 2 * 65536;
    shmemi.order_off = shmemi.scratch_off + scratch;
    shmemi.order_chunk = order / 2 / SHMEMI_ALIGN * SHMEMI_ALIGN;
    shmemi.heap_size = shmemi.user_size + scratch + order;
    void *p = NULL;
    hipError_t e = hipMalloc (&p, shmemi.heap_size + HEAP_STAGGER_SPAN);
    if (e != hipSuccess)
        shmemi_fatal ("hipMalloc of the %zu-byte device symmetric heap failed: %s "
                      "(set SHMEM_DEVICE_HEAP_SIZE / SHMEM_DEVICE_SCRATCH_SIZE)",
                      shmemi.heap_size, hipGetErrorString (e));
    shmemi.heap_arena = (char *) p;
    shmemi.heap = shmemi.heap_arena + heap_skew (shmemi.mype);
    struct shmemi_block *b = (struct shmemi_block *) calloc (1, sizeof *b);
    if (b == NULL)
        shmemi_fatal ("out of host memory");
    b->off = 0;
    b->size = shmemi.user_size;
    shmemi.blocks = b;
    shmemi.peer_heap = (char **) calloc ((size_t) shmemi.npes, sizeof (char *));
    if (shmemi.peer_heap == NULL)
        shmemi_fatal ("out of host memory");
    shmemi.peer_heap[shmemi.mype] = shmemi.heap;
}

static void signal_init (void)
{
    void *h = NULL, *d = NULL;
    SHMEMI_HIP (hipHostMalloc (&h, 128, hipHostMallocCoherent | hipHostMallocMapped));
    SHMEMI_HIP (hipHostGetDevicePointer (&d, h, 0));
    if (d != h)
        shmemi_fatal ("host-coherent signal word maps to a different device address");
    shmemi.sig_flag = (unsigned *) h;
    *shmemi.sig_flag = 0;
    shmemi.stream_err = (unsigned *) ((char *) h + 64); /* own cache line */
    *shmemi.stream_err = 0;
    SHMEMI_HIP (hipMalloc (&d, 64));
    SHMEMI_HIP (hipMemset (d, 0, 64));
    SHMEMI_HIP (hipDeviceSynchronize ());
    shmemi.sig_count = (unsigned *) d;
    shmemi.sig_epoch = 0;
}

/* Creates a stream if it does not exist yet (the staging and server paths
 * call it before use; init creates them). The library's streams are created
 * together at init, so that HIP deals them distinct hardware queues: created
 * later, after other code's streams, the staging copy-in and copy-out
 * streams shared one and host-staged calls serialised their two directions
 * (256 MiB: 10.1 ms against 6.15 ms per call, round 5). Many PEs sharing one
 * GPU are a matter of GPU_MAX_HW_QUEUES (device_wait_test below), not of how
 * many streams a process has. */
void shmemi_lazy_stream (hipStream_t *st, unsigned flags)
{
    if (*st == NULL)
        SHMEMI_HIP (hipStreamCreateWithFlags (st, flags));
}

/* The persistent server's mailbox (host-coherent, same address on both
 * sides) and stream; SHMEM_PERSISTENT=1 turns it on (reduce.c). */
static void server_init (void)
{
    void *h = NULL, *d = NULL;
    SHMEMI_HIP (hipHostMalloc (&h, sizeof (MI355ServerMailbox), hipHostMallocCoherent | hipHostMallocMapped));
    SHMEMI_HIP (hipHostGetDevicePointer (&d, h, 0));
    if (d != h)
        shmemi_fatal ("host-coherent server mailbox maps to a different device address");
    memset (h, 0, sizeof (MI355ServerMailbox));
    shmemi.srv.mb = (MI355ServerMailbox *) h;
    shmemi.srv.seq = 1;
    SHMEMI_HIP (hipStreamCreateWithFlags (&shmemi.srv.st, hipStreamNonBlocking));
    static const char *pe_env[] = {"SHMEM_PERSISTENT", NULL};
    static const char *idle_env[] = {"SHMEM_PERSISTENT_IDLE_US", NULL};
    shmemi.srv.enabled = env_long (pe_env, 0) != 0;
    const long idle_us = env_long (idle_env, 1000);
    shmemi.srv.idle_s = (idle_us < 10 ? 10 : idle_us) * 1e-6;
    shmemi.srv.running = 0;
    shmemi.srv.last_end = -1.0;
}

/* Epochs live in the low 31 bits; bit 31 marks a kernel-side timeout. */
unsigned shmemi_next_epoch (void)
{
    shmemi.sig_epoch = (shmemi.sig_epoch + 1) & 0x7fffffffu;
    if (shmemi.sig_epoch == 0)
        shmemi.sig_epoch = 1;
    return shmemi.sig_epoch;
}

/* Arm the completion signal for the next kernel the combine layer launches. */
void shmemi_arm_signal (void)
{
    mi355_signal_next_launch (shmemi.sig_count, shmemi.sig_flag, shmemi_next_epoch ());
}

void shmemi_wait_signal (void)
{
    if (shmemi_wait_flag (shmemi.sig_epoch) != shmemi.sig_epoch)
        shmemi_fatal ("kernel reported a timeout");
}

/* Wait until the host-coherent flag carries `want` (in its low 31 bits) and
 * return it. A kernel that faults never signals: after the first millisecond
 * the stream is polled every millisecond so its error surfaces. (Polling it
 * from the start cost up to a microsecond per call: hipStreamQuery takes
 * runtime locks and could run just as the flag arrived.) */
unsigned shmemi_wait_flag (unsigned want)
{
    unsigned spins = 0;
    double t0 = 0.0, next_query = 0.0;
    unsigned v;
    while (((v = __atomic_load_n (shmemi.sig_flag, __ATOMIC_ACQUIRE)) & 0x7fffffffu) != want) {
        __builtin_ia32_pause ();
        if ((++spins & 255u) != 0)
            continue;
        const double t = now_s (); /* vDSO clock: tens of ns */
        if (t0 == 0.0) {
            t0 = t;
            next_query = t + 1e-3;
            continue;
        }
        if (t < next_query)
            continue;
        next_query = t + 1e-3;
        hipError_t e = hipStreamQuery (shmemi.stream);
        if (e != hipSuccess && e != hipErrorNotReady)
            shmemi_fatal ("kernel failed: %s", hipGetErrorString (e));
        if (e == hipSuccess && (__atomic_load_n (shmemi.sig_flag, __ATOMIC_ACQUIRE) & 0x7fffffffu) != want)
            shmemi_fatal ("stream drained but the completion signal %u never arrived", want);
        if (t - t0 > shmemi.barrier_timeout)
            shmemi_fatal ("kernel did not complete within %.0f s", shmemi.barrier_timeout);
        check_abort ();
    }
    return v;
}

/* Signal region of the fused kernel: uncached (fine-grained) device memory,
 * so peers' stores over xGMI and this GPU's polls meet in memory. */
static void sigmem_init (void)
{
    void *p = NULL;
    const size_t bytes = 131072;
    _Static_assert (MI355_SIG_WORDS * 8 <= 131072, "signal region too small");
    SHMEMI_HIP (hipExtMallocWithFlags (&p, bytes, hipDeviceMallocUncached));
    SHMEMI_HIP (hipMemset (p, 0, bytes));
    SHMEMI_HIP (hipDeviceSynchronize ());
    shmemi.sigmem = (unsigned long long *) p;
    shmemi.peer_sig = (unsigned long long **) calloc ((size_t) shmemi.npes, sizeof (void *));
    if (shmemi.peer_sig == NULL)
        shmemi_fatal ("out of host memory");
    shmemi.peer_sig[shmemi.mype] = shmemi.sigmem;
}

/* The settings that decide what the members of a collective do together
 * must agree on every PE (one PE on the fused path and another on the
 * multi-launch one would wait on each other for ever): abort at init, naming
 * the environment variable, when a peer's differ. */
static void settings_publish (void)
{
    seg_info (shmemi.mype)->settings =
        (struct shmemi_settings) {shmemi.algorithm, shmemi.order, shmemi.debug != 0, shmemi.srv.enabled,
                                  shmemi.ext_map, shmemi.calib_want, shmemi.order_chunk, shmemi.fused_max, shmemi.oneshot_max, shmemi.scratch_chunk,
                                  shmemi.user_size, shmemi.hheap_size};
}

static void settings_check (void)
{
    const struct shmemi_settings *a = &seg_info (shmemi.mype)->settings;
    for (int pe = 0; pe < shmemi.npes; ++pe) {
        if (pe == shmemi.mype)
            continue;
        const struct shmemi_settings *b = &seg_info (pe)->settings;
#define S(field, env)                                                                                           \
    if (a->field != b->field)                                                                                   \
        shmemi_fatal ("%s differs between PEs: %lld here, %lld on PE %d (every PE must use the same value)", env, \
                      (long long) a->field, (long long) b->field, pe);
        S (algorithm, "SHMEM_REDUCE_ALGORITHM")
        S (order, "SHMEM_REDUCE_ORDER")
        S (debug, "SHMEM_DEBUG")
        S (ext_map, "SHMEM_EXTERNAL_MAP")
        S (calibrate, "SHMEM_THRESHOLD_CALIBRATE (or SHMEM_FUSED_MAX_BYTES / SHMEM_ONESHOT_MAX_BYTES set on some PEs only)")
        S (order_chunk, "SHMEM_DEVICE_ORDER_SIZE")
        S (fused_max, "SHMEM_FUSED_MAX_BYTES")
        S (oneshot_max, "SHMEM_ONESHOT_MAX_BYTES")
        S (scratch_chunk, "SHMEM_DEVICE_SCRATCH_SIZE")
        S (user_size, "SHMEM_DEVICE_HEAP_SIZE")
        S (hheap_size, "SHMEM_SYMMETRIC_HEAP_SIZE")
#undef S
    }
}

/* Publish this PE's heap and map every peer's (after the info barrier). */
static void heap_exchange (void)
{
    struct shmemi_pe_info *me = seg_info (shmemi.mype);
    me->pid = (int32_t) getpid ();
    me->device = shmemi.device;
    if (hipDeviceGetPCIBusId (me->pci_bus_id, (int) sizeof me->pci_bus_id, shmemi.device) != hipSuccess)
        me->pci_bus_id[0] = '\0';
    SHMEMI_HIP (hipIpcGetMemHandle (&me->heap_handle, shmemi.heap_arena));
    SHMEMI_HIP (hipIpcGetMemHandle (&me->sig_handle, shmemi.sigmem));
    me->heap_size = shmemi.heap_size;
    settings_publish ();
    __atomic_store_n (&me->published, 1, __ATOMIC_RELEASE);
    shmemi_barrier_set (0, 1, shmemi.npes);
    settings_check ();

    for (int pe = 0; pe < shmemi.npes; ++pe) {
        if (pe == shmemi.mype)
            continue;
        struct shmemi_pe_info *pi = seg_info (pe);
        if (!__atomic_load_n (&pi->published, __ATOMIC_ACQUIRE))
            shmemi_fatal ("PE %d did not publish its heap", pe);
        if (pi->heap_size != shmemi.heap_size)
            shmemi_fatal ("PE %d has a %llu-byte device heap, this PE %zu: heap sizes must match",
                          pe, (unsigned long long) pi->heap_size, shmemi.heap_size);
        int peer_dev = -1;
        if (pi->pci_bus_id[0] != '\0' && hipDeviceGetByPCIBusId (&peer_dev, pi->pci_bus_id) != hipSuccess)
            peer_dev = -1;
        (void) hipGetLastError ();
        if (peer_dev >= 0 && peer_dev != shmemi.device) {
            int can = 0;
            if (hipDeviceCanAccessPeer (&can, shmemi.device, peer_dev) == hipSuccess && can) {
                hipError_t e = hipDeviceEnablePeerAccess (peer_dev, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
                    fprintf (stderr, "[shmem PE %d] warning: hipDeviceEnablePeerAccess(%d -> %d): %s "
                                     "(the interconnect self-test decides what runs)\n",
                             shmemi.mype, shmemi.device, peer_dev, hipGetErrorString (e));
                (void) hipGetLastError ();
            }
        }
        if (peer_dev != shmemi.device)
            shmemi.peer_acquire = 1; /* a peer on another GPU (or one this process cannot see) */
        if (me->pci_bus_id[0] != '\0' && strcmp (me->pci_bus_id, pi->pci_bus_id) == 0)
            ++shmemi.local_pes; /* shares this GPU: the fused kernels' grids must fit beside each other */
        /* A mapping that cannot be opened is not fatal here: the pointer stays
         * NULL, the self-test below fails for every PE alike and the job falls
         * back (no signal region: host barriers, no fused path; no peer heap:
         * the RCCL schedule). SHMEM_TEST_IPC_FAIL=heap|sig makes PE 1 take
         * that path (tests). */
        const char *fail = shmemi.mype == 1 ? getenv ("SHMEM_TEST_IPC_FAIL") : NULL;
        void *p = NULL;
        hipError_t e = fail != NULL && strcmp (fail, "heap") == 0
                           ? hipErrorInvalidValue
                           : hipIpcOpenMemHandle (&p, pi->heap_handle, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
            fprintf (stderr, "[shmem PE %d] warning: hipIpcOpenMemHandle of PE %d's heap (GPU %s) failed: %s\n",
                     shmemi.mype, pe, pi->pci_bus_id, hipGetErrorString (e));
            (void) hipGetLastError ();
            p = NULL;
        }
        shmemi.peer_heap[pe] = p != NULL ? (char *) p + heap_skew (pe) : NULL;
        p = NULL;
        e = fail != NULL && strcmp (fail, "sig") == 0
                ? hipErrorInvalidValue
                : hipIpcOpenMemHandle (&p, pi->sig_handle, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
            fprintf (stderr, "[shmem PE %d] warning: hipIpcOpenMemHandle of PE %d's signal region failed: %s\n",
                     shmemi.mype, pe, hipGetErrorString (e));
            (void) hipGetLastError ();
            p = NULL;
        }
        shmemi.peer_sig[pe] = (unsigned long long *) p;
    }
    shmemi_barrier_set (0, 1, shmemi.npes);
}

/* Coherence of peer-heap reads (the contract of a blocking get: it returns
 * the remote PE's CURRENT data, src/comms/gasnet/comms-inline.h:2224-2238).
 * A peer GPU's memory is cached in this GPU's L2 without coherence, so a
 * second read of a buffer a peer rewrote may hit the first read's line; the
 * P2P schedules queue mi355_acquire_system before such reads.
 * This checks the protocol on the job's real layout:
 *   1. every PE reads every peer's marker with plain cached loads, from 32
 *      blocks (dealt over the 8 XCDs, so every XCD's L2 holds the lines);
 *   2. barrier; every PE rewrites its own marker with a write-through store;
 *      barrier;
 *   3. re-read without an acquire: an old value = stale_without_acquire
 *      (evidence the acquire is needed; not an error);
 *   4. mi355_acquire_system, re-read: every block must see every new value.
 * SHMEM_TEST_IPC_FAIL=stale makes PE 1 report step 4 stale (tests). */
static void coherence_test (size_t mark_off, int *passed, int *stale, int *sysload)
{
    const int np = shmemi.npes, me = shmemi.mype, nb = 32;
    const unsigned long long newval = 0xC0DE5EE000000000ull;
    unsigned long long **ptrs = (unsigned long long **) calloc ((size_t) np, sizeof (void *));
    unsigned long long *host = (unsigned long long *) calloc ((size_t) np * nb, sizeof (unsigned long long));
    unsigned long long *dev = NULL;
    if (ptrs == NULL || host == NULL)
        shmemi_fatal ("out of host memory");
    SHMEMI_HIP (hipMalloc ((void **) &dev, sizeof (unsigned long long) * (size_t) np * nb));
    for (int q = 0; q < np; ++q)
        ptrs[q] = (unsigned long long *) (shmemi.peer_heap[q] + mark_off);
#define PEEK(what)                                                                                              \
    do {                                                                                                        \
        if (mi355_peek_cached ((const unsigned long long *const *) ptrs, np, dev, nb, shmemi.stream) != 0)      \
            shmemi_fatal ("coherence test: peek launch failed");                                               \
        SHMEMI_HIP (hipMemcpy (host, dev, sizeof (unsigned long long) * (size_t) np * nb,                       \
                               hipMemcpyDeviceToHost));                                                         \
    } while (0)
    PEEK ("first read");
    shmemi_barrier_set (0, 1, np);
    unsigned long long *own = (unsigned long long *) (shmemi.heap + mark_off);
    if (mi355_poke (&own, 1, newval + (unsigned long long) me, shmemi.stream) != 0)
        shmemi_fatal ("coherence test: poke launch failed");
    SHMEMI_HIP (hipStreamSynchronize (shmemi.stream));
    shmemi_barrier_set (0, 1, np);
    /* 3a. system-coherent loads, no acquire (the fused kernel's reads of the
     * members' buffers): every block must see every new value */
    if (mi355_peek_sysload ((const unsigned long long *const *) ptrs, np, dev, nb, shmemi.stream) != 0)
        shmemi_fatal ("coherence test: system-load peek launch failed");
    SHMEMI_HIP (hipMemcpy (host, dev, sizeof (unsigned long long) * (size_t) np * nb, hipMemcpyDeviceToHost));
    *sysload = 1;
    for (int b = 0; b < nb; ++b)
        for (int q = 0; q < np; ++q)
            if (host[(size_t) b * np + q] != newval + (unsigned long long) q)
                *sysload = 0;
    PEEK ("re-read without acquire");
    *stale = 0;
    for (int b = 0; b < nb; ++b)
        for (int q = 0; q < np; ++q)
            if (host[(size_t) b * np + q] != newval + (unsigned long long) q)
                *stale = 1;
    if (mi355_acquire_system (shmemi.stream) != 0)
        shmemi_fatal ("coherence test: acquire launch failed");
    PEEK ("re-read after acquire");
#undef PEEK
    *passed = 1;
    for (int b = 0; b < nb; ++b)
        for (int q = 0; q < np; ++q)
            if (host[(size_t) b * np + q] != newval + (unsigned long long) q)
                *passed = 0;
    const char *fail = me == 1 ? getenv ("SHMEM_TEST_IPC_FAIL") : NULL;
    if (fail != NULL && strcmp (fail, "stale") == 0)
        *passed = 0, *stale = 1, *sysload = 0;
    if (fail != NULL && strcmp (fail, "sysload") == 0)
        *sysload = 0; /* only the system-coherent loads stale: the fused kernel keeps its acquires */
    (void) hipFree (dev);
    free (host);
    free (ptrs);
}

/* The CALLER's producer path (round 4). coherence_test above rewrites its
 * marker with the library's own write-through store; a caller writes its
 * source with plain stores in a kernel of its own and then calls. Here every
 * PE writes 32 marker words with plain stores from 32 blocks of a kernel on
 * the NULL stream (mi355_mark_plain: dirty lines in several XCDs' L2s), and
 * the peers read them, after peer reads of the old values cached them, in the
 * two orderings the library relies on:
 *   F  the fused kernel's: the same-stream flag publish (mi355_poke on the
 *      blocking library stream, so after the caller's kernel) and a device
 *      wait for every member's flag (mi355_producer_read), no host involved;
 *   H  the multi-launch schedules': shmemi_order_after_caller (signal kernel,
 *      host wait), host barrier, then the read kernel.
 * Each read three ways: plain loads with no acquire, 16-byte system-coherent
 * loads (the fused kernel's folds), plain loads after a system-scope acquire.
 * res[] = 1 where every block of this PE saw every member's new words, in
 * shmemi.prod[] order (F plain, F sysload, F acquire, H plain, H sysload,
 * H acquire). SHMEM_TEST_IPC_FAIL=sysload (PE 1) reports F sysload stale;
 * =producer reports H acquire stale; =producer_fused reports F sysload and
 * F acquire stale (the fused kernel is then turned off job-wide). */
static void producer_test (size_t off, int *res)
{
    const int np = shmemi.npes, me = shmemi.mype, nb = 32, W = 32;
    const size_t per = (size_t) np * W, nout = 3 * (size_t) nb * per + 1;
    const unsigned long long *ptrs[64];
    unsigned long long *flags[64];
    unsigned long long *host = (unsigned long long *) calloc (nout, sizeof (unsigned long long));
    unsigned long long *dev = NULL;
    if (host == NULL)
        shmemi_fatal ("out of host memory");
    SHMEMI_HIP (hipMalloc ((void **) &dev, nout * sizeof (unsigned long long)));
    for (int q = 0; q < np; ++q) {
        ptrs[q] = (const unsigned long long *) (shmemi.peer_heap[q] + off);
        flags[q] = shmemi.peer_sig[q] + MI355_SIG_SELFTEST2 + me;
    }
    unsigned long long *own = (unsigned long long *) (shmemi.heap + off);
    const unsigned long long timeout = 1000000000ull; /* 10 s of the 100 MHz s_memrealtime */
    const unsigned long long v_old = 0x01D0000000000000ull, v_f = 0xF05ED00000000000ull,
                             v_h = 0xB05ED00000000000ull, token = 0x70CE000000000001ull;
    for (int i = 0; i < 6; ++i)
        res[i] = 1;
#define RUN(call)                                                                                               \
    do {                                                                                                        \
        if ((call) != 0)                                                                                        \
            shmemi_fatal ("producer-path test: launch failed: %s", #call);                                     \
    } while (0)
#define READ_BACK(first)                                                                                        \
    do {                                                                                                        \
        SHMEMI_HIP (hipStreamSynchronize (shmemi.stream));                                                      \
        SHMEMI_HIP (hipMemcpy (host, dev, nout * sizeof (unsigned long long), hipMemcpyDeviceToHost));          \
        for (int t = 0; t < 3; ++t)                                                                             \
            for (int b = 0; b < nb; ++b)                                                                        \
                for (size_t i = 0; i < per; ++i)                                                                \
                    if (host[((size_t) t * nb + b) * per + i] !=                                                \
                        val + ((unsigned long long) (i / W) << 16) + (i % W))                                   \
                        res[(first) + t] = 0;                                                                   \
        if (host[nout - 1] != 0)                                                                                \
            res[(first)] = res[(first) + 1] = res[(first) + 2] = 0;                                             \
    } while (0)
    /* the old values, cached by every PE's reads */
    RUN (mi355_mark_plain (own, W, v_old + ((unsigned long long) me << 16), NULL));
    SHMEMI_HIP (hipDeviceSynchronize ());
    shmemi_barrier_set (0, 1, np);
    SHMEMI_HIP (hipMemset (dev, 0, nout * sizeof (unsigned long long)));
    RUN (mi355_producer_read (ptrs, np, W, NULL, 0, 0, dev, nb, shmemi.stream));
    SHMEMI_HIP (hipStreamSynchronize (shmemi.stream));
    shmemi_barrier_set (0, 1, np);
    /* F: caller kernel on the null stream, then the fused kernel's ordering */
    unsigned long long val = v_f;
    RUN (mi355_mark_plain (own, W, v_f + ((unsigned long long) me << 16), NULL));
    SHMEMI_HIP (hipMemsetAsync (dev, 0, nout * sizeof (unsigned long long), shmemi.stream));
    RUN (mi355_poke (flags, np, token, shmemi.stream));
    RUN (mi355_producer_read (ptrs, np, W, shmemi.sigmem + MI355_SIG_SELFTEST2, token, timeout, dev, nb,
                              shmemi.stream));
    /* kernel order = PE order of the results (i / W = member q) */
    READ_BACK (0);
    shmemi_barrier_set (0, 1, np); /* nobody reads the F words any more */
    /* H: caller kernel on the null stream, then the multi-launch ordering */
    val = v_h;
    RUN (mi355_mark_plain (own, W, v_h + ((unsigned long long) me << 16), NULL));
    shmemi_order_after_caller (1);
    shmemi_barrier_set (0, 1, np);
    SHMEMI_HIP (hipMemsetAsync (dev, 0, nout * sizeof (unsigned long long), shmemi.stream));
    RUN (mi355_producer_read (ptrs, np, W, NULL, 0, 0, dev, nb, shmemi.stream));
    READ_BACK (3);
    shmemi_barrier_set (0, 1, np);
#undef READ_BACK
#undef RUN
    const char *fail = me == 1 ? getenv ("SHMEM_TEST_IPC_FAIL") : NULL;
    if (fail != NULL && strcmp (fail, "sysload") == 0)
        res[MI355_PROD_F_SYS] = 0;
    if (fail != NULL && strcmp (fail, "producer") == 0)
        res[MI355_PROD_H_ACQ] = 0;
    if (fail != NULL && strcmp (fail, "producer_fused") == 0)
        res[MI355_PROD_F_SYS] = res[MI355_PROD_F_ACQ] = 0;
    (void) hipFree (dev);
    free (host);
}


/* Device-side waits across PEs need every member's hardware queue scheduled
 * at once. With more queues on one GPU than the hardware maps together
 * (PEs sharing a GPU, 4 queues each by default: 6 PEs = 24), the queues are
 * time-sliced and every spin-wait lasts until its peers' turn: a 64 KiB
 * fused call took 22 ms instead of 40 us (bench.py fused_same_gpu at 6 PEs,
 * 40 us with GPU_MAX_HW_QUEUES=2). So init times 8 device barriers over the
 * whole job and counts the queues on this GPU; if any PE finds either too
 * high, every PE runs host barriers and no fused kernel (kernels that never
 * wait on each other run fine time-sliced).
 * The stream-ordered collectives have only device barriers: they stay, slow.
 * SHMEM_TEST_IPC_FAIL=slowwait makes PE 1 report slow waits (tests). */
static void device_wait_test (int np, int me)
{
    double us = 0.0;
    int slow = 0;
    /* A device barrier holds at most MI355_FUSED_MAX_MEMBERS members
     * (MI355FusedArgs), and no active set larger than that ever takes one
     * (device_flags_ok): a bigger job times nothing and keeps only the queue
     * vote below, which still decides the job's smaller active sets. */
    if (np <= MI355_FUSED_MAX_MEMBERS) {
        MI355FusedArgs a;
        shmemi_member_args (&a, 0, 1, np, me);
        /* one untimed barrier (first launch of the kernel), then every PE
         * starts the timed ones together: a late PE would otherwise count as
         * slow waits */
        if (mi355_device_barrier (&a, shmemi.stream) != 0)
            shmemi_fatal ("self-test device barrier launch failed");
        SHMEMI_HIP (hipStreamSynchronize (shmemi.stream));
        shmemi_barrier_set (0, 1, np);
        const int k = 8;
        const double t0 = shmemi_now ();
        for (int i = 0; i < k; ++i)
            if (mi355_device_barrier (&a, shmemi.stream) != 0)
                shmemi_fatal ("self-test device barrier launch failed");
        SHMEMI_HIP (hipStreamSynchronize (shmemi.stream));
        us = (shmemi_now () - t0) / k * 1e6;
        slow = us > 1000.0;
    }
    /* At init each PE has touched only the null stream's and the library
     * stream's queues, so the timing above passes even where the steady
     * state (HIP allocates up to GPU_MAX_HW_QUEUES per process as it runs)
     * is time-sliced: 6 PEs x 4 queues timed 8 barriers fine and still ran
     * fused calls at 22 ms. PEs x queues on this GPU above 16 (4 PEs x 4 ran
     * at full speed) counts as slow too. */
    static const char *hwq_env[] = {"GPU_MAX_HW_QUEUES", NULL};
    const long hwq = env_long (hwq_env, 4);
    slow |= (long) shmemi.local_pes * (hwq > 0 ? hwq : 4) > 16;
    const char *fail = me == 1 ? getenv ("SHMEM_TEST_IPC_FAIL") : NULL;
    slow |= fail != NULL && strcmp (fail, "slowwait") == 0;
    /* SHMEM_DEVICE_WAITS=1 keeps the device-side waits whatever the above says,
     * =0 turns them off (a job-wide setting, like the others) */
    static const char *dw_env[] = {"SHMEM_DEVICE_WAITS", NULL};
    const long force = env_long (dw_env, -1);
    if (force == 0 || force == 1)
        slow = force == 0;
    /* the timing in ns, this PE's vote in bit 63 */
    __atomic_store_n (&seg_info (me)->barrier_ns, (uint64_t) (us * 1e3) | ((uint64_t) slow << 63), __ATOMIC_RELEASE);
    shmemi_barrier_set (0, 1, np);
    double worst = 0;
    int any_slow = 0;
    for (int q = 0; q < np; ++q) {
        const uint64_t r = __atomic_load_n (&seg_info (q)->barrier_ns, __ATOMIC_ACQUIRE);
        const double u = (double) (r & ~(1ull << 63)) * 1e-3;
        worst = u > worst ? u : worst;
        any_slow |= (int) (r >> 63);
    }
    shmemi.dev_barrier_us = worst;
    if (any_slow) {
        if (me == 0)
            fprintf (stderr, "[shmem] warning: device-side waits across PEs would be time-sliced (%d PE(s) on this "
                             "GPU x %ld hardware queues; init barriers %.0f us each; GPU_MAX_HW_QUEUES=2 lowers a PE's "
                             "share): host barriers, no fused kernel\n", shmemi.local_pes, hwq, worst);
        shmemi.dev_wait_slow = 1;
        shmemi.fused_max = 0, shmemi.fused_off = 1;
    }
}

/* Interconnect check at init (PE_size > 1): every PE stores a value into
 * every peer's signal region over the peer mapping (what the fused kernel's
 * flags do) and reads a marker from every peer's heap (what the reduce-scatter
 * does). All PEs learn every PE's outcome through the bootstrap segment and
 * take the same decision: signal stores not seen -> fused path off;
 * peer heap reads wrong -> RCCL schedule (or a loud failure without it). */
static void interconnect_selftest (void)
{
    const int np = shmemi.npes, me = shmemi.mype;
    if (np > 1024)
        return;
    const size_t mark_off = shmemi.scratch_off + 3 * shmemi.scratch_chunk - 8;
    const unsigned long long mark = 0x5E1F7E5700000000ull + (unsigned long long) me;
    SHMEMI_HIP (hipMemcpy (shmemi.heap + mark_off, &mark, 8, hipMemcpyHostToDevice));
    shmemi_barrier_set (0, 1, np);

    unsigned long long **ptrs = (unsigned long long **) calloc ((size_t) np, sizeof (void *));
    unsigned long long *host = (unsigned long long *) calloc ((size_t) np, sizeof (unsigned long long));
    unsigned long long *dev = NULL;
    if (ptrs == NULL || host == NULL)
        shmemi_fatal ("out of host memory");
    SHMEMI_HIP (hipMalloc ((void **) &dev, sizeof (unsigned long long) * (size_t) np));
    int sig_ok = 1, heap_ok = 1;
    int k = 0;
    for (int q = 0; q < np; ++q) {
        if (q == me)
            continue;
        if (shmemi.peer_sig[q] == NULL)
            sig_ok = 0; /* not mapped: nothing to poke */
        else
            ptrs[k++] = shmemi.peer_sig[q] + MI355_SIG_SELFTEST + me;
        if (shmemi.peer_heap[q] == NULL)
            heap_ok = 0;
    }
    if (k > 0 && mi355_poke (ptrs, k, 0xA11CE00000000000ull + (unsigned long long) me, shmemi.stream) != 0)
        shmemi_fatal ("self-test poke launch failed");
    SHMEMI_HIP (hipStreamSynchronize (shmemi.stream));
    shmemi_barrier_set (0, 1, np);

    for (int q = 0; q < np; ++q)
        ptrs[q] = shmemi.sigmem + MI355_SIG_SELFTEST + q;
    if (mi355_peek ((const unsigned long long *const *) ptrs, np, dev, shmemi.stream) != 0)
        shmemi_fatal ("self-test peek launch failed");
    SHMEMI_HIP (hipStreamSynchronize (shmemi.stream));
    SHMEMI_HIP (hipMemcpy (host, dev, sizeof (unsigned long long) * (size_t) np, hipMemcpyDeviceToHost));
    for (int q = 0; q < np; ++q)
        if (q != me && host[q] != 0xA11CE00000000000ull + (unsigned long long) q)
            sig_ok = 0;
    if (heap_ok) { /* every peer heap mapped: read each one's marker */
        for (int q = 0; q < np; ++q)
            ptrs[q] = (unsigned long long *) (shmemi.peer_heap[q] + mark_off);
        if (mi355_peek ((const unsigned long long *const *) ptrs, np, dev, shmemi.stream) != 0)
            shmemi_fatal ("self-test peek launch failed");
        SHMEMI_HIP (hipStreamSynchronize (shmemi.stream));
        SHMEMI_HIP (hipMemcpy (host, dev, sizeof (unsigned long long) * (size_t) np, hipMemcpyDeviceToHost));
        for (int q = 0; q < np; ++q)
            if (host[q] != 0x5E1F7E5700000000ull + (unsigned long long) q)
                heap_ok = 0;
    }
    (void) hipFree (dev);
    free (host);
    free (ptrs);

    /* every PE runs the coherence test when every PE has its peers mapped */
    __atomic_store_n (&seg_info (me)->selftest, sig_ok | (heap_ok << 1), __ATOMIC_RELEASE);
    shmemi_barrier_set (0, 1, np);
    int all_mapped = 1, all_sig_mapped = 1;
    for (int q = 0; q < np; ++q) {
        const int r = __atomic_load_n (&seg_info (q)->selftest, __ATOMIC_ACQUIRE);
        all_mapped &= (r >> 1) & 1;
        all_sig_mapped &= r & 1;
    }
    int coh = 0;
    if (all_mapped) {
        int passed = 1, stale = 0, sysload = 0;
        coherence_test (mark_off, &passed, &stale, &sysload);
        coh = 4 | (passed << 3) | (stale << 4) | (sysload << 5);
        /* mi355_producer_read's member limit; its F round stores flags into
         * every peer's signal region, so every PE must have mapped them all */
        if (np <= 64 && all_sig_mapped) {
            int prod[6];
            producer_test (mark_off + 8 - 1024, prod); /* 32 words below the marker, 16-byte aligned */
            coh |= 1 << 6;
            for (int i = 0; i < 6; ++i)
                coh |= prod[i] << (7 + i);
            /* the multi-launch schedules read peers' buffers the H way */
            passed &= prod[MI355_PROD_H_ACQ];
            coh = (coh & ~(1 << 3)) | (passed << 3);
        }
        if (!passed)
            heap_ok = 0;
    }

    __atomic_store_n (&seg_info (me)->selftest, sig_ok | (heap_ok << 1) | coh, __ATOMIC_RELEASE);
    shmemi_barrier_set (0, 1, np);
    int all_sig = 1, all_heap = 1;
    shmemi.coh_ran = all_mapped;
    shmemi.coh_passed = all_mapped;
    shmemi.coh_stale = 0;
    shmemi.coh_sysload = all_mapped;
    shmemi.prod_ran = all_mapped;
    for (int i = 0; i < 6; ++i)
        shmemi.prod[i] = all_mapped;
    for (int q = 0; q < np; ++q) {
        const int r = __atomic_load_n (&seg_info (q)->selftest, __ATOMIC_ACQUIRE);
        all_sig &= r & 1;
        all_heap &= (r >> 1) & 1;
        shmemi.coh_passed &= (r >> 3) & 1;
        shmemi.coh_stale |= (r >> 4) & 1;
        shmemi.coh_sysload &= (r >> 5) & 1;
        shmemi.prod_ran &= (r >> 6) & 1;
        for (int i = 0; i < 6; ++i)
            shmemi.prod[i] &= (r >> (7 + i)) & 1;
    }
    if (!shmemi.prod_ran)
        for (int i = 0; i < 6; ++i)
            shmemi.prod[i] = 0;
    /* the fused kernel's per-block acquires are redundant when its
     * system-coherent loads read fresh data on every PE, both after the
     * library's own write-through stores and after a caller's kernel wrote
     * with plain stores and the fused kernel's flag ordering passed (the same
     * decision on every PE: from the same records); SHMEM_FUSED_ACQUIRE=1
     * keeps them */
    {
        static const char *acq_env[] = {"SHMEM_FUSED_ACQUIRE", NULL};
        shmemi.fused_no_acquire = shmemi.coh_sysload && shmemi.prod_ran && shmemi.prod[MI355_PROD_F_SYS] &&
                                  shmemi.coh_passed && env_long (acq_env, 0) == 0;
    }
    /* a caller's data not seen through the fused kernel's ordering even
     * after an acquire: the fused kernel is not used */
    if (shmemi.prod_ran && !shmemi.prod[MI355_PROD_F_ACQ] && !shmemi.prod[MI355_PROD_F_SYS]) {
        if (me == 0)
            fprintf (stderr, "[shmem] warning: a caller's plain stores were not visible to peers through the fused "
                             "kernel's flag ordering (init producer-path test); the fused kernel is disabled\n");
        shmemi.fused_max = 0, shmemi.fused_off = 1;
    }
    if (all_mapped && !shmemi.coh_passed && me == 0)
        fprintf (stderr, "[shmem] warning: a peer heap re-read after a system-scope acquire returned stale data "
                         "(init coherence test)\n");
    if (!all_sig) {
        if (me == 0)
            fprintf (stderr, "[shmem] warning: peer signal-region stores are not visible; "
                             "the fused small-message kernel is disabled\n");
        shmemi.fused_max = 0, shmemi.fused_off = 1;
        shmemi.sig_broken = 1;
    } else {
        device_wait_test (np, me);
    }
    if (!all_heap) {
        if (me == 0)
            fprintf (stderr, "[shmem] warning: peer heap reads returned wrong data; "
                             "using the RCCL schedule\n");
        shmemi.algorithm = SHMEMX_REDUCE_RCCL;
        shmemi.p2p_broken = 1;
        shmemi.fused_max = 0, shmemi.fused_off = 1; /* its kernels read the peers' heaps too: every PE takes the same path */
        shmemi.ext_map = 0;   /* peers' other allocations would be mapped the same way (extmap.c) */
    }
    shmemi_barrier_set (0, 1, np);
}

/* shmem_collect's per-PE counts, read by the other members after a barrier */
static size_t local_count;

void shmemi_publish_count (size_t nbytes)
{
    if (shmemi.seg == NULL)
        local_count = nbytes;
    else
        __atomic_store_n (&seg_info (shmemi.mype)->collect_bytes, (uint64_t) nbytes, __ATOMIC_RELEASE);
}

size_t shmemi_peer_count (int pe)
{
    if (shmemi.seg == NULL)
        return local_count;
    return (size_t) __atomic_load_n (&seg_info (pe)->collect_bytes, __ATOMIC_ACQUIRE);
}

void *shmemx_malloc_device (size_t size)
{
    shmemi_init_check ("shmemx_malloc_device");
    if (shmemi.heap == NULL)
        shmemi_fatal ("shmemx_malloc_device: no GPU (SHMEM_BOOTSTRAP_ONLY)");
    void *ret = NULL;
    if (size != 0) {
        const size_t need = round_up (size, SHMEMI_ALIGN);
        for (struct shmemi_block *b = shmemi.blocks; b != NULL; b = b->next) {
            if (b->used || b->size < need)
                continue;
            if (b->size > need) {
                struct shmemi_block *rest = (struct shmemi_block *) calloc (1, sizeof *rest);
                if (rest == NULL)
                    shmemi_fatal ("out of host memory");
                rest->off = b->off + need;
                rest->size = b->size - need;
                rest->next = b->next;
                b->next = rest;
                b->size = need;
            }
            b->used = 1;
            ret = shmemi.heap + b->off;
            break;
        }
        if (ret == NULL)
            SHMEMI_TRACE (SHMEMI_LOG_NOTICE, "shmemx_malloc_device(%zu): device heap exhausted", size);
    }
    SHMEMI_TRACE (SHMEMI_LOG_MEMORY, "shmemx_malloc_device(%zu) = %p (heap offset %zu)", size, ret,
                  ret != NULL ? (size_t) ((char *) ret - shmemi.heap) : (size_t) 0);
    shmem_barrier_all ();
    return ret;
}

static int device_free (void *ptr)
{
    if (!shmemi_in_device_heap (ptr, 0))
        return 0;
    const size_t off = shmemi_heap_offset (ptr);
    struct shmemi_block *prev = NULL;
    for (struct shmemi_block *b = shmemi.blocks; b != NULL; prev = b, b = b->next) {
        if (b->off != off || !b->used)
            continue;
        b->used = 0;
        struct shmemi_block *n = b->next;
        if (n != NULL && !n->used) {
            b->size += n->size;
            b->next = n->next;
            free (n);
        }
        if (prev != NULL && !prev->used) {
            prev->size += b->size;
            prev->next = b->next;
            free (b);
        }
        return 1;
    }
    shmemi_fatal ("shmem_free(%p): not an allocated device-heap block", ptr);
}

void shmemx_free_device (void *ptr)
{
    shmemi_init_check ("shmemx_free_device");
    SHMEMI_TRACE (SHMEMI_LOG_MEMORY, "shmemx_free_device(%p)", ptr);
    shmem_barrier_all ();
    if (ptr != NULL && !device_free (ptr))
        shmemi_fatal ("shmemx_free_device(%p): not in the device symmetric heap", ptr);
}

int shmemx_is_device_symmetric (const void *ptr) { return shmemi_in_device_heap (ptr, 0); }

/* PE pe's copy of the device-heap object at ptr, as an address this PE's GPU
 * can load from and store to (the peer arena's IPC mapping; this PE's own
 * address for pe = this PE); NULL when ptr is not in the device heap or pe's
 * heap is not mapped here. For kernels only: the host cannot dereference it. */
void *shmemx_peer_device_ptr (const void *ptr, int pe)
{
    shmemi_init_check ("shmemx_peer_device_ptr");
    if (pe < 0 || pe >= shmemi.npes || !shmemi_in_device_heap (ptr, 1) || shmemi.peer_heap == NULL ||
        shmemi.peer_heap[pe] == NULL)
        return NULL;
    return shmemi.peer_heap[pe] + shmemi_heap_offset (ptr);
}

/* ---------------------------------------------------------------------- */
/* host heap (shmem_malloc's default: the reference returns host memory)    */
/* ---------------------------------------------------------------------- */
/* SHMEM_SYMMETRIC_HEAP_SIZE (the reference's name, comms-inline.h:675): the
 * size of each PE's symmetric host heap segment; virtual, pages are committed
 * per shmem_malloc block. Default 4 GiB (the reference: 32 MiB). */
static void hheap_setup (void)
{
    shmemi_hheap_create (env_size ("SHMEM_SYMMETRIC_HEAP_SIZE", (size_t) 4 << 30));
}

static int heap_kind_device (void)
{
    const char *v = getenv ("SHMEM_SYMMETRIC_HEAP_KIND");
    return v != NULL && strcasecmp (v, "device") == 0;
}

void *pshmem_malloc (size_t size)
{
    shmemi_init_check ("shmem_malloc");
    if (shmemi.heap != NULL)
        shmemi_server_stop (); /* hipHostRegister below */
    if (heap_kind_device ())
        return shmemx_malloc_device (size);
    void *p = shmemi_host_malloc (size);
    SHMEMI_TRACE (SHMEMI_LOG_MEMORY, "shmem_malloc(%zu) = %p (symmetric host heap)", size, p);
    shmem_barrier_all ();
    return p;
}

/* 1 if PE pe runs on this PE's GPU (same PCI bus id): its device heap is
 * this GPU's own memory. */
int shmemi_pe_same_device (int pe)
{
    if (pe == shmemi.mype)
        return 1;
    if (shmemi.seg == NULL || pe < 0 || pe >= shmemi.npes)
        return 0;
    const char *mine = seg_info (shmemi.mype)->pci_bus_id, *theirs = seg_info (pe)->pci_bus_id;
    return mine[0] != '\0' && strcmp (mine, theirs) == 0;
}

/* MI355X extension (shmemx.h): the same, for callers (bench.py tells an
 * xGMI run from PEs sharing one GPU by PCI bus id, not by the HIP ordinal,
 * which is 0 for every rank under a launcher that gives each one GPU). */
int shmemx_pe_same_device (int pe)
{
    shmemi_init_check ("shmemx_pe_same_device");
    return shmemi_pe_same_device (pe);
}

void pshmem_free (void *ptr)
{
    shmemi_init_check ("shmem_free");
    if (shmemi.heap != NULL)
        shmemi_server_stop (); /* hipHostUnregister below */
    shmem_barrier_all ();
    if (ptr == NULL)
        return;
    if (device_free (ptr))
        return;
    if (shmemi_host_free (ptr))
        return;
    shmemi_fatal ("shmem_free(%p): not allocated by shmem_malloc", ptr);
}

/* ---------------------------------------------------------------------- */
/* init / finalize                                                         */
/* ---------------------------------------------------------------------- */
static void finalize_atexit (void) { pshmem_finalize (); }

/* The fused / one-shot thresholds from measurement on this job's layout
 * (reduce.c shmemi_calibrate_thresholds), where the environment did not set
 * them: every PE decides alike (calib_want is a checked setting, and the
 * self-test outcomes below are job-wide). */
static void calibrate (void)
{
    if (shmemi.npes < 2 || shmemi.calib_want == 0 || shmemi.fused_off || shmemi.sig_broken || shmemi.dev_wait_slow ||
        shmemi.p2p_broken || shmemi.algorithm == SHMEMX_REDUCE_EXACT || shmemi.algorithm == SHMEMX_REDUCE_RCCL)
        return;
    shmemi_calibrate_thresholds (shmemi.calib_want & 1, (shmemi.calib_want >> 1) & 1);
}

void pshmem_init (void)
{
    if (shmemi.initialized)
        return;
    static const char *pe_env[] = {"SHMEM_PE", "RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", NULL};
    static const char *np_env[] = {"SHMEM_NPES", "WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", NULL};
    static const char *dev_env[] = {"SHMEM_DEVICE", "LOCAL_RANK", "SHMEM_LOCAL_PE",
                                    "OMPI_COMM_WORLD_LOCAL_RANK", NULL};
    static const char *to_env[] = {"SHMEM_BARRIER_TIMEOUT", NULL};
    static const char *dbg_env[] = {"SHMEM_DEBUG", NULL};
    shmemi.npes = (int) env_long (np_env, 1);
    shmemi.mype = (int) env_long (pe_env, 0);
    if (shmemi.npes < 1 || shmemi.npes > SHMEMI_MAX_PES || shmemi.mype < 0 || shmemi.mype >= shmemi.npes)
        shmemi_fatal ("invalid PE identity %d of %d (SHMEM_PE/SHMEM_NPES or RANK/WORLD_SIZE)",
                      shmemi.mype, shmemi.npes);
    shmemi_trace_init ();
    shmemi.barrier_timeout = (double) env_long (to_env, 600);
    shmemi.debug = (int) env_long (dbg_env, 0);
    static const char *es_env[] = {"SHMEM_ENTRY_SYNC", NULL};
    shmemi.entry_sync = (int) env_long (es_env, 0);
    static const char *em_env[] = {"SHMEM_EXTERNAL_MAP", NULL};
    shmemi.ext_map = env_long (em_env, 1) != 0;
    shmemi.algorithm = parse_algorithm (getenv ("SHMEM_REDUCE_ALGORITHM"));
    shmemi.order = parse_order (getenv ("SHMEM_REDUCE_ORDER"));

    /* test hook: bring up PEs, barriers and the host heap without a GPU (CPU
     * tests of the bootstrap); every reduction then aborts, there is no CPU path */
    static const char *bo_env[] = {"SHMEM_BOOTSTRAP_ONLY", NULL};
    if (env_long (bo_env, 0) != 0) {
        shmemi.device = -1;
        if (shmemi.npes > 1)
            bootstrap_attach ();
        hheap_setup ();
        if (shmemi.npes > 1) {
            settings_publish ();
            shmemi_barrier_set (0, 1, shmemi.npes);
            settings_check ();
            shmemi_hheap_attach ();
            shmemi_barrier_set (0, 1, shmemi.npes); /* every segment mapped everywhere */
            shmemi_hheap_unlink ();
            if (shmemi.mype == 0) {
                shm_unlink (shmemi.seg_name);
                shmemi.seg_unlinked = 1;
            }
        }
        shmemi.initialized = 1;
        shmemi_trace_show_levels ();
        shmemi_trace_show_info ();
        return;
    }

    int ndev = 0;
    hipError_t e = hipGetDeviceCount (&ndev);
    if (e != hipSuccess || ndev < 1)
        shmemi_fatal ("no HIP device visible (%s): the reduction path runs on the GPU and has "
                      "no CPU fallback", e != hipSuccess ? hipGetErrorString (e) : "0 devices");
    long dev = env_long (dev_env, shmemi.mype);
    shmemi.device = (int) (dev % ndev);
    SHMEMI_HIP (hipSetDevice (shmemi.device));
    /* blocking: ordered after the null stream, see shmemi_order_after_caller */
    SHMEMI_HIP (hipStreamCreateWithFlags (&shmemi.stream, hipStreamDefault));
    SHMEMI_HIP (hipStreamCreateWithFlags (&shmemi.stream_in, hipStreamDefault));
    SHMEMI_HIP (hipStreamCreateWithFlags (&shmemi.stream_out, hipStreamDefault));
    for (int i = 0; i < 2; ++i) {
        SHMEMI_HIP (hipEventCreateWithFlags (&shmemi.ev_in[i], hipEventDisableTiming));
        SHMEMI_HIP (hipEventCreateWithFlags (&shmemi.ev_out[i], hipEventDisableTiming));
    }
    shmemi.local_pes = 1;
    heap_init ();
    signal_init ();
    sigmem_init ();
    server_init ();
    shmemi.fused_max = env_size ("SHMEM_FUSED_MAX_BYTES", (size_t) 2 << 20);
    /* the fused kernel's folds address a member's buffer with 32-bit byte
     * offsets (fused.hip ld16_sys_at) */
    if (shmemi.fused_max > ((size_t) 1 << 30))
        shmemi.fused_max = (size_t) 1 << 30;
    shmemi.oneshot_max = env_size ("SHMEM_ONESHOT_MAX_BYTES", (size_t) 64 << 10);
    /* thresholds not given: measured at init (PE_size > 1, calibrate below);
     * SHMEM_THRESHOLD_CALIBRATE=0 keeps the defaults above */
    {
        static const char *cal_env[] = {"SHMEM_THRESHOLD_CALIBRATE", NULL};
        shmemi.calib_want = env_long (cal_env, 1) == 0 ? 0
                                                       : (getenv ("SHMEM_FUSED_MAX_BYTES") == NULL ? 1 : 0) |
                                                             (getenv ("SHMEM_ONESHOT_MAX_BYTES") == NULL ? 2 : 0);
    }

    if (shmemi.npes == 1)
        hheap_setup ();
    if (shmemi.npes > 1) {
        bootstrap_attach ();
        hheap_setup ();
        heap_exchange (); /* settings agreed, every PE's segments created */
        shmemi_hheap_attach ();
        /* SHMEM_PEER_ACQUIRE=0|1 overrides the choice made from the peers' devices */
        static const char *pa_env[] = {"SHMEM_PEER_ACQUIRE", NULL};
        shmemi.peer_acquire = (int) env_long (pa_env, shmemi.peer_acquire) != 0;
        /* SHMEM_FUSED_GRID_SHARE=k: size the spin-waiting grids as if k PEs shared this GPU */
        static const char *gs_env[] = {"SHMEM_FUSED_GRID_SHARE", NULL};
        shmemi.local_pes = (int) env_long (gs_env, shmemi.local_pes);
        if (shmemi.local_pes < 1)
            shmemi.local_pes = 1;
        interconnect_selftest (); /* its barriers: every PE has mapped every host segment */
        shmemi_hheap_unlink ();
        if (shmemi.mype == 0 && !shmemi.seg_unlinked) {
            shm_unlink (shmemi.seg_name); /* every PE is attached: drop the name */
            shmemi.seg_unlinked = 1;
        }
    }
    shmemi.initialized = 1;
    calibrate ();
    shmemi_trace_show_levels ();
    if (shmemi_trace_mask & (1u << SHMEMI_LOG_INIT)) {
        char bus[64] = "";
        (void) hipDeviceGetPCIBusId (bus, (int) sizeof bus, shmemi.device);
        static const char *const alg[] = {"auto", "p2p", "exact", "rccl"};
        SHMEMI_TRACE (SHMEMI_LOG_INIT, "%s: PE %d of %d on GPU %d (%s)", SHMEMX_VERSION_STRING, shmemi.mype,
                      shmemi.npes, shmemi.device, bus);
        SHMEMI_TRACE (SHMEMI_LOG_INIT,
                      "device heap %zu bytes (user %zu, scratch 3 x %zu, version areas 2 x %zu), signal region %s",
                      shmemi.heap_size, shmemi.user_size, shmemi.scratch_chunk, shmemi.order_chunk,
                      shmemi.sig_broken ? "off (self-test failed)" : "on");
        SHMEMI_TRACE (SHMEMI_LOG_INIT,
                      "reduce algorithm %s, result order %s, fused path up to %zu bytes, peer heap reads %s, "
                      "peer L2 acquire %s",
                      alg[shmemi.algorithm & 3], shmemi.order == SHMEMX_ORDER_REFERENCE ? "reference (per PE)" : "PE_start",
                      shmemi.fused_max, shmemi.p2p_broken ? "FAILED (RCCL)" : "ok", shmemi.peer_acquire ? "on" : "off");
    }
    shmemi_trace_show_info ();
    static int registered = 0;
    if (!registered) {
        atexit (finalize_atexit);
        registered = 1;
    }
}

void pstart_pes (int npes)
{
    (void) npes; /* the reference ignores the argument too */
    pshmem_init ();
}

void pshmem_finalize (void)
{
    if (!shmemi.initialized)
        return;
    SHMEMI_TRACE (SHMEMI_LOG_FINALIZE, "finalizing (PE %d of %d)", shmemi.mype, shmemi.npes);
    if (shmemi.device >= 0 && shmemi.heap != NULL)
        shmemi_server_stop ();
    /* stream-ordered collectives still queued on the caller's streams finish
     * first (they only wait on peers' kernels that are already enqueued) */
    if (shmemi.device >= 0 && shmemi.heap != NULL)
        (void) hipDeviceSynchronize ();
    shmem_barrier_all ();
    if (shmemi.rccl_comm != NULL) {
        extern void shmemi_rccl_destroy (void);
        shmemi_rccl_destroy ();
    }
    shmemi_ext_finalize (); /* peers' buffers mapped by calls (extmap.c) */
    if (shmemi.peer_heap != NULL) {
        for (int pe = 0; pe < shmemi.npes; ++pe) {
            if (pe != shmemi.mype && shmemi.peer_heap[pe] != NULL)
                (void) hipIpcCloseMemHandle (shmemi.peer_heap[pe] - heap_skew (pe));
            if (pe != shmemi.mype && shmemi.peer_sig != NULL && shmemi.peer_sig[pe] != NULL)
                (void) hipIpcCloseMemHandle (shmemi.peer_sig[pe]);
        }
        /* the peers may still read this heap until they have closed theirs */
        shmem_barrier_all ();
        free (shmemi.peer_heap);
        shmemi.peer_heap = NULL;
    }
    while (shmemi.blocks != NULL) {
        struct shmemi_block *n = shmemi.blocks->next;
        free (shmemi.blocks);
        shmemi.blocks = n;
    }
    shmemi_hheap_finalize (); /* after the barrier above: no peer reads it any more */
    free (shmemi.pair_calls);
    shmemi.pair_calls = NULL;
    if (shmemi.heap_arena != NULL)
        (void) hipFree (shmemi.heap_arena);
    shmemi.heap = shmemi.heap_arena = NULL;
    if (shmemi.sigmem != NULL)
        (void) hipFree (shmemi.sigmem);
    shmemi.sigmem = NULL;
    free (shmemi.peer_sig);
    shmemi.peer_sig = NULL;
    shmemi.stream_err = NULL;
    if (shmemi.srv.mb != NULL)
        (void) hipHostFree (shmemi.srv.mb);
    shmemi.srv.mb = NULL;
    if (shmemi.srv.st != NULL)
        (void) hipStreamDestroy (shmemi.srv.st);
    shmemi.srv.st = NULL;
    if (shmemi.sig_flag != NULL)
        (void) hipHostFree (shmemi.sig_flag);
    if (shmemi.sig_count != NULL)
        (void) hipFree (shmemi.sig_count);
    shmemi.sig_flag = NULL;
    shmemi.sig_count = NULL;
    if (shmemi.ev != NULL) {
        for (int i = 0; i < 2 * shmemi.timed_cap; ++i)
            (void) hipEventDestroy (shmemi.ev[i]);
        free (shmemi.ev);
        shmemi.ev = NULL;
        free (shmemi.timed_phase);
        shmemi.timed_phase = NULL;
        shmemi.timed_cap = 0;
    }
    if (shmemi.stream != NULL) {
        for (int i = 0; i < 2; ++i) {
            (void) hipEventDestroy (shmemi.ev_in[i]);
            (void) hipEventDestroy (shmemi.ev_out[i]);
        }
        if (shmemi.stream_in != NULL)
            (void) hipStreamDestroy (shmemi.stream_in);
        if (shmemi.stream_out != NULL)
            (void) hipStreamDestroy (shmemi.stream_out);
        shmemi.stream_in = shmemi.stream_out = NULL;
        (void) hipStreamDestroy (shmemi.stream);
    }
    shmemi.stream = NULL;
    if (shmemi.seg != NULL) {
        munmap (shmemi.seg, shmemi.seg_size);
        shmemi.seg = NULL;
    }
    free (shmemi.bar_count);
    shmemi.bar_count = NULL;
    free (shmemi.dbg_count);
    shmemi.dbg_count = NULL;
    shmemi.initialized = 0;
    shmemi_trace_fini ();
}

void pshmem_global_exit (int status)
{
    server_quit_nowait ();
    if (shmemi.seg != NULL) {
        int zero = 0;
        if (atomic_compare_exchange_strong (&shmemi.seg->abort_flag, &zero, 1)) {
            shmemi.seg->abort_pe = shmemi.mype;
            shmemi.seg->abort_status = status;
            snprintf (shmemi.seg->abort_msg, sizeof shmemi.seg->abort_msg,
                      "shmem_global_exit(%d)", status);
        }
    }
    fflush (NULL);
    _exit (status);
}

int pshmem_my_pe (void) { return shmemi.mype; }
int pshmem_n_pes (void) { return shmemi.initialized ? shmemi.npes : 1; }

void pshmem_barrier_all (void)
{
    shmemi_init_check ("shmem_barrier_all");
    shmemi_check_stream_err ("shmem_barrier_all");
    SHMEMI_TRACE (SHMEMI_LOG_BARRIER, "shmem_barrier_all");
    if (shmemi.stream != NULL)
        SHMEMI_HIP (hipStreamSynchronize (shmemi.stream));
    shmemi_barrier_set (0, 1, shmemi.npes);
}

void pshmem_barrier (int PE_start, int logPE_stride, int PE_size, long *pSync)
{
    (void) pSync; /* counters live in the bootstrap segment; pSync stays SHMEM_SYNC_VALUE */
    shmemi_init_check ("shmem_barrier");
    if (logPE_stride < 0 || logPE_stride > 30 || PE_size < 1 || PE_start < 0 ||
        PE_start + (long) (PE_size - 1) * (1L << logPE_stride) >= shmemi.npes)
        shmemi_fatal ("shmem_barrier: active set (%d, %d, %d) outside the %d PEs", PE_start,
                      logPE_stride, PE_size, shmemi.npes);
    SHMEMI_TRACE (SHMEMI_LOG_BARRIER, "shmem_barrier(PE_start %d, logPE_stride %d, PE_size %d)", PE_start,
                  logPE_stride, PE_size);
    if (shmemi.stream != NULL)
        SHMEMI_HIP (hipStreamSynchronize (shmemi.stream));
    shmemi_barrier_set (PE_start, 1 << logPE_stride, PE_size);
}

void pshmem_quiet (void)
{
    if (shmemi.initialized && shmemi.stream != NULL)
        SHMEMI_HIP (hipStreamSynchronize (shmemi.stream));
    if (shmemi.initialized)
        shmemi_check_stream_err ("shmem_quiet");
}

/* shmem_ names are weak aliases of the pshmem_ ones (PSHMEM, reference
 * src/profiling/profiling.c and src/reduce/reduce-op.c:291-380) */
#define WEAK(name) __attribute__ ((weak, alias ("p" #name)))
void start_pes (int npes) WEAK (start_pes);
void shmem_init (void) WEAK (shmem_init);
void shmem_finalize (void) WEAK (shmem_finalize);
void shmem_global_exit (int status) WEAK (shmem_global_exit);
int shmem_my_pe (void) WEAK (shmem_my_pe);
int shmem_n_pes (void) WEAK (shmem_n_pes);
int _my_pe (void) __attribute__ ((weak, alias ("pshmem_my_pe")));
int _num_pes (void) __attribute__ ((weak, alias ("pshmem_n_pes")));
void *shmem_malloc (size_t size) WEAK (shmem_malloc);
void shmem_free (void *ptr) WEAK (shmem_free);
void shmem_barrier_all (void) WEAK (shmem_barrier_all);
void shmem_barrier (int PE_start, int logPE_stride, int PE_size, long *pSync) WEAK (shmem_barrier);
void shmem_quiet (void) WEAK (shmem_quiet);

/* ---------------------------------------------------------------------- */
/* extensions                                                              */
/* ---------------------------------------------------------------------- */
int shmemx_set_reduce_algorithm (int algorithm)
{
    if (algorithm < SHMEMX_REDUCE_AUTO || algorithm > SHMEMX_REDUCE_RCCL)
        shmemi_fatal ("shmemx_set_reduce_algorithm(%d): unknown algorithm", algorithm);
    int old = shmemi.algorithm;
    if (old != algorithm && shmemi.initialized && shmemi.heap != NULL)
        shmemi_server_stop (); /* a resident server keeps the schedule it was started for */
    shmemi.algorithm = algorithm;
    return old;
}

int shmemx_get_reduce_algorithm (void) { return shmemi.algorithm; }

/* MI355X extensions (shmemx.h): the schedule thresholds at run time. Like
 * the algorithm, every PE must set the same value (SHMEM_DEBUG checks it per
 * call). A fused path a failed init self-test turned off stays off. */
size_t shmemx_set_fused_max_bytes (size_t bytes)
{
    const size_t old = shmemi.fused_max;
    if (bytes > ((size_t) 1 << 30)) /* 32-bit byte offsets in the fused folds (fused.hip ld16_sys_at) */
        bytes = (size_t) 1 << 30;
    if (shmemi.fused_off)
        bytes = 0;
    if (old != bytes && shmemi.initialized && shmemi.heap != NULL)
        shmemi_server_stop (); /* a resident server serves fused calls only */
    shmemi.fused_max = bytes;
    return old;
}

size_t shmemx_get_fused_max_bytes (void) { return shmemi.fused_max; }
size_t shmemx_get_oneshot_max_bytes (void) { return shmemi.oneshot_max; }

size_t shmemx_set_oneshot_max_bytes (size_t bytes)
{
    const size_t old = shmemi.oneshot_max;
    if (old != bytes && shmemi.initialized && shmemi.heap != NULL)
        shmemi_server_stop (); /* a resident server keeps the one-shot choice it was started with */
    shmemi.oneshot_max = bytes;
    return old;
}

int shmemx_set_reduce_order (int order)
{
    if (order != SHMEMX_ORDER_REFERENCE && order != SHMEMX_ORDER_PE_START)
        shmemi_fatal ("shmemx_set_reduce_order(%d): unknown order", order);
    int old = shmemi.order;
    if (old != order && shmemi.initialized && shmemi.heap != NULL)
        shmemi_server_stop (); /* a resident server keeps the result order it was started with */
    shmemi.order = order;
    return old;
}

void shmemx_coherence_selftest (int *ran, int *passed, int *stale_without_acquire)
{
    if (ran != NULL)
        *ran = shmemi.coh_ran;
    if (passed != NULL)
        *passed = shmemi.coh_passed;
    if (stale_without_acquire != NULL)
        *stale_without_acquire = shmemi.coh_stale;
}

void shmemx_coherence_sysload (int *sysload_fresh, int *acquires_skipped)
{
    if (sysload_fresh != NULL)
        *sysload_fresh = shmemi.coh_sysload;
    if (acquires_skipped != NULL)
        *acquires_skipped = shmemi.fused_no_acquire;
}

/* MI355X extension (shmemx.h): the init producer-path test's job-wide outcomes */
void shmemx_coherence_producer (int *ran, int *fresh)
{
    if (ran != NULL)
        *ran = shmemi.prod_ran;
    if (fresh != NULL)
        for (int i = 0; i < 6; ++i)
            fresh[i] = shmemi.prod[i];
}

int shmemx_threshold_calibration (double *us, int n)
{
    for (int k = 0; us != NULL && k < n && k < SHMEMI_CALIB_SLOTS; ++k)
        us[k] = shmemi.calib_us[k];
    return shmemi.calib_ran;
}

void shmemx_device_wait_report (int *slow, double *us)
{
    if (slow != NULL)
        *slow = shmemi.dev_wait_slow;
    if (us != NULL)
        *us = shmemi.dev_barrier_us;
}

int shmemx_get_reduce_order (void) { return shmemi.order; }

int shmemx_device_id (void) { return shmemi.initialized ? shmemi.device : -1; }

/* Link between this PE's GPU and PE pe's (bench.py's xgmi record):
 * hsa_amd_link_info_type_t (4 = xGMI, 2 = PCIe) and hop count. -1 when pe is
 * this PE, shares its GPU, or its GPU is not visible to this process. */
int shmemx_peer_link (int pe, int *link_type, int *hops)
{
    if (!shmemi.initialized || shmemi.seg == NULL || pe < 0 || pe >= shmemi.npes || pe == shmemi.mype)
        return -1;
    int peer_dev = -1;
    const char *bus = seg_info (pe)->pci_bus_id;
    if (bus[0] == '\0' || hipDeviceGetByPCIBusId (&peer_dev, bus) != hipSuccess || peer_dev == shmemi.device) {
        (void) hipGetLastError ();
        return -1;
    }
    uint32_t t = 0, h = 0;
    if (hipExtGetLinkTypeAndHopCount (shmemi.device, peer_dev, &t, &h) != hipSuccess) {
        (void) hipGetLastError ();
        return -1;
    }
    if (link_type != NULL)
        *link_type = (int) t;
    if (hops != NULL)
        *hops = (int) h;
    return 0;
}

void shmemx_device_synchronize (void)
{
    if (shmemi.initialized && shmemi.heap != NULL)
        shmemi_server_stop (); /* a resident server would hold the synchronization until it idles out */
    SHMEMI_HIP (hipDeviceSynchronize ());
}

int shmemx_set_persistent (int enable)
{
    shmemi_init_check ("shmemx_set_persistent");
    const int prev = shmemi.srv.enabled;
    shmemi.srv.enabled = enable != 0;
    if (!enable && shmemi.heap != NULL)
        shmemi_server_stop ();
    return prev;
}

void shmemx_persistent_stats (long *served, long *launched)
{
    if (served != NULL)
        *served = shmemi.srv.served;
    if (launched != NULL)
        *launched = shmemi.srv.launched;
}

void shmemx_memcpy (void *dst, const void *src, size_t nbytes)
{
    if (nbytes == 0)
        return;
    SHMEMI_HIP (hipMemcpy (dst, src, nbytes, hipMemcpyDefault));
}

void shmemx_kernel_timing (int enable)
{
    if (enable)
        SHMEMI_HIP (hipStreamSynchronize (shmemi.stream));
    shmemi.timing = enable ? 1 : 0;
    if (enable)
        shmemi.ntimed = 0;
}

/* Device-resident buffers: the caller's kernels that wrote them must be done
 * before the reduction reads them. The library stream is a BLOCKING stream,
 * so (legacy default-stream semantics) everything it runs is ordered after
 * work queued on the null stream -- hipMemcpy, kernels on the default stream
 * (PyTorch's default stream among them) -- at no host cost. Work on other
 * streams must be synchronized by the caller first, as for any GPU-aware
 * communication library, or SHMEM_ENTRY_SYNC=1 makes every call start with
 * hipDeviceSynchronize.
 * When peers will read this PE's buffers after a host barrier (PE_size > 1),
 * the host must also know that point has been reached: a one-block kernel
 * carries the completion signal (6.5 us round trip on MI355X, against 17 us
 * for hipDeviceSynchronize right after the previous call's signal). */
void shmemi_order_after_caller (int host_wait)
{
    if (shmemi.entry_sync) {
        shmemi_server_stop ();
        SHMEMI_HIP (hipDeviceSynchronize ());
        return;
    }
    if (!host_wait)
        return;
    shmemi_arm_signal ();
    int rc = mi355_signal_launch (shmemi.stream);
    if (rc != 0)
        shmemi_fatal ("signal kernel launch failed: %d", rc);
    shmemi_wait_signal ();
}

/* Before a kernel reads buffers that other PEs wrote since this GPU last read
 * them: their GPUs' memory is cached in this GPU's L2 without coherence, so
 * queue a system-scope acquire on every XCD first (mi355_acquire_system).
 * Only when some peer is on another GPU (PEs sharing one GPU read their own
 * device's memory, coherent in its L2), or SHMEM_PEER_ACQUIRE=1. */
void shmemi_peer_acquire (hipStream_t st)
{
    if (!shmemi.peer_acquire)
        return;
    const int rc = mi355_acquire_system (st);
    if (rc != 0)
        shmemi_fatal ("acquire kernel launch failed: %d", rc);
}

/* Kernel timing without marker packets: the next kernel the combine layer
 * launches carries the event pair itself (hipExtLaunchKernel stamps). Each
 * timed launch has a phase: 0 = the call's dominant kernel (the fold, or the
 * copy of a 1-PE call), 1 = the all-gather copy of the P2P schedule. */
void shmemi_timed_begin_phase (int phase)
{
    if (!shmemi.timing)
        return;
    if (shmemi.ntimed == shmemi.timed_cap) {
        int cap = shmemi.timed_cap ? 2 * shmemi.timed_cap : 256;
        hipEvent_t *ev = (hipEvent_t *) realloc (shmemi.ev, sizeof (hipEvent_t) * 2 * (size_t) cap);
        int *ph = (int *) realloc (shmemi.timed_phase, sizeof (int) * (size_t) cap);
        if (ev == NULL || ph == NULL)
            shmemi_fatal ("out of host memory");
        shmemi.ev = ev;
        shmemi.timed_phase = ph;
        for (int i = 2 * shmemi.timed_cap; i < 2 * cap; ++i)
            SHMEMI_HIP (hipEventCreate (&ev[i]));
        shmemi.timed_cap = cap;
    }
    shmemi.timed_phase[shmemi.ntimed] = phase;
    mi355_time_next_launch (shmemi.ev[2 * shmemi.ntimed], shmemi.ev[2 * shmemi.ntimed + 1]);
}

void shmemi_timed_begin (void) { shmemi_timed_begin_phase (0); }

void shmemi_timed_end (void)
{
    if (!shmemi.timing)
        return;
    mi355_time_next_launch (NULL, NULL);
    shmemi.ntimed++;
}

/* For launches the combine layer does not make (ncclAllReduce): markers. */
void shmemi_timed_marker (int end)
{
    if (!shmemi.timing)
        return;
    if (!end) {
        shmemi_timed_begin ();
        mi355_time_next_launch (NULL, NULL);
        SHMEMI_HIP (hipEventRecord (shmemi.ev[2 * shmemi.ntimed], shmemi.stream));
    } else {
        SHMEMI_HIP (hipEventRecord (shmemi.ev[2 * shmemi.ntimed + 1], shmemi.stream));
        shmemi.ntimed++;
    }
}

void shmemx_kernel_timing_phase_stats (int phase, long *launches, double *total_ms, double *avg_ms)
{
    double tot = 0.0;
    long k = 0;
    if (shmemi.ntimed > 0)
        SHMEMI_HIP (hipStreamSynchronize (shmemi.stream));
    for (int i = 0; i < shmemi.ntimed; ++i) {
        if (shmemi.timed_phase[i] != phase)
            continue;
        float ms = 0.f;
        SHMEMI_HIP (hipEventElapsedTime (&ms, shmemi.ev[2 * i], shmemi.ev[2 * i + 1]));
        tot += ms;
        ++k;
    }
    if (launches) *launches = k;
    if (total_ms) *total_ms = tot;
    if (avg_ms) *avg_ms = k ? tot / (double) k : 0.0;
}

void shmemx_kernel_timing_stats (long *launches, double *total_ms, double *avg_ms)
{
    shmemx_kernel_timing_phase_stats (0, launches, total_ms, avg_ms);
}
