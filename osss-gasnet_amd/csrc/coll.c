/*
 * coll.c -- the data-movement neighbours of the reduction path (SURVEY.md
 * section 8f rows 3-4): one-sided put/get and the broadcast / collect /
 * fcollect collectives, over the same device symmetric heap and peer
 * mappings as the reductions.
 *
 * Reference semantics followed:
 *   shmem_putmem/getmem, put/get32/64/128, shmem_<T>_put/get
 *       src/ptp/putget.c:116-256 -> shmemi_comms_put_bulk / get_bulk: blocking
 *       byte copies to/from a symmetric address on another PE
 *   shmem_broadcast32/64   src/broadcast/broadcast.c:69-110,
 *       linear form broadcast-linear.c:61-82: barrier, then every PE but the
 *       root copies the root's source into its target; the root's target is
 *       untouched (the reference's default tree form, broadcast-tree.c, also
 *       overwrites the non-root PEs' SOURCE with the data as it forwards it;
 *       that side effect is not part of the API and is not reproduced)
 *   shmem_fcollect32/64    src/fcollect/fcollect-linear.c:60-93: PE i's
 *       nelems elements land at offset i*nelems of every member's target
 *   shmem_collect32/64     src/collect/collect-linear.c:60-156: like fcollect
 *       with per-PE counts; offsets are the running sum in active-set order
 *
 * The remote side of put/get, and every collective's source, is symmetric:
 * in the device symmetric heap (shmemx_malloc_device), which peers read over
 * xGMI, or in shmem_malloc's symmetric host heap (hostheap.c), whose every
 * PE's segment is mapped in every PE, as the reference's segment exchange
 * makes them reachable (comms-inline.h:766-845). Host-heap objects move with
 * plain memory copies when the other side is host memory too (the
 * reference's transport does the same over GASNet), and with hipMemcpy when
 * it is device memory; everything else below is the device path. Local sides
 * may be any host or device memory. A put into
 * another GPU's memory goes through hipMemcpy on the peer-mapped pointer (the
 * HIP runtime's P2P copy contract makes the bytes visible to the peer's later
 * kernels; this library's kernels only ever write their own GPU's memory, so
 * no coherence question about a peer GPU's L2 arises); a put whose target is
 * on this GPU (a PE sharing it, or this PE) runs the copy kernel. A get into device
 * memory, and every collective, PULLS with the streaming copy kernel: every
 * PE reads the members' sources over xGMI into its own target, between two
 * barriers -- the same producer/consumer pattern as the reduction's
 * all-gather leg. Host-memory local sides use hipMemcpy. Broadcast and
 * fcollect queue barrier, copies and barrier on the library stream (device
 * barriers, one host wait); collect exchanges its counts through the host
 * bootstrap segment and keeps host barriers.
 */
#define _GNU_SOURCE
#include <complex.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mi355_reduce.h"
#include "pshmem.h"
#include "shmem.h"
#include "shmemx.h"
#include "shmemi.h"

/* ---------------------------------------------------------------------- */
/* helpers                                                                 */
/* ---------------------------------------------------------------------- */
static void check_pe (const char *fn, int pe)
{
    if (pe < 0 || pe >= shmemi.npes)
        shmemi_fatal ("%s: PE %d outside 0..%d", fn, pe, shmemi.npes - 1);
}

/* Address of symmetric object `sym` (nbytes long) on PE `pe`: in the peer's
 * device heap, or in its host heap segment as mapped here. */
static void *remote_addr (const char *fn, const void *sym, size_t nbytes, int pe)
{
    if (pe == shmemi.mype)
        return (void *) sym;
    if (shmemi_in_device_heap (sym, nbytes))
        return shmemi_peer_ptr (pe, shmemi_heap_offset (sym));
    if (shmemi_in_host_heap (sym, nbytes))
        return shmemi_host_peer_ptr (pe, sym);
    shmemi_fatal ("%s: remote address %p is not symmetric (allocate it with shmem_malloc or "
                  "shmemx_malloc_device)", fn, sym);
}

static int is_device_ptr (const void *p);

/* p is host memory (no GPU at all: everything is) */
static int host_side (const void *p)
{
    return shmemi.heap == NULL || !is_device_ptr (p);
}

static void need_gpu (const char *fn)
{
    if (shmemi.heap == NULL)
        shmemi_fatal ("%s: no GPU (SHMEM_BOOTSTRAP_ONLY): only host-memory copies run without one", fn);
}

static void blocking_copy (void *dst, const void *src, size_t nbytes)
{
    if (nbytes == 0 || dst == src)
        return;
    SHMEMI_HIP (hipMemcpyAsync (dst, src, nbytes, hipMemcpyDefault, shmemi.stream));
    SHMEMI_HIP (hipStreamSynchronize (shmemi.stream));
}

static void pull (void **dsts, const void **srcs, size_t *nbytes, int nseg);

static void put_bytes (const char *fn, void *dest, const void *src, size_t nbytes, int pe)
{
    shmemi_init_check (fn);
    if (nbytes > 0 && (dest == NULL || src == NULL))
        shmemi_fatal ("%s: NULL %s (%zu bytes, PE %d)", fn, dest == NULL ? "dest" : "source", nbytes, pe);
    if (shmemi.heap != NULL)
        shmemi_server_stop ();
    check_pe (fn, pe);
    if (nbytes == 0)
        return;
    void *to = remote_addr (fn, dest, nbytes, pe);
    const int to_host = shmemi_in_host_heap (dest, nbytes) || (pe == shmemi.mype && host_side (dest));
    if (to_host && host_side (src)) {
        /* host memory both sides (a peer's host heap segment is mapped
         * here): the bytes are in place when memmove returns, and the
         * barriers' release/acquire make them visible to the peer */
        memmove (to, src, nbytes);
        return;
    }
    need_gpu (fn);
    const void *from = is_device_ptr (src) ? src : shmemi_host_dev_ptr (src, nbytes);
    if (!to_host && from != NULL && from != to && shmemi_pe_same_device (pe)) {
        /* target memory on this GPU (this PE's own heap, or a PE sharing the
         * GPU) <- device or page-locked host: the streaming copy kernel; the
         * call returns once every store has drained (local completion), and
         * shmem_quiet / the barriers wait for the kernel's end. A target on
         * ANOTHER GPU keeps the runtime's P2P copy below: this library's
         * kernels never write another GPU's memory (see the file header). */
        shmemi_order_after_caller (0);
        size_t nb = nbytes;
        shmemi_arm_signal ();
        const int rc = mi355_copy_segments (&to, &from, &nb, 1, shmemi.stream);
        if (rc != 0)
            shmemi_fatal ("%s: copy kernel launch failed: %d", fn, rc);
        shmemi_wait_signal ();
        return;
    }
    blocking_copy (to, src, nbytes);
}

static void get_bytes (const char *fn, void *dest, const void *src, size_t nbytes, int pe)
{
    shmemi_init_check (fn);
    if (nbytes > 0 && (dest == NULL || src == NULL))
        shmemi_fatal ("%s: NULL %s (%zu bytes, PE %d)", fn, dest == NULL ? "dest" : "source", nbytes, pe);
    if (shmemi.heap != NULL)
        shmemi_server_stop ();
    check_pe (fn, pe);
    if (nbytes == 0)
        return;
    const void *from = remote_addr (fn, src, nbytes, pe);
    const int from_host = shmemi_in_host_heap (src, nbytes) || (pe == shmemi.mype && host_side (src));
    if (from_host && host_side (dest)) {
        memmove (dest, from, nbytes);
        return;
    }
    need_gpu (fn);
    if (!from_host && is_device_ptr (dest) && dest != from) {
        /* device <- (peer) device: the streaming copy kernel pulls over xGMI
         * (2-3x the rate of hipMemcpy's D2D path, profiles/r01/coll_bench) */
        shmemi_order_after_caller (0);
        pull (&dest, &from, &nbytes, 1);
    } else {
        blocking_copy (dest, from, nbytes);
    }
}

/* ---------------------------------------------------------------------- */
/* put / get                                                               */
/* ---------------------------------------------------------------------- */
void pshmem_putmem (void *dest, const void *src, size_t nelems, int pe)
{
    put_bytes ("shmem_putmem", dest, src, nelems, pe);
}
void pshmem_getmem (void *dest, const void *src, size_t nelems, int pe)
{
    get_bytes ("shmem_getmem", dest, src, nelems, pe);
}
void pshmem_put32 (void *dest, const void *src, size_t nelems, int pe)
{
    put_bytes ("shmem_put32", dest, src, 4 * nelems, pe);
}
void pshmem_put64 (void *dest, const void *src, size_t nelems, int pe)
{
    put_bytes ("shmem_put64", dest, src, 8 * nelems, pe);
}
void pshmem_put128 (void *dest, const void *src, size_t nelems, int pe)
{
    put_bytes ("shmem_put128", dest, src, 16 * nelems, pe);
}
void pshmem_get32 (void *dest, const void *src, size_t nelems, int pe)
{
    get_bytes ("shmem_get32", dest, src, 4 * nelems, pe);
}
void pshmem_get64 (void *dest, const void *src, size_t nelems, int pe)
{
    get_bytes ("shmem_get64", dest, src, 8 * nelems, pe);
}
void pshmem_get128 (void *dest, const void *src, size_t nelems, int pe)
{
    get_bytes ("shmem_get128", dest, src, 16 * nelems, pe);
}

#define TYPED_PUTGET(Name, Type)                                                                    \
    void pshmem_##Name##_put (Type *dest, const Type *src, size_t nelems, int pe)                   \
    {                                                                                               \
        put_bytes ("shmem_" #Name "_put", dest, src, sizeof (Type) * nelems, pe);                  \
    }                                                                                               \
    void pshmem_##Name##_get (Type *dest, const Type *src, size_t nelems, int pe)                   \
    {                                                                                               \
        get_bytes ("shmem_" #Name "_get", dest, src, sizeof (Type) * nelems, pe);                  \
    }                                                                                               \
    void shmem_##Name##_put (Type *dest, const Type *src, size_t nelems, int pe)                    \
        __attribute__ ((weak, alias ("pshmem_" #Name "_put")));                                     \
    void shmem_##Name##_get (Type *dest, const Type *src, size_t nelems, int pe)                    \
        __attribute__ ((weak, alias ("pshmem_" #Name "_get")));

TYPED_PUTGET (char, char)
TYPED_PUTGET (short, short)
TYPED_PUTGET (int, int)
TYPED_PUTGET (long, long)
TYPED_PUTGET (longlong, long long)
TYPED_PUTGET (longdouble, long double)
TYPED_PUTGET (double, double)
TYPED_PUTGET (float, float)

/* ---------------------------------------------------------------------- */
/* collectives                                                             */
/* ---------------------------------------------------------------------- */
struct cset {
    int start, stride, size, me;
};

static struct cset make_set (const char *fn, int PE_start, int logPE_stride, int PE_size)
{
    shmemi_init_check (fn);
    if (shmemi.heap != NULL)
        shmemi_server_stop ();
    if (logPE_stride < 0 || logPE_stride > 30 || PE_size < 1 || PE_start < 0 ||
        PE_start + (long) (PE_size - 1) * (1L << logPE_stride) >= shmemi.npes)
        shmemi_fatal ("%s: active set (PE_start %d, logPE_stride %d, PE_size %d) outside the %d PEs", fn,
                      PE_start, logPE_stride, PE_size, shmemi.npes);
    struct cset s = {PE_start, 1 << logPE_stride, PE_size, -1};
    for (int i = 0; i < PE_size; ++i)
        if (PE_start + i * s.stride == shmemi.mype)
            s.me = i;
    if (s.me < 0)
        shmemi_fatal ("%s: PE %d is not in the active set (PE_start %d, logPE_stride %d, PE_size %d)", fn,
                      shmemi.mype, PE_start, logPE_stride, PE_size);
    return s;
}

static int is_device_ptr (const void *p)
{
    if (shmemi.heap == NULL)
        return 0;
    if (shmemi_in_device_heap (p, 0))
        return 1;
    hipPointerAttribute_t a;
    memset (&a, 0, sizeof a);
    hipError_t e = hipPointerGetAttributes (&a, p);
    (void) hipGetLastError ();
    return e == hipSuccess && (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged);
}

/* Pull nseg byte ranges of peers' symmetric HOST heap segments (mapped here)
 * into local memory: plain copies into host memory, hipMemcpy into device
 * memory (the GPU does not read the peers' segments: they are not
 * registered with this process's HIP). */
static void pull_host (const char *fn, void **dsts, const void **srcs, size_t *nbytes, int nseg)
{
    for (int i = 0; i < nseg; ++i) {
        if (nbytes[i] == 0)
            continue;
        if (host_side (dsts[i])) {
            memmove (dsts[i], srcs[i], nbytes[i]);
        } else {
            need_gpu (fn);
            SHMEMI_HIP (hipMemcpyAsync (dsts[i], srcs[i], nbytes[i], hipMemcpyDefault, shmemi.stream));
            SHMEMI_HIP (hipStreamSynchronize (shmemi.stream));
        }
    }
}

/* Pull nseg byte ranges from peers into local memory: one copy kernel when
 * the destination is device memory, DMA copies otherwise. wait: block until
 * done (the copy kernel's completion signal, or a stream synchronize);
 * otherwise only queue them on the library stream. */
static void pull_impl (void **dsts, const void **srcs, size_t *nbytes, int nseg, int wait)
{
    int dev = 1;
    for (int i = 0; i < nseg; ++i)
        dev &= is_device_ptr (dsts[i]);
    if (dev) {
        shmemi_peer_acquire (shmemi.stream); /* the sources are other PEs' memory */
        for (int base = 0; base < nseg; base += 64) {
            const int k = nseg - base < 64 ? nseg - base : 64;
            const int last = base + k == nseg;
            if (last && wait)
                shmemi_arm_signal ();
            int rc = mi355_copy_segments (dsts + base, srcs + base, nbytes + base, k, shmemi.stream);
            if (rc != 0)
                shmemi_fatal ("copy kernel launch failed: %d", rc);
        }
        if (wait)
            shmemi_wait_signal ();
    } else {
        for (int i = 0; i < nseg; ++i)
            if (nbytes[i] != 0)
                SHMEMI_HIP (hipMemcpyAsync (dsts[i], srcs[i], nbytes[i], hipMemcpyDefault, shmemi.stream));
        if (wait)
            SHMEMI_HIP (hipStreamSynchronize (shmemi.stream));
    }
}

static void pull (void **dsts, const void **srcs, size_t *nbytes, int nseg)
{
    pull_impl (dsts, srcs, nbytes, nseg, 1);
}

/* Opening barrier: every source is ready. With device barriers the rest of
 * the collective is queued behind it (dev = 1); else a host barrier after the
 * host has seen the caller's work done. */
/* 1: source in the symmetric host heap; 0: in the device heap (or nothing to
 * read); fatal otherwise */
static int source_kind (const char *fn, const void *source, size_t nbytes)
{
    if (nbytes == 0 || shmemi_in_device_heap (source, nbytes))
        return 0;
    if (shmemi_in_host_heap (source, nbytes))
        return 1;
    shmemi_fatal ("%s: source %p is not symmetric (allocate it with shmem_malloc or shmemx_malloc_device)", fn,
                  source);
}

/* PE pe's copy of a symmetric source (device or host heap) */
static const void *source_on (int pe, const void *source, int host)
{
    return host ? shmemi_host_peer_ptr (pe, source) : shmemi_peer_ptr (pe, shmemi_heap_offset (source));
}

static int collective_entry (const char *fn, const void *source, size_t nbytes, const struct cset *s,
                             int allow_dev)
{
    if (source_kind (fn, source, nbytes) != 0 || shmemi.heap == NULL)
        allow_dev = 0; /* the host heap: host barriers, the copies below run on the host */
    if (shmemi.heap == NULL) {
        shmemi_barrier_set (s->start, s->stride, s->size);
        return 0;
    }
    if (allow_dev && shmemi_dev_barrier_ok (s->start, s->stride, s->size)) {
        shmemi_order_after_caller (0); /* SHMEM_ENTRY_SYNC */
        shmemi_dev_barrier (s->start, s->stride, s->size, s->me, 0);
        return 1;
    }
    shmemi_order_after_caller (1);
    shmemi_barrier_set (s->start, s->stride, s->size);
    return 0;
}

/* Closing barrier: nobody reads this PE's source any more. */
static void collective_exit (const struct cset *s, int dev)
{
    if (dev)
        shmemi_dev_barrier (s->start, s->stride, s->size, s->me, 1);
    else
        shmemi_barrier_set (s->start, s->stride, s->size);
}

/* Small broadcast / fcollect in ONE launch (mi355_fused_pull): arrive, pull
 * this PE's segments, "done reading" -- instead of device barrier, copy
 * kernel and device barrier. The choice depends on the call's arguments only
 * (every member must make it alike); a member whose target the kernel cannot
 * write (pageable host memory) pulls into its scratch C and copies out. */
static int fused_pull_ok (const struct cset *s, size_t total)
{
    return shmemi.heap != NULL && s->size >= 2 && shmemi.fused_max != 0 && total <= shmemi.fused_max &&
           total <= shmemi.scratch_chunk && shmemi_dev_barrier_ok (s->start, s->stride, s->size);
}

/* segments: byte offsets into this PE's target of `total` bytes */
static void fused_pull (const char *fn, const struct cset *s, void *target, size_t total, const size_t *toff,
                        const void *const *srcs, const size_t *nb, int k)
{
    char *t = NULL;
    int copy_out = 0;
    if (total != 0) {
        t = is_device_ptr (target) ? (char *) target : (char *) shmemi_host_dev_ptr (target, total);
        if (t == NULL) {
            t = shmemi.heap + shmemi.scratch_off + 2 * shmemi.scratch_chunk; /* scratch C */
            copy_out = 1;
        }
    }
    MI355PullArgs p;
    memset (&p, 0, sizeof p);
    shmemi_member_args (&p.m, s->start, s->stride, s->size, s->me);
    p.nseg = k;
    for (int i = 0; i < k; ++i) {
        p.dst[i] = t + toff[i];
        p.src[i] = srcs[i];
        p.nbytes[i] = nb[i];
    }
    p.m.host_flag = shmemi.sig_flag;
    p.m.epoch = shmemi_next_epoch ();
    shmemi_order_after_caller (0); /* SHMEM_ENTRY_SYNC */
    const int rc = mi355_fused_pull (&p, shmemi.stream);
    if (rc != 0)
        shmemi_fatal ("%s: fused pull launch failed: %d", fn, rc);
    if (shmemi_wait_flag (p.m.epoch) != p.m.epoch)
        shmemi_fatal ("%s: timed out waiting for the other PEs of the active set", fn);
    if (copy_out)
        for (int i = 0; i < k; ++i)
            blocking_copy ((char *) target + toff[i], t + toff[i], nb[i]);
}

static void broadcast_bytes (const char *fn, void *target, const void *source, size_t nbytes, int PE_root,
                             int PE_start, int logPE_stride, int PE_size)
{
    struct cset s = make_set (fn, PE_start, logPE_stride, PE_size);
    if (PE_root < 0 || PE_root >= PE_size)
        shmemi_fatal ("%s: PE_root %d outside the active set of %d PEs", fn, PE_root, PE_size);
    const int root = PE_start + PE_root * s.stride;
    const int host = source_kind (fn, source, nbytes);
    if (s.size == 1)
        return; /* the root does not write its own target, and there is nobody to wait for */
    if (!host && fused_pull_ok (&s, nbytes)) {
        SHMEMI_TRACE (SHMEMI_LOG_BROADCAST, "%s: %zu bytes from PE %d, one fused launch", fn, nbytes, root);
        const void *src = nbytes != 0 ? shmemi_peer_ptr (root, shmemi_heap_offset (source)) : NULL;
        const size_t toff = 0;
        fused_pull (fn, &s, target, nbytes, &toff, &src, &nbytes, shmemi.mype != root && nbytes != 0 ? 1 : 0);
        return;
    }
    const int dev = collective_entry (fn, source, nbytes, &s, 1);
    if (shmemi.mype != root && nbytes != 0) {
        void *d = target;
        const void *src = source_on (root, source, host);
        if (host)
            pull_host (fn, &d, &src, &nbytes, 1);
        else
            pull_impl (&d, &src, &nbytes, 1, !dev);
    }
    collective_exit (&s, dev); /* nobody reads the root's source any more */
}

void pshmem_broadcast32 (void *target, const void *source, size_t nelems, int PE_root, int PE_start,
                         int logPE_stride, int PE_size, long *pSync)
{
    (void) pSync;
    broadcast_bytes ("shmem_broadcast32", target, source, 4 * nelems, PE_root, PE_start, logPE_stride, PE_size);
}

void pshmem_broadcast64 (void *target, const void *source, size_t nelems, int PE_root, int PE_start,
                         int logPE_stride, int PE_size, long *pSync)
{
    (void) pSync;
    broadcast_bytes ("shmem_broadcast64", target, source, 8 * nelems, PE_root, PE_start, logPE_stride, PE_size);
}

/* counts[i] bytes from member i land at the running offset in target */
static void gather_bytes (const char *fn, void *target, const void *source, const size_t *counts,
                          const struct cset *s, int wait, int host)
{
    void **dsts = (void **) malloc (sizeof (void *) * (size_t) s->size);
    const void **srcs = (const void **) malloc (sizeof (void *) * (size_t) s->size);
    size_t *nb = (size_t *) malloc (sizeof (size_t) * (size_t) s->size);
    if (dsts == NULL || srcs == NULL || nb == NULL)
        shmemi_fatal ("out of host memory");
    size_t off = 0;
    int k = 0;
    for (int i = 0; i < s->size; ++i) {
        const int pe = s->start + i * s->stride;
        if (counts[i] != 0) {
            dsts[k] = (char *) target + off;
            srcs[k] = source_on (pe, source, host);
            nb[k] = counts[i];
            ++k;
        }
        off += counts[i];
    }
    if (k > 0 && host)
        pull_host (fn, dsts, srcs, nb, k);
    else if (k > 0)
        pull_impl (dsts, srcs, nb, k, wait);
    free (nb);
    free (srcs);
    free (dsts);
}

static void fcollect_bytes (const char *fn, void *target, const void *source, size_t nbytes, int PE_start,
                            int logPE_stride, int PE_size)
{
    struct cset s = make_set (fn, PE_start, logPE_stride, PE_size);
    const int host = source_kind (fn, source, nbytes);
    if (s.size == 1) { /* one member: target = source, nobody to wait for */
        if (nbytes != 0 && target != source) {
            void *d = target;
            const void *src = source;
            if (host) {
                pull_host (fn, &d, &src, &nbytes, 1);
            } else {
                shmemi_order_after_caller (0);
                pull (&d, &src, &nbytes, 1);
            }
        }
        return;
    }
    if (!host && s.size <= MI355_PULL_MAX_SEGS && nbytes != 0 && fused_pull_ok (&s, nbytes * (size_t) s.size)) {
        size_t toff[MI355_PULL_MAX_SEGS], nb[MI355_PULL_MAX_SEGS];
        const void *srcs[MI355_PULL_MAX_SEGS];
        for (int i = 0; i < s.size; ++i) {
            toff[i] = (size_t) i * nbytes;
            srcs[i] = shmemi_peer_ptr (s.start + i * s.stride, shmemi_heap_offset (source));
            nb[i] = nbytes;
        }
        SHMEMI_TRACE (SHMEMI_LOG_COLLECT, "%s: %d x %zu bytes, one fused launch", fn, s.size, nbytes);
        fused_pull (fn, &s, target, nbytes * (size_t) s.size, toff, srcs, nb, s.size);
        return;
    }
    const int dev = collective_entry (fn, source, nbytes, &s, 1);
    size_t *counts = (size_t *) malloc (sizeof (size_t) * (size_t) s.size);
    if (counts == NULL)
        shmemi_fatal ("out of host memory");
    for (int i = 0; i < s.size; ++i)
        counts[i] = nbytes;
    gather_bytes (fn, target, source, counts, &s, !dev, host);
    free (counts);
    collective_exit (&s, dev); /* nobody reads our source any more */
}

void pshmem_fcollect32 (void *target, const void *source, size_t nelems, int PE_start, int logPE_stride,
                        int PE_size, long *pSync)
{
    (void) pSync;
    fcollect_bytes ("shmem_fcollect32", target, source, 4 * nelems, PE_start, logPE_stride, PE_size);
}

void pshmem_fcollect64 (void *target, const void *source, size_t nelems, int PE_start, int logPE_stride,
                        int PE_size, long *pSync)
{
    (void) pSync;
    fcollect_bytes ("shmem_fcollect64", target, source, 8 * nelems, PE_start, logPE_stride, PE_size);
}

/* collect: the per-PE byte counts travel through the bootstrap segment; the
 * closing barrier keeps a count alive until every member has read it */
static void collect_bytes (const char *fn, void *target, const void *source, size_t nbytes, int PE_start,
                           int logPE_stride, int PE_size)
{
    struct cset s = make_set (fn, PE_start, logPE_stride, PE_size);
    const int host = source_kind (fn, source, nbytes);
    shmemi_publish_count (nbytes);
    (void) collective_entry (fn, source, nbytes, &s, 0);
    size_t *counts = (size_t *) malloc (sizeof (size_t) * (size_t) s.size);
    if (counts == NULL)
        shmemi_fatal ("out of host memory");
    for (int i = 0; i < s.size; ++i)
        counts[i] = shmemi_peer_count (s.start + i * s.stride);
    gather_bytes (fn, target, source, counts, &s, 1, host);
    free (counts);
    shmemi_barrier_set (s.start, s.stride, s.size);
}

void pshmem_collect32 (void *target, const void *source, size_t nelems, int PE_start, int logPE_stride,
                       int PE_size, long *pSync)
{
    (void) pSync;
    collect_bytes ("shmem_collect32", target, source, 4 * nelems, PE_start, logPE_stride, PE_size);
}

void pshmem_collect64 (void *target, const void *source, size_t nelems, int PE_start, int logPE_stride,
                       int PE_size, long *pSync)
{
    (void) pSync;
    collect_bytes ("shmem_collect64", target, source, 8 * nelems, PE_start, logPE_stride, PE_size);
}

#define WEAK(name) __attribute__ ((weak, alias ("p" #name)))
void shmem_putmem (void *dest, const void *src, size_t nelems, int pe) WEAK (shmem_putmem);
void shmem_getmem (void *dest, const void *src, size_t nelems, int pe) WEAK (shmem_getmem);
void shmem_put32 (void *dest, const void *src, size_t nelems, int pe) WEAK (shmem_put32);
void shmem_put64 (void *dest, const void *src, size_t nelems, int pe) WEAK (shmem_put64);
void shmem_put128 (void *dest, const void *src, size_t nelems, int pe) WEAK (shmem_put128);
void shmem_get32 (void *dest, const void *src, size_t nelems, int pe) WEAK (shmem_get32);
void shmem_get64 (void *dest, const void *src, size_t nelems, int pe) WEAK (shmem_get64);
void shmem_get128 (void *dest, const void *src, size_t nelems, int pe) WEAK (shmem_get128);
void shmem_broadcast32 (void *target, const void *source, size_t nelems, int PE_root, int PE_start,
                        int logPE_stride, int PE_size, long *pSync) WEAK (shmem_broadcast32);
void shmem_broadcast64 (void *target, const void *source, size_t nelems, int PE_root, int PE_start,
                        int logPE_stride, int PE_size, long *pSync) WEAK (shmem_broadcast64);
void shmem_fcollect32 (void *target, const void *source, size_t nelems, int PE_start, int logPE_stride,
                       int PE_size, long *pSync) WEAK (shmem_fcollect32);
void shmem_fcollect64 (void *target, const void *source, size_t nelems, int PE_start, int logPE_stride,
                       int PE_size, long *pSync) WEAK (shmem_fcollect64);
void shmem_collect32 (void *target, const void *source, size_t nelems, int PE_start, int logPE_stride,
                      int PE_size, long *pSync) WEAK (shmem_collect32);
void shmem_collect64 (void *target, const void *source, size_t nelems, int PE_start, int logPE_stride,
                      int PE_size, long *pSync) WEAK (shmem_collect64);
