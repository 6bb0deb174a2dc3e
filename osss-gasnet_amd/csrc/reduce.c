/*
 * reduce.c -- the 44 shmem_<TYPE>_<OP>_to_all collectives on MI355X.
 *
 * Reference: src/reduce/reduce-op.c. There, every PE copies its source into
 * the target (:226-229), barriers (:230), then pulls every other PE's source
 * in 64-element chunks with shmem_getmem and folds them in with one indirect
 * call per element (:232-264), barriers again (:266) and copies back from a
 * temporary if target and source overlapped (:267-275).
 *
 * Here the combine runs on the PE's GPU (combine.hip, C ABI mi355_reduce.h)
 * and the cross-PE movement is xGMI peer access to the device symmetric heap:
 *
 *   P2P (default)  split the nreduce elements into PE_size contiguous shards
 *                  (256-byte aligned); PE i folds shard i of every member's
 *                  source into its own target shard; barrier; PE i gathers
 *                  the other shards from the members' targets. Result order
 *                  (shmemx.h): where the reference's members disagree
 *                  (floating point; see ordered_pair), PE i folds shard i in
 *                  EVERY member's reference order at once -- own source first,
 *                  then the others ascending (:226-264) -- keeps its own
 *                  version and leaves member q's in slot q of its version
 *                  area, from which q gathers it: every PE ends with the
 *                  reference's result for itself. Elsewhere (and with
 *                  SHMEM_REDUCE_ORDER=pe_start) every PE gets PE_start's
 *                  result, the fold in ascending active-set order.
 *   EXACT          every PE folds the full arrays in ITS reference order
 *                  (own source first, then the others ascending): bit-identical
 *                  to the reference on every PE, at PE_size x the xGMI reads.
 *   RCCL           ncclAllReduce for the op/type pairs RCCL has, when the
 *                  active set is the whole job; P2P otherwise.
 *
 * Buffers outside the device symmetric heap (host memory from shmem_malloc,
 * static arrays, other device memory) are staged through the heap's scratch
 * area in chunks: copy in, reduce device-resident, copy out.
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mi355_reduce.h"
#include "pshmem.h"
#include "shmem.h"
#include "shmemx.h"
#include "shmemi.h"

enum { SHMEMI_CHAN_HOST = 0, SHMEMI_CHAN_STREAM = 1 }; /* signal-region channels */

struct aset {
    int start, stride, size, me; /* me = index of this PE in the set */
};

static int aset_pe (const struct aset *s, int i) { return s->start + i * s->stride; }

/* What the call ran (shmemx_last_call_info): called right after the
 * dominant kernel's launch, so the combine layer's last kernel is it.
 * sources/outputs buffers of `bytes` each; extra_alg / extra_peer: bytes
 * beyond those (the fused two-shot's gather). Rounds add launches. */
static const char *cur_schedule = "none";

static void note_call (int ordered, int sources, int outputs, int peer_sources, unsigned long long bytes,
                       unsigned long long extra_alg, unsigned long long extra_peer, const void *kernel)
{
    shmemi.last.valid = 1;
    shmemi.last.schedule = cur_schedule;
    shmemi.last.kernel = kernel;
    shmemi.last.ordered = ordered;
    shmemi.last.sources = sources;
    shmemi.last.outputs = outputs;
    shmemi.last.peer_sources = peer_sources;
    shmemi.last.bytes_per_buffer = bytes;
    shmemi.last.alg_bytes = (unsigned long long) (sources + outputs) * bytes + extra_alg;
    shmemi.last.peer_bytes = (unsigned long long) peer_sources * bytes + extra_peer;
    shmemi.last.launches++;
}

static void begin_call (const char *schedule)
{
    cur_schedule = schedule;
    shmemi.last.valid = 1;
    shmemi.last.schedule = schedule;
    shmemi.last.kernel = NULL;
    shmemi.last.launches = 0;
    shmemi.last.ordered = shmemi.last.sources = shmemi.last.outputs = shmemi.last.peer_sources = 0;
    shmemi.last.bytes_per_buffer = shmemi.last.alg_bytes = shmemi.last.peer_bytes = 0;
}

int shmemx_last_call_info (shmemx_call_info *info)
{
    if (info == NULL || !shmemi.last.valid)
        return -1;
    memset (info, 0, sizeof *info);
    snprintf (info->schedule, sizeof info->schedule, "%s", shmemi.last.schedule);
    if (shmemi.last.kernel != NULL && mi355_kernel_name (shmemi.last.kernel, info->kernel, sizeof info->kernel) != 0)
        info->kernel[0] = '\0';
    info->ordered = shmemi.last.ordered;
    info->sources = shmemi.last.sources;
    info->outputs = shmemi.last.outputs;
    info->peer_sources = shmemi.last.peer_sources;
    info->launches = shmemi.last.launches;
    info->bytes_per_buffer = shmemi.last.bytes_per_buffer;
    info->alg_bytes = shmemi.last.alg_bytes;
    info->peer_bytes = shmemi.last.peer_bytes;
    return 0;
}

/* Launch the fold and wait for its completion signal (the kernel's last
 * block writes a host-coherent word; ~4 us sooner than a stream sync). */
static void combine_wait (int op, int dtype, void *dst, const void *const *srcs, int nsrc, size_t n, int timed)
{
    if (timed)
        shmemi_timed_begin ();
    shmemi_arm_signal ();
    int rc = mi355_combine (op, dtype, dst, srcs, nsrc, n, shmemi.stream);
    if (timed)
        shmemi_timed_end ();
    if (rc != 0)
        shmemi_fatal ("combine kernel launch failed (op %d, dtype %d, %d sources, %zu elements): %d",
                      op, dtype, nsrc, n, rc);
    shmemi_wait_signal ();
}

/* Byte copies, 64 segments per launch; the last launch carries the signal
 * (and, when kernel timing is on, the event pair of timing phase `phase`;
 * phase < 0: not timed). */
static void copy_wait (void *const *dsts, const void *const *srcs, const size_t *nbytes, int nseg, int phase)
{
    const int timed = phase >= 0;
    if (nseg <= 0)
        return;
    for (int base = 0; base < nseg; base += 64) {
        const int k = nseg - base < 64 ? nseg - base : 64;
        const int last = base + k == nseg;
        if (last) {
            if (timed)
                shmemi_timed_begin_phase (phase);
            shmemi_arm_signal ();
        }
        int rc = mi355_copy_segments (dsts + base, srcs + base, nbytes + base, k, shmemi.stream);
        if (last && timed)
            shmemi_timed_end ();
        if (rc != 0)
            shmemi_fatal ("copy kernel launch failed: %d", rc);
    }
    shmemi_wait_signal ();
}

static int ranges_overlap (size_t a, size_t b, size_t nbytes)
{
    return a < b + nbytes && b < a + nbytes;
}

/* Elements per shard: ceil(n / size) rounded up so every shard starts on a
 * 256-byte boundary. */
static size_t shard_chunk (size_t n, size_t es, int size)
{
    size_t align = es >= 256 ? 1 : 256 / es;
    size_t chunk = (n + (size_t) size - 1) / (size_t) size;
    return (chunk + align - 1) / align * align;
}

/* Shard bounds of member i for n elements of es bytes over `size` members. */
void mi355_shard_bounds (size_t n, size_t es, int size, int i, size_t *lo, size_t *hi)
{
    const size_t chunk = shard_chunk (n, es, size);
    size_t l = (size_t) i * chunk;
    *lo = l < n ? l : n;
    *hi = l + chunk < n ? l + chunk : n;
}

/* ---------------------------------------------------------------------- */
/* result order (shmemx.h, SHMEMX_ORDER_REFERENCE)                          */
/* ---------------------------------------------------------------------- */
/* The reference's members disagree on this reduction: floating point (the
 * integer and bitwise operators wrap, select identical bits or are exact, so
 * any order gives the same bits), and either 3+ members (the rounding follows
 * the order), min/max (`a < b ? a : b` picks by position when a NaN or a +-0
 * pair is involved, reduce-op.c:138-150, from 2 members on), or a two-member
 * float, double or complex sum/prod: a + b and b + a have the same value, but
 * where both operands are NaNs SSE returns the FIRST one (ops.h x86_result),
 * so the two members' results differ in payload. x87 long double returns the
 * NaN with the larger significand whatever the order (x80.h), so its
 * two-member sum/prod agree. */
static int order_sensitive (int op, int dtype, int size)
{
    if (shmemi.order != SHMEMX_ORDER_REFERENCE || size < 2)
        return 0;
    if (dtype != MI355_FLOAT && dtype != MI355_DOUBLE && dtype != MI355_LONGDOUBLE && dtype != MI355_COMPLEXF &&
        dtype != MI355_COMPLEXD)
        return 0;
    return size > 2 || op == MI355_OP_MIN || op == MI355_OP_MAX || dtype != MI355_LONGDOUBLE;
}

/* The shard schedules deliver every member's order up to
 * MI355_ORDERS_MAX_SOURCES members (mi355_combine_orders); larger
 * order-sensitive active sets run the EXACT schedule instead. */
static int ordered_pair (int op, int dtype, int size)
{
    return order_sensitive (op, dtype, size) && size <= MI355_ORDERS_MAX_SOURCES;
}

/* Two members, float or double sum/prod, each member's own order: the
 * members' results differ only where both operands are NaNs (SSE keeps the
 * first). The multi-launch schedules then skip the version areas: each owner
 * folds its shard in ITS order (own source first) and the other member
 * gathers it NaN-patched from its own source (mi355_nan_patch_copy): one
 * output per shard, one more local read in the gather. (Complex types keep
 * the version areas: the imaginary part of gcc's float complex add takes the
 * incoming operand first, and Annex G's product is not a plain pair.) */
static int nan_pair (int op, int dtype, const struct aset *s)
{
    return shmemi.order == SHMEMX_ORDER_REFERENCE && s->size == 2 && (dtype == MI355_FLOAT || dtype == MI355_DOUBLE) &&
           (op == MI355_OP_SUM || op == MI355_OP_PROD);
}

/* Version areas: on every PE, one per signal-region channel, (size - 1)
 * slots of one shard each; slot s of owner i holds member q's version of
 * shard i, s = q < i ? q : q - 1. Each slot starts at the target's offset
 * within 256 bytes, so the gather copies run as aligned vectors.
 * Consecutive slots are VER_STAGGER bytes further apart than a shard needs:
 * the every-member fold writes all its outputs at the same element offset,
 * and outputs a power-of-two shard size apart land in the same HBM channels
 * (tools/probes/cold_probe orders_skew2, 8 x 32 MiB double sum: 0.62 of peak from
 * HBM with 256-byte gaps, 0.68-0.70 with 4 KiB-granular ones). */
#define VER_STAGGER 4096
static size_t ver_slot_bytes (size_t n, size_t es, int size)
{
    const size_t b = shard_chunk (n, es, size) * es;
    return (b + 255) / 256 * 256 + 256 + VER_STAGGER;
}

static size_t ver_off (int chan, int owner, int q, size_t slot_bytes, size_t dst_off)
{
    return shmemi.order_off + (size_t) chan * shmemi.order_chunk + (size_t) (q < owner ? q : q - 1) * slot_bytes +
           (dst_off & 255);
}

/* Elements per round of an ordered P2P reduction: the largest message whose
 * versions fit one channel's version area (longer messages run in rounds). */
static size_t ordered_round_elems (size_t es, int size)
{
    const size_t align = es >= 256 ? 1 : 256 / es;
    const size_t per_slot = shmemi.order_chunk / (size_t) (size - 1);
    if (per_slot < 512 + VER_STAGGER + align * es)
        shmemi_fatal ("SHMEM_DEVICE_ORDER_SIZE (%zu bytes per channel) is too small for %d PEs", shmemi.order_chunk,
                      size);
    return (per_slot - 512 - VER_STAGGER) / es / align * align * (size_t) size;
}

/* ---------------------------------------------------------------------- */
/* device-resident schedules on symmetric heap offsets                     */
/* ---------------------------------------------------------------------- */

/* Member list of the active set for the device-flag kernels (fused.hip), on
 * one signal-region channel. */
static void member_args (MI355FusedArgs *a, const struct aset *s, int chan)
{
    memset (a, 0, sizeof *a);
    a->nmembers = s->size;
    a->me = s->me;
    for (int i = 0; i < s->size; ++i) {
        a->pe[i] = aset_pe (s, i);
        a->sig[i] = shmemi.peer_sig[a->pe[i]] + (size_t) chan * MI355_SIG_CHANNEL_WORDS;
    }
    a->err_flag = shmemi.stream_err;
    a->timeout_ticks = (unsigned long long) (shmemi.barrier_timeout * 1e8);
    a->share = shmemi.local_pes;
    a->no_acquire = shmemi.fused_no_acquire;
}

/* The device-flag kernels can carry this active set's synchronization. */
static int device_flags_ok (const struct aset *s)
{
    return s->size <= MI355_FUSED_MAX_MEMBERS && shmemi.npes <= MI355_SIG_RSDONE && shmemi.sigmem != NULL &&
           !shmemi.sig_broken && !shmemi.dev_wait_slow;
}

static void device_barrier (const MI355FusedArgs *a, hipStream_t st)
{
    shmemi_server_stop (); /* two spin-waiting grids need not fit beside each other */
    const int rc = mi355_device_barrier (a, st);
    if (rc != 0)
        shmemi_fatal ("device barrier launch failed: %d", rc);
}

/* For coll.c: the member list of an active set on the host channel. */
void shmemi_member_args (MI355FusedArgs *a, int PE_start, int stride, int PE_size, int me)
{
    struct aset s = {PE_start, stride, PE_size, me};
    member_args (a, &s, SHMEMI_CHAN_HOST);
}

/* For coll.c: a device barrier over an active set on the library stream
 * (host channel); `last` makes it carry the completion flag and waits. */
int shmemi_dev_barrier_ok (int PE_start, int stride, int PE_size)
{
    struct aset s = {PE_start, stride, PE_size, 0};
    return device_flags_ok (&s);
}

void shmemi_dev_barrier (int PE_start, int stride, int PE_size, int me, int last)
{
    struct aset s = {PE_start, stride, PE_size, me};
    MI355FusedArgs a;
    member_args (&a, &s, SHMEMI_CHAN_HOST);
    if (last) {
        a.host_flag = shmemi.sig_flag;
        a.epoch = shmemi_next_epoch ();
    }
    device_barrier (&a, shmemi.stream);
    if (last && shmemi_wait_flag (a.epoch) != a.epoch)
        shmemi_fatal ("device barrier timed out waiting for the other PEs of the active set");
}

/* nan_pair's NaN word can carry the owner's "no NaN" to the other member:
 * the owner's signal region is mapped there and peers' stores into signal
 * regions were seen at init (without that, sig_broken: host barriers, and the
 * gather patches unconditionally). */
static int nan_word_ok (const struct aset *s)
{
    const int other_pe = aset_pe (s, 1 - s->me);
    return !shmemi.sig_broken && shmemi.sigmem != NULL && shmemi.peer_sig[other_pe] != NULL;
}

/* nan_pair: this call's number among the two-member calls with the other
 * member on channel chan -- the same on both members (every member makes the
 * same collective calls) -- whose parity picks the NaN word the owner's fold
 * sets (MI355_SIG_NANFLAG_AT; it clears the other parity's, which the previous
 * call's gather has finished reading) and the other member's gather reads. */
static long long pair_next (int chan, const struct aset *s)
{
    if (shmemi.pair_calls == NULL) {
        shmemi.pair_calls = (uint64_t *) calloc ((size_t) MI355_SIG_CHANNELS * (size_t) shmemi.npes, sizeof (uint64_t));
        if (shmemi.pair_calls == NULL)
            shmemi_fatal ("out of host memory");
    }
    return (long long) ++shmemi.pair_calls[(size_t) chan * (size_t) shmemi.npes + (size_t) aset_pe (s, 1 - s->me)];
}

/* The reduce-scatter leg: fold this PE's shard of every member's source
 * into its target shard -- in member order, or (ordered) in every member's
 * reference order with the other members' versions going to this PE's
 * version area on channel `chan`. Returns the launch's status (0: queued, or
 * nothing to do: empty shard). */
static int fold_shard (int op, int dtype, size_t es, size_t dst_off, size_t src_off, size_t n, const struct aset *s,
                       int ordered, long long pair_k, int chan, hipStream_t st)
{
    const int pair = pair_k >= 0;
    const void *sp[MI355_FUSED_MAX_MEMBERS > MI355_ORDERS_MAX_SOURCES ? MI355_FUSED_MAX_MEMBERS
                                                                       : MI355_ORDERS_MAX_SOURCES];
    size_t lo, hi;
    mi355_shard_bounds (n, es, s->size, s->me, &lo, &hi);
    if (hi <= lo) {
        /* no fold: clear the word the next call's fold would have (this
         * call's stays as the previous call of its parity left it, but the
         * other member's gather of an empty shard reads nothing) */
        if (pair && nan_word_ok (s)) {
            const int other = aset_pe (s, 1 - s->me);
            const hipError_t e = hipMemsetAsync (shmemi.sigmem + MI355_SIG_NANFLAG_AT (chan, (pair_k + 1) & 1, other),
                                                 0, sizeof (unsigned long long), st);
            if (e != hipSuccess)
                return (int) e;
        }
        return 0;
    }
    const void **spp = sp;
    if (s->size > (int) (sizeof sp / sizeof sp[0])) {
        spp = (const void **) malloc (sizeof (void *) * (size_t) s->size);
        if (spp == NULL)
            shmemi_fatal ("out of host memory");
    }
    for (int i = 0; i < s->size; ++i)
        spp[i] = shmemi_peer_ptr (aset_pe (s, i), src_off + lo * es);
    if (pair && s->me == 1) { /* nan_pair: this owner's order, its own source first */
        const void *t = spp[0];
        spp[0] = spp[1];
        spp[1] = t;
    }
    void *dst = shmemi_peer_ptr (shmemi.mype, dst_off + lo * es);
    int rc;
    if (pair && nan_word_ok (s)) {
        const int other = aset_pe (s, 1 - s->me);
        mi355_nan_flag_next_launch (shmemi.sigmem + MI355_SIG_NANFLAG_AT (chan, pair_k & 1, other),
                                    shmemi.sigmem + MI355_SIG_NANFLAG_AT (chan, (pair_k + 1) & 1, other));
    }
    if (!ordered) {
        rc = mi355_combine (op, dtype, dst, spp, s->size, hi - lo, st);
    } else {
        void *dsts[MI355_ORDERS_MAX_SOURCES];
        const size_t slot = ver_slot_bytes (n, es, s->size);
        for (int q = 0; q < s->size; ++q)
            dsts[q] = q == s->me ? dst : shmemi_peer_ptr (shmemi.mype, ver_off (chan, s->me, q, slot, dst_off));
        rc = mi355_combine_orders (op, dtype, dsts, spp, s->size, hi - lo, st);
    }
    if (rc == 0)
        note_call (ordered, s->size, ordered ? s->size : 1, s->size - 1, (unsigned long long) ((hi - lo) * es), 0, 0,
                   mi355_last_kernel ());
    if (spp != sp)
        free (spp);
    return rc;
}

/* The all-gather leg's segments: the other members' shards, from their
 * targets, or (ordered) this PE's version of them from their version areas.
 * Returns the number of segments (arrays of s->size entries). */
static int gather_segments (size_t es, size_t dst_off, size_t n, const struct aset *s, int ordered, int chan,
                            void **dsts, const void **sp, size_t *nb)
{
    const size_t slot = ver_slot_bytes (n, es, s->size);
    int k = 0;
    for (int i = 0; i < s->size; ++i) {
        size_t l, h;
        mi355_shard_bounds (n, es, s->size, i, &l, &h);
        if (i == s->me || h <= l)
            continue;
        dsts[k] = shmemi_peer_ptr (shmemi.mype, dst_off + l * es);
        sp[k] = ordered ? shmemi_peer_ptr (aset_pe (s, i), ver_off (chan, i, s->me, slot, dst_off))
                        : shmemi_peer_ptr (aset_pe (s, i), dst_off + l * es);
        nb[k] = (h - l) * es;
        ++k;
    }
    return k;
}

/* nan_pair's gather: the other member's shard from its target, where this
 * PE's own source is a NaN that NaN quieted instead. 0: queued, or nothing to
 * do (an empty shard: fires an armed signal). */
static int pair_gather (int dtype, size_t es, size_t dst_off, size_t src_off, size_t n, const struct aset *s,
                        long long pair_k, int chan, hipStream_t st)
{
    const int other = 1 - s->me, other_pe = aset_pe (s, other);
    size_t l, h;
    mi355_shard_bounds (n, es, 2, other, &l, &h);
    return mi355_nan_patch_copy (dtype, shmemi_peer_ptr (shmemi.mype, dst_off + l * es),
                                 shmemi_peer_ptr (other_pe, dst_off + l * es),
                                 shmemi_peer_ptr (shmemi.mype, src_off + l * es), h > l ? h - l : 0,
                                 nan_word_ok (s) ? shmemi.peer_sig[other_pe] +
                                                       MI355_SIG_NANFLAG_AT (chan, pair_k & 1, shmemi.mype)
                                                 : NULL, /* no word: always patch */
                                 st);
}

/* P2P shard schedule, dst and src disjoint or identical, with the three
 * barriers as one-block device-barrier kernels on the library stream: five
 * launches queued back to back, one host wait (the last barrier carries the
 * completion flag). The first barrier also orders the sources: each PE's
 * arrival is stream-ordered after its caller's work. */
static void p2p_range_dev (int op, int dtype, size_t es, size_t dst_off, size_t src_off, size_t n,
                           const struct aset *s, int ordered, int pair)
{
    MI355FusedArgs a;
    member_args (&a, s, SHMEMI_CHAN_HOST);
    void *dsts[MI355_FUSED_MAX_MEMBERS];
    const void *sp[MI355_FUSED_MAX_MEMBERS];
    size_t nb[MI355_FUSED_MAX_MEMBERS];

    const long long pk = pair ? pair_next (SHMEMI_CHAN_HOST, s) : -1;
    device_barrier (&a, shmemi.stream); /* every source is ready */
    shmemi_peer_acquire (shmemi.stream);
    shmemi_timed_begin ();
    int rc = fold_shard (op, dtype, es, dst_off, src_off, n, s, ordered, pk, SHMEMI_CHAN_HOST, shmemi.stream);
    shmemi_timed_end ();
    if (rc != 0)
        shmemi_fatal ("combine kernel launch failed (op %d, dtype %d, %d sources, %zu elements): %d", op, dtype,
                      s->size, n, rc);
    device_barrier (&a, shmemi.stream); /* every shard is reduced */
    shmemi_peer_acquire (shmemi.stream);
    const int k = pair ? 0 : gather_segments (es, dst_off, n, s, ordered, SHMEMI_CHAN_HOST, dsts, sp, nb);
    if (pair) {
        shmemi_timed_begin_phase (1);
        rc = pair_gather (dtype, es, dst_off, src_off, n, s, pk, SHMEMI_CHAN_HOST, shmemi.stream);
        shmemi_timed_end ();
        if (rc != 0)
            shmemi_fatal ("gather kernel launch failed: %d", rc);
    }
    if (k > 0) {
        shmemi_timed_begin_phase (1);
        rc = mi355_copy_segments (dsts, sp, nb, k, shmemi.stream);
        shmemi_timed_end ();
        if (rc != 0)
            shmemi_fatal ("copy kernel launch failed: %d", rc);
    }
    a.host_flag = shmemi.sig_flag; /* peers are done reading us: the call is over */
    a.epoch = shmemi_next_epoch ();
    device_barrier (&a, shmemi.stream);
    if (shmemi_wait_flag (a.epoch) != a.epoch)
        shmemi_fatal ("device barrier timed out waiting for the other PEs of the active set");
}

/* Before a host barrier lets peers read this PE's caller-written buffers,
 * the host must know the caller's queued work is done (one signal kernel,
 * shmemi_order_after_caller). Set per call by reduce_impl; the device-flag
 * schedules never need it. */
static int caller_order_pending;

static void host_order (void)
{
    if (caller_order_pending) {
        shmemi_order_after_caller (1);
        caller_order_pending = 0;
    }
}

/* P2P shard schedule (host barriers), dst and src disjoint or identical. */
static void p2p_range (int op, int dtype, size_t es, size_t dst_off, size_t src_off, size_t n,
                       const struct aset *s, int ordered, int pair)
{
    const void **sp = (const void **) malloc (sizeof (void *) * (size_t) s->size);
    void **dsts = (void **) malloc (sizeof (void *) * (size_t) s->size);
    size_t *nb = (size_t *) malloc (sizeof (size_t) * (size_t) s->size);
    if (sp == NULL || dsts == NULL || nb == NULL)
        shmemi_fatal ("out of host memory");

    size_t lo, hi;
    mi355_shard_bounds (n, es, s->size, s->me, &lo, &hi);

    const long long pk = pair ? pair_next (SHMEMI_CHAN_HOST, s) : -1;
    host_order ();
    shmemi_barrier_set (s->start, s->stride, s->size); /* every source is ready */
    if (hi > lo) {
        shmemi_peer_acquire (shmemi.stream);
        shmemi_timed_begin ();
        shmemi_arm_signal ();
        int rc = fold_shard (op, dtype, es, dst_off, src_off, n, s, ordered, pk, SHMEMI_CHAN_HOST, shmemi.stream);
        shmemi_timed_end ();
        if (rc != 0)
            shmemi_fatal ("combine kernel launch failed (op %d, dtype %d, %d sources, %zu elements): %d", op,
                          dtype, s->size, n, rc);
        shmemi_wait_signal ();
    } else if (pair) { /* an empty shard: fold_shard only clears the next call's NaN word */
        const int rc = fold_shard (op, dtype, es, dst_off, src_off, n, s, ordered, pk, SHMEMI_CHAN_HOST, shmemi.stream);
        if (rc != 0)
            shmemi_fatal ("NaN word clear failed: %d", rc);
    }
    shmemi_barrier_set (s->start, s->stride, s->size); /* every shard is reduced */
    shmemi_peer_acquire (shmemi.stream);

    /* gather the other members' shards: one launch */
    if (pair) {
        shmemi_arm_signal ();
        const int rc = pair_gather (dtype, es, dst_off, src_off, n, s, pk, SHMEMI_CHAN_HOST, shmemi.stream);
        if (rc != 0)
            shmemi_fatal ("gather kernel launch failed: %d", rc);
        shmemi_wait_signal ();
    } else {
        const int k = gather_segments (es, dst_off, n, s, ordered, SHMEMI_CHAN_HOST, dsts, sp, nb);
        copy_wait (dsts, sp, nb, k, 1);
    }
    shmemi_barrier_set (s->start, s->stride, s->size); /* peers are done reading us */
    free (nb);
    free (dsts);
    free (sp);
}

/* The multi-launch P2P schedule over [0, n): one round, or (ordered, when the
 * versions outgrow the version area) several, each a complete schedule. */
static void p2p_any (int op, int dtype, size_t es, size_t dst_off, size_t src_off, size_t n, const struct aset *s)
{
    const int pair = nan_pair (op, dtype, s);
    const int ordered = ordered_pair (op, dtype, s->size) && !pair;
    const int dev = device_flags_ok (s);
    const size_t round = ordered ? ordered_round_elems (es, s->size) : n;
    SHMEMI_TRACE (SHMEMI_LOG_REDUCTION, "schedule: P2P shards, %s barriers, %s (%zu elements, %d members%s)",
                  dev ? "device" : "host",
                  pair      ? "each member's reference order (own-order fold, NaN-patched gather)"
                  : ordered ? "every member's reference order"
                            : "PE_start order",
                  n, s->size, ordered && n > round ? ", several rounds" : "");
    begin_call (dev ? (n > round ? "p2p-rounds" : "p2p") : (n > round ? "p2p-host-rounds" : "p2p-host"));
    size_t b = 0;
    do {
        const size_t cn = n - b < round ? n - b : round;
        if (dev)
            p2p_range_dev (op, dtype, es, dst_off + b * es, src_off + b * es, cn, s, ordered, pair);
        else
            p2p_range (op, dtype, es, dst_off + b * es, src_off + b * es, cn, s, ordered, pair);
        b += cn;
    } while (b < n);
}

/* The fused one-launch schedule (fused.hip) applies: small enough, few
 * enough members, 16-byte aligned symmetric offsets, dst == src or disjoint,
 * and (ordered) the versions fit the version area. */
static int fused_eligible (int op, int dtype, size_t es, size_t dst_off, size_t src_off, size_t n,
                           const struct aset *s)
{
    return s->size > 1 && s->size <= MI355_FUSED_MAX_MEMBERS && n * es <= shmemi.fused_max &&
           shmemi.npes <= MI355_SIG_RSDONE &&
           shmemi.sigmem != NULL && ((dst_off | src_off) & 15) == 0 && es <= 256 &&
           (dst_off == src_off || !ranges_overlap (dst_off, src_off, n * es)) &&
           shmemi.algorithm != SHMEMX_REDUCE_EXACT &&
           (!ordered_pair (op, dtype, s->size) ||
            (size_t) (s->size - 1) * shard_chunk (n, es, s->size) * es <= shmemi.order_chunk);
}

/* The fused kernel's result order: ordered two-shot calls read and write the
 * members' version areas of channel `chan` (mi355_reduce.h). */
static void fused_order (MI355FusedArgs *a, const struct aset *s, int chan)
{
    a->ordered = ordered_pair (a->op, a->dtype, s->size);
    if (a->ordered && !a->oneshot)
        for (int i = 0; i < s->size; ++i)
            a->ver[i] = shmemi_peer_ptr (aset_pe (s, i), shmemi.order_off + (size_t) chan * shmemi.order_chunk);
}

/* The fused kernel's bytes: one-shot = every member's whole source read
 * (N - 1 of them from peers), one output; two-shot = the shard of every
 * member folded into 1 (or, ordered, N) outputs, then the other N - 1 shards
 * gathered from peers and written here. A one-member "fused" call is the
 * persistent server's identity copy. */
static void note_fused (int size, int ordered, int oneshot, size_t n, size_t es, const void *kernel)
{
    if (size == 1) {
        note_call (0, 1, 1, 0, (unsigned long long) (n * es), 0, 0, kernel);
        return;
    }
    if (oneshot) {
        note_call (ordered, size, 1, size - 1, (unsigned long long) (n * es), 0, 0, kernel);
        return;
    }
    const unsigned long long shard = (unsigned long long) (shard_chunk (n, es, size) * es);
    note_call (ordered, size, ordered ? size : 1, size - 1, shard, 2ull * (unsigned long long) (size - 1) * shard,
               (unsigned long long) (size - 1) * shard, kernel);
}

/* ---------------------------------------------------------------------- */
/* persistent fused server (opt-in: SHMEM_PERSISTENT=1, shmemx_set_persistent) */
/* ---------------------------------------------------------------------- */
/* A blocking call pays a launch and its dispatch (~6 us, profiles/r02/
 * kernarg_probe.txt) before the first block runs. When fused calls of one
 * (op, dtype, active set) come back to back (the second within
 * SHMEM_PERSISTENT_IDLE_US of the first), the fused kernel is left resident
 * on a stream of its own (mi355_fused_server): a call then writes its
 * offsets, sizes and epoch into the mailbox and waits for the epoch as
 * usual. The server leaves after SHMEM_PERSISTENT_IDLE_US without a call, or
 * when any other GPU operation of the library needs the device (device
 * barriers, other fused or pull kernels, RCCL, stream-ordered calls,
 * shmemx_device_synchronize, host heap changes, finalize). Not ordered after
 * the caller's queued GPU work: the caller's writes to the source must be
 * complete (synchronized) before the call -- hence opt-in. */
static int server_matches (int op, int dtype, const struct aset *s)
{
    return shmemi.srv.running && shmemi.srv.op == op && shmemi.srv.dtype == dtype && shmemi.srv.start == s->start &&
           shmemi.srv.stride == s->stride && shmemi.srv.size == s->size &&
           shmemi.srv.ordered == ordered_pair (op, dtype, s->size);
}

/* The server has left (EXITED): later servers start past its last seq. */
static void server_gone (void)
{
    const unsigned after = shmemi.srv.mb->state_seq + 1;
    if ((int) (after - shmemi.srv.seq) > 0)
        shmemi.srv.seq = after;
    shmemi.srv.running = 0;
    SHMEMI_HIP (hipStreamSynchronize (shmemi.srv.st)); /* the grid has drained */
}

static void server_wait_exited (void)
{
    const double t0 = shmemi_now ();
    unsigned spins = 0;
    while (__atomic_load_n (&shmemi.srv.mb->state, __ATOMIC_ACQUIRE) != MI355_SERVER_EXITED) {
        __builtin_ia32_pause ();
        if ((++spins & 1023u) == 0) {
            const hipError_t e = hipStreamQuery (shmemi.srv.st);
            if (e != hipSuccess && e != hipErrorNotReady)
                shmemi_fatal ("persistent fused server failed: %s", hipGetErrorString (e));
            if (shmemi_now () - t0 > shmemi.barrier_timeout)
                shmemi_fatal ("persistent fused server did not exit within %.0f s", shmemi.barrier_timeout);
        }
    }
}

void shmemi_server_stop (void)
{
    if (!shmemi.srv.running)
        return;
    MI355ServerMailbox *mb = shmemi.srv.mb;
    if (__atomic_load_n (&mb->state, __ATOMIC_ACQUIRE) != MI355_SERVER_EXITED) {
        mb->cmd = MI355_SERVER_QUIT;
        const unsigned seq = shmemi.srv.seq++;
        mb->check = mi355_mailbox_check (mb, seq);
        __atomic_store_n (&mb->seq_head, seq, __ATOMIC_RELEASE);
        __atomic_store_n (&mb->seq_tail, seq, __ATOMIC_RELEASE);
        server_wait_exited ();
    }
    server_gone ();
    SHMEMI_TRACE (SHMEMI_LOG_REDUCTION, "persistent fused server stopped");
}

/* Serve one call; 0 when the server had already left (the caller launches). */
static int server_call (size_t dst_off, size_t src_off, size_t n, size_t shard, int oneshot)
{
    MI355ServerMailbox *mb = shmemi.srv.mb;
    const unsigned epoch = shmemi_next_epoch ();
    mb->src_off = src_off;
    mb->dst_off = dst_off;
    mb->n = n;
    mb->shard = shard;
    mb->epoch = epoch;
    mb->oneshot = oneshot;
    mb->cmd = MI355_SERVER_RUN;
    const unsigned seq = shmemi.srv.seq++;
    mb->check = mi355_mailbox_check (mb, seq);
    __atomic_store_n (&mb->seq_head, seq, __ATOMIC_RELEASE);
    __atomic_store_n (&mb->seq_tail, seq, __ATOMIC_RELEASE);
    const double t0 = shmemi_now ();
    unsigned spins = 0;
    for (;;) {
        const unsigned v = __atomic_load_n (shmemi.sig_flag, __ATOMIC_ACQUIRE);
        if ((v & 0x7fffffffu) == epoch) {
            if (v & 0x80000000u)
                shmemi_fatal ("fused reduction timed out waiting for the other PEs of the active set");
            ++shmemi.srv.served;
            return 1;
        }
        if (__atomic_load_n (&mb->state, __ATOMIC_ACQUIRE) == MI355_SERVER_EXITED) {
            /* it left without taking this call (idle): the flag cannot come */
            if ((__atomic_load_n (shmemi.sig_flag, __ATOMIC_ACQUIRE) & 0x7fffffffu) == epoch)
                continue;
            server_gone ();
            return 0;
        }
        __builtin_ia32_pause ();
        if ((++spins & 1023u) == 0) {
            const hipError_t e = hipStreamQuery (shmemi.srv.st);
            if (e != hipSuccess && e != hipErrorNotReady)
                shmemi_fatal ("persistent fused server failed: %s", hipGetErrorString (e));
            if (shmemi_now () - t0 > shmemi.barrier_timeout)
                shmemi_fatal ("persistent fused server: call not completed within %.0f s", shmemi.barrier_timeout);
        }
    }
}

static void server_start (int op, int dtype, size_t es, size_t n, int oneshot, const struct aset *s)
{
    MI355FusedArgs a;
    member_args (&a, s, SHMEMI_CHAN_HOST);
    a.op = op;
    a.dtype = dtype;
    for (int i = 0; i < s->size; ++i) {
        a.src[i] = shmemi_peer_ptr (a.pe[i], 0);
        a.dst[i] = shmemi_peer_ptr (a.pe[i], 0);
    }
    a.host_flag = shmemi.sig_flag;
    a.ordered = ordered_pair (op, dtype, s->size);
    if (a.ordered)
        for (int i = 0; i < s->size; ++i)
            a.ver[i] = shmemi_peer_ptr (a.pe[i], shmemi.order_off + (size_t) SHMEMI_CHAN_HOST * shmemi.order_chunk);
    MI355ServerMailbox *mb = shmemi.srv.mb;
    mb->state = MI355_SERVER_RUNNING;
    mb->state_seq = 0;
    /* the grid of this call's launch (mi355_fused_allreduce) */
    const unsigned long long vecs = oneshot || s->size == 1 ? (n * es + 15) / 16
                                                            : shard_chunk (n, es, s->size) * es / 16 * (s->size - 1);
    shmemi_lazy_stream (&shmemi.srv.st, hipStreamNonBlocking);
    const int rc = mi355_fused_server (&a, mb, shmemi.srv.seq, (unsigned long long) (shmemi.srv.idle_s * 1e8), vecs,
                                       shmemi.srv.st);
    if (rc != 0) {
        SHMEMI_TRACE (SHMEMI_LOG_REDUCTION, "persistent fused server not started: %d", rc);
        return;
    }
    shmemi.srv.running = 1;
    shmemi.srv.op = op;
    shmemi.srv.dtype = dtype;
    shmemi.srv.start = s->start;
    shmemi.srv.stride = s->stride;
    shmemi.srv.size = s->size;
    shmemi.srv.ordered = a.ordered;
    shmemi.srv.kernel = mi355_last_kernel ();
    shmemi.srv.grid_elems = n;
    ++shmemi.srv.launched;
    SHMEMI_TRACE (SHMEMI_LOG_REDUCTION, "persistent fused server started (%d members, sized for %zu elements)",
                  s->size, n);
}

static void copy_local (size_t dst_off, size_t src_off, size_t nbytes, int timed);

static void fused_launch (int op, int dtype, size_t es, size_t n, const struct aset *s, const void *const *srcs,
                          void *const *dsts, int same, const void *host_src, void *host_dst);

/* host_src/host_dst: device-accessible page-locked host buffers of this PE
 * staged in-kernel into src_off / out of dst_off (mi355_reduce.h), or NULL.
 * A one-member set (the 1-PE identity copy) comes here only with the
 * persistent server enabled: served, or else one copy kernel. */
static void fused_range (int op, int dtype, size_t es, size_t dst_off, size_t src_off, size_t n,
                         const struct aset *s, const void *host_src, void *host_dst)
{
    const int servable = shmemi.srv.enabled && host_src == NULL && host_dst == NULL && dst_off < SHMEMI_EXT_TARGET &&
                         src_off < SHMEMI_EXT_TARGET; /* it addresses the members' heaps */
    const double t_call = servable ? shmemi_now () : 0.0;
    if (servable && server_matches (op, dtype, s) && n <= 2 * shmemi.srv.grid_elems) {
        SHMEMI_TRACE (SHMEMI_LOG_REDUCTION, "schedule: persistent fused server (%zu elements, %d members)", n, s->size);
        const int oneshot = n * es <= shmemi.oneshot_max && dst_off != src_off;
        if (server_call (dst_off, src_off, n, shard_chunk (n, es, s->size), oneshot)) {
            shmemi.srv.last_end = shmemi_now ();
            begin_call ("persistent");
            note_fused (s->size, shmemi.srv.ordered, oneshot, n, es, shmemi.srv.kernel);
            return;
        }
    }
    shmemi_server_stop (); /* a different call: the launched grid must fit */
    if (s->size == 1) {
        SHMEMI_TRACE (SHMEMI_LOG_REDUCTION, "schedule: 1-PE identity, one copy of %zu bytes", n * es);
        begin_call ("identity");
        copy_local (dst_off, src_off, n * es, 1);
    } else {
        const void *srcs[MI355_FUSED_MAX_MEMBERS];
        void *dsts[MI355_FUSED_MAX_MEMBERS];
        for (int i = 0; i < s->size; ++i) {
            srcs[i] = shmemi_peer_ptr (aset_pe (s, i), src_off);
            dsts[i] = shmemi_peer_ptr (aset_pe (s, i), dst_off);
        }
        fused_launch (op, dtype, es, n, s, srcs, dsts, dst_off == src_off, host_src, host_dst);
    }
    if (servable) {
        /* the second call of a burst leaves the kernel resident for the next */
        if (shmemi.srv.last_end >= 0.0 && t_call - shmemi.srv.last_end < shmemi.srv.idle_s)
            server_start (op, dtype, es, n, n * es <= shmemi.oneshot_max && dst_off != src_off, s);
        shmemi.srv.last_end = shmemi_now ();
    }
}

/* One launch of the fused kernel over the members' buffers srcs[i] / dsts[i]
 * (this PE's = member s->me's), waited for. `same`: target = source (no
 * one-shot: it would overwrite a source others still read). */
static void fused_launch (int op, int dtype, size_t es, size_t n, const struct aset *s, const void *const *srcs,
                          void *const *dsts, int same, const void *host_src, void *host_dst)
{
    {
        SHMEMI_TRACE (SHMEMI_LOG_REDUCTION, "schedule: fused one-launch P2P, %s, %s (%zu elements, %d members)%s",
                      n * es <= shmemi.oneshot_max && !same ? "one-shot" : "reduce-scatter + all-gather",
                      ordered_pair (op, dtype, s->size) ? "every member's reference order" : "PE_start order", n,
                      s->size, host_src != NULL ? ", staging host buffers in-kernel" : "");
        MI355FusedArgs a;
        memset (&a, 0, sizeof a);
        a.op = op;
        a.dtype = dtype;
        a.nmembers = s->size;
        a.me = s->me;
        a.n = n;
        a.shard = shard_chunk (n, es, s->size);
        for (int i = 0; i < s->size; ++i) {
            const int pe = aset_pe (s, i);
            a.pe[i] = pe;
            a.src[i] = srcs[i];
            a.dst[i] = dsts[i];
            a.sig[i] = shmemi.peer_sig[pe] + SHMEMI_CHAN_HOST * MI355_SIG_CHANNEL_WORDS;
        }
        a.host_flag = shmemi.sig_flag;
        a.epoch = shmemi_next_epoch ();
        a.err_flag = shmemi.stream_err;
        a.timeout_ticks = (unsigned long long) (shmemi.barrier_timeout * 1e8);
        a.host_src = host_src;
        a.host_dst = host_dst;
        a.share = shmemi.local_pes;
        a.no_acquire = shmemi.fused_no_acquire;
        a.oneshot = n * es <= shmemi.oneshot_max && !same;
        fused_order (&a, s, SHMEMI_CHAN_HOST);
        shmemi_timed_begin (); /* the call's one (dominant) kernel */
        const int rc = mi355_fused_allreduce (&a, shmemi.stream);
        shmemi_timed_end ();
        if (rc != 0)
            shmemi_fatal ("fused reduction launch failed (op %d, dtype %d, %d PEs, %zu elements): %d", op, dtype,
                          s->size, n, rc);
        begin_call (a.oneshot ? "fused-oneshot" : "fused-twoshot");
        note_fused (s->size, a.ordered, a.oneshot, n, es, mi355_last_kernel ());
        if (shmemi_wait_flag (a.epoch) != a.epoch)
            shmemi_fatal ("fused reduction timed out waiting for the other PEs of the active set");
    }
}

/* EXACT: fold everything in this PE's reference order into dst; dst must
 * not overlap any source (callers route overlaps through scratch). */
static void exact_into (int op, int dtype, size_t dst_off, size_t src_off, size_t n, const struct aset *s)
{
    const void **sp = (const void **) malloc (sizeof (void *) * (size_t) s->size);
    if (sp == NULL)
        shmemi_fatal ("out of host memory");
    shmemi_peer_acquire (shmemi.stream);
    sp[0] = shmemi_peer_ptr (shmemi.mype, src_off);
    int k = 1;
    for (int i = 0; i < s->size; ++i)
        if (i != s->me)
            sp[k++] = shmemi_peer_ptr (aset_pe (s, i), src_off);
    combine_wait (op, dtype, shmemi_peer_ptr (shmemi.mype, dst_off), sp, s->size, n, 1);
    note_call (1, s->size, 1, s->size - 1, (unsigned long long) (n * mi355_dtype_size (dtype)), 0, 0,
               mi355_last_kernel ());
    free (sp);
}

/* timed: the copy is the call's dominant kernel (the PE_size == 1 identity) */
static void copy_local (size_t dst_off, size_t src_off, size_t nbytes, int timed)
{
    void *d = shmemi_peer_ptr (shmemi.mype, dst_off);
    const void *sv = shmemi_peer_ptr (shmemi.mype, src_off);
    size_t nb = nbytes;
    copy_wait (&d, &sv, &nb, 1, timed ? 0 : -1);
    if (timed)
        note_call (0, 1, 1, 0, (unsigned long long) nbytes, 0, 0, mi355_last_kernel ());
}

/* Reduce n elements at symmetric offsets. Handles aliasing like the
 * reference's temporary target (reduce-op.c:174-215), but chunked through
 * scratch in memmove order so any overlap is safe. */
static void reduce_symmetric (int op, int dtype, size_t es, size_t dst_off, size_t src_off, size_t n,
                              const struct aset *s)
{
    const size_t nbytes = n * es;
    /* EXACT by request, or for an order-sensitive set too large for the
     * shard schedules' every-order fold (ordered_pair) */
    const int exact = shmemi.algorithm == SHMEMX_REDUCE_EXACT ||
                      (order_sensitive (op, dtype, s->size) && !ordered_pair (op, dtype, s->size));
    const int same = dst_off == src_off;
    if (s->size > 1 && shmemi.p2p_broken)
        shmemi_fatal ("peer GPU memory reads failed the init self-test; only the RCCL pairs "
                      "(sum/prod/min/max on short/int/long/float/double, complex sum) over all PEs can run");
    const int overlap = ranges_overlap (dst_off, src_off, nbytes);

    if (s->size == 1) {
        /* a one-PE fold is the identity: target = source (reduce-op.c:226-229) */
        if (same) {
            SHMEMI_TRACE (SHMEMI_LOG_REDUCTION, "schedule: 1-PE identity in place, nothing to move");
            begin_call ("identity");
            return;
        }
        if (!overlap) {
            if (shmemi.srv.enabled && nbytes <= shmemi.fused_max && ((dst_off | src_off) & 15) == 0) {
                fused_range (op, dtype, es, dst_off, src_off, n, s, NULL, NULL); /* persistent server */
                return;
            }
            SHMEMI_TRACE (SHMEMI_LOG_REDUCTION, "schedule: 1-PE identity, one copy of %zu bytes", nbytes);
            begin_call ("identity");
            copy_local (dst_off, src_off, nbytes, 1);
            return;
        }
    } else if (!exact && (same || !overlap)) {
        if (fused_eligible (op, dtype, es, dst_off, src_off, n, s))
            fused_range (op, dtype, es, dst_off, src_off, n, s, NULL, NULL);
        else
            p2p_any (op, dtype, es, dst_off, src_off, n, s);
        return;
    } else if (exact && !overlap) {
        SHMEMI_TRACE (SHMEMI_LOG_REDUCTION, "schedule: EXACT reference order, host barriers");
        begin_call ("exact");
        host_order ();
        shmemi_barrier_set (s->start, s->stride, s->size);
        exact_into (op, dtype, dst_off, src_off, n, s);
        shmemi_barrier_set (s->start, s->stride, s->size);
        return;
    }

    /* overlapping target/source: through scratch buffer C, chunk by chunk,
     * walking down when target lies above source (memmove order) */
    const size_t tmp_off = shmemi.scratch_off + 2 * shmemi.scratch_chunk;
    const size_t per = shmemi.scratch_chunk / es;
    const size_t nchunks = (n + per - 1) / per;
    const int down = dst_off > src_off;
    SHMEMI_TRACE (SHMEMI_LOG_REDUCTION, "schedule: overlapping target, %zu chunk(s) through scratch, %s", nchunks,
                  down ? "top down" : "bottom up");
    if (s->size == 1 || exact)
        begin_call (exact ? "exact" : "identity");
    for (size_t c = 0; c < nchunks; ++c) {
        const size_t idx = down ? nchunks - 1 - c : c;
        const size_t b = idx * per;
        const size_t cn = n - b < per ? n - b : per;
        if (s->size == 1) {
            copy_local (tmp_off, src_off + b * es, cn * es, 0);
        } else if (!exact) {
            p2p_any (op, dtype, es, tmp_off, src_off + b * es, cn, s);
        } else {
            host_order ();
            shmemi_barrier_set (s->start, s->stride, s->size);
            exact_into (op, dtype, tmp_off, src_off + b * es, cn, s);
            shmemi_barrier_set (s->start, s->stride, s->size);
        }
        copy_local (dst_off + b * es, tmp_off, cn * es, 0);
        /* nobody reads our target chunk; the next chunk's first barrier orders
         * our write before any peer reads the source bytes it may cover */
    }
    if (s->size > 1)
        shmemi_barrier_set (s->start, s->stride, s->size);
}

/* ---------------------------------------------------------------------- */
/* RCCL                                                                    */
/* ---------------------------------------------------------------------- */
int shmemi_rccl_allreduce (int op, int dtype, const void *src, void *dst, size_t n);
int shmemi_rccl_supported (int op, int dtype);

/* ---------------------------------------------------------------------- */
/* entry                                                                   */
/* ---------------------------------------------------------------------- */
enum { PK_HOST = SHMEMI_PK_HOST, PK_DEV_SYM = SHMEMI_PK_DEV_SYM, PK_DEV_OTHER = SHMEMI_PK_DEV_OTHER };

static int ptr_kind (const void *p, size_t nbytes)
{
    if (shmemi_in_device_heap (p, nbytes))
        return PK_DEV_SYM;
    hipPointerAttribute_t a;
    memset (&a, 0, sizeof a);
    hipError_t e = hipPointerGetAttributes (&a, p);
    (void) hipGetLastError ();
    if (e == hipSuccess && (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged))
        return PK_DEV_OTHER;
    return PK_HOST;
}

/* Buffers outside the device heap: stream them through scratch in chunks,
 * double-buffered so the copy-in of chunk k+1 (stream in) and the copy-out of
 * chunk k-1 (stream out) run while chunk k is reduced: with host buffers the
 * two PCIe directions then work at the same time.
 *   A0/A1 = halves of scratch A (sources), B0/B1 = halves of scratch B (results)
 * PE_size == 1 is the identity: each chunk goes in to A and straight back out.
 * A target that overlaps the source from above is walked top down (memmove
 * order, like the reference's temporary target, reduce-op.c:174-215): the
 * copy-out of a chunk then only writes source bytes already copied in, while
 * the copy-in of the next chunk (below) runs beside it. */
static void staged (int op, int dtype, const char *fn, void *target, const void *source, size_t n,
                    const struct aset *s, int ks, int kt, int use_rccl)
{
    const size_t es = mi355_dtype_size (dtype);
    shmemi_lazy_stream (&shmemi.stream_in, hipStreamDefault);
    shmemi_lazy_stream (&shmemi.stream_out, hipStreamDefault);
    const size_t half = shmemi.scratch_chunk / 2 / SHMEMI_ALIGN * SHMEMI_ALIGN;
    const size_t per = half / es;
    const size_t nchunks = (n + per - 1) / per;
    const size_t a_off[2] = {shmemi.scratch_off, shmemi.scratch_off + half};
    const size_t b_off[2] = {shmemi.scratch_off + shmemi.scratch_chunk,
                             shmemi.scratch_off + shmemi.scratch_chunk + half};
    const hipMemcpyKind in_kind = ks == PK_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
    const hipMemcpyKind out_kind = kt == PK_HOST ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    const int identity = s->size == 1;
    const int down = (const char *) target > (const char *) source &&
                     (const char *) target < (const char *) source + n * es;

#define CHUNK_ID(k) (down ? nchunks - 1 - (k) : (k)) /* the k-th chunk processed */
#define CHUNK_N(c) (n - (c) * per < per ? n - (c) * per : per)
    for (size_t k = 0; k < nchunks + 1; ++k) {
        /* copy-in of the k-th chunk (issued one chunk ahead of its reduction) */
        if (k < nchunks) {
            const int j = (int) (k & 1);
            const size_t c = CHUNK_ID (k);
            if (k >= 2) /* A[j] was last read by the copy-out (identity) or reduction of the (k-2)-th chunk */
                SHMEMI_HIP (hipStreamWaitEvent (shmemi.stream_in, shmemi.ev_out[j], 0));
            SHMEMI_HIP (hipMemcpyAsync (shmemi.heap + a_off[j], (const char *) source + c * per * es,
                                        CHUNK_N (c) * es, in_kind, shmemi.stream_in));
            SHMEMI_HIP (hipEventRecord (shmemi.ev_in[j], shmemi.stream_in));
        }
        if (k == 0)
            continue;
        /* reduce and copy out the (k-1)-th chunk */
        const size_t q = k - 1, c = CHUNK_ID (q);
        const int j = (int) (q & 1);
        const size_t cn = CHUNK_N (c);
        size_t out_off = a_off[j];
        if (identity) {
            SHMEMI_HIP (hipStreamWaitEvent (shmemi.stream_out, shmemi.ev_in[j], 0));
        } else {
            SHMEMI_HIP (hipEventSynchronize (shmemi.ev_in[j])); /* peers read A[j] after the barrier */
            if (q >= 2) /* B[j] is still being copied out for the (q-2)-th chunk */
                SHMEMI_HIP (hipStreamWaitEvent (shmemi.stream, shmemi.ev_out[j], 0));
            out_off = b_off[j];
            if (use_rccl) {
                if (shmemi_rccl_allreduce (op, dtype, shmemi.heap + a_off[j], shmemi.heap + b_off[j], cn) != 0)
                    shmemi_fatal ("%s: ncclAllReduce failed", fn);
            } else {
                reduce_symmetric (op, dtype, es, b_off[j], a_off[j], cn, s);
            }
        }
        SHMEMI_HIP (hipMemcpyAsync ((char *) target + c * per * es, shmemi.heap + out_off, cn * es, out_kind,
                                    shmemi.stream_out));
        SHMEMI_HIP (hipEventRecord (shmemi.ev_out[j], shmemi.stream_out));
    }
#undef CHUNK_N
#undef CHUNK_ID
    SHMEMI_HIP (hipStreamSynchronize (shmemi.stream_out));
    SHMEMI_HIP (hipStreamSynchronize (shmemi.stream_in));
}

/* Buffers outside the device symmetric heap that this GPU can still reach:
 * plain device memory (hipMalloc, e.g. a framework's tensors) and page-locked
 * host arrays (shmem_malloc's default heap). Instead of separate H2D/D2D/D2H
 * copies around the reduction:
 *   1 PE          one copy kernel straight from source to target (device to
 *                 device at any size; with a host side up to 1 MiB -- above,
 *                 the DMA double buffering of staged() is faster);
 *   N PEs, small  the fused kernel stages this PE's source into its scratch A
 *                 and the result out of scratch B itself (one launch) -- the
 *                 same scratch offsets and the same single collective as
 *                 staged()'s one-chunk case, so PEs that take staged() (pageable
 *                 host arrays) still meet it.
 * Host arrays: ~30 -> ~11 us at 1 PE and ~58 -> ~19 us at 2 PEs for 8 B -
 * 8 KiB. Returns 0 when it does not apply. */
#define SHMEMI_SMALL_LOCAL_MAX ((size_t) 1 << 20)
static const void *reachable (const void *p, size_t nbytes, int kind)
{
    return kind == PK_HOST ? shmemi_host_dev_ptr (p, nbytes) : p;
}

static int local_direct (int op, int dtype, void *target, const void *source, size_t n, int overlap, int kt,
                         int ks, const struct aset *s)
{
    const size_t es = mi355_dtype_size (dtype), nbytes = n * es;
    if (overlap && target != source)
        return 0;
    void *ht = (void *) reachable (target, nbytes, kt);
    const void *hs = reachable (source, nbytes, ks);
    if (ht == NULL || hs == NULL)
        return 0;
    const int any_host = kt == PK_HOST || ks == PK_HOST;
    if (s->size == 1) {
        if (any_host && nbytes > SHMEMI_SMALL_LOCAL_MAX)
            return 0;
        SHMEMI_TRACE (SHMEMI_LOG_REDUCTION, "schedule: 1-PE identity, one copy kernel source -> target (%zu bytes)",
                      nbytes);
        begin_call ("identity");
        if (target != source) {
            void *d = ht;
            size_t nb = nbytes;
            copy_wait (&d, &hs, &nb, 1, -1);
            note_call (0, 1, 1, 0, (unsigned long long) nbytes, 0, 0, mi355_last_kernel ());
        }
        return 1;
    }
    const size_t half = shmemi.scratch_chunk / 2 / SHMEMI_ALIGN * SHMEMI_ALIGN;
    if (nbytes > SHMEMI_SMALL_LOCAL_MAX || nbytes > half)
        return 0;
    const size_t a_off = shmemi.scratch_off, b_off = shmemi.scratch_off + shmemi.scratch_chunk;
    if (!fused_eligible (op, dtype, es, b_off, a_off, n, s))
        return 0;
    fused_range (op, dtype, es, b_off, a_off, n, s, hs, ht);
    return 1;
}

/* SHMEM_DEBUG=1: the members compare their arguments before anything else
 * of the call happens (runtime.c, shmemi_debug_exchange). */
static void debug_check (const char *fn, int op, int dtype, const void *target, const void *source, int nreduce,
                         int PE_start, int logPE_stride, int PE_size)
{
    if (PE_size < 2)
        return;
    struct shmemi_dbg_rec r;
    memset (&r, 0, sizeof r);
    r.op = op;
    r.dtype = dtype;
    r.nreduce = nreduce;
    r.pe_start = PE_start;
    r.log_stride = logPE_stride;
    r.pe_size = PE_size;
    r.tkind = r.skind = -1;
    if (nreduce > 0) {
        const size_t nbytes = (size_t) nreduce * mi355_dtype_size (dtype);
        r.tkind = ptr_kind (target, nbytes);
        r.skind = ptr_kind (source, nbytes);
        if (r.tkind == PK_DEV_SYM)
            r.toff = shmemi_heap_offset (target);
        if (r.skind == PK_DEV_SYM)
            r.soff = shmemi_heap_offset (source);
        /* the staging path walks its chunks in an order the members share */
        const char *t = (const char *) target, *sr = (const char *) source;
        r.overlap = t == sr ? 1 : t > sr && t < sr + nbytes ? 2 : sr > t && sr < t + nbytes ? 3 : 0;
    }
    r.algorithm = shmemi.algorithm;
    r.order = shmemi.order;
    r.fused_max = shmemi.fused_max;
    r.oneshot_max = shmemi.oneshot_max;
    snprintf (r.fn, sizeof r.fn, "%s", fn);
    shmemi_debug_exchange (&r, PE_start, 1 << logPE_stride, PE_size);
}

/* SHMEM_FUSED_MAX_BYTES and SHMEM_ONESHOT_MAX_BYTES from measurement, at
 * init, on this job's own layout (PE_size > 1, the variable not given): the
 * fused one-launch schedule saves the multi-launch schedule's barrier
 * launches (barrier-linear.c:57-85's two barriers and the gather's own) but
 * pays its device-side flag round trips in one grid; where it stops paying
 * depends on the links (round 5, two PEs on one GPU: 1 MiB, not the 2 MiB
 * default; bench.py threshold_sweep). Double sums over the whole job between
 * scratch buffers A and B: each size timed both ways (median of 9 blocking
 * calls after 2 warm-ups, entry to return), the medians max-reduced over the
 * PEs through the bootstrap segment, and the threshold set to the largest
 * size of the prefix of sizes where the fused (one-shot) call was no slower
 * -- the same decision on every PE. About 250 calls, a few ms. */
void shmemi_calibrate_thresholds (int fused, int oneshot)
{
    static const size_t fsz[SHMEMI_CALIB_NF] = {64 << 10, 256 << 10, 512 << 10, 1 << 20, 2 << 20, 4 << 20};
    static const size_t osz[SHMEMI_CALIB_NO] = {16 << 10, 32 << 10, 64 << 10, 128 << 10, 256 << 10};
    const int np = shmemi.npes, me = shmemi.mype, K = 9, W = 2;
    struct aset s = {0, 1, np, me};
    const size_t src_off = shmemi.scratch_off, dst_off = shmemi.scratch_off + shmemi.scratch_chunk;
    const size_t f0 = shmemi.fused_max, o0 = shmemi.oneshot_max;
    const unsigned mask0 = shmemi_trace_mask;
    shmemi_trace_mask &= ~(1u << SHMEMI_LOG_REDUCTION); /* no schedule lines for these calls */
    SHMEMI_HIP (hipMemset (shmemi.heap + src_off, 0, shmemi.scratch_chunk));
    SHMEMI_HIP (hipDeviceSynchronize ());
    shmemi_barrier_set (0, 1, np);
    uint64_t mine[SHMEMI_CALIB_SLOTS] = {0};
    /* slot of (kind, size): kind 0 fused / 1 multi-launch / 2 one-shot / 3 two-shot */
#define SLOT(kind, i) ((kind) < 2 ? (kind) * SHMEMI_CALIB_NF + (i) : 2 * SHMEMI_CALIB_NF + ((kind) - 2) * SHMEMI_CALIB_NO + (i))
    for (int kind = 0; kind < 4; ++kind) {
        if ((kind < 2 && !fused) || (kind >= 2 && !oneshot))
            continue;
        const int nsz = kind < 2 ? SHMEMI_CALIB_NF : SHMEMI_CALIB_NO;
        for (int i = 0; i < nsz; ++i) {
            const size_t bytes = kind < 2 ? fsz[i] : osz[i];
            if (bytes > shmemi.scratch_chunk)
                continue; /* 0 = not measured: ends the prefix below */
            shmemi.fused_max = kind == 1 ? 0 : (size_t) 1 << 30;
            shmemi.oneshot_max = kind == 2 ? (size_t) 1 << 30 : kind == 3 ? 0 : o0;
            double t[16];
            for (int r = 0; r < W + K; ++r) {
                caller_order_pending = 1;
                const double t0 = shmemi_now ();
                reduce_symmetric (MI355_OP_SUM, MI355_DOUBLE, 8, dst_off, src_off, bytes / 8, &s);
                if (r >= W)
                    t[r - W] = shmemi_now () - t0;
            }
            for (int a = 1; a < K; ++a) /* median: insertion sort of 9 */
                for (int b = a; b > 0 && t[b] < t[b - 1]; --b) {
                    const double x = t[b];
                    t[b] = t[b - 1];
                    t[b - 1] = x;
                }
            mine[SLOT (kind, i)] = (uint64_t) (t[K / 2] * 1e9) + 1;
        }
    }
    struct shmemi_pe_info *info = shmemi_seg_info (me);
    for (int k = 0; k < SHMEMI_CALIB_SLOTS; ++k)
        __atomic_store_n (&info->calib_ns[k], mine[k], __ATOMIC_RELEASE);
    shmemi_barrier_set (0, 1, np);
    for (int k = 0; k < SHMEMI_CALIB_SLOTS; ++k) {
        uint64_t w = 0;
        for (int q = 0; q < np; ++q) {
            const uint64_t v = __atomic_load_n (&shmemi_seg_info (q)->calib_ns[k], __ATOMIC_ACQUIRE);
            w = v == 0 || w == UINT64_MAX ? UINT64_MAX : v > w ? v : w; /* unmeasured anywhere: unmeasured */
        }
        shmemi.calib_us[k] = w == UINT64_MAX ? 0.0 : (double) w * 1e-3;
    }
    shmemi_barrier_set (0, 1, np); /* nobody reads the records any more */
    /* the largest size of the prefix where the fused / one-shot call was no slower */
    size_t fm = f0, om = o0;
    if (fused) {
        fm = 0;
        for (int i = 0; i < SHMEMI_CALIB_NF; ++i) {
            const double a = shmemi.calib_us[SLOT (0, i)], b = shmemi.calib_us[SLOT (1, i)];
            if (a <= 0.0 || b <= 0.0 || a > b)
                break;
            fm = fsz[i];
        }
    }
    if (oneshot) {
        om = 0;
        for (int i = 0; i < SHMEMI_CALIB_NO; ++i) {
            const double a = shmemi.calib_us[SLOT (2, i)], b = shmemi.calib_us[SLOT (3, i)];
            if (a <= 0.0 || b <= 0.0 || a > b)
                break;
            om = osz[i];
        }
    }
#undef SLOT
    shmemi.fused_max = fm;
    shmemi.oneshot_max = om;
    shmemi.calib_ran = 1;
    shmemi_trace_mask = mask0;
    SHMEMI_TRACE (SHMEMI_LOG_INIT, "thresholds from measurement: fused path up to %zu bytes, one-shot up to %zu bytes",
                  fm, om);
}

static void reduce_impl (int op, int dtype, const char *fn, void *target, const void *source,
                         int nreduce, int PE_start, int logPE_stride, int PE_size, long *pSync)
{
    shmemi_init_check (fn);
    if (logPE_stride < 0 || logPE_stride > 30 || PE_size < 1 || PE_start < 0 ||
        PE_start + (long) (PE_size - 1) * (1L << logPE_stride) >= shmemi.npes)
        shmemi_fatal ("%s: active set (PE_start %d, logPE_stride %d, PE_size %d) outside the %d PEs",
                      fn, PE_start, logPE_stride, PE_size, shmemi.npes);
    struct aset s = {PE_start, 1 << logPE_stride, PE_size, -1};
    for (int i = 0; i < PE_size; ++i)
        if (aset_pe (&s, i) == shmemi.mype)
            s.me = i;
    if (s.me < 0)
        shmemi_fatal ("%s: PE %d is not in the active set (PE_start %d, logPE_stride %d, PE_size %d)",
                      fn, shmemi.mype, PE_start, logPE_stride, PE_size);
    if (nreduce < 0)
        shmemi_fatal ("%s: nreduce %d < 0", fn, nreduce);
    if (shmemi.debug && pSync != NULL && (pSync[0] != SHMEM_SYNC_VALUE || pSync[1] != SHMEM_SYNC_VALUE))
        shmemi_fatal ("%s: pSync not initialised to SHMEM_SYNC_VALUE", fn);

    const size_t es = mi355_dtype_size (dtype);
    const size_t n = (size_t) nreduce;
    if (shmemi.debug)
        debug_check (fn, op, dtype, target, source, nreduce, PE_start, logPE_stride, PE_size);
    if (n == 0) {
        begin_call ("barrier-only");
        /* both barriers of reduce-op.c:230,266 still run (host only: no GPU work) */
        shmemi_barrier_set (s.start, s.stride, s.size);
        shmemi_barrier_set (s.start, s.stride, s.size);
        return;
    }
    if (shmemi.heap == NULL)
        shmemi_fatal ("%s: no GPU: this library reduces on the GPU only (SHMEM_BOOTSTRAP_ONLY set?)", fn);
    if (target == NULL || source == NULL)
        shmemi_fatal ("%s: NULL target or source", fn);
    const size_t nbytes = n * es;
    const int kt = ptr_kind (target, nbytes), ks = ptr_kind (source, nbytes);
    /* Device buffers: the library stream is ordered after the caller's
     * null-stream work. The device-flag schedules (fused kernel, device
     * barriers) then learn on the GPU that peers' sources are ready; a
     * schedule with host barriers first waits for that point on the host. */
    if (kt != PK_HOST || ks != PK_HOST)
        shmemi_order_after_caller (0); /* SHMEM_ENTRY_SYNC */
    caller_order_pending = s.size > 1 && kt == PK_DEV_SYM && ks == PK_DEV_SYM;

    const int overlap = target != source && ranges_overlap ((size_t) target, (size_t) source, nbytes);
    if (shmemi_trace_mask & (1u << SHMEMI_LOG_REDUCTION)) {
        static const char *const kind[] = {"host", "device heap", "device, not symmetric"};
        SHMEMI_TRACE (SHMEMI_LOG_REDUCTION,
                      "%s: nreduce %d, PE_start %d, logPE_stride %d, PE_size %d; target %p (%s), source %p (%s)", fn,
                      nreduce, PE_start, logPE_stride, PE_size, target, kind[kt], source, kind[ks]);
        /* the reference's overlap trace (reduce-op.c:210-223) */
        SHMEMI_TRACE (SHMEMI_LOG_REDUCTION, "target (%p) and source (%p, size %zu) %s", target, source, nbytes,
                      target == source ? "are the same buffer" : overlap ? "overlap, using temporary target"
                                                                          : "do not overlap");
    }
    /* RCCL by request, or whenever the init self-test found peer heap reads
     * broken (whatever the selected algorithm): the pairs RCCL has still run */
    const int use_rccl = (shmemi.algorithm == SHMEMX_REDUCE_RCCL || shmemi.p2p_broken) && s.size == shmemi.npes &&
                         s.size > 1 && shmemi_rccl_supported (op, dtype);
    if (use_rccl && kt != PK_HOST && ks != PK_HOST && !overlap) {
        SHMEMI_TRACE (SHMEMI_LOG_REDUCTION, "schedule: RCCL allreduce");
        shmemi_server_stop ();
        if (shmemi_rccl_allreduce (op, dtype, source, target, n) != 0)
            shmemi_fatal ("%s: ncclAllReduce failed", fn);
        /* RCCL's own kernels: bytes as a full-mesh exchange would move them */
        begin_call ("rccl");
        note_call (0, 1, 1, 0, (unsigned long long) nbytes, 0,
                   2ull * (unsigned long long) (s.size - 1) * nbytes / (unsigned long long) s.size, NULL);
        return;
    }
    if (kt == PK_DEV_SYM && ks == PK_DEV_SYM) {
        reduce_symmetric (op, dtype, es, shmemi_heap_offset (target), shmemi_heap_offset (source), n, &s);
        return;
    }
    /* device buffers outside the heap (a framework's tensors): the members
     * map each other's allocations for this call and run the heap schedules
     * on them, or, when one of them cannot, all stage (extmap.c) */
    if (s.size > 1 && !use_rccl) {
        size_t toff, soff;
        if (shmemi_ext_begin (fn, target, source, nbytes, kt, ks, s.start, s.stride, s.size, &toff, &soff)) {
            SHMEMI_TRACE (SHMEMI_LOG_REDUCTION, "device buffers outside the heap mapped by the peers for this call");
            caller_order_pending = 1; /* peers read this PE's buffers directly */
            reduce_symmetric (op, dtype, es, toff, soff, n, &s);
            shmemi_ext_end ();
            static char name[80];
            snprintf (name, sizeof name, "mapped-%s", shmemi.last.schedule);
            shmemi.last.schedule = name;
            return;
        }
    }

    if (!use_rccl && local_direct (op, dtype, target, source, n, overlap, kt, ks, &s))
        return;
    SHMEMI_TRACE (SHMEMI_LOG_REDUCTION, "staged through the scratch buffers (%s)", use_rccl ? "RCCL" : "P2P");
    begin_call ("staged");
    staged (op, dtype, fn, target, source, n, &s, ks, kt, use_rccl);
    shmemi.last.schedule = "staged"; /* the kernel fields: the last chunk's reduction */
}

/* ---------------------------------------------------------------------- */
/* stream-ordered collectives (shmemx.h)                                   */
/* ---------------------------------------------------------------------- */
/* The same P2P schedule, enqueued on the caller's stream with no host wait:
 * cross-PE ordering is device-side (fused.hip's pair counts), so a caller can
 * overlap the reduction with its own kernels or capture it into a HIP graph.
 *   fused-eligible   one launch of the fused kernel
 *   otherwise        device barrier, fold of shard `me`, device barrier,
 *                    gather, device barrier -- the host schedule's three
 *                    barriers, each a one-block kernel instead of a host wait
 They use their own signal-region channel, so a host-launched fused call may
 * run while they are in flight; among themselves they must run one at a time
 * per PE (one stream, or streams the caller orders). Errors of device-side
 * waits (a peer never arrives within SHMEM_BARRIER_TIMEOUT) surface at the
 * next library call. */

void shmemi_check_stream_err (const char *fn)
{
    if (shmemi.stream_err != NULL && __atomic_load_n (shmemi.stream_err, __ATOMIC_ACQUIRE) != 0)
        shmemi_fatal ("%s: a stream-ordered collective timed out waiting for another PE", fn);
}

static void stream_begin (const char *fn)
{
    shmemi_init_check (fn);
    if (shmemi.heap == NULL)
        shmemi_fatal ("%s: no GPU (SHMEM_BOOTSTRAP_ONLY set?)", fn);
    shmemi_server_stop (); /* its grid and the stream-ordered ones need not fit together */
    shmemi_check_stream_err (fn);
}

static void stream_aset (const char *fn, struct aset *s, int PE_start, int logPE_stride, int PE_size)
{
    if (logPE_stride < 0 || logPE_stride > 30 || PE_size < 1 || PE_start < 0 ||
        PE_start + (long) (PE_size - 1) * (1L << logPE_stride) >= shmemi.npes)
        shmemi_fatal ("%s: active set (PE_start %d, logPE_stride %d, PE_size %d) outside the %d PEs",
                      fn, PE_start, logPE_stride, PE_size, shmemi.npes);
    s->start = PE_start;
    s->stride = 1 << logPE_stride;
    s->size = PE_size;
    s->me = -1;
    for (int i = 0; i < PE_size; ++i)
        if (aset_pe (s, i) == shmemi.mype)
            s->me = i;
    if (s->me < 0)
        shmemi_fatal ("%s: PE %d is not in the active set (PE_start %d, logPE_stride %d, PE_size %d)",
                      fn, shmemi.mype, PE_start, logPE_stride, PE_size);
    if (PE_size > MI355_FUSED_MAX_MEMBERS || shmemi.npes > MI355_SIG_RSDONE)
        shmemi_fatal ("%s: stream-ordered collectives take at most %d PEs per active set (of at most %d)",
                      fn, MI355_FUSED_MAX_MEMBERS, MI355_SIG_RSDONE);
    if (PE_size > 1 && (shmemi.sigmem == NULL || shmemi.p2p_broken || shmemi.sig_broken))
        shmemi_fatal ("%s: peer GPU memory failed the init self-test", fn);
}

static void stream_barrier (const char *fn, const struct aset *s, hipStream_t st)
{
    if (s->size < 2)
        return;
    MI355FusedArgs a;
    member_args (&a, s, SHMEMI_CHAN_STREAM);
    const int rc = mi355_device_barrier (&a, st);
    if (rc != 0)
        shmemi_fatal ("%s: device barrier launch failed: %d", fn, rc);
}

static void stream_copy (const char *fn, void *const *dsts, const void *const *srcs, const size_t *nb, int k,
                         hipStream_t st)
{
    for (int base = 0; base < k; base += 64) {
        const int m = k - base < 64 ? k - base : 64;
        const int rc = mi355_copy_segments (dsts + base, srcs + base, nb + base, m, st);
        if (rc != 0)
            shmemi_fatal ("%s: copy kernel launch failed: %d", fn, rc);
    }
}

static void reduce_on_stream (int op, int dtype, const char *fn, void *target, const void *source, int nreduce,
                              int PE_start, int logPE_stride, int PE_size, void *stream)
{
    hipStream_t st = (hipStream_t) stream;
    stream_begin (fn);
    struct aset s;
    stream_aset (fn, &s, PE_start, logPE_stride, PE_size);
    if (nreduce < 0)
        shmemi_fatal ("%s: nreduce %d < 0", fn, nreduce);
    const size_t es = mi355_dtype_size (dtype);
    const size_t n = (size_t) nreduce;
    const size_t nbytes = n * es;
    if (n > 0 && (target == NULL || source == NULL || !shmemi_in_device_heap (target, nbytes) ||
                  !shmemi_in_device_heap (source, nbytes)))
        shmemi_fatal ("%s: target and source must lie in the device symmetric heap (shmemx_malloc_device)", fn);
    if (n > 0 && target != source && ranges_overlap ((size_t) target, (size_t) source, nbytes))
        shmemi_fatal ("%s: target and source overlap without being equal", fn);
    if (shmemi.debug)
        debug_check (fn, op, dtype, target, source, nreduce, PE_start, logPE_stride, PE_size);

    if (n == 0) {
        begin_call ("barrier-only");
        stream_barrier (fn, &s, st);
    } else if (s.size == 1) {
        begin_call ("stream-identity");
        if (target != source) {
            void *d = target;
            const void *sv = source;
            stream_copy (fn, &d, &sv, &nbytes, 1, st);
            note_call (0, 1, 1, 0, (unsigned long long) nbytes, 0, 0, mi355_last_kernel ());
        }
    } else {
        const size_t dst_off = shmemi_heap_offset (target), src_off = shmemi_heap_offset (source);
        MI355FusedArgs a;
        member_args (&a, &s, SHMEMI_CHAN_STREAM);
        const int ordered = ordered_pair (op, dtype, s.size);
        if (order_sensitive (op, dtype, s.size) && !ordered)
            shmemi_fatal ("%s: %d PEs: the stream-ordered schedules deliver each PE's reference order up to %d "
                          "PEs (set SHMEM_REDUCE_ORDER=pe_start)", fn, s.size, MI355_ORDERS_MAX_SOURCES);
        if (n * es <= shmemi.fused_max && ((dst_off | src_off) & 15) == 0 && es <= 256 &&
            (!ordered || (size_t) (s.size - 1) * shard_chunk (n, es, s.size) * es <= shmemi.order_chunk)) {
            a.op = op;
            a.dtype = dtype;
            a.n = n;
            a.shard = shard_chunk (n, es, s.size);
            for (int i = 0; i < s.size; ++i) {
                a.src[i] = shmemi_peer_ptr (a.pe[i], src_off);
                a.dst[i] = shmemi_peer_ptr (a.pe[i], dst_off);
            }
            a.oneshot = n * es <= shmemi.oneshot_max && dst_off != src_off;
            fused_order (&a, &s, SHMEMI_CHAN_STREAM);
            const int rc = mi355_fused_allreduce (&a, st);
            if (rc != 0)
                shmemi_fatal ("%s: fused reduction launch failed: %d", fn, rc);
            begin_call (a.oneshot ? "stream-fused-oneshot" : "stream-fused-twoshot");
            note_fused (s.size, a.ordered, a.oneshot, n, es, mi355_last_kernel ());
        } else {
            void *dsts[MI355_FUSED_MAX_MEMBERS];
            const void *sp[MI355_FUSED_MAX_MEMBERS];
            size_t nb[MI355_FUSED_MAX_MEMBERS];
            const int pair = nan_pair (op, dtype, &s);
            const int ord = ordered && !pair;
            const size_t round = ord ? ordered_round_elems (es, s.size) : n;
            begin_call (n > round ? "stream-p2p-rounds" : "stream-p2p");
            for (size_t b = 0; b < n; b += round) {
                const size_t cn = n - b < round ? n - b : round;
                const size_t d0 = dst_off + b * es, s0 = src_off + b * es;
                const long long pk = pair ? pair_next (SHMEMI_CHAN_STREAM, &s) : -1;
                stream_barrier (fn, &s, st); /* every source is ready */
                shmemi_peer_acquire (st);
                const int rc = fold_shard (op, dtype, es, d0, s0, cn, &s, ord, pk, SHMEMI_CHAN_STREAM, st);
                if (rc != 0)
                    shmemi_fatal ("%s: combine kernel launch failed: %d", fn, rc);
                stream_barrier (fn, &s, st); /* every shard is reduced */
                shmemi_peer_acquire (st);
                if (pair) {
                    if (pair_gather (dtype, es, d0, s0, cn, &s, pk, SHMEMI_CHAN_STREAM, st) != 0)
                        shmemi_fatal ("%s: gather kernel launch failed", fn);
                } else {
                    const int k = gather_segments (es, d0, cn, &s, ord, SHMEMI_CHAN_STREAM, dsts, sp, nb);
                    stream_copy (fn, dsts, sp, nb, k, st);
                }
                stream_barrier (fn, &s, st); /* peers are done reading this target and version area */
            }
        }
    }
}

void shmemx_barrier_on_stream (int PE_start, int logPE_stride, int PE_size, void *stream)
{
    hipStream_t st = (hipStream_t) stream;
    stream_begin ("shmemx_barrier_on_stream");
    struct aset s;
    stream_aset ("shmemx_barrier_on_stream", &s, PE_start, logPE_stride, PE_size);
    stream_barrier ("shmemx_barrier_on_stream", &s, st);
}

/* ---------------------------------------------------------------------- */
/* the 44 entry points (reduce-op.c:388-448), pshmem_ strong, shmem_ weak  */
/* ---------------------------------------------------------------------- */
#define SHMEMI_REDUCE(Name, Op, Type, DT, OPC)                                                      \
    void pshmem_##Name##_##Op##_to_all (Type *target, Type *source, int nreduce, int PE_start,       \
                                        int logPE_stride, int PE_size, Type *pWrk, long *pSync)      \
    {                                                                                                \
        (void) pWrk; /* scratch lives in the device heap; pWrk is not touched */                   \
        reduce_impl (OPC, DT, "shmem_" #Name "_" #Op "_to_all", target, source, nreduce, PE_start,  \
                     logPE_stride, PE_size, pSync);                                                  \
    }                                                                                                \
    void shmemx_##Name##_##Op##_to_all_on_stream (Type *target, Type *source, int nreduce,           \
                                                  int PE_start, int logPE_stride, int PE_size,       \
                                                  Type *pWrk, long *pSync, void *stream)             \
    {                                                                                                \
        (void) pWrk;                                                                                 \
        (void) pSync;                                                                                \
        reduce_on_stream (OPC, DT, "shmemx_" #Name "_" #Op "_to_all_on_stream", target, source,     \
                          nreduce, PE_start, logPE_stride, PE_size, stream);                         \
    }                                                                                                \
    void shmem_##Name##_##Op##_to_all (Type *target, Type *source, int nreduce, int PE_start,        \
                                       int logPE_stride, int PE_size, Type *pWrk, long *pSync)       \
        __attribute__ ((weak, alias ("pshmem_" #Name "_" #Op "_to_all")));

#define SUMPROD(Name, Type, DT)                          \
    SHMEMI_REDUCE (Name, sum, Type, DT, MI355_OP_SUM)    \
    SHMEMI_REDUCE (Name, prod, Type, DT, MI355_OP_PROD)
#define LOGIC(Name, Type, DT)                            \
    SHMEMI_REDUCE (Name, and, Type, DT, MI355_OP_AND)    \
    SHMEMI_REDUCE (Name, or, Type, DT, MI355_OP_OR)      \
    SHMEMI_REDUCE (Name, xor, Type, DT, MI355_OP_XOR)
#define MINMAX(Name, Type, DT)                           \
    SHMEMI_REDUCE (Name, max, Type, DT, MI355_OP_MAX)    \
    SHMEMI_REDUCE (Name, min, Type, DT, MI355_OP_MIN)

SUMPROD (short, short, MI355_SHORT)
SUMPROD (int, int, MI355_INT)
SUMPROD (long, long, MI355_LONG)
SUMPROD (longlong, long long, MI355_LONGLONG)
SUMPROD (double, double, MI355_DOUBLE)
SUMPROD (float, float, MI355_FLOAT)
SUMPROD (longdouble, long double, MI355_LONGDOUBLE)
SUMPROD (complexd, double _Complex, MI355_COMPLEXD)
SUMPROD (complexf, float _Complex, MI355_COMPLEXF)
LOGIC (short, short, MI355_SHORT)
LOGIC (int, int, MI355_INT)
LOGIC (long, long, MI355_LONG)
LOGIC (longlong, long long, MI355_LONGLONG)
MINMAX (short, short, MI355_SHORT)
MINMAX (int, int, MI355_INT)
MINMAX (long, long, MI355_LONG)
MINMAX (longlong, long long, MI355_LONGLONG)
MINMAX (double, double, MI355_DOUBLE)
MINMAX (float, float, MI355_FLOAT)
MINMAX (longdouble, long double, MI355_LONGDOUBLE)
