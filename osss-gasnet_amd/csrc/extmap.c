/*
 * extmap.c -- *_to_all on device buffers outside the symmetric heap without
 * staging copies.
 *
 * The reference reduces symmetric objects only (src/reduce/reduce-op.c:
 * 179-276 fetches `source` at the same address on every PE). A framework's
 * tensors (hipMalloc / a caching allocator's segments) are device memory
 * the peers have not mapped; staged through the heap's scratch buffers they
 * cost two extra local copies and a host barrier per scratch chunk (N = 2 on
 * one GPU, 256 MiB: 673 us against 218 us for heap buffers,
 * profiles/r03/external_buffers_before_n2.jsonl; mapped: 222 us,
 * profiles/r03/external_buffers.jsonl). Here the members of the call
 * instead:
 *   1. export the allocation holding each of their buffers (hipIpcGetMemHandle
 *      of its base, cached per allocation) and publish handle + offset in the
 *      bootstrap segment;
 *   2. pass one host barrier (a member passing host memory, which stages
 *      anyway, publishes a record that says so and only arrives);
 *   3. read every member's record. All members read the same records and
 *      take the same decision: map when every member could export both
 *      buffers, passed the same kinds of memory, 16-byte aligned, no partial
 *      overlap of target and source; otherwise every member stages as before;
 *   4. open the peers' handles (cached per (PE, handle): a reallocated buffer
 *      gets a new handle, hip_runtime_api.h hipIpcGetMemHandle) and run the
 *      heap schedules on virtual offsets (shmemi.h SHMEMI_EXT_*), which
 *      shmemi_peer_ptr turns into each member's real address.
 * A member cannot leave the call before every member has read the records
 * (each member's result needs every member's source, which a member offers
 * only after reading them), so one barrier suffices: the next call may
 * rewrite the record.
 *   5. opening a peer's handle can fail: HIP refuses the handle of an
 *      allocation its owner has since freed ("invalid device pointer", HIP
 *      logging "IPC Attach: Invalid IPC handle"), and once in round 3's
 *      random stress an open failed on live buffers. Round 3 blamed re-opening
 *      a handle whose every importer had closed it; the deterministic probe
 *      (tools/ipc_reopen_probe.py, profiles/r04/ipc_reopen_probe.json) refutes
 *      that: a live allocation's handle re-opens after every close (3,000
 *      open/close cycles, no file descriptor growth on either side), a
 *      re-export returns the same handle bytes, and a buffer freed and
 *      allocated again at the same address gets new bytes (so no cached
 *      mapping goes stale). The round-3 failure stays unexplained, so the
 *      guard stays: after opening, the members publish whether they opened
 *      everything and pass a second barrier; if one did not, every member
 *      stages this call and drops its cached exports of the call's buffers,
 *      and the next call maps again (tests/test_gpu_multipe.py
 *      test_external_buffer_open_failure_recovers).
 *
 * Imported mappings hold the peer's memory alive; the cache keeps at most
 * SHMEM_EXTERNAL_MAP_CACHE of them (default 64, least recently used closed
 * first), shmemx_external_map_flush closes them all. SHMEM_EXTERNAL_MAP=0
 * turns the mapping off (staging, as before).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "shmemi.h"
#include "shmemx.h"

/* this call's per-member addresses: [0] target, [1] source */
static char **tab[2];
static int active;
static const char *call_fn = "";

/* exports of this PE's allocations */
struct export {
    void *base;
    size_t size;
    unsigned long long id;
    hipIpcMemHandle_t h;
    unsigned long long tick;
};
#define N_EXPORTS 16
static struct export exports[N_EXPORTS];
static int n_exports;

/* peers' allocations mapped here */
struct import {
    int pe;
    hipIpcMemHandle_t h;
    char *base;
    unsigned long long tick;
};
static struct import *imports;
static int n_imports, cap_imports;
static long n_fallbacks; /* calls staged because a member could not open a peer's handle */
static unsigned long long tick;
static long n_opened, n_closed, n_open_failed;
static int cache_limit; /* SHMEM_EXTERNAL_MAP_CACHE */

static int export_of (const void *p, size_t nbytes, hipIpcMemHandle_t *h, uint64_t *off)
{
    hipDeviceptr_t base = NULL;
    size_t size = 0;
    if (hipMemGetAddressRange (&base, &size, (hipDeviceptr_t) p) != hipSuccess || base == NULL) {
        (void) hipGetLastError ();
        return 0;
    }
    if ((const char *) p + nbytes > (const char *) base + size)
        return 0;
    /* a buffer freed and allocated again at the same address has a new id */
    unsigned long long id = 0;
    if (hipPointerGetAttribute (&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t) p) != hipSuccess) {
        (void) hipGetLastError ();
        id = 0;
    }
    *off = (uint64_t) ((const char *) p - (const char *) base);
    int lru = 0;
    for (int i = 0; i < n_exports; ++i) {
        if (exports[i].base == base && exports[i].size == size && exports[i].id == id && id != 0) {
            exports[i].tick = ++tick;
            *h = exports[i].h;
            return 1;
        }
        if (exports[i].tick < exports[lru].tick)
            lru = i;
    }
    hipIpcMemHandle_t nh;
    if (hipIpcGetMemHandle (&nh, base) != hipSuccess) {
        (void) hipGetLastError ();
        return 0; /* e.g. virtual-memory (hipMemCreate) allocations */
    }
    const int slot = n_exports < N_EXPORTS ? n_exports++ : lru;
    exports[slot] = (struct export) {base, size, id, nh, ++tick};
    *h = nh;
    return 1;
}

static void import_close (int i)
{
    (void) hipIpcCloseMemHandle (imports[i].base);
    (void) hipGetLastError ();
    imports[i] = imports[--n_imports];
    ++n_closed;
}

/* The mapped base of PE pe's allocation with handle h; entries used by the
 * current call (tick >= first) are never evicted for it. */
static char *import_of (int pe, const hipIpcMemHandle_t *h, unsigned long long first)
{
    for (int i = 0; i < n_imports; ++i)
        if (imports[i].pe == pe && memcmp (&imports[i].h, h, sizeof *h) == 0) {
            imports[i].tick = ++tick;
            return imports[i].base;
        }
    if (cache_limit == 0) {
        const char *v = getenv ("SHMEM_EXTERNAL_MAP_CACHE");
        cache_limit = v != NULL && atoi (v) > 0 ? atoi (v) : 64;
    }
    const int limit = cache_limit;
    while (n_imports >= limit) {
        int lru = -1;
        for (int i = 0; i < n_imports; ++i)
            if (imports[i].tick < first && (lru < 0 || imports[i].tick < imports[lru].tick))
                lru = i;
        if (lru < 0)
            break; /* every entry serves this call: grow past the limit */
        /* the calls that used it have completed (blocking), and nothing else
         * reads a call's mappings */
        import_close (lru);
    }
    if (n_imports == cap_imports) {
        const int nc = cap_imports ? 2 * cap_imports : 16;
        struct import *ni = (struct import *) realloc (imports, sizeof *ni * (size_t) nc);
        if (ni == NULL)
            shmemi_fatal ("out of host memory");
        imports = ni;
        cap_imports = nc;
    }
    void *p = NULL;
    /* SHMEM_TEST_IPC_FAIL=extopen: PE 1 cannot open peers' buffers;
     * =extopen1: only its first open fails (tests) */
    const char *fail = shmemi.mype == 1 ? getenv ("SHMEM_TEST_IPC_FAIL") : NULL;
    static int failed_once;
    const int simulate = fail != NULL && (strcmp (fail, "extopen") == 0 ||
                                          (strcmp (fail, "extopen1") == 0 && !failed_once++));
    const hipError_t e = simulate ? hipErrorInvalidDevicePointer
                                  : hipIpcOpenMemHandle (&p, *h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
        (void) hipGetLastError ();
        ++n_open_failed;
        SHMEMI_TRACE (SHMEMI_LOG_REDUCTION, "%s: mapping PE %d's device buffer failed (%s): the call stages",
                      call_fn, pe, hipGetErrorString (e));
        return NULL;
    }
    imports[n_imports++] = (struct import) {pe, *h, (char *) p, ++tick};
    ++n_opened;
    return (char *) p;
}

int shmemi_ext_begin (const char *fn, void *target, const void *source, size_t nbytes, int kt, int ks, int PE_start,
                      int stride, int PE_size, size_t *toff, size_t *soff)
{
    if (!shmemi.ext_map || shmemi.seg == NULL || PE_size < 2)
        return 0;
    call_fn = fn;
    const int same = target == source;
    struct shmemi_ext_rec r;
    memset (&r, 0, sizeof r);
    r.same = same;
    r.tkind = kt;
    r.skind = ks;
    if (kt == SHMEMI_PK_HOST || ks == SHMEMI_PK_HOST) {
        /* host memory is staged whatever the peers pass: say so and go on
         * (the members that wait for the records see this one) */
        shmemi_seg_info (shmemi.mype)->ext = r;
        atomic_thread_fence (memory_order_release);
        shmemi_barrier_arrive (PE_start, stride, PE_size);
        return 0;
    }
    const char *t = (const char *) target, *s = (const char *) source;
    int ok = ((((uintptr_t) t) | ((uintptr_t) s)) & 15) == 0 && (same || t + nbytes <= s || s + nbytes <= t);
    if (ok)
        ok = kt == SHMEMI_PK_DEV_SYM ? (r.toff = shmemi_heap_offset (target), 1)
                                     : export_of (target, nbytes, &r.th, &r.toff);
    if (ok) {
        if (same) {
            r.sh = r.th;
            r.soff = r.toff;
        } else {
            ok = ks == SHMEMI_PK_DEV_SYM ? (r.soff = shmemi_heap_offset (source), 1)
                                         : export_of (source, nbytes, &r.sh, &r.soff);
        }
    }
    r.ok = ok;
    shmemi_seg_info (shmemi.mype)->ext = r;
    atomic_thread_fence (memory_order_release);
    shmemi_barrier_set (PE_start, stride, PE_size);
    atomic_thread_fence (memory_order_acquire);

    /* the same decision on every member: from the same records */
    struct shmemi_ext_rec *rec = (struct shmemi_ext_rec *) malloc (sizeof *rec * (size_t) PE_size);
    if (rec == NULL)
        shmemi_fatal ("out of host memory");
    int all = 1;
    for (int i = 0; i < PE_size; ++i) {
        rec[i] = shmemi_seg_info (PE_start + i * stride)->ext;
        all &= rec[i].ok && rec[i].same == same && rec[i].tkind == kt && rec[i].skind == ks &&
               (kt != SHMEMI_PK_DEV_SYM || rec[i].toff == r.toff) && (ks != SHMEMI_PK_DEV_SYM || rec[i].soff == r.soff);
    }
    if (!all) {
        free (rec);
        return 0;
    }
    for (int w = 0; w < 2; ++w)
        if (tab[w] == NULL && (tab[w] = (char **) calloc ((size_t) shmemi.npes, sizeof (char *))) == NULL)
            shmemi_fatal ("out of host memory");
    const unsigned long long first = tick + 1;
    int opened = 1;
    for (int i = 0; i < PE_size; ++i) {
        const int pe = PE_start + i * stride;
        if (pe == shmemi.mype) {
            tab[0][pe] = (char *) target;
            tab[1][pe] = (char *) source;
            continue;
        }
        char *tb = kt == SHMEMI_PK_DEV_OTHER ? import_of (pe, &rec[i].th, first) : NULL;
        char *sb = ks == SHMEMI_PK_DEV_OTHER && !same ? import_of (pe, &rec[i].sh, first) : NULL;
        if ((kt == SHMEMI_PK_DEV_OTHER && tb == NULL) || (ks == SHMEMI_PK_DEV_OTHER && !same && sb == NULL))
            opened = 0;
        tab[0][pe] = tb != NULL ? tb + rec[i].toff : NULL;
        tab[1][pe] = same ? tab[0][pe] : sb != NULL ? sb + rec[i].soff : NULL;
    }
    free (rec);
    /* second round: did every member open everything? (the same answer on
     * every member, read after the barrier from the same records) */
    shmemi_seg_info (shmemi.mype)->ext.open_ok = opened;
    atomic_thread_fence (memory_order_release);
    shmemi_barrier_set (PE_start, stride, PE_size);
    atomic_thread_fence (memory_order_acquire);
    int all_opened = 1;
    for (int i = 0; i < PE_size; ++i)
        all_opened &= shmemi_seg_info (PE_start + i * stride)->ext.open_ok;
    if (!all_opened) {
        /* stage this call; export this call's buffers afresh next time */
        for (int i = 0; i < n_exports; ++i)
            if ((kt == SHMEMI_PK_DEV_OTHER && memcmp (&exports[i].h, &r.th, sizeof r.th) == 0) ||
                (ks == SHMEMI_PK_DEV_OTHER && memcmp (&exports[i].h, &r.sh, sizeof r.sh) == 0)) {
                exports[i] = exports[--n_exports];
                --i;
            }
        ++n_fallbacks;
        return 0;
    }
    *toff = kt == SHMEMI_PK_DEV_SYM ? r.toff : SHMEMI_EXT_TARGET;
    *soff = ks == SHMEMI_PK_DEV_SYM ? r.soff : same ? SHMEMI_EXT_TARGET : SHMEMI_EXT_SOURCE;
    active = 1;
    return 1;
}

void shmemi_ext_end (void) { active = 0; }

void *shmemi_ext_ptr (int pe, size_t off)
{
    const int w = off >= SHMEMI_EXT_SOURCE;
    if (!active || tab[w] == NULL || tab[w][pe] == NULL)
        shmemi_fatal ("internal: virtual offset %#zx of a mapped device buffer used outside its call (PE %d)", off,
                      pe);
    return tab[w][pe] + (off - (w ? SHMEMI_EXT_SOURCE : SHMEMI_EXT_TARGET));
}

void shmemi_ext_finalize (void)
{
    while (n_imports > 0)
        import_close (n_imports - 1);
    free (imports);
    imports = NULL;
    cap_imports = 0;
    n_exports = 0;
    for (int w = 0; w < 2; ++w) {
        free (tab[w]);
        tab[w] = NULL;
    }
    active = 0;
}

void shmemx_external_map_flush (void)
{
    shmemi_init_check ("shmemx_external_map_flush");
    while (n_imports > 0)
        import_close (n_imports - 1);
    n_exports = 0;
}

long shmemx_external_map_fallbacks (void) { return n_fallbacks; }

void shmemx_external_map_stats (long *mapped, long *opened, long *closed)
{
    if (mapped != NULL)
        *mapped = n_imports;
    if (opened != NULL)
        *opened = n_opened;
    if (closed != NULL)
        *closed = n_closed;
}
