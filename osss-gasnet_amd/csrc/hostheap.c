/*
 * hostheap.c -- shmem_malloc's symmetric heap in host memory.
 *
 * The reference's symmetric heap is one host segment per PE
 * (comms-inline.h:766-845: posix_memalign of SHMEM_SYMMETRIC_HEAP_SIZE bytes,
 * 32 MiB by default, comms-shared.h:82), carved by one allocator per PE
 * (memalloc.c:71-154, dlmalloc mspace): every PE makes the same sequence of
 * collective shmem_malloc calls, so a block has the same OFFSET in every PE's
 * segment, and a peer's copy of a symmetric object is that peer's segment
 * base + the offset (comms-inline.h:559-585, SHMEM_SYMMETRIC_HEAP_BASE(pe)).
 * shmem_getmem / putmem and the collectives reach peers' objects that way
 * (putget.c:249-256, broadcast-linear.c:61-82, fcollect-linear.c:60-93).
 *
 * Here (one node, one process per PE): each PE's segment is a POSIX
 * shared-memory object that every PE of the job maps at init, so a peer's
 * copy is plain host memory this process can read and write
 * (shmemi_host_peer_ptr). The names are dropped once every PE has mapped
 * every segment, so nothing outlives the job. The allocator is first fit
 * over page-aligned blocks, deterministic in the call sequence like the
 * reference's. Each allocated block is page-locked with hipHostRegister (the
 * reductions stage it over PCIe at full rate; their kernels may read and
 * write it directly), and the pages of a freed block are returned.
 * Space is committed at shmem_malloc (posix_fallocate), so a full /dev/shm
 * is a clear fatal error there, never a SIGBUS later.
 *
 * One PE: an anonymous mapping (nothing to share).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "shmemi.h"

struct shmemi_hostblk {
    size_t off, size;   /* in the segment; size rounded up to pages */
    int registered;
    char *dev;          /* device-accessible address of the block (registered), else NULL */
    struct shmemi_hostblk *next;  /* sorted by offset */
};

#define PAGE ((size_t) 4096)

static size_t page_up (size_t x) { return (x + PAGE - 1) / PAGE * PAGE; }

static void seg_name_of (int pe, char *out, size_t len)
{
    snprintf (out, len, "%s-h%d", shmemi.seg_name, pe);
}

/* This PE's segment of `size` bytes (virtual: pages are committed per block). */
void shmemi_hheap_create (size_t size)
{
    shmemi.hheap_size = page_up (size);
    shmemi.hheap_fd = -1;
    if (shmemi.npes > 1) {
        char name[160];
        seg_name_of (shmemi.mype, name, sizeof name);
        shm_unlink (name); /* a crashed job's leftover */
        const int fd = shm_open (name, O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0)
            shmemi_fatal ("shm_open(%s) for the symmetric host heap: %s", name, strerror (errno));
        if (ftruncate (fd, (off_t) shmemi.hheap_size) != 0)
            shmemi_fatal ("ftruncate(%s, %zu): %s (SHMEM_SYMMETRIC_HEAP_SIZE)", name, shmemi.hheap_size,
                          strerror (errno));
        void *p = mmap (NULL, shmemi.hheap_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        if (p == MAP_FAILED)
            shmemi_fatal ("mmap of the %zu-byte symmetric host heap: %s", shmemi.hheap_size, strerror (errno));
        shmemi.hheap = (char *) p;
        shmemi.hheap_fd = fd;
        shmemi.hheap_named = 1;
    } else {
        void *p = mmap (NULL, shmemi.hheap_size, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE,
                        -1, 0);
        if (p == MAP_FAILED)
            shmemi_fatal ("mmap of the %zu-byte symmetric host heap: %s", shmemi.hheap_size, strerror (errno));
        shmemi.hheap = (char *) p;
    }
}

/* After a barrier that follows every PE's shmemi_hheap_create: map every
 * peer's segment (the sizes agree: settings_check). */
void shmemi_hheap_attach (void)
{
    const int np = shmemi.npes;
    shmemi.peer_hheap = (char **) calloc ((size_t) np, sizeof (char *));
    if (shmemi.peer_hheap == NULL)
        shmemi_fatal ("out of host memory");
    shmemi.peer_hheap[shmemi.mype] = shmemi.hheap;
    for (int pe = 0; pe < np; ++pe) {
        if (pe == shmemi.mype)
            continue;
        char name[160];
        seg_name_of (pe, name, sizeof name);
        const int fd = shm_open (name, O_RDWR, 0600);
        if (fd < 0)
            shmemi_fatal ("shm_open(%s), PE %d's symmetric host heap: %s", name, pe, strerror (errno));
        struct stat st;
        if (fstat (fd, &st) != 0 || (size_t) st.st_size != shmemi.hheap_size)
            shmemi_fatal ("PE %d's symmetric host heap is not %zu bytes (SHMEM_SYMMETRIC_HEAP_SIZE)", pe,
                          shmemi.hheap_size);
        void *p = mmap (NULL, shmemi.hheap_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close (fd);
        if (p == MAP_FAILED)
            shmemi_fatal ("mmap of PE %d's symmetric host heap: %s", pe, strerror (errno));
        shmemi.peer_hheap[pe] = (char *) p;
    }
}

/* After a barrier that follows every PE's shmemi_hheap_attach. */
void shmemi_hheap_unlink (void)
{
    if (!shmemi.hheap_named)
        return;
    char name[160];
    seg_name_of (shmemi.mype, name, sizeof name);
    shm_unlink (name);
    shmemi.hheap_named = 0;
}

int shmemi_in_host_heap (const void *p, size_t nbytes)
{
    const char *c = (const char *) p;
    return shmemi.hheap != NULL && c >= shmemi.hheap && c - shmemi.hheap < (ptrdiff_t) shmemi.hheap_size &&
           nbytes <= shmemi.hheap_size - (size_t) (c - shmemi.hheap);
}

/* PE pe's copy of the symmetric host-heap object at p (this PE's address). */
void *shmemi_host_peer_ptr (int pe, const void *p)
{
    const size_t off = (size_t) ((const char *) p - shmemi.hheap);
    if (pe == shmemi.mype)
        return (void *) p;
    if (shmemi.peer_hheap == NULL || shmemi.peer_hheap[pe] == NULL)
        shmemi_fatal ("PE %d's symmetric host heap is not mapped here", pe);
    return shmemi.peer_hheap[pe] + off;
}

static void release_pages (size_t off, size_t size)
{
    if (shmemi.hheap_fd >= 0)
        (void) fallocate (shmemi.hheap_fd, FALLOC_FL_PUNCH_HOLE | FALLOC_FL_KEEP_SIZE, (off_t) off, (off_t) size);
    else
        (void) madvise (shmemi.hheap + off, size, MADV_DONTNEED);
}

/* First fit over the gaps between blocks, in offset order: the same call
 * sequence gives the same offsets on every PE (symmetric). */
void *shmemi_host_malloc (size_t size)
{
    if (size == 0)
        return NULL;
    const size_t need = page_up (size);
    size_t off = 0;
    struct shmemi_hostblk **pp = &shmemi.host_blocks;
    for (; *pp != NULL; pp = &(*pp)->next) {
        if ((*pp)->off - off >= need)
            break;
        off = (*pp)->off + (*pp)->size;
    }
    /* No room, or no pages to commit: NULL, as the reference's shmalloc
     * (symmem.c:150-153: a NOTICE trace, malloc_error set, the caller's
     * barrier still entered by pshmem_malloc). Every PE sees the same
     * exhaustion (same call sequence, same heap size); a full /dev/shm is
     * this PE's alone, and its caller's NULL check is the reference's. */
    if (need > shmemi.hheap_size - off) {
        SHMEMI_TRACE (SHMEMI_LOG_NOTICE, "shmem_malloc(%zu) failed: the symmetric host heap (%zu bytes) has no room "
                                         "left (SHMEM_SYMMETRIC_HEAP_SIZE)", size, shmemi.hheap_size);
        return NULL;
    }
    if (shmemi.hheap_fd >= 0) {
        const int e = posix_fallocate (shmemi.hheap_fd, (off_t) off, (off_t) need);
        if (e != 0) {
            SHMEMI_TRACE (SHMEMI_LOG_NOTICE, "shmem_malloc(%zu) failed: committing the symmetric host heap's pages: "
                                             "%s (is /dev/shm full?)", size, strerror (e));
            release_pages (off, need); /* whatever part was committed */
            return NULL;
        }
    }
    struct shmemi_hostblk *h = (struct shmemi_hostblk *) calloc (1, sizeof *h);
    if (h == NULL)
        shmemi_fatal ("out of host memory");
    h->off = off;
    h->size = need;
    char *p = shmemi.hheap + off;
    /* page-locked so the staging copies run at full PCIe rate */
    if (shmemi.device >= 0) {
        h->registered = hipHostRegister (p, need, hipHostRegisterDefault) == hipSuccess;
        void *d = NULL;
        if (h->registered && hipHostGetDevicePointer (&d, p, 0) == hipSuccess)
            h->dev = (char *) d;
        (void) hipGetLastError ();
    }
    h->next = *pp;
    *pp = h;
    return p;
}

static void free_block (struct shmemi_hostblk *h)
{
    if (h->registered)
        (void) hipHostUnregister (shmemi.hheap + h->off);
    release_pages (h->off, h->size);
    free (h);
}

/* 1 if p was a block of this heap (now freed), 0 if not this heap's */
int shmemi_host_free (void *p)
{
    for (struct shmemi_hostblk **pp = &shmemi.host_blocks; *pp != NULL; pp = &(*pp)->next) {
        if (shmemi.hheap + (*pp)->off == (char *) p) {
            struct shmemi_hostblk *h = *pp;
            *pp = h->next;
            free_block (h);
            return 1;
        }
    }
    return 0;
}

/* Device-accessible address of [p, p + nbytes) when it lies inside one
 * page-locked shmem_malloc block (kernels can then read and write it over
 * PCIe directly), else NULL. */
void *shmemi_host_dev_ptr (const void *p, size_t nbytes)
{
    const char *c = (const char *) p;
    for (const struct shmemi_hostblk *h = shmemi.host_blocks; h != NULL; h = h->next) {
        const char *b = shmemi.hheap + h->off;
        if (h->dev != NULL && c >= b && c + nbytes <= b + h->size)
            return h->dev + (c - b);
    }
    return NULL;
}

void shmemi_hheap_finalize (void)
{
    while (shmemi.host_blocks != NULL) {
        struct shmemi_hostblk *n = shmemi.host_blocks->next;
        free_block (shmemi.host_blocks);
        shmemi.host_blocks = n;
    }
    if (shmemi.peer_hheap != NULL) {
        for (int pe = 0; pe < shmemi.npes; ++pe)
            if (pe != shmemi.mype && shmemi.peer_hheap[pe] != NULL)
                munmap (shmemi.peer_hheap[pe], shmemi.hheap_size);
        free (shmemi.peer_hheap);
        shmemi.peer_hheap = NULL;
    }
    shmemi_hheap_unlink ();
    if (shmemi.hheap != NULL)
        munmap (shmemi.hheap, shmemi.hheap_size);
    if (shmemi.hheap_fd >= 0)
        close (shmemi.hheap_fd);
    shmemi.hheap = NULL;
    shmemi.hheap_fd = -1;
}
