/*
 * trace.c -- env-gated trace messages, the reference's logging facility
 * restated for this build ("Tracing / profiling").
 *
 * Reference: src/utils/trace.h:59-83 (levels), trace.c:227-243 (SHMEM_LOG_FILE,
 * appended, stderr otherwise), :266-301 (SHMEM_INFO/SMA_INFO -> "info",
 * SHMEM_VERSION/SMA_VERSION -> "init"), :304-321 (SHMEM_LOG_LEVELS: names
 * separated by , : or ;, "all"), :438-466 (line format
 * "[elapsed] PE n: LEVEL: message", one flushed write per line).
 *
 * Differences: always compiled in (the reference needs --enable-trace); a
 * disabled level costs one bit test at the call site (SHMEMI_TRACE); FATAL
 * messages keep going through shmemi_fatal, which aborts the whole job.
 */
#define _POSIX_C_SOURCE 200809L
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>
#include <time.h>

#include "shmemi.h"

unsigned shmemi_trace_mask;

static FILE *trace_out;
static double trace_t0;

static const char *const level_names[SHMEMI_LOG_NLEVELS] = {
    [SHMEMI_LOG_DEBUG] = "DEBUG",         [SHMEMI_LOG_INFO] = "INFO",
    [SHMEMI_LOG_VERSION] = "VERSION",     [SHMEMI_LOG_INIT] = "INIT",
    [SHMEMI_LOG_FINALIZE] = "FINALIZE",   [SHMEMI_LOG_BARRIER] = "BARRIER",
    [SHMEMI_LOG_BROADCAST] = "BROADCAST", [SHMEMI_LOG_REDUCTION] = "REDUCTION",
    [SHMEMI_LOG_COLLECT] = "COLLECT",     [SHMEMI_LOG_QUIET] = "QUIET",
    [SHMEMI_LOG_MEMORY] = "MEMORY",       [SHMEMI_LOG_NOTICE] = "NOTICE",
};

static double mono_s (void)
{
    struct timespec ts;
    clock_gettime (CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

static int env_set (const char *a, const char *b)
{
    return (getenv (a) != NULL) || (b != NULL && getenv (b) != NULL);
}

static void enable_name (const char *name)
{
    if (strcasecmp (name, "all") == 0) {
        shmemi_trace_mask = ~0u;
        return;
    }
    for (int l = 0; l < SHMEMI_LOG_NLEVELS; ++l)
        if (level_names[l] != NULL && strcasecmp (name, level_names[l]) == 0)
            shmemi_trace_mask |= 1u << l;
    /* unknown names are ignored, as in the reference (trace.c:304-321) */
}

void shmemi_trace_init (void)
{
    trace_t0 = mono_s ();
    shmemi_trace_mask = 0;
    if (env_set ("SHMEM_INFO", "SMA_INFO"))
        enable_name ("info");
    if (env_set ("SHMEM_VERSION", "SMA_VERSION"))
        enable_name ("init");
    const char *levels = getenv ("SHMEM_LOG_LEVELS");
    if (levels != NULL) {
        char buf[512];
        snprintf (buf, sizeof buf, "%s", levels);
        char *save = NULL;
        for (char *t = strtok_r (buf, ",:;", &save); t != NULL; t = strtok_r (NULL, ",:;", &save))
            enable_name (t);
    }
    trace_out = stderr;
    const char *file = getenv ("SHMEM_LOG_FILE");
    if (shmemi_trace_mask != 0 && file != NULL && *file != '\0') {
        FILE *f = fopen (file, "a");
        if (f != NULL)
            trace_out = f;
    }
}

void shmemi_trace_fini (void)
{
    if (trace_out != NULL && trace_out != stderr)
        fclose (trace_out);
    trace_out = NULL;
    shmemi_trace_mask = 0;
}

void shmemi_trace_emit (int level, const char *fmt, ...)
{
    char line[640];
    const int k = snprintf (line, sizeof line, "[%-8.6f] PE %d: %s: ", mono_s () - trace_t0, shmemi.mype,
                            level >= 0 && level < SHMEMI_LOG_NLEVELS && level_names[level] ? level_names[level]
                                                                                           : "?");
    va_list ap;
    va_start (ap, fmt);
    vsnprintf (line + k, sizeof line - (size_t) k - 1, fmt, ap);
    va_end (ap);
    strcat (line, "\n");
    FILE *out = trace_out != NULL ? trace_out : stderr;
    fputs (line, out); /* one write per line, flushed */
    fflush (out);
}

/* SHMEM_INFO: PE 0 lists the environment this build understands
 * (reference trace.c:335-372 does the same for its own variables). */
void shmemi_trace_show_info (void)
{
    if (shmemi.mype != 0 || !(shmemi_trace_mask & (1u << SHMEMI_LOG_INFO)))
        return;
    static const char *const vars[][2] = {
        {"{SHMEM,SMA}_VERSION", "print the library version (INIT trace)"},
        {"{SHMEM,SMA}_INFO", "print this list"},
        {"SHMEM_LOG_LEVELS", "trace levels to enable (names separated by , : ; or \"all\")"},
        {"SHMEM_LOG_FILE", "append trace lines to this file instead of stderr"},
        {"SHMEM_PE, SHMEM_NPES", "PE identity (else RANK/WORLD_SIZE, OMPI_COMM_WORLD_*, PMI_*)"},
        {"SHMEM_DEVICE", "GPU of this PE (else LOCAL_RANK, or the PE number)"},
        {"SHMEM_JOB_ID", "name of the node-local bootstrap segment"},
        {"SHMEM_DEVICE_HEAP_SIZE", "device symmetric heap per PE (default 2G)"},
        {"SHMEM_DEVICE_SCRATCH_SIZE", "staging/temporary scratch per PE (3 buffers)"},
        {"SHMEM_SYMMETRIC_HEAP_KIND", "\"device\": shmem_malloc returns device memory"},
        {"SHMEM_REDUCE_ALGORITHM", "auto | p2p | exact | rccl"},
        {"SHMEM_REDUCE_ORDER", "reference (each PE gets the reference's result for itself) | pe_start"},
        {"SHMEM_DEVICE_ORDER_SIZE", "version areas of the per-PE-order schedule (default 512M, 2 channels)"},
        {"SHMEM_FUSED_GRID_SHARE", "size the spin-waiting grids as if this many PEs shared the GPU"},
        {"SHMEM_PERSISTENT", "1: back-to-back fused calls served by a resident fused kernel (opt-in; shmemx.h)"},
        {"SHMEM_PERSISTENT_IDLE_US", "the persistent server leaves after this long without a call (default 1000)"},
        {"SHMEM_FUSED_MAX_BYTES", "largest message for the one-launch fused reduction (default 2M)"},
        {"SHMEM_DEVICE_WAITS", "1: keep device-side waits (fused kernel, device barriers) even where init finds them time-sliced; 0: host barriers"},
        {"SHMEM_ONESHOT_MAX_BYTES", "largest fused message folded one-shot, not reduce-scatter + all-gather (default 64K)"},
        {"SHMEM_BARRIER_TIMEOUT", "seconds before a barrier wait aborts the job (default 600)"},
        {"SHMEM_BOOTSTRAP_TIMEOUT", "seconds a PE waits at init for PE 0 to create the job's segment (default: "
                                    "SHMEM_BARRIER_TIMEOUT)"},
        {"SHMEM_DEBUG", "1: check pSync and exchange every collective's arguments between its members, aborting "
                        "with the first differing field"},
        {"SHMEM_ENTRY_SYNC", "1: every call starts with hipDeviceSynchronize"},
        {"SHMEM_EXTERNAL_MAP", "1 (default) / 0: peers map device buffers outside the heap for a call instead of "
                               "staging them through scratch"},
        {"SHMEM_EXTERNAL_MAP_CACHE", "peers' mapped allocations kept open (default 64, least recently used closed)"},
        {"SHMEM_PEER_ACQUIRE", "1/0: system-scope L2 acquire before reading peers' buffers (default: on if a peer is on another GPU)"},
    };
    shmemi_trace_emit (SHMEMI_LOG_INFO, "environment variables understood by this build:");
    for (size_t i = 0; i < sizeof vars / sizeof vars[0]; ++i)
        shmemi_trace_emit (SHMEMI_LOG_INFO, "%-28s %s", vars[i][0], vars[i][1]);
}

/* INIT: which levels are on (reference trace.c:398-425) */
void shmemi_trace_show_levels (void)
{
    if (!(shmemi_trace_mask & (1u << SHMEMI_LOG_INIT)))
        return;
    char buf[256] = "enabled messages:";
    for (int l = 0; l < SHMEMI_LOG_NLEVELS; ++l)
        if (level_names[l] != NULL && (shmemi_trace_mask & (1u << l))) {
            strncat (buf, " ", sizeof buf - strlen (buf) - 1);
            strncat (buf, level_names[l], sizeof buf - strlen (buf) - 1);
        }
    shmemi_trace_emit (SHMEMI_LOG_INIT, "%s", buf);
}
