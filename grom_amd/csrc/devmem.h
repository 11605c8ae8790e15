/* devmem.h -- device memory of the library: every buffer the scan contexts,
 * stages and the BAM decoder grow is allocated here.
 *
 * One process per GPU holds a few large buffers per chromosome in flight
 * (DESIGN.md 3 and 8).  An allocation that fails does not fail the run at
 * once: it first frees idle memory (reclaim hooks: e.g. the blocks of stages
 * no chromosome holds), then waits for memory this process releases (a scan
 * giving its stage back) or another process releases (the previous run's
 * memory, cleared by the driver after it exits), and retries, for up to
 * GROM_ALLOC_WAIT_S seconds (default 60).
 *
 * GROM_TEST_HBM_CAP=<bytes> (test hook) makes every allocation that would
 * take this process's accounted device memory above the cap fail, so the
 * reclaim and wait path runs on a small case. */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { GROM_DEVCAT_SCAN, GROM_DEVCAT_SV, GROM_DEVCAT_CNV, GROM_DEVCAT_STAGE, GROM_DEVCAT_DECODE, GROM_DEVCAT_ARENA,
       GROM_DEVCAT_OTHER, GROM_DEVCAT_N };

/* hipMalloc on the calling thread's device, accounted under `cat`, with the
 * reclaim / wait / retry path above; 0 or -1 (the memory did not come free) */
int grom_dev_malloc(void **p, size_t bytes, int cat);
/* hipFree + accounting; wakes allocations that wait */
void grom_dev_free(void *p, size_t bytes, int cat);
/* memory of this process may have come free (a stage given back): wake waiters */
void grom_dev_release_notify(void);

/* reclaim hook: free idle memory on `device`, return the bytes freed */
typedef int64_t (*grom_reclaim_fn)(void *arg, int device, size_t want);
void grom_dev_add_reclaim(grom_reclaim_fn fn, void *arg);
void grom_dev_remove_reclaim(grom_reclaim_fn fn, void *arg);

/* A phase arena: one device block that a scan context's transient buffers of
 * one phase are carved from, reused by the next phase.  The pileup and
 * breakpoint phase (per-read records, event sorts, range sums) and the CNV
 * phase (window means, classification words, walk links) never live at the
 * same time, so a context holds the larger of the two instead of their sum.
 * grom_arena_begin starts a phase (everything taken before is dead; the
 * caller has waited for the kernels that used it), first growing the block
 * to the largest phase seen so far; take is thread-safe (the CNV kinds grow
 * their buffers from two threads). */
typedef struct grom_arena grom_arena;
grom_arena *grom_arena_new(int cat);
void grom_arena_free(grom_arena *a);
int grom_arena_begin(grom_arena *a);
/* bytes of the current phase (256-aligned), or NULL when the block is full:
 * the caller then allocates on its own (grom_dev_malloc) and the arena grows
 * to hold it at the next begin */
void *grom_arena_take(grom_arena *a, size_t bytes);
/* grom_arena_hint: the next grom_arena_begin sizes the arena for at least
 * this many bytes (an estimate of the phase to come; a phase that needs more
 * overflows into allocations of its own, and the arena grows after it). */
void grom_arena_hint(grom_arena *a, size_t bytes);
int64_t grom_arena_bytes(const grom_arena *a);

/* accounting only (allocations made elsewhere) */
void grom_dev_note(int cat, int64_t delta);
/* peak[k] / now[k] for k < GROM_DEVCAT_N, [GROM_DEVCAT_N] = their sum */
void grom_dev_peaks(int64_t *peak, int64_t *now);
/* allocations that waited, and the seconds they waited */
void grom_dev_waits(int64_t *n, double *secs);
/* hipMalloc calls that took over 0.1 s (each is also logged to stderr) */
void grom_dev_slow(int64_t *n, double *secs);

#ifdef __cplusplus
}
#endif
