/*
 * pdecode.h -- parallel BAM decode for the streamed CLI path (SURVEY §8
 * rows A1 and N1).
 *
 * The reference reads the BAM serially through htslib (my_samread,
 * GROM.c:981-992) on one thread per process.  This decoder splits the file
 * at record boundaries the BAI already names -- each reference's first/last
 * record offsets (pseudo-bin 37450) and the 16 kb linear index -- into pieces
 * of ~64k records that a pool of threads inflates and parses independently,
 * straight into pinned structure-of-arrays buffers.  One thread (the
 * caller's) takes the pieces in file order, applies the few order-dependent
 * facts (global CIGAR/base/aux offsets, read-name ids across piece borders,
 * the two records lost at each chromosome boundary) and appends
 * them to a device stage (grom_stage_append), so decode, host->device copies
 * and the scans of earlier chromosomes overlap.  The facts that need the
 * insert statistics (the walk's skip prefix, the last base reached, -S) are
 * applied when a chromosome is finished; the insert statistics themselves
 * (find_insert_mean, GROM.c:1205-1318) are accumulated from the same pieces
 * in file order.
 *
 * The serial stream semantics are kept exactly: which records each processed
 * chromosome's scan receives follows the reference's loop (GROM.c:5740,
 * 11075-11083, 14960-14976: Q1 and Q21), computed on the runs of records per
 * reference that the index counts.  If the index cannot support this (no
 * pseudo-bins, unsorted offsets) or a piece does not decode to exactly the
 * counted records, the session reports it and the CLI uses the serial reader.
 */
#ifndef GROM_AMD_PDECODE_H
#define GROM_AMD_PDECODE_H

#include <stdint.h>

#include "../../include/grom_amd.h"
#include "bamio.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pd_session pd_session;

/* per processed chromosome, in plan order */
typedef struct pd_chrom_in {
    int32_t tid;             /* BAM target (-1: none) */
    const char *target_name; /* the SA/XP chromosome test's name (GROM.c:1894-1961) */
    int64_t len;             /* its reference length (device mode reserves the stage's room for it) */
} pd_chrom_in;

/* what the serial stream gives one chromosome (grom_chrom's stream facts) */
typedef struct pd_chrom_facts {
    int64_t n_reads;   /* kept reads after the skip prefix */
    int64_t n_drop;
    int32_t n_skip, p_last, lseq_tail;
} pd_chrom_facts;

/* Open the streamed decoder on a BAM whose index supports it, for the
 * preliminary plan (every candidate chromosome; pd_set_walk gives the final
 * one).  Returns NULL with a reason in `why` when the index lacks what the
 * plan needs (the caller then reads serially). */
pd_session *pd_open(const char *bam_path, const bam_hdr *hdr, const pd_chrom_in *plan, int n_plan, int splitread,
                    int read_name_len, int n_threads, char *why, int why_len);
/* before pd_start: only the plan chromosomes with want[k] != 0 are decoded,
 * staged and handed out (GROM_CHROMS: one rank's share of the genome); the
 * others keep their place in the serial stream's plan (their records still
 * decide Q1/Q21 for the rest) but are skipped */
void pd_set_wanted(pd_session *s, const int *want);
/* before pd_start: decode on the GPUs (ddecode.hip: each device's worker
 * reads its chromosomes' compressed runs, inflates and parses them into the
 * stages) instead of the host decoder threads; same results, same API */
void pd_set_device_mode(pd_session *s, int on);
/* before pd_set_wanted / pd_start: GROM -P n semantics (GROM.c:21051-21064,
 * 549-599): every chromosome is given its own target's records as bam_fetch
 * returns them -- no records consumed by the chromosome before it (no Q1
 * drops), no starvation after an empty one (no Q21), its stream ending at its
 * own last record -- instead of the serial stream's */
void pd_set_fetch_mode(pd_session *s, int on);
/* device decode workers per GPU (GROM_DD_WORKERS, 1..8; default 1): the one
 * place that decides it (pd_start_device, the CLI's start-up thread) */
int pd_dd_workers(void);
/* device mode: each GPU's chromosomes are decoded longest first (plan order
 * among equal lengths); the caller takes them in that order */
int pd_device_mode(const pd_session *s);
/* start the decoder threads and the uploader.  dev_of[k]: the GPU of plan
 * chromosome k.  plan_only: no device; chromosomes go to host mirrors. */
int pd_start(pd_session *s, int min_mapq, int n_dev, const int *dev_of, int plan_only);
/* a stage the uploader may fill (the caller creates them per device) */
int pd_add_stage(pd_session *s, grom_stage *st, int device);
/* find_insert_mean's sample (GROM.c:1205-1318) as the pieces go by: blocks
 * until the first 10,000,000 qualifying records (or the file) have been
 * decoded; same outputs as grom_insert_stats.  Returns the mean, -1 if no
 * read qualified, -2 if the session failed. */
int pd_insert_stats(pd_session *s, double prob2, int min_mapq, int *lseq, int *imin, int *imax, long *mapped);
/* the walk's index start (cdp_one_base_index_start, GROM.c:2918), the facts
 * grom_batch_finish needs, and the final plan: keep[k] = 0 drops preliminary
 * chromosome k (the length test of find_disc_svs needs the insert size) */
/* before pd_start: the caller has the insert statistics (<bam>.mean, as the
 * reference's -c children load them, GROM.c:22253-22257); no statistics pass */
void pd_stats_given(pd_session *s);
void pd_set_walk(pd_session *s, int32_t index_start, int32_t overlap_mult, int32_t insert_max, const int *keep);
/* wait for plan chromosome k (kept, in order) to be staged and finalised:
 * 0 with its stage and facts; 1 if the index-based plan was contradicted by
 * the data (read serially instead); negative on failure (pd_error) */
int pd_wait_chrom(pd_session *s, int k, grom_stage **stage, pd_chrom_facts *facts);
/* the scan of a handed-out stage is done: the uploader may refill it */
void pd_release_stage(pd_session *s, grom_stage *st);
const char *pd_error(pd_session *s);
/* plan-only: the host mirror of chromosome k, in the serial reader's form */
int pd_mirror_view(pd_session *s, int k, grom_reads *out);

/* decode statistics: records parsed, pieces, bytes inflated, seconds in the
 * decoders (summed over threads) and in the uploader's fix-up/append loop */
typedef struct pd_counters {
    int64_t records, pieces, inflated_bytes, compressed_bytes, h2d_bytes;
    double decode_thread_s, inflate_s, upload_s, wait_s, io_s;
    int threads, libdeflate;
    int device;          /* runs decoded on the GPU (device mode) */
    int64_t rewalked, subchunks; /* device mode: record-walk sub-chunks re-walked / all */
    double gpu_ms[4];    /* device mode: inflate, record walk, parse (HIP events, summed); buffer growth (wall) */
    int64_t reclaimed;   /* idle stage blocks freed for allocations short of device memory */
    int dd_workers;      /* device mode: decode workers (all GPUs) */
    int64_t stats_only_runs; /* device mode: runs decoded for the insert statistics alone */
} pd_counters;
void pd_get_counters(pd_session *s, pd_counters *c);
void pd_close(pd_session *s);

/* GROM_TRACE=<path>: a host timeline of the streamed run (CSV: seconds since
 * the session opened, thread, event, two arguments), written by pd_close.
 * The CLI adds its own events (scan start/end per chromosome). */
enum {
    PD_EV_DECODE = 1,   /* a: piece, b: 0 start / 1 end */
    PD_EV_UPLOAD = 2,   /* a: piece, b: 0 start / 1 end */
    PD_EV_FINAL = 3,    /* a: chromosome */
    PD_EV_STATS = 4,    /* insert statistics complete */
    PD_EV_STAGE = 5,    /* a: chromosome, b: 0 wait start / 1 got / 2 made */
    PD_EV_SCAN = 6,     /* a: chromosome, b: 0 start / 1 end (CLI workers) */
    PD_EV_HANDED = 7,   /* a: chromosome handed to the scans (CLI) */
    PD_EV_PHASE = 8,    /* a: CLI phase id, b: 0 start / 1 end */
};
void pd_trace(pd_session *s, int ev, int64_t a, int64_t b);

/* a digest of one chromosome's read batch as the scan receives it (every
 * array, CIGAR/base/aux contents per read, the dropped records, and which
 * overlapping reads share a read name); used by the CPU tests to show the
 * streamed and the serial decoders hand the scan the same input */
uint64_t pd_digest(const grom_reads *r);

#ifdef __cplusplus
}
#endif
#endif
