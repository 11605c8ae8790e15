/*
 * stream.h -- host front end: FASTA index/load, insert-size pre-pass, and the
 * serial BAM record stream split into per-chromosome read batches.
 *
 * The reference reads one shared `samfile_t` serially (GROM.c:20471,
 * 5740-14976); which records each chromosome's scan sees depends on that
 * stream (two records lost at each chromosome boundary; a
 * processed chromosome with no reads swallowing the rest of the file, Q21).
 * `grom_batch_plan` reproduces that consumption while decoding the file once,
 * so every chromosome can be scanned independently (and on any GPU) with the
 * records the serial run would have given it.
 */
#ifndef GROM_AMD_STREAM_H
#define GROM_AMD_STREAM_H

#include <stdint.h>
#include <stdio.h>

#include "../../include/grom_amd.h"
#include "bamio.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GROM_MAX_CHR_NAMES 30000 /* max_chr_names, GROM.c:45 */
#define GROM_MAX_CHR_NAME_LEN 50 /* max_chr_name_len, GROM.c:638 */

typedef struct grom_fasta {
    FILE *fh;
    int n;                 /* g_chr_names_index */
    char (*names)[GROM_MAX_CHR_NAME_LEN];
    int *name_len;
    long *file_pos;
    long *len;
    long mappable;         /* g_mappable_genome_length */
    int loader_line_len;   /* state carried across loads (GROM.c:21014-21029) */
    int loader_alpha_len;
} grom_fasta;

int grom_fasta_open(grom_fasta *f, const char *path); /* find_genome_length */
/* the CLI's open: the <fasta>.info cache when it loads (load_genome_info),
 * else grom_fasta_open + save_genome_info (GROM.c:22308-22311) */
int grom_fasta_open_cached(grom_fasta *f, const char *path);
void grom_fasta_close(grom_fasta *f);
/* load chromosome `i` into buf (capacity cap); returns its length */
long grom_fasta_load(grom_fasta *f, int i, char *buf, long cap);
/* the same load without the shared stream (thread-safe, pread + memchr);
 * -2 when the chromosome holds a NUL byte (use grom_fasta_load), -1 on error */
long grom_fasta_load_at(const grom_fasta *f, int i, char *buf, long cap);
/* lengths of chromosomes idx[0..n) (grom_fasta_load_at) on up to `threads`
 * threads; -1 if any failed (out[k] < 0 for those) */
int grom_fasta_lengths(const grom_fasta *f, const int *idx, int n, long *out, int threads);

/* FASTA index of a BAM target under find_disc_svs' name rules
 * (GROM.c:20898-20975), -1 if none */
int grom_match_target(const grom_fasta *f, const char *target_name);
/* lower-cased, trimmed BAM target name (GROM.c:20893-20906); returns length */
int grom_target_name_lc(const char *target, char *out, int cap);

/* find_insert_mean (GROM.c:1205-1318) on an already-open stream positioned
 * after the header; returns the insert mean, fills lseq/min/max. */
int grom_insert_stats(bgzf_reader *r, double prob2, int *lseq, int *imin, int *imax, long *mapped_reads,
                      int min_mapq);
/* ascending sort of n ints (O(n) radix; same result as qsort) */
void grom_sort_ints(int *a, int64_t n);
/* g_prob2 of calculate_normal_binom_constants for `-s num_sd` */
double grom_prob2(double num_sd);

/* A growable host batch of one chromosome's ingested reads. */
typedef struct grom_batch {
    int32_t tid;
    int32_t n_skip;
    int32_t p_last;
    int32_t last_pos;
    int64_t n, cap;
    int64_t n_cig, cap_cig;
    int64_t n_bases, cap_bases;
    int32_t *pos;
    uint16_t *flag;
    uint8_t *mapq;
    int32_t *mtid, *mpos, *isize, *l_qseq;
    uint32_t *cigar_off, *cigar;
    int64_t *base_off;
    uint8_t *seq, *qual;
    uint32_t *name_id;
    /* read-name interning */
    /* open-addressing table: name offset into the arena (+1, 0 = empty),
     * its 64-bit hash and id */
    int64_t *nkeys;
    uint64_t *nhash;
    uint32_t *nids;
    int64_t ncap, nn;
    char *narena;          /* NUL-terminated names, appended */
    int64_t narena_len, narena_cap;
    int32_t max_ref_span;  /* max over reads of the M/D/N/=/X extent */
    int read_name_len;
    int any_ingested;
    /* split-read alignments (SA:Z / XP:Z) of the kept reads */
    int32_t *aux_idx;
    grom_aux *aux;
    int64_t n_aux, cap_aux;
    /* records dropped by the flag filter (unmapped / duplicate) */
    int32_t *drop_pos, *drop_lq;
    int64_t *drop_before;
    int64_t n_drop, cap_drop;
    int32_t lseq_tail;     /* grom_chrom.lseq_tail */
    const char *target_name; /* BAM name of the chromosome (the SA chromosome test) */
    int splitread;         /* g_splitread: -S gates the ingest-loop fetch only */
    int n_seen, prev_skipped;
} grom_batch;

void grom_batch_init(grom_batch *b, int32_t tid, int read_name_len);
/* the chromosome's BAM target name and -S (before the first add) */
void grom_batch_set_sv(grom_batch *b, const char *target_name, int splitread);
/* the record of another chromosome that ends this one's stream (its length
 * is what the walk's last evaluated base sees) */
void grom_batch_end_record(grom_batch *b, const bam_rec *r);
/* GROM's SA/XP parse of one record (GROM.c:5763-5826, 6683-6733); returns 1
 * and fills *out when the record carries one it would read */
int grom_parse_aux(const bam_rec *r, const char *target_name, grom_aux *out);
void grom_batch_free(grom_batch *b);
/* feed one record of this chromosome's stream (in stream order) */
void grom_batch_add(grom_batch *b, const bam_rec *r, int32_t index_start);
/* finish: compute p_last (GROM.c:5842, 6406-6412) */
void grom_batch_finish(grom_batch *b, int32_t index_start, int32_t overlap_mult, int32_t insert_max);
/* view as the C-ABI struct (pointers alias the batch) */
void grom_batch_view(const grom_batch *b, grom_reads *out);

/* Serial-stream planner.  Given processed target ids in processing order, it
 * is fed every record of the file in order and tells which processed
 * chromosome's stream (index into `order`) the record belongs to, or -1. */
typedef struct grom_planner {
    const int32_t *order;
    int n_order;
    int k;          /* current processed chromosome */
    int state;      /* 0: seeking its first record, 1: inside, 2: dropping */
    int drop_left;
    int eof_all;
} grom_planner;

void grom_planner_init(grom_planner *p, const int32_t *order, int n_order);
int grom_planner_feed(grom_planner *p, int32_t tid);

#ifdef __cplusplus
}
#endif
#endif
