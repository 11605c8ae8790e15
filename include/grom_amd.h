/*
 * grom_amd.h -- C ABI of the MI355X-native GROM per-chromosome scan.
 *
 * The reference has no library or FFI: its seam is the C function
 *
 *   void count_discordant_pairs(samfile_t*, char* bam_name, char* chr_fasta,
 *        long chr_len, char* chr_name, int chr_name_len, FILE* vcf, ...,
 *        FILE* ctx, int** sample_hi, ..., double* pval2sd_p, ...)   GROM.c:1432
 *
 * called once per chromosome by find_disc_svs (GROM.c:21057) with every
 * parameter in globals (GROM.c:710-979) and the BAM record stream positioned
 * where the previous chromosome left it.  This header replaces that seam:
 *
 *   - grom_params     <- the g_* globals the scan reads (set by main,
 *                        GROM.c:21907-22290)
 *   - grom_chrom      <- chr_fasta / chr_len / chr_name (GROM.c:1432 args 3-6)
 *                        plus the two facts of the serial record stream the
 *                        scan depends on (records skipped before the walk,
 *                        GROM.c:14859-14969, and the last base reached,
 *                        GROM.c:5842)
 *   - grom_reads      <- the records `my_samread` would return for this
 *                        chromosome (GROM.c:981-992), decoded into
 *                        structure-of-arrays form
 *   - grom_out        <- the VCF / CTX text the scan appends to its FILE*s
 *
 * Plain pointers and sizes only; no torch or HIP types cross the boundary.
 * Ownership: the caller owns every input and grom_out's buffers (grown with
 * realloc by the library); the library owns device memory between
 * grom_dev_init and grom_dev_fini.  Errors: negative return codes, message via
 * grom_last_error(); the library never calls exit().  Threading: one host
 * thread per device; calls on different devices may run concurrently.
 */
#ifndef GROM_AMD_H
#define GROM_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GROM_AMD_ABI_VERSION 7
#define GROM_MAX_TRIALS 1000 /* max_trials, GROM.c:631 */

enum {
    GROM_OK = 0,
    GROM_E_ARG = -1,      /* invalid argument / unsupported parameter value */
    GROM_E_HIP = -2,      /* HIP runtime failure */
    GROM_E_NOMEM = -3,    /* host or device allocation failed */
    GROM_E_NODEV = -4,    /* device not initialised */
    GROM_E_OVERFLOW = -5, /* a per-tile event buffer overflowed */
};

/* Every global the scan reads.  Names follow GROM.c's g_* variables. */
typedef struct grom_params {
    int32_t min_mapq;          /* g_min_mapq (-q), GROM.c:803 */
    int32_t rd_min_mapq;       /* g_rd_min_mapq (= -q, GROM.c:22102) */
    int32_t min_base_qual;     /* g_min_base_qual (-b), GROM.c:892 */
    int32_t min_snv;           /* g_min_snv (-n), GROM.c:891 */
    int32_t ploidy;            /* g_ploidy (-p) */
    int32_t gender;            /* g_gender (-g) */
    int32_t splitread;         /* g_splitread (-S clears) */
    int32_t rmdup;             /* g_rmdup (-M) */
    int32_t vcf;               /* g_vcf (-f clears) */
    int32_t overlap_mult;      /* g_overlap_mult (-l) */
    int32_t sv_list_len;       /* g_sv_list_len (-G) */
    int32_t rmdup_list_len;    /* g_rmdup_list_len, GROM.c:864 */
    int32_t read_name_len;     /* g_read_name_len, GROM.c:887 */
    int32_t sc_min;            /* g_sc_min, GROM.c:808 */
    double min_snv_ratio;      /* g_min_snv_ratio (-a), GROM.c:895 */
    double min_ave_bq;         /* g_min_ave_bq (-x), GROM.c:904 */
    double snv_rd_min_factor;  /* g_snv_rd_min_factor, GROM.c:906 */
    double high_cov_min_snv_ratio; /* g_high_cov_min_snv_ratio, GROM.c:907 */
    /* derived by main from the insert-size pre-pass, GROM.c:22255-22290 */
    int32_t insert_mean, insert_min_size, insert_max_size, lseq;
    int32_t one_base_rd_len;      /* full ring length (2 * half) */
    int32_t half_one_base_rd_len;
    int32_t r14_one_base_rd_len;  /* g_14_one_base_rd_len */
    int32_t r34_one_base_rd_len;  /* g_34_one_base_rd_len */
    /* read-depth CNV path (detect_del_dup and its callers) */
    int32_t ranks_stdev;          /* g_ranks_stdev (-K), GROM.c:925 */
    int32_t chr_rd_threshold_factor; /* g_chr_rd_threshold_factor (-U), GROM.c:737 */
    int64_t min_repeat;           /* g_min_repeat (-D), GROM.c:733 */
    int64_t min_blocks;           /* g_min_blocks (-Y), GROM.c:739 */
    int64_t block_min;            /* g_block_min (-Z), GROM.c:758 */
    int64_t min_rd_window_len;    /* g_min_rd_window_len (-W), GROM.c:931 */
    int64_t max_rd_window_len;    /* g_max_rd_window_len (-X), GROM.c:933 */
    int64_t windows_sampling_factor; /* g_windows_sampling_factor (-A), GROM.c:727 */
    int64_t dup_threshold_factor; /* g_dup_threshold_factor (-L), GROM.c:731 */
    double min_repeat_stdev;      /* g_min_repeat_stdev (-E), GROM.c:734 */
    double rd_pval_threshold;     /* g_rd_pval_threshold (-V), GROM.c:722 */
    double mapq_factor;           /* g_mapq_factor (-F), GROM.c:719 */
    /* breakpoint path (rows A8-A13), ABI 4 */
    int32_t min_disc;             /* g_min_disc (-d), GROM.c:810 */
    int32_t sc_range;             /* g_sc_range, GROM.c:812 */
    int32_t max_split_loss;       /* g_max_split_loss (-y), GROM.c:967 */
    int32_t min_sr_len;           /* g_min_sr_len (-z), GROM.c:969 */
    int32_t max_homopolymer;      /* g_max_homopolymer (-k), GROM.c:898 */
    int32_t max_ins_range;        /* g_max_ins_range (-w), GROM.c:899 */
    int32_t sv_list2_len;         /* g_sv_list2_len (-G sets it to G/10), GROM.c:831 */
    int32_t pad_sv;
    double pval_threshold;        /* g_pval_threshold (-v), GROM.c:942 */
    double pval_threshold1;       /* g_pval_threshold1 = g_pval_threshold, GROM.c:22101 */
    double pval_insertion1;       /* g_pval_insertion1, GROM.c:943 */
    double pval_insertion;        /* g_pval_insertion (-e), GROM.c:944 */
    double min_sv_ratio;          /* g_min_sv_ratio (-j), GROM.c:901 */
    double min_indel_ratio;       /* g_min_indel_ratio (-m), GROM.c:902 */
    double max_evidence_ratio;    /* g_max_evidence_ratio (-u), GROM.c:900 */
    double range_mult;            /* g_range_mult, GROM.c:828 */
    double max_inv_rd_diff;       /* g_max_inv_rd_diff, GROM.c:907 */
    double min_overlap_ratio;     /* g_min_overlap_ratio, GROM.c:817 */
    /* ABI 6 */
    int64_t gen1000_window;       /* g_1000gen_window (-N), GROM.c:746: the .1000gen side file when > 0 */
} grom_params;

/* One chromosome.  `ref` holds exactly what find_disc_svs loaded
 * (GROM.c:21009-21045), `name` the lower-cased FASTA name it passes. */
typedef struct grom_chrom {
    const char *ref;
    int64_t len;
    const char *name;
    int32_t tid;        /* BAM target id of the records below */
    int32_t n_skip;     /* stream records with pos < index_start, skipped
                           before the per-base walk (GROM.c:14859-14969) */
    int32_t p_last;     /* last base the walk reaches (the base at which the
                           chromosome's final record is ingested), or -1 if
                           the walk never ingests a record */
    int32_t cnv;        /* 1: run the read-depth CNV path (the reference runs it
                           when the FASTA name matched a BAM target) */
    uint32_t seed;      /* CNV sampling seed: replaces srand(time()) at
                           GROM.c:1584 */
    int32_t lseq_tail;  /* cdp_lseq when the walk evaluates p_last: l_qseq of
                           the record that ended the chromosome's stream, or
                           at end of file the last record's (plus its hard
                           clips when it was ingested).  The breakpoint tests
                           read the pending record's length (GROM.c:12047) */
    int32_t pad;
} grom_chrom;

/* The SA:Z / XP:Z alignment of a read as GROM parses it (GROM.c:5763-5826,
 * 6683-6733): only when the record's aux block is 1..99 bytes, and under -S
 * only for records not fetched inside the ingest loop. */
typedef struct grom_aux {
    int32_t pos;            /* as written in the tag (1-based, kept as is) */
    int32_t start_adj;      /* leading 'S' of its CIGAR */
    int32_t end_adj;        /* trailing 'S' */
    int32_t end_adj_indel;  /* sum I - sum D */
    int16_t mq;             /* atoi of the mapq field */
    uint8_t strand;         /* 0 '+', 1 otherwise */
    uint8_t same_chr;       /* strncmp(target_name, tag_chr, strlen(target_name)) == 0 */
    int32_t pad;
} grom_aux;

/* The records the chromosome's scan ingests (stream order, after the serial
 * stream's boundary drops and the n_skip prefix), minus records flagged
 * unmapped or duplicate, which the ingest body ignores (GROM.c:6418).
 * seq is BAM 4-bit packed; read i's bases start at nibble base_off[i]
 * (always even) and its qualities at qual[base_off[i]]. */
typedef struct grom_reads {
    int64_t n;
    int64_t n_cigar_ops;  /* length of cigar[] */
    int64_t n_bases;      /* length of qual[] (seq[] holds n_bases/2 bytes) */
    const int32_t *pos;
    const uint16_t *flag;
    const uint8_t *mapq;
    const int32_t *mtid;
    const int32_t *mpos;
    const int32_t *isize;
    const int32_t *l_qseq;
    const uint32_t *cigar_off;  /* n+1 prefix offsets into cigar[] */
    const uint32_t *cigar;      /* BAM-encoded ops (len<<4 | op) */
    const int64_t *base_off;
    const uint8_t *seq;
    const uint8_t *qual;
    const uint32_t *name_id;    /* equal ids <=> equal read names; 0 = a
                                   name that is never stored (len >= 50) */
    /* ABI 4: split-read alignments: aux_idx[i] indexes aux[] or is -1 */
    int64_t n_aux;
    const int32_t *aux_idx;
    const grom_aux *aux;
    /* ABI 4: the records of the stream dropped from the arrays above
     * (unmapped / duplicate flag): position, l_qseq, and how many kept
     * reads precede each in stream order.  The breakpoint tests read the
     * length of the next record in the stream (GROM.c:12047). */
    int64_t n_drop;
    const int32_t *drop_pos;
    const int32_t *drop_lq;
    const int64_t *drop_before;
} grom_reads;

/* Growable output text (the two FILE*s of count_discordant_pairs). */
typedef struct grom_out {
    char *vcf;
    size_t vcf_len, vcf_cap;
    char *ctx;
    size_t ctx_len, ctx_cap;
    /* ABI 6: the chromosome's <results>.1000gen.<chr> side file (-N,
     * GROM.c:20234-20345), written whenever its CNV pass ran and -N > 0 */
    char *side;
    size_t side_len, side_cap;
    int32_t side_written, side_pad;
} grom_out;

/* Per-chromosome run statistics (for benchmarks / logs). */
typedef struct grom_stats {
    double ms_total;        /* device time of the whole scan */
    double ms_pileup;       /* device time of the SNV pileup/evaluation kernel */
    double ms_cnv;          /* device time of the CNV kernels */
    int64_t cnv_rows;       /* <DEL>/<DUP> rows written */
    int64_t bases_evaluated;
    int64_t snv_candidates;
    int64_t mismatch_events;
} grom_stats;

int grom_abi_version(void);
/* number of visible GPUs (hipGetDeviceCount); 0 if none */
int grom_device_count(void);
/* sizeof of the ABI structs, for bindings to check their layout:
 * 0 grom_params, 1 grom_chrom, 2 grom_reads, 3 grom_out, 4 grom_stats,
 * 5 grom_indel_rec, 6 grom_aux, 7 grom_sv_rec */
size_t grom_abi_struct_size(int which);
/* The message of the last failing call made FROM THE CALLING HOST THREAD
 * (errors are kept per thread, since contexts run concurrently).
 * grom_cli_main copies the first failing worker's message into the caller's
 * thread before it returns. */
const char *grom_last_error(void);
/* Set the calling thread's error text (used by the CLI to hand a worker's
 * failure to its caller). */
void grom_set_last_error(const char *msg);
/* Free device memory in bytes (hipMemGetInfo), or -1. */
int64_t grom_device_mem_free(int device);

/* Initialise `device`: upload the two binomial tables (each
 * (GROM_MAX_TRIALS+1)^2 doubles, row-major: g_hez_prob_binom_cdf_table and
 * g_mq_prob_binom_cdf_table, GROM.c:780-783) and the parameters. */
int grom_dev_init(int device, const grom_params *params, const double *hez_table, const double *mq_table);
/* A scan context in `slot` (0..63) on physical `device`.  Every entry point
 * below takes a slot: grom_dev_init(d, ...) is grom_ctx_init(d, d, ...).
 * Several slots may share one GPU; each has its own stream and scratch, so
 * scans in different slots run concurrently when called from different host
 * threads (two chromosomes in flight per GPU).  Device-resident reads from
 * grom_upload in one slot may be scanned from another slot on the same GPU. */
int grom_ctx_init(int slot, int device, const grom_params *params, const double *hez_table, const double *mq_table);
/* replace an initialised context's parameters (e.g. once the insert statistics
 * are known: the CLI creates its contexts while the BAM's head is decoded) */
int grom_ctx_set_params(int slot, const grom_params *params);
void grom_dev_fini(int device);

/* Scan one chromosome whose reads are in host memory; appends its VCF rows to
 * out->vcf (the rows count_discordant_pairs writes for that chromosome). */
int grom_scan_chrom(int device, const grom_chrom *chrom, const grom_reads *reads, grom_out *out, grom_stats *stats);

/* Same, with every grom_reads pointer (and chrom->ref) already in device
 * memory of `device`.  Used to time the scan with inputs resident in HBM.
 * qual and seq must be 16-byte aligned and readable up to the next 16-byte
 * boundary past their end (the kernel copies them in 16-byte words);
 * grom_upload guarantees both. */
int grom_scan_chrom_device(int device, const grom_chrom *chrom, const grom_reads *dev_reads, grom_out *out,
                           grom_stats *stats);

/* Test hook: per-base counters of every evaluated base p (p > 2*insert_max and
 * p <= chrom->p_last), NCOUNT int32 per base in the order of the reference's
 * declarations (see grom_amd/csrc/scan_common.h), plus the three
 * whole-chromosome read-depth arrays (3 * len int32).  Buffers are caller
 * owned: counts must hold (p_last - first + 1) * GROM_NCOUNT int32. */
#define GROM_NCOUNT 40
int grom_debug_counts(int device, const grom_chrom *chrom, const grom_reads *reads, int32_t *first_pos,
                      int32_t *counts, int64_t counts_cap, int32_t *caf3);

/* CIGAR indel evidence of one evaluated base (row A7; replaces the reference's
 * cdp_one_base_indel_* ring arrays, GROM.c:7187-7423): primary insertion,
 * forward-deletion and reverse-deletion counters (+6 per MAPQ >= -q read, 0
 * otherwise) with their lengths, the deletion read depths, the number of
 * occupied "other" slots as the evaluation counts them (GROM.c:11415-11425;
 * the slots are shared with the breakpoint clusters) and the 50-byte inserted-sequence
 * buffer (zero-filled when the base enters the window). */
typedef struct grom_indel_rec {
    int32_t pos;
    int32_t ins, ins_len;
    int32_t del_f, del_f_len, del_f_rd;
    int32_t del_r, del_r_len, del_r_rd;
    int32_t other_len;
    char ins_seq[52];
    int32_t pad;
} grom_indel_rec;

/* Test hook: the indel evidence records of the last scan on `device` (one per
 * evaluated base that a CIGAR I/D op or a split-read deletion reached, in
 * position order).  Copies at
 * most `cap` records to `out` (may be NULL with cap 0) and returns how many
 * the scan produced, or a negative GROM_E_* code. */
int64_t grom_debug_indels(int device, grom_indel_rec *out, int64_t cap);

/* Breakpoint cluster state of one evaluated base (rows A8/A9; replaces the
 * reference's cdp_one_base_{del,dup,inv,ctx}_* ring arrays and the "other"
 * slots, GROM.c:7431-10953) as the per-base tests see it: per cluster type
 * (DEL_F, DEL_R, DUP_F, DUP_R, INV_F1, INV_R1, INV_F2, INV_R2, CTX_F, CTX_R)
 * the weighted count, running-mean distance (the mate position for CTX) and
 * first/last read positions; the CTX mate chromosomes; the number of
 * occupied "other" slots; and the order-free range sums at the base: depth
 * adds, concordant pairs, short-insert pairs and unmapped-mate reads. */
typedef struct grom_sv_rec {
    int32_t pos, other_len;
    int32_t cnt[10], rs[10], re[10];
    double dist[10];
    int32_t ctx_mchr[2];
    int32_t rd_add, conc, ins, mun_f, mun_r, pad;
} grom_sv_rec;

/* Test hook: the breakpoint records of the last scan on `device`: one per
 * evaluated base with a nonzero cluster count or an occupied "other" slot,
 * in position order; same calling convention as grom_debug_indels.  Needs the
 * scan to run with GROM_SV_DEBUG set in the environment. */
int64_t grom_debug_sv(int device, grom_sv_rec *out, int64_t cap);

/* Host helpers shared by the CLI and the tests (grom_amd/csrc/tables.c):
 * the tables exactly as a run with -q min_mapq uses them. */
void grom_build_tables(int32_t min_mapq, double *hez_table, double *mq_table);
void grom_default_params(grom_params *p);
/* derive insert-dependent window sizes (GROM.c:22260-22290) */
void grom_params_set_insert(grom_params *p, int32_t insert_mean, int32_t insert_min, int32_t insert_max,
                            int32_t lseq);

void grom_out_free(grom_out *out);

/* Test hook: checks the VCF writer's exact "%.2f" conversion against printf
 * on n pseudo-random integer ratios (plus edge cases); returns mismatches. */
int64_t grom_fmt_selftest(int64_t n, uint64_t seed);

/* Copy a host chromosome + reads into library-owned device buffers of
 * `device` and return device-side views of them (valid until the next upload
 * or grom_dev_fini).  Lets callers time grom_scan_chrom_device with the inputs
 * already resident in HBM. */
int grom_upload(int device, const grom_chrom *chrom, const grom_reads *reads, grom_chrom *dev_chrom,
                grom_reads *dev_reads);

/* A device-resident copy of one chromosome's inputs in a single allocation
 * the library makes on physical `device` (not owned by any context), so a
 * caller can keep a whole genome in HBM and scan any chromosome from any slot
 * on that device.  Fills *dev_chrom / *dev_reads with device views (valid
 * until grom_resident_free).  NULL on failure (grom_last_error). */
typedef struct grom_resident grom_resident;
grom_resident *grom_resident_new(int device, const grom_chrom *chrom, const grom_reads *reads, grom_chrom *dev_chrom,
                                 grom_reads *dev_reads);
int64_t grom_resident_bytes(const grom_resident *r);
void grom_resident_free(grom_resident *r);

/* ---- streamed input (ABI 5) ----
 * The reference pulls records one at a time from htslib into its ring
 * (my_samread, GROM.c:981-992; the reader thread GROM.c:82-324).  Here a
 * caller decodes pieces of a chromosome (runs of consecutive records) into
 * PINNED host memory (grom_pinned_alloc) in grom_reads form and appends them
 * to a stage: every append is a set of async host->device copies on the
 * stage's own stream, so a decoder refills one piece while the previous one
 * is in flight and a chromosome's copies overlap the scan of the one before
 * it (which runs on a context's stream).  A piece's offsets must already be
 * global for the chromosome: cigar_off (n+1 entries) and base_off count from
 * the start of the chromosome's arrays, aux_idx indexes its aux array,
 * drop_before counts every kept read appended before (the stage concatenates
 * pieces as given).  n_bases must be even (every read starts on a byte). */
typedef struct grom_stage grom_stage;
typedef struct grom_stage_sizes {
    int64_t n, n_cigar_ops, n_bases, n_aux, n_drop, ref_len; /* capacity hints */
} grom_stage_sizes;
void *grom_pinned_alloc(size_t bytes); /* page-locked host memory, NULL on failure */
void grom_pinned_free(void *p);
grom_stage *grom_stage_new(int device);
void grom_stage_free(grom_stage *s);
/* start a new chromosome (waits for the stage's previous copies; the caller
 * must not reuse a stage whose scan is still running); est may be NULL */
int grom_stage_begin(grom_stage *s, const grom_stage_sizes *est);
/* async upload of the chromosome's reference bases (host memory) */
int grom_stage_set_ref(grom_stage *s, const char *ref, int64_t len);
/* append one piece; returns a ticket >= 0 (or a negative GROM_E_* code).
 * The piece's host memory may be reused once grom_stage_ticket_done returns 1
 * or grom_stage_ticket_wait returns. */
int64_t grom_stage_append(grom_stage *s, const grom_reads *piece);
int grom_stage_ticket_done(grom_stage *s, int64_t ticket);
int grom_stage_ticket_wait(grom_stage *s, int64_t ticket);
/* views start after the first n_front appended reads (the walk's skip prefix,
 * known once the insert statistics are): cigar_off/base_off/aux_idx stay
 * absolute, drop_before must count kept reads after the trim */
int grom_stage_trim(grom_stage *s, int64_t n_front);
/* give appended read `read_index` (counted before any trim) the split-read
 * alignment *aux (the one record -S still parses) */
int grom_stage_patch_aux(grom_stage *s, int64_t read_index, const grom_aux *aux);
/* host->device bytes issued for the current chromosome */
int64_t grom_stage_bytes(const grom_stage *s);
/* device views of the staged chromosome (chrom->len must equal the staged
 * reference); the arrays stay valid until the next grom_stage_begin */
int grom_stage_view(grom_stage *s, const grom_chrom *chrom, grom_chrom *dev_chrom, grom_reads *dev_reads);
/* scan the staged chromosome from context `slot` (same device): the scan's
 * stream waits for the stage's copies; chrom->ref is the HOST copy of the
 * reference (the breakpoint rows read it) */
int grom_scan_chrom_staged(int slot, grom_stage *s, const grom_chrom *chrom, grom_out *out, grom_stats *stats);
/* grom_debug_counts on a staged chromosome */
int grom_debug_counts_staged(int slot, grom_stage *s, const grom_chrom *chrom, int32_t *first_pos, int32_t *counts,
                             int64_t counts_cap, int32_t *caf3);

/* main's translocation post-pass (GROM.c:22400-22770) over the raw CTX rows
 * of every chromosome (grom_out.ctx of each scan, concatenated in chromosome
 * order): pairs each breakpoint with its mate row, drops the weaker of two
 * nearby pairs and appends the BND rows of .ctx.vcf (no header) to out->ctx.
 * target_names: the BAM header's target names (the mate chromosome ids index
 * them).  Used by the CLI and by a multi-rank caller on rank 0. */
int grom_ctx_postpass(const char *raw, size_t raw_len, const char *const *target_names, int32_t n_targets,
                      int32_t insert_max, int32_t lseq, grom_out *out);

/* The drop-in command line (GROM's main, GROM.c:21865) as a library call:
 * argv as for `GROM -i BAM -r FASTA -o OUT [options]`; returns the exit code.
 * The `grom` executable is a wrapper around it. */
int grom_cli_main(int argc, char **argv);

/* ---- host conveniences for tests and benchmarks (grom_amd/csrc/hostapi.c) ---- */
typedef struct grom_batch_handle grom_batch_handle;

/* Generate one synthetic chromosome (grom_amd/csrc/synth.c) and the read
 * batch its scan ingests.  Insert statistics are measured on the generated
 * pairs exactly as find_insert_mean does (GROM.c:1205-1318) and written into
 * *params (with grom_params_set_insert); *params must hold the other options. */
grom_batch_handle *grom_synth_batch(int64_t chr_len, double coverage, int32_t read_len, double insert_mean,
                                    double insert_sd, uint64_t seed, grom_params *params);
/* One chromosome of a multi-chromosome synthetic genome (the BASELINE
 * configs[2]-[4] shapes: human-like contig lengths and names, breakpoint SVs
 * with split reads and discordant pairs, copy-number regions, PCR duplicates,
 * a ploidy other than 2).  Chromosome `chrom` is generated exactly as the
 * genome's BAM would hold it (grom_synth), and turned into the batch its scan
 * ingests with tid = chrom and the chromosome's own name.  When
 * params->half_one_base_rd_len is already set, the insert statistics are kept
 * (one genome-wide find_insert_mean, as the reference runs it once per BAM);
 * otherwise they are measured on this chromosome's pairs first. */
typedef struct grom_synth_spec {
    int32_t n_chr;
    int32_t chrom;             /* the chromosome to generate, 0..n_chr-1 */
    const int64_t *chr_len;    /* n_chr lengths */
    const char *names;         /* comma-separated names, NULL: chr1..chrN */
    double coverage;
    int32_t read_len;
    int32_t ploidy;            /* donor haplotypes (0 = 2) */
    double insert_mean, insert_sd;
    double dup_frac;           /* fragments emitted twice (the -M filter's work) */
    double sv_per_mb;          /* breakpoint SVs per Mb (DEL/DUP/INV/INS/CTX) */
    double cnv_rate;           /* copy-number regions per base */
    int64_t cnv_min, cnv_max;  /* their length range (0: 10 kb - 300 kb) */
    const double *chr_cov;     /* per-chromosome depth (n_chr), NULL: coverage
                                  everywhere (a male genome halves chrX/chrY) */
    double munmap_frac;        /* pairs with an unmapped mate */
    uint64_t seed;
} grom_synth_spec;
grom_batch_handle *grom_synth_chrom(const grom_synth_spec *spec, grom_params *params);
/* ABI 7: chromosome `chrom` as its scan sees it inside the whole genome's BAM
 * (grom_synth's file, every chromosome processed in order, as the CLI's
 * serial-stream plan gives it): the previous chromosome's loop consumed its
 * first two records (GROM.c:5740, 14960-14976), and lseq_tail is
 * the next chromosome's first record's length (GROM.c:12047).  The insert
 * statistics must already be set in *params.  bench.py scans these resident
 * and compares the rows with the CLI's whole run over the BAM. */
grom_batch_handle *grom_synth_chrom_stream(const grom_synth_spec *spec, grom_params *params);
/* ABI 7: the digest the CLI's plan-only mode prints for a chromosome's input
 * (every array, CIGAR/base/quality/SA-XP contents, dropped records, which
 * overlapping reads share a name id); host arrays.  Test helper. */
uint64_t grom_reads_digest(const grom_reads *reads);
/* views into the handle (valid until grom_batch_release) */
int grom_batch_get(grom_batch_handle *h, grom_chrom *chrom, grom_reads *reads);
void grom_batch_release(grom_batch_handle *h);

/* ---- BAM index (replaces htslib's bam_index_build / bam_index_load /
 * bam_fetch, GROM.c:216-261 and 22128-22138; SAM v1 section 5.2) ---- */
/* index <bam> into <bam>.bai: 0, or negative */
int grom_bai_build(const char *bam_path);
/* parse an index file; out = {n_ref, bins, chunks, linear intervals,
 * unplaced-read count or -1 when absent}.  0, or negative */
int grom_bai_summary(const char *bai_path, int64_t out[5]);
/* n_queries seeded random regions of <bam> fetched through <bam>.bai and by a
 * full scan: the number of regions whose record sets differ (0 = all equal),
 * negative on error.  *visited gets the records the fetches returned. */
int64_t grom_bai_selftest(const char *bam_path, int64_t n_queries, uint64_t seed, int64_t *visited);

#ifdef __cplusplus
}
#endif
#endif
