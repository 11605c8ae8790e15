/*
 * tools/gromc_binding.c -- the GROM.c-side binding of INTEGRATION.md §2,
 * compiled as written, inside a minimal stand-in for GROM's main and
 * find_disc_svs loop.
 *
 * The block between the BEGIN/END markers is the stub a GROM maintainer adds
 * to src/GROM.c; tests/test_gpu_parity.py::test_integration_stub checks that
 * INTEGRATION.md shows exactly this text and that this program's rows equal
 * grom_cli_main's on the same files.  Everything outside the markers plays
 * GROM's part:
 *   - the g_* globals the stub reads, with GROM.c's defaults (GROM.c:710-979)
 *     and the options that set them (main's getopt, GROM.c:21908-22103);
 *   - find_insert_mean and the insert-derived window sizes (GROM.c:22255-22290);
 *   - find_disc_svs' chromosome loop over the serial record stream
 *     (GROM.c:20826-21065), with the library's host stream helpers
 *     (grom_amd/csrc/stream.h) standing in for htslib + count_discordant_pairs'
 *     own record loop;
 *   - main's translocation post-pass (GROM.c:22400-22770) via grom_ctx_postpass.
 * It writes only the rows (no VCF header): OUT gets the VCF rows of every
 * chromosome in order, OUT.ctx.vcf the BND rows.
 *
 *   gromc_binding -i BAM -r FASTA -o OUT [GROM options]
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "../grom_amd/csrc/bamio.h"
#include "../grom_amd/csrc/stream.h"

/* ---- GROM's globals the binding reads (names and defaults of GROM.c) ---- */
int g_min_mapq = 20;                 /* GROM.c:803 */
int g_rd_min_mapq = 20;              /* GROM.c:917, = g_min_mapq (GROM.c:22102) */
int g_min_base_qual = 20;            /* GROM.c:892 */
int g_min_snv = 3;                   /* GROM.c:891 */
int g_ploidy = 2;                    /* GROM.c:918 */
int g_gender = 0;                    /* GROM.c:916 */
int g_splitread = 1;                 /* GROM.c:852 */
int g_rmdup = 0;                     /* GROM.c:853 */
int g_vcf = 1;                       /* GROM.c:813 */
int g_overlap_mult = 1;              /* GROM.c:845 */
int g_sv_list_len = 1000000;         /* GROM.c:841 */
int g_sv_list2_len = 100000;         /* GROM.c:842 */
double g_min_snv_ratio = 0.2;        /* GROM.c:895 */
double g_min_ave_bq = 15;            /* GROM.c:904 */
int g_ranks_stdev = 1;               /* GROM.c:925 */
int g_chr_rd_threshold_factor = 2;   /* GROM.c:737 */
long g_min_repeat = 20;              /* GROM.c:733 */
long g_min_blocks = 4;               /* GROM.c:739 */
long g_block_min = 10000;            /* GROM.c:758 */
long g_min_rd_window_len = 100;      /* GROM.c:931 */
long g_max_rd_window_len = 10000;    /* GROM.c:933 */
long g_windows_sampling_factor = 2;  /* GROM.c:727 */
long g_dup_threshold_factor = 2;     /* GROM.c:731 */
double g_min_repeat_stdev = 1.5;     /* GROM.c:734 */
double g_rd_pval_threshold = 0.000000001; /* GROM.c:722 */
double g_mapq_factor = 0.5;          /* GROM.c:719 */
long g_1000gen_window = 0;           /* GROM.c:746 */
int g_min_disc = 3;                  /* GROM.c:810 */
int g_max_split_loss = 20;           /* GROM.c:967 */
int g_min_sr_len = 30;               /* GROM.c:969 */
int g_max_homopolymer = 10;          /* GROM.c:898 */
int g_max_ins_range = 10;            /* GROM.c:899 */
double g_pval_threshold = 0.001;     /* GROM.c:942 */
double g_pval_threshold1 = 0.01;     /* GROM.c:941, = g_pval_threshold (GROM.c:22101) */
double g_pval_insertion = 0.0000000001; /* GROM.c:944 */
double g_min_sv_ratio = 0.05;        /* GROM.c:901 */
double g_min_indel_ratio = 0.125;    /* GROM.c:902 */
double g_max_evidence_ratio = 0.25;  /* GROM.c:900 */
int g_insert_mean, g_insert_min_size, g_insert_max_size, g_lseq; /* GROM.c:956, 834, 831 */

/* ---- BEGIN INTEGRATION.md §2 stub ---- */
#include "grom_amd.h"

static int g_dev = 0;                          /* one host thread per device */

/* once, after main() has parsed options and run find_insert_mean (GROM.c:22255) */
static void grom_gpu_init(void) {
    grom_params p;
    grom_default_params(&p);           /* GROM's fixed constants (g_sc_min, g_read_name_len, ...) */
    p.min_mapq = g_min_mapq;           p.rd_min_mapq = g_rd_min_mapq;
    p.min_base_qual = g_min_base_qual; p.min_snv = g_min_snv;
    p.ploidy = g_ploidy;               p.gender = g_gender;
    p.splitread = g_splitread;         p.rmdup = g_rmdup;         p.vcf = g_vcf;
    p.overlap_mult = g_overlap_mult;   p.sv_list_len = g_sv_list_len;  p.sv_list2_len = g_sv_list2_len;
    p.min_snv_ratio = g_min_snv_ratio; p.min_ave_bq = g_min_ave_bq;
    /* read-depth CNV path (detect_del_dup and its callers), -N side file */
    p.ranks_stdev = g_ranks_stdev;       p.chr_rd_threshold_factor = g_chr_rd_threshold_factor;
    p.min_repeat = g_min_repeat;         p.min_blocks = g_min_blocks;   p.block_min = g_block_min;
    p.min_rd_window_len = g_min_rd_window_len;  p.max_rd_window_len = g_max_rd_window_len;
    p.windows_sampling_factor = g_windows_sampling_factor;
    p.dup_threshold_factor = g_dup_threshold_factor;
    p.min_repeat_stdev = g_min_repeat_stdev;    p.rd_pval_threshold = g_rd_pval_threshold;
    p.mapq_factor = g_mapq_factor;              p.gen1000_window = g_1000gen_window;
    /* breakpoint path (-d -y -z -k -w -v -e -j -m -u) */
    p.min_disc = g_min_disc;             p.max_split_loss = g_max_split_loss;
    p.min_sr_len = g_min_sr_len;         p.max_homopolymer = g_max_homopolymer;
    p.max_ins_range = g_max_ins_range;   p.pval_threshold = g_pval_threshold;
    p.pval_threshold1 = g_pval_threshold1;  p.pval_insertion = g_pval_insertion;
    p.min_sv_ratio = g_min_sv_ratio;     p.min_indel_ratio = g_min_indel_ratio;
    p.max_evidence_ratio = g_max_evidence_ratio;
    /* the insert-derived window sizes, as main derives them (GROM.c:22260-22290) */
    grom_params_set_insert(&p, g_insert_mean, g_insert_min_size, g_insert_max_size, g_lseq);
    static double hez[(GROM_MAX_TRIALS + 1) * (GROM_MAX_TRIALS + 1)];
    static double mq[(GROM_MAX_TRIALS + 1) * (GROM_MAX_TRIALS + 1)];
    /* the tables GROM reads from its %e text files (GROM.c:21345-21373) */
    grom_build_tables(g_min_mapq, hez, mq);
    if (grom_dev_init(g_dev, &p, hez, mq) != GROM_OK) {
        printf("%s\n", grom_last_error());
        exit(1);
    }
}

/* what srand() gets at GROM.c:1584 (GROM_SEED pins it, as the CLI does) */
static uint32_t grom_cnv_seed(void) {
    const char *e = getenv("GROM_SEED");
    return e ? (uint32_t)strtoul(e, NULL, 10) : (uint32_t)time(NULL);
}

/* in find_disc_svs, instead of count_discordant_pairs(...) (GROM.c:21057) */
static void grom_gpu_scan(const char *fasta, long len, const char *name, int tid,
                          const grom_reads *reads,   /* SoA view of this chromosome's records */
                          int32_t n_skip, int32_t p_last, int32_t lseq_tail,
                          FILE *vcf, FILE *ctx_raw) {
    /* cnv: GROM runs detect_del_dup when cdp_chr_match != -1 (GROM.c:16633);
     * lseq_tail: cdp_lseq when the walk evaluates p_last (GROM.c:12047) */
    grom_chrom c = { fasta, len, name, tid, n_skip, p_last, tid >= 0, grom_cnv_seed(), lseq_tail, 0 };
    grom_out out = { 0 };
    grom_stats st;
    if (grom_scan_chrom(g_dev, &c, reads, &out, &st) != GROM_OK) {
        printf("%s\n", grom_last_error());
        exit(1);
    }
    fwrite(out.vcf, 1, out.vcf_len, vcf);
    /* raw CTX rows: main pairs them after the last chromosome (GROM.c:22400-22770) */
    if (out.ctx_len) fwrite(out.ctx, 1, out.ctx_len, ctx_raw);
    grom_out_free(&out);
}
/* ---- END INTEGRATION.md §2 stub ---- */

/* ---------------- GROM's part (test harness) ---------------- */
typedef struct {
    int fasta_idx, tid;
    long len;
    char name[GROM_MAX_CHR_NAME_LEN + 1];
    char *target;
} chrom_t;

int main(int argc, char **argv) {
    const char *bam_name = NULL, *fasta_name = NULL, *out_name = NULL;
    double num_sd = 3; /* g_insert_num_st_devs, GROM.c:805 */
    int opt;
    /* main's getopt string (GROM.c:21908); options of the orchestration are accepted and ignored */
    while ((opt = getopt(argc, argv,
                         "Z:W:X:Q:A:Y:B:D:E:K:N:V:U:L:F:SP:c:R:MG:i:r:o:p:q:s:v:g:l:d:b:n:a:y:z:e:fj:k:m:u:w:x:h")) != -1) {
        switch (opt) {
        case 'S': g_splitread = 0; break;
        case 'G': g_sv_list_len = atoi(optarg); g_sv_list2_len = g_sv_list_len / 10; break;
        case 'M': g_rmdup = 1; break;
        case 'i': bam_name = optarg; break;
        case 'r': fasta_name = optarg; break;
        case 'o': out_name = optarg; break;
        case 'p': g_ploidy = atoi(optarg); break;
        case 'q': g_min_mapq = atoi(optarg); break;
        case 's': num_sd = atof(optarg); break;
        case 'g': g_gender = atoi(optarg); break;
        case 'l': g_overlap_mult = atoi(optarg); break;
        case 'b': g_min_base_qual = atoi(optarg); break;
        case 'n': g_min_snv = atoi(optarg); break;
        case 'a': g_min_snv_ratio = atof(optarg); break;
        case 'f': g_vcf = 0; break;
        case 'x': g_min_ave_bq = atof(optarg); break;
        case 'Z': g_block_min = atol(optarg); break;
        case 'W': g_min_rd_window_len = atol(optarg); break;
        case 'X': g_max_rd_window_len = atol(optarg); break;
        case 'A': g_windows_sampling_factor = atol(optarg); break;
        case 'Y': g_min_blocks = atol(optarg); break;
        case 'D': g_min_repeat = atol(optarg); break;
        case 'E': g_min_repeat_stdev = atof(optarg); break;
        case 'K': g_ranks_stdev = atoi(optarg); break;
        case 'V': g_rd_pval_threshold = atof(optarg); break;
        case 'U': g_chr_rd_threshold_factor = atoi(optarg); break;
        case 'L': g_dup_threshold_factor = atol(optarg); break;
        case 'F': g_mapq_factor = atof(optarg); break;
        case 'v': g_pval_threshold = atof(optarg); break;
        case 'd': g_min_disc = atoi(optarg); break;
        case 'y': g_max_split_loss = atoi(optarg); break;
        case 'z': g_min_sr_len = atoi(optarg); break;
        case 'e': g_pval_insertion = atof(optarg); break;
        case 'j': g_min_sv_ratio = atof(optarg); break;
        case 'k': g_max_homopolymer = atoi(optarg); break;
        case 'm': g_min_indel_ratio = atof(optarg); break;
        case 'u': g_max_evidence_ratio = atof(optarg); break;
        case 'w': g_max_ins_range = atoi(optarg); break;
        case 'N': g_1000gen_window = atol(optarg); break;
        case '?': return 2;
        default: break;
        }
    }
    g_pval_threshold1 = g_pval_threshold; /* GROM.c:22101 */
    g_rd_min_mapq = g_min_mapq;           /* GROM.c:22102 */
    if (!bam_name || !fasta_name || !out_name) {
        fprintf(stderr, "usage: gromc_binding -i BAM -r FASTA -o OUT [options]\n");
        return 2;
    }
    bgzf_reader br;
    bam_hdr hdr;
    if (bgzf_open_read(&br, bam_name) != 0 || bam_read_header(&br, &hdr) != 0) {
        fprintf(stderr, "cannot read %s\n", bam_name);
        return 1;
    }
    /* find_insert_mean on the first records (GROM.c:22255) */
    long mapped = 0;
    g_insert_mean = grom_insert_stats(&br, grom_prob2(num_sd), &g_lseq, &g_insert_min_size, &g_insert_max_size,
                                      &mapped, g_min_mapq);
    bgzf_close_read(&br);
    if (g_insert_mean < 0) { fprintf(stderr, "no reads\n"); return 1; }
    grom_gpu_init();
    grom_params P; /* the derived sizes the harness needs for the stream (same formulas as GROM.c:22282-22290) */
    grom_default_params(&P);
    P.overlap_mult = g_overlap_mult;
    grom_params_set_insert(&P, g_insert_mean, g_insert_min_size, g_insert_max_size, g_lseq);
    const int32_t s0 = P.one_base_rd_len / 4 + 1; /* cdp_one_base_index_start, GROM.c:2918 */
    /* find_disc_svs: FASTA chromosomes that match a BAM target, in BAM order
     * (GROM.c:20826-21050), chrY skipped for a female sample, the length test */
    grom_fasta fa;
    if (grom_fasta_open(&fa, fasta_name) != 0) { fprintf(stderr, "cannot read %s\n", fasta_name); return 1; }
    chrom_t *ch = calloc(hdr.n_ref > 0 ? hdr.n_ref : 1, sizeof(chrom_t));
    int32_t *order = calloc(hdr.n_ref > 0 ? hdr.n_ref : 1, sizeof(int32_t));
    int n = 0;
    for (int t = 0; t < hdr.n_ref; t++) {
        int fi = grom_match_target(&fa, hdr.ref_name[t]);
        char lc[GROM_MAX_CHR_NAMES];
        int bl = grom_target_name_lc(hdr.ref_name[t], lc, (int)sizeof(lc));
        if (g_gender == 0 && ((bl == 4 && strncmp(lc, "chry", 4) == 0) || (bl == 1 && lc[0] == 'y'))) fi = -1;
        if (fi < 0) continue;
        long len = grom_fasta_load(&fa, fi, NULL, 0);
        if (!(len > s0 + (long)g_overlap_mult * g_insert_max_size) || !(len > 0 && len <= 300000000)) continue;
        int32_t tid2 = -1;
        for (int a = 0; a < hdr.n_ref; a++)
            if (grom_match_target(&fa, hdr.ref_name[a]) == fi) { tid2 = a; break; }
        ch[n].fasta_idx = fi;
        ch[n].tid = tid2;
        ch[n].len = len;
        ch[n].target = hdr.ref_name[tid2 >= 0 ? tid2 : hdr.n_ref - 1];
        snprintf(ch[n].name, sizeof(ch[n].name), "%.*s", fa.name_len[fi], fa.names[fi]);
        order[n++] = tid2;
    }
    char ctx_path[4096], raw_path[4096];
    snprintf(ctx_path, sizeof(ctx_path), "%s.ctx.vcf", out_name);
    snprintf(raw_path, sizeof(raw_path), "%s.ctx_raw", out_name);
    FILE *vcf = fopen(out_name, "w"), *ctx_raw = fopen(raw_path, "w+");
    if (!vcf || !ctx_raw) { fprintf(stderr, "cannot write %s\n", out_name); return 1; }
    /* one serial pass over the records: each processed chromosome takes the
     * records its count_discordant_pairs loop would */
    if (bgzf_open_read(&br, bam_name) != 0) return 1;
    {
        bam_hdr h2;
        if (bam_read_header(&br, &h2) != 0) return 1;
        bam_free_header(&h2);
    }
    grom_planner pl;
    grom_planner_init(&pl, order, n);
    grom_batch batch;
    bam_rec rec;
    memset(&rec, 0, sizeof(rec));
    int cur = 0, ended = 0;
    if (n > 0) {
        grom_batch_init(&batch, order[0], 50 /* g_read_name_len */);
        grom_batch_set_sv(&batch, ch[0].target, g_splitread);
    }
#define SCAN_CUR()                                                                                      \
    do {                                                                                                \
        grom_batch_finish(&batch, s0, g_overlap_mult, g_insert_max_size);                               \
        grom_reads rd;                                                                                  \
        grom_batch_view(&batch, &rd);                                                                   \
        char *ref = malloc(ch[cur].len + 1);                                                            \
        grom_fasta_load(&fa, ch[cur].fasta_idx, ref, ch[cur].len);                                      \
        grom_gpu_scan(ref, ch[cur].len, ch[cur].name, ch[cur].tid, &rd, batch.n_skip, batch.p_last,     \
                      batch.lseq_tail, vcf, ctx_raw);                                                   \
        free(ref);                                                                                      \
        grom_batch_free(&batch);                                                                        \
        if (++cur < n) {                                                                                \
            grom_batch_init(&batch, order[cur], 50);                                                    \
            grom_batch_set_sv(&batch, ch[cur].target, g_splitread);                                     \
            ended = 0;                                                                                  \
        }                                                                                               \
    } while (0)
    while (cur < n && bam_read_rec(&br, &rec) > 0) {
        if (!ended && batch.n_seen > 0 && rec.tid != order[cur]) {
            grom_batch_end_record(&batch, &rec);
            ended = 1;
        }
        int k = grom_planner_feed(&pl, rec.tid);
        while (cur < n && pl.k > cur) SCAN_CUR();
        if (k >= 0 && k == cur) grom_batch_add(&batch, &rec, s0);
    }
    while (cur < n) SCAN_CUR();
#undef SCAN_CUR
    bam_free_rec(&rec);
    bgzf_close_read(&br);
    fclose(vcf);
    /* main's translocation post-pass over every chromosome's raw CTX rows */
    long raw_len = ftell(ctx_raw);
    char *raw = malloc(raw_len + 1);
    rewind(ctx_raw);
    if (raw_len && fread(raw, 1, raw_len, ctx_raw) != (size_t)raw_len) return 1;
    fclose(ctx_raw);
    remove(raw_path);
    grom_out post = {0};
    if (grom_ctx_postpass(raw, (size_t)raw_len, (const char *const *)hdr.ref_name, hdr.n_ref, g_insert_max_size,
                          g_lseq, &post) != GROM_OK) {
        fprintf(stderr, "%s\n", grom_last_error());
        return 1;
    }
    FILE *ctx = fopen(ctx_path, "w");
    if (!ctx) return 1;
    if (post.ctx_len) fwrite(post.ctx, 1, post.ctx_len, ctx);
    fclose(ctx);
    grom_out_free(&post);
    free(raw);
    grom_dev_fini(g_dev);
    grom_fasta_close(&fa);
    free(ch);
    free(order);
    bam_free_header(&hdr);
    return 0;
}
