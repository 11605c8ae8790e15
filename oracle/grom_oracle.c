/*
 * grom_oracle.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of GROM v1.0.1's
 * per-chromosome scan.  Used by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the checker; never linked into or called by
 * the product path (grom_amd/).
 *
 * Pinning status (see DESIGN.md "Oracle"): the reference cannot be built here
 * (it needs the missing samtools-1.3.1 tarball, Makefile:3-8) and its shipped
 * binary `dist/GROM` is prebuilt machine code that this project does not run.
 * The restatement is pinned against the only golden vectors the reference
 * ships, test_data/test_outuput_tilapia_*.vcf: VCF header text, record layout
 * and the binomial-table values behind every SNV `PR` field.  Per-base counter
 * values are "parity unpinned" beyond that: they follow GROM.c line by line
 * (citations inline) and are cross-checked against the independent HIP path.
 *
 * Scope of this restatement (round 1): the serial read stream with its
 * chromosome-boundary quirks, -M duplicate filtering, whole-chromosome read
 * depth (caf_rd_*), the per-base SNV tally with read-name de-duplication,
 * soft-clip evidence, physical read depth, SNV calling, SNV list flushes and
 * the VCF header/SNV rows.  The per-position sliding ring of the reference
 * (GROM.c:2897-3680, 5846-6402) is restated as a modular window of
 * g_half_one_base_rd_len positions indexed by absolute coordinate; the ring
 * index `cdp_one_base_index` is still tracked because the SNV flush range
 * depends on it (GROM.c:11207, 15066).
 */
#include "grom_oracle.h"

#include <ctype.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "orc_bam.h" /* the oracle's own BAM reader: nothing from grom_amd/ */

#define MAX_TRIALS 1000
#define MAX_CHR_NAMES 30000
#define MAX_CHR_NAME_LEN 50

/* ---------------- globals (GROM.c:710-979) ---------------- */
static int g_min_mapq = 20;             /* -q, GROM.c:803 */
static int g_rd_min_mapq = 20;          /* = g_min_mapq, GROM.c:22102 */
static double g_insert_num_st_devs = 3; /* -s, GROM.c:805 */
static int g_min_snv = 3;               /* -n, GROM.c:891 */
static int g_min_base_qual = 20;        /* -b, GROM.c:892 */
static double g_min_snv_ratio = 0.2;    /* -a, GROM.c:895 */
static double g_min_ave_bq = 15;        /* -x, GROM.c:904 */
static double g_snv_rd_min_factor = 1.75;
static double g_high_cov_min_snv_ratio = 0.4;
static int g_ploidy = 2;                /* -p */
static int g_gender = 0;                /* -g */
static int g_splitread = 1;             /* -S */
static int g_rmdup = 0;                 /* -M */
static int g_rmdup_list_len = 10000;
static int g_vcf = 1;                   /* -f */
static int g_overlap_mult = 1;          /* -l */
static int g_sv_list_len = 1000000;     /* -G */
static long g_max_chr_fasta_len = 300000000; /* -B */
static int g_read_name_len = 50;
static int g_sc_min = 1;
static int g_insert_max_mult = 5;
static int insert_sample_size = 10000000;
/* breakpoint-path parameters (GROM.c:807-974) */
static int g_min_disc = 3;              /* -d */
static int g_sc_range = 35;
static int g_max_split_loss = 20;       /* -y */
static int g_min_sr_len = 30;           /* -z */
static double g_pval_threshold = 0.001; /* -v; g_pval_threshold1 is set from it, GROM.c:22101 */
static double g_pval_threshold1 = 0.01;
static double g_pval_insertion1 = 0.01;
static double g_pval_insertion = 0.0000000001; /* -e */
static double g_min_sv_ratio = 0.05;    /* -j */
static int g_max_homopolymer = 10;      /* -k */
static double g_min_indel_ratio = 0.125; /* -m */
static double g_max_evidence_ratio = 0.25; /* -u */
static int g_max_ins_range = 10;        /* -w */
static double g_range_mult = 0.75;
static double g_max_inv_rd_diff = 1.75;
static double g_min_overlap_ratio = 0.5;

static double g_prob2, g_mq_prob;
static int g_insert_mean, g_insert_min_size, g_insert_max_size, g_lseq;
static long g_one_base_window_size, g_one_base_window_size_total;
static int g_one_base_rd_len, g_half_one_base_rd_len, g_14_one_base_rd_len, g_34_one_base_rd_len;

static double g_mq_table[MAX_TRIALS + 1][MAX_TRIALS + 1];
static double g_hez_table[MAX_TRIALS + 1][MAX_TRIALS + 1];

static char g_chr_names[MAX_CHR_NAMES][MAX_CHR_NAME_LEN];
static int g_chr_names_len[MAX_CHR_NAMES];
static long g_fasta_file_position[MAX_CHR_NAMES];
static long g_chr_len[MAX_CHR_NAMES];
static int g_chr_names_index = 0;
static long g_mappable_genome_length = 0;

static const char g_dna[4] = {'A', 'C', 'G', 'T'};
static const char *g_dump_prefix = NULL;

/* ---------------- binomial tables (GROM.c:21134-21626) ---------------- */

/* GROM.c:21589-21626 */
static void calculate_normal_binom_constants(void) {
    double p = 0.3275911, a1 = 0.254829592, a2 = -0.284496736, a3 = 1.421413741, a4 = -1.453152027,
           a5 = 1.061405429;
    double xc = g_insert_num_st_devs / sqrt(2);
    double t = 1.0 / (1.0 + p * xc);
    double erf = 1.0 - (a1 * t + a2 * pow(t, 2) + a3 * pow(t, 3) + a4 * pow(t, 4) + a5 * pow(t, 5)) * exp(-pow(xc, 2));
    g_prob2 = (1.0 - erf) / 2.0;
    g_mq_prob = pow(10, (-g_min_mapq / 10.0));
}

/* one cell of the Poisson / normal / exact CDF (GROM.c:21226-21301, 21401-21476);
 * `norm_min_k` is 17 for the hez table and 20 for the mq table. */
static double binom_cdf_cell(long n, long successes, double prob, long norm_min_k) {
    const double p = 0.3275911, a1 = 0.254829592, a2 = -0.284496736, a3 = 1.421413741, a4 = -1.453152027,
                 a5 = 1.061405429;
    double cdf;
    if ((n >= 20 && prob <= 0.05) || (n >= 100 && n * prob <= 10)) {
        double lambda = n * prob;
        cdf = 0;
        /* GROM keeps k! in a `long`; it wraps past 20! exactly as the x86-64
         * imul does, which the unsigned arithmetic below reproduces. */
        uint64_t kf = 1;
        for (long k = 0; k < successes; k++) {
            if (k > 1) kf = kf * (uint64_t)k;
            cdf += pow(lambda, k) * exp(-lambda) / (double)(int64_t)kf;
        }
    } else if (n * prob * (1 - prob) >= 5 && successes >= norm_min_k) {
        double stdev = sqrt(n * prob * (1.0 - prob));
        double mean = n * prob;
        double ns = (mean - successes + 0.5) / stdev;
        double x = ns / sqrt(2.0);
        double t = 1.0 / (1.0 + p * x);
        double erf = 1.0 - (a1 * t + a2 * pow(t, 2) + a3 * pow(t, 3) + a4 * pow(t, 4) + a5 * pow(t, 5)) * exp(-pow(x, 2));
        if (ns >= 0) cdf = (1.0 - erf) / 2.0;
        else cdf = 1 - (erf + (1.0 - erf) / 2.0);
    } else {
        cdf = 0;
        long n_minus_k = n;
        long comb = 1;
        for (long k = 0; k < successes; k++) {
            cdf += comb * pow(prob, k) * pow((1 - prob), n_minus_k);
            /* `long = double` conversion: out-of-range values become
             * LONG_MIN on x86-64 (cvttsd2si), reproduced explicitly. */
            double nc = (k > 0) ? (comb / (k + 1.0)) * n_minus_k : (double)comb * n_minus_k;
            if (nc >= 9223372036854775808.0 || nc < -9223372036854775808.0 || nc != nc) comb = INT64_MIN;
            else comb = (long)nc;
            n_minus_k -= 1;
        }
    }
    if (cdf < 0) cdf = 0;
    if (cdf > 1) cdf = 1;
    return 1.0 - cdf;
}

/* The reference parses the tables back from "%e" text on every run that
 * finds them next to the executable (GROM.c:21343-21355, 21531-21545). */
static double pct_e_roundtrip(double v) {
    char buf[64];
    snprintf(buf, sizeof(buf), "%e", v);
    return atof(buf);
}

static void build_binom_tables(void) {
    memset(g_hez_table, 0, sizeof(g_hez_table));
    memset(g_mq_table, 0, sizeof(g_mq_table));
    /* hez table, GROM.c:21219-21325 */
    for (long n = 1; n < MAX_TRIALS + 1; n++)
        for (long s = 0; s < n + 1; s++) g_hez_table[n][s] = binom_cdf_cell(n, s, 0.5, 17);
    for (int r = 0; r < MAX_TRIALS; r++) {
        for (int c = 0; c < MAX_TRIALS; c++) {
            g_hez_table[r][c] = 1.0 - g_hez_table[r][c + 1];
            if (g_hez_table[r][c] < 0) g_hez_table[r][c] = 0;
            if (c > 0 && g_hez_table[r][c - 1] == 1) g_hez_table[r][c] = 1;
        }
        g_hez_table[r][MAX_TRIALS] = 1.0;
    }
    /* mq table, GROM.c:21392-21485 */
    for (long n = 1; n < MAX_TRIALS + 1; n++) {
        for (long s = 0; s < n + 1; s++) {
            if ((s > 0 && g_mq_table[n][s - 1] == 0) || (s > 1 && g_mq_table[n][s - 1] == g_mq_table[n][s - 2]))
                g_mq_table[n][s] = 0;
            else
                g_mq_table[n][s] = binom_cdf_cell(n, s, g_mq_prob, 20);
        }
    }
    for (int r = 0; r <= MAX_TRIALS; r++)
        for (int c = 0; c <= MAX_TRIALS; c++) {
            g_hez_table[r][c] = pct_e_roundtrip(g_hez_table[r][c]);
            g_mq_table[r][c] = pct_e_roundtrip(g_mq_table[r][c]);
        }
}

/* ---------------- record stream (GROM.c:981-992) ---------------- */
typedef struct {
    bgzf_reader bg;
    bam_hdr hdr;
    int open;
    int only_tid; /* -1: every record (the serial stream); else bam_fetch's records of that target */
} stream_t;

/* -P n (1 <= n <= 256, GROM.c:21923-21927): every chromosome reads its own
 * records through bam_fetch over [g_sub_region_start, g_sub_region_end - 1] =
 * [0, MAX_REGION) (the reader thread of find_disc_svs, GROM.c:21051-21064,
 * single_chromosome_read GROM.c:304-324; the -c children of -P n > 1 do the
 * same, GROM.c:549-599): the target's records with a position, in file
 * order, then the end of the stream -- no records of the next chromosome are
 * consumed (no Q1 drops) and an empty chromosome starves nothing (no Q21). */
static int g_fetch_mode = 0;

static int stream_open(stream_t *s, const char *path) {
    memset(s, 0, sizeof(*s));
    s->only_tid = -1;
    if (bgzf_open_read(&s->bg, path) != 0) return -1;
    if (bam_read_header(&s->bg, &s->hdr) != 0) return -1;
    s->open = 1;
    return 0;
}
static void stream_close(stream_t *s) {
    if (!s->open) return;
    bgzf_close_read(&s->bg);
    bam_free_header(&s->hdr);
    s->open = 0;
}
static int my_samread(stream_t *s, bam_rec *b) {
    for (;;) {
        int rc = bam_read_rec(&s->bg, b);
        if (rc <= 0) return -1;
        /* bam_fetch over [0, MAX_REGION): the target's records that overlap
         * it, i.e. every one with a position (an unmapped read placed at its
         * mate's position included) */
        if (s->only_tid < 0 || (b->tid == s->only_tid && b->pos >= 0 && b->pos < 300000000)) return 1;
    }
}

/* ---------------- find_insert_mean (GROM.c:1205-1318) ---------------- */
static int cmp_int(const void *a, const void *b) { return (*(const int *)a - *(const int *)b); }

static int find_insert_mean(stream_t *s, int *gc_lseq, int *imin, int *imax) {
    int *sizes = (int *)malloc((size_t)insert_sample_size * sizeof(int));
    int *lseqs = (int *)malloc((size_t)insert_sample_size * sizeof(int));
    int count = 0;
    bam_rec b;
    memset(&b, 0, sizeof(b));
    while (my_samread(s, &b) > 0 && count < insert_sample_size) {
        int flag = b.flag;
        if ((flag & GF_UNMAP) == 0 && (flag & GF_DUP) == 0) {
            if ((flag & GF_PAIRED) == 0) {
                sizes[count] = b.l_qseq;
                lseqs[count] = b.l_qseq;
                count++;
            } else if ((flag & GF_MUNMAP) == 0 && b.tid == b.mtid) {
                if (b.pos < b.mpos && (flag & GF_PROPER) != 0 && b.isize > 0) {
                    sizes[count] = b.isize;
                    lseqs[count] = b.l_qseq;
                    count++;
                }
            }
        }
    }
    bam_free_rec(&b);
    qsort(sizes, count, sizeof(int), cmp_int);
    int mean = sizes[count / 2];
    int max_insert = mean * g_insert_max_mult;
    int start = 0, end = 0;
    for (int a = count - 1; a >= 0; a--)
        if (sizes[a] <= max_insert) { end = a; break; }
    end += 1;
    mean = sizes[start + (end - start) / 2];
    int min_index = (int)(g_prob2 * (end - start) / 2) + start;
    int max_index = end - min_index;
    *imin = sizes[min_index];
    *imax = sizes[max_index];
    printf("insert_min_size, insert_max_size %d %d\n", *imin, *imax);
    qsort(lseqs, count, sizeof(int), cmp_int);
    *gc_lseq = lseqs[count / 2];
    free(sizes);
    free(lseqs);
    return mean;
}

/* ---------------- FASTA (GROM.c:1321-1428, 21009-21045) ---------------- */
static void find_genome_length(FILE *fh) {
    char line[1000];
    long pos = 0, chr_len = 0;
    while (fgets(line, sizeof(line), fh)) {
        if (line[0] != '>') {
            size_t L = strlen(line);
            for (size_t a = 0; a < L; a++)
                if (isalpha((unsigned char)line[a])) {
                    if (line[a] != 'N' && line[a] != 'n') g_mappable_genome_length += 1;
                    chr_len += 1;
                }
        } else {
            pos = ftell(fh);
            int name_len = (int)strlen(line);
            int w = name_len - 1, alpha_len = name_len;
            while (w > 0) {
                if (isgraph((unsigned char)line[w]) == 0) alpha_len = w;
                w -= 1;
            }
            if (g_chr_names_index < MAX_CHR_NAMES) {
                if (alpha_len >= MAX_CHR_NAME_LEN) alpha_len = MAX_CHR_NAME_LEN;
                for (int a = 1; a < alpha_len; a++)
                    g_chr_names[g_chr_names_index][a - 1] = (char)tolower((unsigned char)line[a]);
                g_fasta_file_position[g_chr_names_index] = pos;
                if (g_chr_names_index > 0) g_chr_len[g_chr_names_index - 1] = chr_len;
                g_chr_names_len[g_chr_names_index] = alpha_len - 1;
            }
            g_chr_names_index += 1;
            chr_len = 0;
        }
    }
    if (g_chr_names_index > 0 && g_chr_names_index < MAX_CHR_NAMES) g_chr_len[g_chr_names_index - 1] = chr_len;
    fseek(fh, 0, SEEK_SET);
}

/* name match rules shared by find_disc_svs (GROM.c:20908-20975) and
 * count_discordant_pairs (GROM.c:1916-1961): exact, BAM "chrX" vs FASTA "X",
 * BAM "X" vs FASTA "chrX". */
static int names_match(const char *bam, int bam_len, const char *fa, int fa_len) {
    char tmp[MAX_CHR_NAME_LEN + 8];
    if (bam_len == fa_len && strncmp(bam, fa, fa_len) == 0) return 1;
    if (bam_len - 3 == fa_len && strncmp(bam, "chr", 3) == 0) {
        snprintf(tmp, sizeof(tmp), "chr%.*s", fa_len, fa);
        if (strncmp(bam, tmp, bam_len) == 0) return 1;
    } else if (bam_len + 3 == fa_len && strncmp(fa, "chr", 3) == 0) {
        snprintf(tmp, sizeof(tmp), "chr%.*s", bam_len, bam);
        if (strncmp(fa, tmp, fa_len) == 0) return 1;
    }
    return 0;
}

/* lower-case BAM target name, trimmed at the first non-graph char after
 * index 0 (GROM.c:1899-1912) */
static int bam_name_lc(const char *target, char *out, int cap) {
    int L = (int)strlen(target);
    if (L > cap - 1) L = cap - 1;
    for (int i = 0; i < L; i++) out[i] = (char)tolower((unsigned char)target[i]);
    out[L] = 0;
    int i = L - 1;
    while (i > 0) {
        if (isgraph((unsigned char)out[i]) == 0) L = i;
        i -= 1;
    }
    return L;
}

#include "cnv_oracle.c"
#include "sv_oracle.c"

/* ---------------- per-chromosome scan state ---------------- */
typedef struct {
    /* current record as loaded by the fetch sites (GROM.c:5744-5837) */
    bam_rec b;
    int32_t pos, mpos, tlen, lseq, chr, mchr;
    uint16_t flag, mq;
    int add;
    int aux_pos, aux_mq, aux_strand;
    char aux_str[128];
    char *aux_chr, *aux_cigar;
} cur_t;

/* window of per-position state (modular restatement of the ring) */
typedef struct {
    int W;          /* window length = g_half_one_base_rd_len */
    orc_counts *c;  /* counters (pos field unused here) */
    int32_t *names; /* g_min_snv name ids per position */
    orc_indel *ind; /* CIGAR indel evidence per position (row A7) */
    uint8_t *ind_touched;            /* some I/D op reached the base */
    int32_t *conc, *ins;             /* cdp_one_base_conc / cdp_one_base_ins (row A9) */
    int32_t *rd_add;                 /* the A9 part of cdp_one_base_rd (dump only) */
} win_t;

#define ORC_OTHER_LEN 50 /* g_other_len, GROM.c:837 */
#define ORC_INDEL_SEQ 50 /* g_indel_i_seq_len, GROM.c:904 */
enum { OT_EMPTY = 0, OT_INDEL_I = 11, OT_INDEL_D_F = 12, OT_INDEL_D_R = 13 }; /* GROM.c:668-681 */

static inline long wslot(const win_t *w, long x) { return ((x % w->W) + w->W) % w->W; }

/* ---------------- read-name interning ---------------- */
typedef struct { char **keys; int32_t *ids; long cap, n; } nametab;

static uint64_t fnv1a(const char *s) {
    uint64_t h = 1469598103934665603ULL;
    while (*s) { h ^= (unsigned char)*s++; h *= 1099511628211ULL; }
    return h;
}
static int32_t name_id(nametab *t, const char *s) {
    if (t->n * 2 >= t->cap) {
        long ncap = t->cap ? t->cap * 2 : 1 << 16;
        char **nk = (char **)calloc(ncap, sizeof(char *));
        int32_t *ni = (int32_t *)calloc(ncap, sizeof(int32_t));
        for (long i = 0; i < t->cap; i++)
            if (t->keys[i]) {
                long j = (long)(fnv1a(t->keys[i]) & (uint64_t)(ncap - 1));
                while (nk[j]) j = (j + 1) & (ncap - 1);
                nk[j] = t->keys[i];
                ni[j] = t->ids[i];
            }
        free(t->keys);
        free(t->ids);
        t->keys = nk;
        t->ids = ni;
        t->cap = ncap;
    }
    long j = (long)(fnv1a(s) & (uint64_t)(t->cap - 1));
    while (t->keys[j]) {
        if (strcmp(t->keys[j], s) == 0) return t->ids[j];
        j = (j + 1) & (t->cap - 1);
    }
    t->keys[j] = strdup(s);
    t->ids[j] = (int32_t)(++t->n);
    return t->ids[j];
}
static void nametab_free(nametab *t) {
    for (long i = 0; i < t->cap; i++) free(t->keys[i]);
    free(t->keys);
    free(t->ids);
    memset(t, 0, sizeof(*t));
}

/* aux parsing at a fetch site (GROM.c:5757-5826, 10990-11066, 14885-14950) */
static void load_record(cur_t *c, int parse_aux) {
    bam_rec *b = &c->b;
    c->pos = b->pos;
    c->flag = b->flag;
    c->mq = b->mapq;
    c->chr = b->tid;
    c->mchr = b->mtid;
    c->mpos = b->mpos;
    c->tlen = b->isize;
    c->lseq = b->l_qseq;
    c->add = (c->mq >= g_min_mapq) ? 6 : 0; /* GROM.c:5829-5836 */
    c->aux_pos = -1;
    c->aux_mq = -1;
    int l_aux = bam_l_aux(b);
    if (parse_aux && l_aux > 0 && l_aux < 100) {
        int is_xp = 1;
        uint8_t *a = bam_aux_find(b, "XP");
        if (!a) { is_xp = 0; a = bam_aux_find(b, "SA"); }
        if (a) {
            const uint8_t *src = (a[0] == 'Z') ? a + 1 : a;
            const uint8_t *end = b->data + b->data_len;
            int k = 0;
            while (src + k < end && src[k] && k < (int)sizeof(c->aux_str) - 1) { c->aux_str[k] = (char)src[k]; k++; }
            c->aux_str[k] = 0;
            char *save = NULL;
            c->aux_chr = strtok_r(c->aux_str, ",", &save);
            char *t = strtok_r(NULL, ",", &save);
            if (is_xp) {
                if (t) {
                    c->aux_strand = (t[0] == '+') ? 0 : 1;
                    c->aux_pos = atoi(t + 1);
                }
                c->aux_cigar = strtok_r(NULL, ",", &save);
                t = strtok_r(NULL, ",", &save);
                c->aux_mq = t ? atoi(t) : 0;
            } else {
                c->aux_pos = t ? atoi(t) : -1;
                t = strtok_r(NULL, ",", &save);
                c->aux_strand = (t && t[0] == '+') ? 0 : 1;
                c->aux_cigar = strtok_r(NULL, ",", &save);
                t = strtok_r(NULL, ",", &save);
                c->aux_mq = t ? atoi(t) : 0;
            }
            if (!c->aux_chr || !c->aux_cigar) c->aux_pos = -1;
        }
    }
}

typedef struct {
    int n;
    int cap;
    int32_t *pos, *base;
    double *ratio, *binom, *hez;
    int32_t (*snv)[4], (*lowmq)[4], (*pir)[4], (*fs)[4];
    int32_t *bq, *bq_all, *mq, *mq_all, *bq_rc, *mq_rc, *rc_all;
} snv_list;

static void snv_list_init(snv_list *l, int cap) {
    memset(l, 0, sizeof(*l));
    l->cap = cap;
    l->pos = (int32_t *)malloc(cap * sizeof(int32_t));
    l->base = (int32_t *)malloc(cap * sizeof(int32_t));
    l->ratio = (double *)malloc(cap * sizeof(double));
    l->binom = (double *)malloc(cap * sizeof(double));
    l->hez = (double *)malloc(cap * sizeof(double));
    l->snv = malloc(cap * sizeof(*l->snv));
    l->lowmq = malloc(cap * sizeof(*l->lowmq));
    l->pir = malloc(cap * sizeof(*l->pir));
    l->fs = malloc(cap * sizeof(*l->fs));
    l->bq = (int32_t *)malloc(cap * sizeof(int32_t));
    l->bq_all = (int32_t *)malloc(cap * sizeof(int32_t));
    l->mq = (int32_t *)malloc(cap * sizeof(int32_t));
    l->mq_all = (int32_t *)malloc(cap * sizeof(int32_t));
    l->bq_rc = (int32_t *)malloc(cap * sizeof(int32_t));
    l->mq_rc = (int32_t *)malloc(cap * sizeof(int32_t));
    l->rc_all = (int32_t *)malloc(cap * sizeof(int32_t));
}
static void snv_list_free(snv_list *l) {
    free(l->pos); free(l->base); free(l->ratio); free(l->binom); free(l->hez);
    free(l->snv); free(l->lowmq); free(l->pir); free(l->fs);
    free(l->bq); free(l->bq_all); free(l->mq); free(l->mq_all); free(l->bq_rc); free(l->mq_rc); free(l->rc_all);
}

/* SNV rows of one list flush (GROM.c:11203-11326 mid-scan, 15035-15160 final) */
static void snv_flush(snv_list *l, const char *fasta, long chr_len, const int32_t *caf_rd, const int32_t *caf_low,
                      long *last_group_pos, long range_end, long *rc_total, long *base_total, const char *chr_name,
                      FILE *vcf, int cur_lseq) {
    for (long a = *last_group_pos; a < range_end; a++) {
        if (fasta[a] != 'N' && fasta[a] != 'n') {
            *rc_total += (long)caf_rd[a] + (long)caf_low[a];
            *base_total += 1;
        }
    }
    double ave_rd = (double)*rc_total / (double)*base_total;
    *last_group_pos = range_end;
    /* GROM.c:1477 keeps the GT text in 100 bytes: -p above 50 writes past
     * it (undefined); both sides print the whole 2*p-1 character string */
    char *gt = (char *)malloc(2 * (size_t)(g_ploidy > 0 ? g_ploidy : 1) + 2);
    gt[0] = 0;
    for (int a = 0; a < l->n; a++) {
        if (!(l->rc_all[a] <= round(g_snv_rd_min_factor * ave_rd) || l->ratio[a] >= g_high_cov_min_snv_ratio)) continue;
        int b = l->base[a];
        if (g_vcf == 1) {
            int cn = (int)round(l->ratio[a] * g_ploidy);
            if (cn == 0) cn = 1;
            for (int k = 0; k < g_ploidy; k++) {
                gt[2 * k] = (k < cn) ? '1' : '0';
                gt[2 * k + 1] = (k < g_ploidy - 1) ? '/' : '\0';
            }
            fprintf(vcf,
                    "%s\t%d\t\t%c\t%c\t.\t.\t.\tGT:PR:AF:A:C:G:T:AL:CL:GL:TL:BQ:MQ:PIR:FS\t%s:%e:%e:%d:%d:%d:%d:%d:%d:%d:%d:"
                    "%.2f:%.2f:%.2f:%.2f\n",
                    chr_name, l->pos[a] + 1, fasta[l->pos[a]], g_dna[b], gt, l->binom[a], l->ratio[a], l->snv[a][0],
                    l->snv[a][1], l->snv[a][2], l->snv[a][3], l->lowmq[a][0], l->lowmq[a][1], l->lowmq[a][2],
                    l->lowmq[a][3], (double)l->bq_all[a] / (double)l->rc_all[a],
                    (double)l->mq_all[a] / (double)l->rc_all[a], (double)l->pir[a][b] / (double)l->snv[a][b],
                    (double)l->fs[a][b] / (double)l->snv[a][b]);
        } else {
            /* GROM.c:11276-11323 (-f tab format) */
            fprintf(vcf, "SNV\t%s\t%d\t%c\t%e\t%d\t%d", chr_name, l->pos[a], g_dna[b], l->ratio[a], 0, 0);
            for (int k = 0; k < 4; k++) fprintf(vcf, "\t%d", l->snv[a][k]);
            for (int k = 0; k < 4; k++) fprintf(vcf, "\t%d", l->lowmq[a][k]);
            fprintf(vcf, "\t%d\t%d\t%d\t%d\t%d\t%d\t%d", l->bq[a], l->bq_all[a], l->mq[a], l->mq_all[a], l->bq_rc[a],
                    l->mq_rc[a], l->rc_all[a]);
            double pir = (double)l->pir[a][b] / (double)l->snv[a][b], fs = (double)l->fs[a][b] / (double)l->snv[a][b];
            if (l->pos[a] > 0 && l->pos[a] < chr_len - 1)
                fprintf(vcf, "\t%.2f\t%.2f\t%c%c%c", pir, fs, fasta[l->pos[a] - 1], fasta[l->pos[a]], fasta[l->pos[a] + 1]);
            else
                fprintf(vcf, "\t%.2f\t%.2f\t%c%c%c", pir, fs, '.', '.', '.');
            fprintf(vcf, "\t");
            for (int k = 0; k < cur_lseq; k++) {
                long x = l->pos[a] - cur_lseq + 1 + k;
                fputc(x < 0 ? 'N' : fasta[x], vcf);
            }
            for (int k = 0; k < cur_lseq - 1; k++) {
                long x = l->pos[a] + cur_lseq - 1 - k;
                fputc(x >= chr_len - 1 ? 'N' : fasta[x], vcf);
            }
            fprintf(vcf, "\t%e\t%e\n", l->binom[a], l->hez[a]);
        }
    }
    free(gt);
    l->n = 0;
}

typedef struct {
    const char *fasta;
    long chr_len;
    win_t w;
    int32_t *caf_mq, *caf_rd, *caf_low;
    nametab names;
    /* -M state (GROM.c:5451-5498) */
    int *rm_mchr, *rm_mpos, *rm_lseq, *rm_tlen, *rm_svtype;
    int rm_index, old_pos;
    int p, one_base_index;
    sv_ring ring;      /* cluster arrays with the reference's ring semantics (sv_oracle.c) */
    sv_lists lists;    /* candidate lists of the per-base tests */
    const char *target_name; /* cdp_target_name: the split-read chromosome test, GROM.c:7431 */
} scan_t;

enum { SV_DEL = 0, SV_DUP = 1, SV_INV_F = 8, SV_INV_R = 9, SV_CTX_FF = 11, SV_CTX_FR = 12, SV_CTX_RF = 13, SV_CTX_RR = 14 };

/* -M pair-orientation class (GROM.c:6432-6529) */
static int rmdup_svtype(const cur_t *c) {
    int rev = (c->flag & GF_REVERSE) != 0, mrev = (c->flag & GF_MREVERSE) != 0;
    if (c->chr == c->mchr) {
        if (c->mpos > c->pos) {
            if (!rev && mrev) return SV_DEL;
            if (!rev && !mrev) return SV_INV_F;
            return mrev ? SV_INV_R : SV_DUP;
        }
        if (rev && !mrev) return SV_DEL;
        if (!rev && !mrev) return SV_INV_F;
        if (mrev) return rev ? SV_INV_R : SV_DUP;
        return -1;
    }
    if (!rev) return mrev ? SV_CTX_FR : SV_CTX_FF;
    return mrev ? SV_CTX_RR : SV_CTX_RF;
}

/* one record through the ingest body (GROM.c:6418-7185) */
/* One CIGAR indel event folded into its base (GROM.c:7209-7283 for I,
 * 7289-7420 for the two deletion ends): the primary counter takes the first
 * length seen while its count is 0, a same-length event adds, and a different
 * length goes to the "other" slots, where an entry that overtakes the primary
 * swaps with it. */
static void indel_fold(scan_t *s, long x, int type, int add, long len, const char *seq) {
    win_t *w = &s->w;
    long sl = wslot(w, x);
    orc_indel *k = &w->ind[sl];
    w->ind_touched[sl] = 1;
    int32_t *cnt, *dist;
    if (type == OT_INDEL_I) { cnt = &k->ins; dist = &k->ins_len; }
    else if (type == OT_INDEL_D_F) { cnt = &k->del_f; dist = &k->del_f_len; k->del_f_rd += 1; }
    else { cnt = &k->del_r; dist = &k->del_r_len; k->del_r_rd += 1; }
    if (*cnt == 0) {
        *cnt = add;
        *dist = (int32_t)len;
        if (type == OT_INDEL_I && len <= ORC_INDEL_SEQ)
            for (long q = 0; q < len; q++) k->ins_seq[q] = seq[q];
    } else if ((uint32_t)len == (uint32_t)*dist) {
        *cnt += add;
    } else {
        /* the "other" slots are shared with the breakpoint clusters (ring) */
        sv_indel_other(&s->ring, s->one_base_index + (int)(x - s->p), type, add, len, cnt, dist);
    }
}

/* window accessors for the breakpoint restatement (sv_oracle.c) */
/* the pair binning's depth adds go into cdp_one_base_rd; rd_add keeps them
 * apart for the breakpoint-record dump (grom_sv_rec.rd_add) */
static void acc_rd_inc(void *u, long x) {
    scan_t *s = (scan_t *)u;
    const long sl = wslot(&s->w, x);
    s->w.c[sl].rd += 1;
    s->w.rd_add[sl] += 1;
}
static int32_t *acc_conc(void *u, long x) { scan_t *s = (scan_t *)u; return &s->w.conc[wslot(&s->w, x)]; }
static int32_t *acc_ins(void *u, long x) { scan_t *s = (scan_t *)u; return &s->w.ins[wslot(&s->w, x)]; }
static void acc_indel(void *u, long x, int type, int add, long len) { indel_fold((scan_t *)u, x, type, add, len, NULL); }

static void ingest(scan_t *s, cur_t *c) {
    const char *fasta = s->fasta;
    long chr_len = s->chr_len;
    bam_rec *b = &c->b;
    if ((c->flag & GF_UNMAP) != 0 || (c->flag & GF_DUP) != 0) return;
    int add_to_list = 1;
    if (g_rmdup > 0 && (c->flag & GF_PAIRED) != 0 && (c->flag & GF_MUNMAP) == 0) {
        int svtype = rmdup_svtype(c);
        if (svtype >= 0) {
            if (c->pos != s->old_pos) {
                s->rm_index = 0;
                s->old_pos = c->pos;
            } else {
                for (int a = 0; a < s->rm_index; a++) {
                    if (c->mpos == s->rm_mpos[a] && c->mchr == s->rm_mchr[a] && s->rm_lseq[a] == c->lseq &&
                        s->rm_tlen[a] == c->tlen && c->mq >= g_min_mapq && s->rm_svtype[a] == svtype) {
                        add_to_list = 0;
                        break;
                    }
                }
            }
            if (add_to_list == 1 && s->rm_index < g_rmdup_list_len) {
                s->rm_mchr[s->rm_index] = c->mchr;
                s->rm_mpos[s->rm_index] = c->mpos;
                s->rm_lseq[s->rm_index] = c->lseq;
                s->rm_tlen[s->rm_index] = c->tlen;
                s->rm_svtype[s->rm_index] = svtype;
                s->rm_index += 1;
            }
        }
    }
    if (add_to_list != 1) return;
    int n_cigar = b->n_cigar;
    /* an aligned copy of the CIGAR (it sits at any byte offset in the record) */
    uint32_t cig_buf[512], *cig = n_cigar <= 512 ? cig_buf : (uint32_t *)malloc(4 * (size_t)n_cigar);
    memcpy(cig, bam_cigar(b), 4 * (size_t)n_cigar);

    /* whole-chromosome read depth, GROM.c:6605-6671 */
    long caf_pos = c->pos;
    for (int a = 0; a < n_cigar; a++) {
        int op = cig[a] & 0xf;
        long len = cig[a] >> 4;
        if (op == GC_MATCH || op == GC_EQUAL || op == GC_DIFF) {
            if (caf_pos >= 0 && caf_pos + len < chr_len) {
                for (long x = caf_pos; x < caf_pos + len; x++) {
                    s->caf_mq[x] += c->mq;
                    if (c->mq >= g_rd_min_mapq) s->caf_rd[x] += 1;
                    else s->caf_low[x] += 1;
                }
            }
            caf_pos += len;
        } else if (op == GC_DEL) {
            caf_pos += len;
        }
    }

    /* CIGAR copy limited to 1000 ops, GROM.c:6740-6750 */
    int cigar_len = n_cigar > 1000 ? 1000 : n_cigar;
    int c_type[1000];
    long c_len[1000];
    for (int a = 0; a < cigar_len; a++) { c_type[a] = cig[a] & 0xf; c_len[a] = cig[a] >> 4; }
    if (cig != cig_buf) free(cig);

    const char *rname = bam_qname(b);
    int name_storable = strlen(rname) < (size_t)g_read_name_len && rname[0] != 0;
    int32_t nid = name_id(&s->names, rname);
    const uint8_t *seq4 = bam_seq(b);
    const uint8_t *qual = bam_qual(b);
    int lseq_q = b->l_qseq;
    int snv_base = 0, snv_ref_base = 0, last_cigar_id = 0;
    int rev = (c->flag & GF_REVERSE) != 0;
    (void)last_cigar_id;

    /* per-base SNV tally, GROM.c:6769-7059 */
    for (int a = 0; a < cigar_len; a++) {
        int op = c_type[a];
        if (op == GC_MATCH || op == GC_EQUAL || op == GC_DIFF) {
            if (c->pos >= 0 && c->pos < chr_len) {
                long loop_end;
                if (c->pos + snv_ref_base + c_len[a] >= chr_len) loop_end = chr_len - c->pos;
                else loop_end = c_len[a];
                for (long bl = 0; bl < loop_end; bl++) {
                    long x = c->pos + snv_ref_base;
                    /* bytes past the read's own qual/seq or past the chromosome are
                     * only reached for reads running off the chromosome end; those
                     * positions are never evaluated ("edge semantics") */
                    int q = snv_base < lseq_q ? qual[snv_base] : 0;
                    char sb = snv_base < lseq_q ? grom_nt16_rev[bam_seqi(seq4, snv_base)] : 'N';
                    char rb = x < chr_len ? (char)toupper((unsigned char)fasta[x]) : 'N';
                    orc_counts *k = &s->w.c[wslot(&s->w, x)];
                    if (c->mq >= g_min_mapq && q >= g_min_base_qual) {
                        int found = 0;
                        if (rb != sb) {
                            int32_t *slots = &s->w.names[wslot(&s->w, x) * g_min_snv];
                            for (int cl = 0; cl < g_min_snv; cl++) {
                                if (slots[cl] == 0) {
                                    if (name_storable) slots[cl] = nid;
                                    break;
                                } else if (slots[cl] == nid) {
                                    found = 1;
                                    break;
                                }
                            }
                        }
                        if (!found) {
                            for (int cl = 0; cl < 4; cl++) {
                                if (sb != g_dna[cl]) continue;
                                if (rb == sb) {
                                    k->snv[cl] += 1;
                                    k->bq += q; k->bq_all += q;
                                    k->mq += c->mq; k->mq_all += c->mq;
                                    k->bq_rc += 1; k->mq_rc += 1; k->rc_all += 1;
                                    if (!rev) { k->pir[cl] += snv_base; k->fs[cl] += 1; }
                                    else k->pir[cl] += c->lseq - snv_base;
                                } else {
                                    /* guard at GROM.c:6889 compares a length with an
                                     * op code; both ids are >= 0, so always taken */
                                    k->snv[cl] += 1;
                                    k->bq += q; k->bq_all += q;
                                    k->mq += c->mq; k->mq_all += c->mq;
                                    k->bq_rc += 1; k->mq_rc += 1; k->rc_all += 1;
                                    k->pir[cl] += snv_base;
                                    if (!rev) k->fs[cl] += 1;
                                }
                                break;
                            }
                        }
                    } else {
                        for (int cl = 0; cl < 4; cl++) {
                            if (sb != g_dna[cl]) continue;
                            k->snv_lowmq[cl] += 1;
                            k->bq_all += q;
                            k->mq_all += c->mq;
                            k->rc_all += 1;
                            break;
                        }
                    }
                    snv_base += 1;
                    snv_ref_base += 1;
                }
                last_cigar_id = 0;
            }
        } else if (op == GC_SOFT_CLIP || op == GC_HARD_CLIP) {
            if (op == GC_HARD_CLIP) c->lseq += (int)c_len[a];
            else snv_base += (int)c_len[a];
            last_cigar_id = 0;
        } else if (op == GC_INS) {
            snv_base += (int)c_len[a];
            last_cigar_id = 1;
        } else if (op == GC_DEL) {
            snv_ref_base += (int)c_len[a];
            last_cigar_id = 1;
        } else if (op == GC_REF_SKIP) {
            snv_ref_base += (int)c_len[a];
            last_cigar_id = 0;
        } else {
            last_cigar_id = 0;
        }
    }

    /* clip lengths, GROM.c:7067-7100 */
    int start_adj = (c_type[0] == GC_SOFT_CLIP || c_type[0] == GC_HARD_CLIP) ? (int)c_len[0] : 0;
    int end_adj = (c_type[cigar_len - 1] == GC_SOFT_CLIP || c_type[cigar_len - 1] == GC_HARD_CLIP)
                      ? (int)c_len[cigar_len - 1] : 0;
    int end_adj_indel = 0;
    for (int a = 0; a < cigar_len; a++) {
        if (c_type[a] == GC_INS) end_adj_indel += (int)c_len[a];
        else if (c_type[a] == GC_DEL) end_adj_indel -= (int)c_len[a];
    }
    int paired = (c->flag & GF_PAIRED) != 0, munmap = (c->flag & GF_MUNMAP) != 0;
    long E = (long)c->pos - start_adj + c->lseq - end_adj - end_adj_indel;

    /* soft-clip evidence, GROM.c:7105-7169 */
    if (start_adj >= g_sc_min) {
        orc_counts *k = &s->w.c[wslot(&s->w, (long)c->pos - 1)];
        if (!paired || (!rev && (munmap || (!munmap && c->chr == c->mchr && c->mpos > c->pos)))) {
            k->sc_left += c->add; k->sc_left_rd += 1; k->sc_rd += 1;
        }
        if (paired && !munmap && c->chr != c->mchr && rev) {
            k->ctx_sc_left += c->add; k->ctx_sc_left_rd += 1; k->ctx_sc_rd += 1;
        }
        if (paired && !munmap && c->chr == c->mchr && rev && abs(c->tlen) <= g_insert_max_size && c->mpos < c->pos) {
            k->indel_sc_left += c->add; k->indel_sc_left_rd += 1; k->indel_sc_rd += 1;
        }
    }
    if (end_adj >= g_sc_min) {
        orc_counts *k = &s->w.c[wslot(&s->w, E)];
        if (!paired || (rev && (munmap || (!munmap && c->chr == c->mchr && c->mpos < c->pos)))) {
            k->sc_right += c->add; k->sc_right_rd += 1; k->sc_rd += 1;
        }
        if (paired && !munmap && c->chr != c->mchr && !rev) {
            k->ctx_sc_right += c->add; k->ctx_sc_right_rd += 1; k->ctx_sc_rd += 1;
        }
        if (paired && !munmap && c->chr == c->mchr && !rev && abs(c->tlen) <= g_insert_max_size && c->mpos > c->pos) {
            k->indel_sc_right += c->add; k->indel_sc_right_rd += 1; k->indel_sc_rd += 1;
        }
    }
    /* physical read depth over [pos, E), GROM.c:7173-7181 */
    for (long x = c->pos; x < E; x++) s->w.c[wslot(&s->w, x)].rd += 1;

    /* CIGAR indel evidence, GROM.c:7187-7423: every ingested read; I at the
     * base after the preceding aligned block, D at its first and last base */
    {
        long tp = c->pos;
        int sb = 0;
        char iseq[ORC_INDEL_SEQ];
        for (int a = 0; a < cigar_len; a++) {
            int op = c_type[a];
            if (op == GC_SOFT_CLIP) {
                sb += (int)c_len[a];
            } else if (op == GC_MATCH || op == GC_REF_SKIP || op == GC_EQUAL || op == GC_DIFF) {
                tp += c_len[a];
                if (op != GC_REF_SKIP) sb += (int)c_len[a];
            } else if (op == GC_INS) {
                if (c_len[a] <= ORC_INDEL_SEQ)
                    for (long q = 0; q < c_len[a]; q++)
                        iseq[q] = (sb + q < lseq_q) ? grom_nt16_rev[bam_seqi(seq4, sb + q)] : 0;
                indel_fold(s, tp, OT_INDEL_I, c->add, c_len[a], iseq);
                sb += (int)c_len[a];
            } else if (op == GC_DEL) {
                indel_fold(s, tp, OT_INDEL_D_F, c->add, c_len[a], NULL);
                indel_fold(s, tp + c_len[a] - 1, OT_INDEL_D_R, c->add, c_len[a], NULL);
                tp += c_len[a];
            }
        }
    }

    /* split-read and read-pair breakpoint evidence (rows A8/A9, sv_oracle.c) */
    sv_read r;
    memset(&r, 0, sizeof(r));
    r.pos = c->pos; r.mpos = c->mpos; r.tlen = c->tlen; r.lseq = c->lseq; r.chr = c->chr; r.mchr = c->mchr;
    r.mq = c->mq; r.flag = c->flag; r.add = c->add;
    r.start_adj = start_adj; r.end_adj = end_adj; r.end_adj_indel = end_adj_indel;
    r.aux_pos = c->aux_pos; r.aux_mq = c->aux_mq; r.aux_strand = c->aux_strand;
    if (c->aux_pos >= 0) {
        r.aux_same_chr = strncmp(s->target_name, c->aux_chr, strlen(s->target_name)) == 0;
        sv_aux_cigar(c->aux_cigar, &r.aux_start_adj, &r.aux_end_adj, &r.aux_end_adj_indel); /* GROM.c:6683-6733 */
    }
    sv_ctx X = {&s->ring, s->one_base_index, s->p, acc_rd_inc, acc_conc, acc_ins, acc_indel, s,
                g_insert_max_size, g_insert_min_size, g_insert_mean, g_sc_min, g_min_mapq, g_max_split_loss,
                g_min_sr_len, g_lseq};
    sv_ingest(&X, &r);
}

static void scan_chromosome(stream_t *st, cur_t *c, const char *target_name_of_match, int chr_match,
                            const char *fasta, long chr_len, const char *chr_name, FILE *vcf, FILE *ctx_raw,
                            FILE *dump_cnt, FILE *dump_ind, FILE *dump_sv) {
    scan_t s;
    memset(&s, 0, sizeof(s));
    /* srand(time()) per chromosome, GROM.c:1584; GROM_SEED pins it */
    {
        const char *e = getenv("GROM_SEED");
        glibc_srand(&g_rng, e ? (unsigned)strtoul(e, NULL, 10) : (unsigned)time(NULL));
    }
    cnv_pre pre;
    cnv_prepass(fasta, chr_len, &pre); /* GROM.c:1586-1881 */
    s.fasta = fasta;
    s.chr_len = chr_len;
    s.w.W = g_half_one_base_rd_len;
    s.w.c = (orc_counts *)calloc(s.w.W, sizeof(orc_counts));
    s.w.names = (int32_t *)calloc((size_t)s.w.W * g_min_snv, sizeof(int32_t));
    s.w.ind = (orc_indel *)calloc(s.w.W, sizeof(orc_indel));
    s.w.ind_touched = (uint8_t *)calloc(s.w.W, 1);
    s.w.conc = (int32_t *)calloc(s.w.W, sizeof(int32_t));
    s.w.rd_add = (int32_t *)calloc(s.w.W, sizeof(int32_t));
    s.w.ins = (int32_t *)calloc(s.w.W, sizeof(int32_t));
    sv_ring_init(&s.ring, g_one_base_rd_len);
    sv_lists_init(&s.lists, g_sv_list_len);
    s.target_name = target_name_of_match ? target_name_of_match : "";
    s.caf_mq = (int32_t *)calloc(chr_len, sizeof(int32_t));
    s.caf_rd = (int32_t *)calloc(chr_len, sizeof(int32_t));
    s.caf_low = (int32_t *)calloc(chr_len, sizeof(int32_t));
    s.rm_mchr = (int *)malloc(g_rmdup_list_len * sizeof(int));
    s.rm_mpos = (int *)malloc(g_rmdup_list_len * sizeof(int));
    s.rm_lseq = (int *)malloc(g_rmdup_list_len * sizeof(int));
    s.rm_tlen = (int *)malloc(g_rmdup_list_len * sizeof(int));
    s.rm_svtype = (int *)malloc(g_rmdup_list_len * sizeof(int));
    s.old_pos = -1;

    snv_list sl;
    snv_list_init(&sl, g_sv_list_len);
    long last_group_pos = 0, rc_total = 0, base_total = 0;

    int idx_start = g_one_base_rd_len / 4 + 1; /* GROM.c:2918 */
    int idx = idx_start;
    int p = idx_start;
    int begin = 0;
    int H2 = s.w.W / 2;
    long n_skipped = 0, n_ingested = 0;

    if (chr_match >= 0) {
        while (my_samread(st, &c->b) > 0 && begin < 2) {
            load_record(c, 1);
            if (c->chr == chr_match) {
                begin = 1;
                while (begin < 2) {
                    idx += 1;
                    if (idx == g_34_one_base_rd_len) { /* ring shift, GROM.c:5847-6401 */
                        idx = g_14_one_base_rd_len;
                        sv_ring_shift(&s.ring);
                    }
                    if (begin < 2 && c->pos >= idx_start) {
                        if (c->pos - g_overlap_mult * g_insert_max_size <= p) {
                            while (c->pos - g_overlap_mult * g_insert_max_size <= p && begin < 2) {
                                s.p = p;
                                s.one_base_index = idx;
                                ingest(&s, c);
                                n_ingested++;
                                if (my_samread(st, &c->b) > 0) {
                                    load_record(c, g_splitread == 1);
                                    if (c->chr != chr_match) begin = 2;
                                } else {
                                    begin = 2;
                                }
                            }
                        }
                        if (p > 2 * g_insert_max_size) {
                            orc_counts *k = &s.w.c[wslot(&s.w, p)];
                            if (dump_cnt) {
                                orc_counts o = *k;
                                o.pos = p;
                                fwrite(&o, sizeof(o), 1, dump_cnt);
                                long sl_ = wslot(&s.w, p);
                                if (dump_ind && s.w.ind_touched[sl_]) {
                                    orc_indel r = s.w.ind[sl_];
                                    r.pos = p;
                                    r.other_len = sv_other_len(&s.ring, idx); /* GROM.c:11415-11425 */
                                    fwrite(&r, sizeof(r), 1, dump_ind);
                                }
                                /* breakpoint cluster state of the base (rows A8/A9), the
                                 * records grom_debug_sv returns: every base with a cluster
                                 * count or an occupied "other" slot */
                                if (dump_sv) {
                                    orc_sv_rec v;
                                    memset(&v, 0, sizeof(v));
                                    v.pos = p;
                                    v.other_len = sv_other_len(&s.ring, idx);
                                    int any = v.other_len > 0;
                                    for (int t = 0; t < CL_N; t++) {
                                        const clus_t *q = &s.ring.cl[t][idx];
                                        v.cnt[t] = q->cnt;
                                        v.rs[t] = q->rs;
                                        v.re[t] = q->re;
                                        v.dist[t] = q->dist;
                                        any = any || q->cnt != 0;
                                    }
                                    v.ctx_mchr[0] = s.ring.ctx_mchr[0][idx];
                                    v.ctx_mchr[1] = s.ring.ctx_mchr[1][idx];
                                    v.rd_add = s.w.rd_add[sl_];
                                    v.conc = s.w.conc[sl_];
                                    v.ins = s.w.ins[sl_];
                                    v.mun_f = s.ring.mun[0][idx];
                                    v.mun_r = s.ring.mun[1][idx];
                                    if (any) fwrite(&v, sizeof(v), 1, dump_sv);
                                }
                            }
                            /* SNV test, GROM.c:11096-11199 */
                            if (k->rd + k->indel_sc_rd > 0 && fasta[p] != 'N' && fasta[p] != 'n') {
                                int total = 0;
                                for (int a = 0; a < 4; a++) total += k->snv[a];
                                /* the alt kept at this base: the first passing base with the
                                 * largest ratio (a later base replaces it only when strictly
                                 * larger, GROM.c:11150-11156) */
                                const int a = grom_oracle_snv_pick(k->snv, fasta[p], k->bq_all, k->rc_all, g_min_snv,
                                                                   g_min_snv_ratio, g_min_ave_bq);
                                if (a >= 0) {
                                    const float ratio = (float)k->snv[a] / (float)total;
                                    double binom, hez;
                                    if (total > MAX_TRIALS) {
                                        binom = g_mq_table[MAX_TRIALS][k->snv[a] * MAX_TRIALS / total];
                                        hez = g_hez_table[MAX_TRIALS][k->snv[a] * MAX_TRIALS / total];
                                    } else {
                                        binom = g_mq_table[total][k->snv[a]];
                                        hez = g_hez_table[total][k->snv[a]];
                                    }
                                    int n = sl.n;
                                    sl.pos[n] = p;
                                    for (int bb = 0; bb < 4; bb++) {
                                        sl.snv[n][bb] = k->snv[bb];
                                        sl.lowmq[n][bb] = k->snv_lowmq[bb];
                                        sl.pir[n][bb] = k->pir[bb];
                                        sl.fs[n][bb] = k->fs[bb];
                                    }
                                    sl.ratio[n] = ratio;
                                    sl.base[n] = a;
                                    sl.binom[n] = binom;
                                    sl.hez[n] = hez;
                                    sl.bq[n] = k->bq; sl.bq_all[n] = k->bq_all;
                                    sl.mq[n] = k->mq; sl.mq_all[n] = k->mq_all;
                                    sl.bq_rc[n] = k->bq_rc; sl.mq_rc[n] = k->mq_rc;
                                    sl.rc_all[n] = k->rc_all;
                                    sl.n += 1;
                                }
                                if (sl.n >= g_sv_list_len - 10)
                                    snv_flush(&sl, fasta, chr_len, s.caf_rd, s.caf_low, &last_group_pos, (long)p - idx,
                                              &rc_total, &base_total, chr_name, vcf, c->lseq);
                            }
                            /* indel, insertion and breakpoint tests, GROM.c:11338-13553 */
                            {
                                const orc_counts *k1 = &s.w.c[wslot(&s.w, (long)p + 1)];
                                const orc_indel *in = &s.w.ind[wslot(&s.w, p)];
                                sv_base B;
                                B.rd = k->rd; B.sc_rd = k->sc_rd; B.indel_sc_rd = k->indel_sc_rd;
                                B.sc_left = k->sc_left; B.sc_right = k->sc_right;
                                B.sc_left_rd = k->sc_left_rd; B.sc_right_rd = k->sc_right_rd;
                                B.indel_sc_left = k->indel_sc_left; B.indel_sc_right = k->indel_sc_right;
                                B.sc_left_next = k1->sc_left; B.sc_left_rd_next = k1->sc_left_rd;
                                B.snv_all = 0;
                                for (int a = 0; a < 4; a++) B.snv_all += k->snv[a] + k->snv_lowmq[a];
                                B.conc = s.w.conc[wslot(&s.w, p)];
                                B.ins = s.w.ins[wslot(&s.w, p)];
                                B.indel_i = in->ins; B.indel_idist = in->ins_len;
                                B.indel_d_f = in->del_f; B.indel_d_f_rd = in->del_f_rd;
                                B.indel_d_r = in->del_r; B.indel_d_rdist = in->del_r_len; B.indel_d_r_rd = in->del_r_rd;
                                B.ins_seq = in->ins_seq;
                                sv_eval_prm E = {&g_mq_table[0][0], &g_hez_table[0][0], g_min_disc, g_insert_max_size,
                                                 g_insert_min_size, g_insert_mean, g_lseq, g_sc_range, g_pval_threshold1,
                                                 g_pval_insertion1, g_max_evidence_ratio, g_range_mult};
                                sv_eval(&E, &s.lists, &s.ring, idx, p, &B, c->lseq);
                            }
                        }
                        p += 1;
                        /* slide the modular window: the slot of p-H/2-1 now holds p+H/2-1 */
                        {
                            long x = (long)p + H2 - 1;
                            long sl_ = wslot(&s.w, x);
                            memset(&s.w.c[sl_], 0, sizeof(orc_counts));
                            memset(&s.w.names[sl_ * g_min_snv], 0, sizeof(int32_t) * g_min_snv);
                            memset(&s.w.ind[sl_], 0, sizeof(orc_indel));
                            s.w.ind_touched[sl_] = 0;
                            s.w.conc[sl_] = 0;
                            s.w.ins[sl_] = 0;
                            s.w.rd_add[sl_] = 0;
                        }
                    } else {
                        n_skipped++;
                        if (my_samread(st, &c->b) > 0) {
                            load_record(c, 1);
                            if (c->chr != chr_match) begin = 2;
                        } else {
                            begin = 2;
                        }
                    }
                }
            } else if (begin == 1) {
                begin = 2;
            }
        }
    }
    /* final SNV flush, GROM.c:15063-15160 */
    snv_flush(&sl, fasta, chr_len, s.caf_rd, s.caf_low, &last_group_pos, (long)p - idx, &rc_total, &base_total,
              chr_name, vcf, c->lseq);
    /* SV assembly and rows, GROM.c:15163-16580 */
    {
        sv_out_prm O = {g_insert_max_size, g_lseq, g_vcf, 0, g_pval_threshold, g_pval_insertion, g_min_sv_ratio,
                        g_min_indel_ratio, g_max_inv_rd_diff, g_min_overlap_ratio, g_max_homopolymer, g_max_ins_range};
        sv_write_rows(&O, &s.lists, chr_name, fasta, chr_len, s.caf_rd, s.caf_low, vcf, ctx_raw);
    }

    if (g_dump_prefix) {
        char path[4096];
        snprintf(path, sizeof(path), "%s.%s.caf", g_dump_prefix, chr_name);
        FILE *f = fopen(path, "wb");
        if (f) {
            fwrite(s.caf_mq, sizeof(int32_t), chr_len, f);
            fwrite(s.caf_rd, sizeof(int32_t), chr_len, f);
            fwrite(s.caf_low, sizeof(int32_t), chr_len, f);
            fclose(f);
        }
        snprintf(path, sizeof(path), "%s.%s.meta", g_dump_prefix, chr_name);
        f = fopen(path, "w");
        if (f) {
            fprintf(f, "p_end %d\nidx_end %d\nn_skip %ld\nn_ingested %ld\n", p, idx, n_skipped, n_ingested);
            fclose(f);
        }
    }
    /* read-depth CNV path, GROM.c:16633-17300 (only for a matched target);
     * after the dump above, since it divides caf_mq in place */
    if (chr_match != -1) cnv_chromosome(chr_len, fasta, &pre, s.caf_mq, s.caf_rd, s.caf_low, chr_name, vcf);
    cnv_pre_free(&pre);
    snv_list_free(&sl);
    nametab_free(&s.names);
    free(s.w.c); free(s.w.names);
    free(s.w.ind); free(s.w.ind_touched); free(s.w.conc); free(s.w.ins); free(s.w.rd_add);
    sv_ring_free(&s.ring);
    sv_lists_free(&s.lists);
    free(s.caf_mq); free(s.caf_rd); free(s.caf_low);
    free(s.rm_mchr); free(s.rm_mpos); free(s.rm_lseq); free(s.rm_tlen); free(s.rm_svtype);
}

/* VCF header, GROM.c:20517-20565; the .ctx.vcf variant (GROM.c:22612-22651)
 * omits the GT and the four CNV FORMAT lines.  fileDate may be pinned by
 * GROM_FILEDATE for reproducible comparisons. */
static void write_header(FILE *f, const char *fasta_file_name, int ctx);
static const char *g_hdr_fasta = "";
static void write_ctx_header(FILE *f) { write_header(f, g_hdr_fasta, 1); }
/* -f: the insert statistics and the column header instead of the VCF
 * header, GROM.c:20566-20671 */
static const char TAB_COLUMNS[] =
    "SV\tChromosome\tStart (Tumor)\tEnd (Tumor)\tLength (Tumor)\tP-val (Start, Tumor)\t"
    "P-val (End, Tumor)\tConcordant Pairs (Start, Tumor)\tConcordant Pairs (End, Tumor)\t"
    "Start or End?\tRead Depth (High MapQ, Normal)\tRead Depth (Low MapQ, Normal)\t"
    "Concordant Pairs (Normal)\tINS (Normal)\tDEL (For, Normal)\tDEL (Rev, Normal)\t"
    "DEL (For, Length, Normal)\tDEL (Rev, Length, Normal)\tDUP (Rev, Normal)\tDUP (For, Normal)\t"
    "DUP (Rev, Length, Normal)\tDUP (For, Length, Normal)\tINV (For, Start, Normal)\t"
    "INV (Rev, Start, Normal)\tINV (For, End, Normal)\tINV (Rev, End, Normal)\t"
    "INV (For, Start, Length, Normal)\tINV (Rev, Start, Length, Normal)\t"
    "INV (For, End, Length, Normal)\tINV (Rev, End, Length, Normal)\tUnmapped Mate (For, Normal)\t"
    "Unmapped Mate (Rev, Normal)\tSoft-clipping (Left, Normal)\tSoft-clipping (Right, Normal)\t"
    "Soft-clipping Read Depth (Left, Normal)\tSoft-clipping Read Depth (Right, Normal)\t"
    "Soft-clipping Read Depth (Left+Right, Normal)\tINS Indel (Normal)\tDEL Indel (Start, Normal)\t"
    "DEL Indel (End, Normal)\tDEL Indel (Start, Length, Normal)\tDEL Indel (End, Length, Normal)\t"
    "CTX Soft-clipping (Left, Normal)\tCTX Soft-clipping (Right, Normal)\t"
    "CTX Soft-clipping Read Depth (Left, Normal)\tCTX Soft-clipping Read Depth (Right, Normal)\t"
    "CTX Soft-clipping Read Depth (Left+Right, Normal)\tIndel Soft-clipping (Left, Normal)\t"
    "Indel Soft-clipping (Right, Normal)\tIndel Soft-clipping Read Depth (Left, Normal)\t"
    "Indel Soft-clipping Read Depth (Right, Normal)\t"
    "Indel Soft-clipping Read Depth (Left+Right, Normal)\t"
    "Soft-clipping (Left Max including CTX, Normal)\t"
    "Soft-clipping (Right Max including CTX, Normal)\tOther (Number of Non-Empty, Normal)\t"
    "CTX (For, Normal)\tCTX (Rev, Normal)\tSV Overlap (Normal)\tOther (Number of Non-Empty, Tumor)\t"
    "Read Start (Start, Tumor)\tRead End (Start, Tumor)\tRead Start (End, Tumor)\t"
    "Read End (End, Tumor)\tDEL Read Start (For/Rev, Normal)\tDEL Read End (For/Rev, Normal)\t"
    "DUP Read Start (Rev/For, Normal)\tDUP Read End (Rev/For, Normal)\tINV Read Start (For, Normal)\t"
    "INV Read End (For, Normal)\tINV Read Start (Rev, Normal)\tINV Read End (Rev, Normal)\t"
    "CTX Read Start (For, Normal)\tCTX Read End (For, Normal)\tCTX Read Start (Rev, Normal)\t"
    "CTX Read End (Rev, Normal)\tMate Chr (CTX only, Tumor)\tMate Pos (CTX only, Tumor)\t"
    "Mate Chr (For, Normal)\tMate Pos (For, Normal)\tMate Chr (Rev, Normal)\tMate Pos (Rev, Normal)\t"
    "Reference Base\tSNV Base (Tumor)\tSNV Ratio (Tumor)\tSNV Count (A, Tumor)\t"
    "SNV Count (C, Tumor)\tSNV Count (G, Tumor)\tSNV Count (T, Tumor)\tSNV Count (A, Normal)\t"
    "SNV Count (C, Normal)\tSNV Count (G, Normal)\tSNV Count (T, Normal)\t\n";
static void write_tab_header(FILE *f) {
    fprintf(f, "%d\t%d\t%d\t%d\n", g_insert_mean, g_insert_min_size, g_insert_max_size, g_lseq);
    fputs(TAB_COLUMNS, f);
}
/* -f: the trimmed .ctx file's column header, GROM.c:22652-22700 */
static void write_ctx_tab_header(FILE *f) {
    fprintf(f, "SV\tChromosome\tStart\tID\tMate ID\tBinom Prob (Start)\tCTX evidence\tRead Depth (High MapQ)\t"
               "Concordant Pairs\tOther (Number of Non-Empty)\tMate Chr\tMate Pos\tRead Start\tRead End\tHez binom prob\n");
}
static void write_header(FILE *f, const char *fasta_file_name, int ctx) {
    const char *pin = getenv("GROM_FILEDATE");
    fprintf(f, "##fileformat=VCFv4.2\n");
    if (pin) fprintf(f, "##fileDate=%s\n", pin);
    else {
        time_t t = time(NULL);
        struct tm tm = *localtime(&t);
        fprintf(f, "##fileDate=%d%d%d\n", tm.tm_year + 1900, tm.tm_mon + 1, tm.tm_mday);
    }
    fprintf(f, "##reference=%s\n", fasta_file_name);
    static const char *rest0 =
        "##ALT=<ID=DEL,Description=\"Deletion\">\n"
        "##ALT=<ID=DUP,Description=\"Duplication\">\n"
        "##ALT=<ID=INS,Description=\"Insertion\">\n"
        "##ALT=<ID=INV,Description=\"Inversion\">\n"
        "##INFO=<ID=END,Number=1,Type=Integer,Description=\"End position of the structural variant\">\n"
""; fputs(rest0, f); if (!ctx) fputs("##FORMAT=<ID=GT,Number=1,Type=String,Description=\"Genotype\">\n", f);
    static const char *rest =
        "##FORMAT=<ID=SPR,Number=1,Type=Float,Description=\"Probability of start breakpoint evidence occurring by chance\">\n"
        "##FORMAT=<ID=EPR,Number=1,Type=Float,Description=\"Probability of end breakpoint evidence occurring by chance\">\n"
        "##FORMAT=<ID=SEV,Number=1,Type=Integer,Description=\"Evidence supporting variant at start breakpoint\">\n"
        "##FORMAT=<ID=EEV,Number=1,Type=Integer,Description=\"Evidence supporting variant at end breakpoint\">\n"
        "##FORMAT=<ID=SRD,Number=1,Type=Integer,Description=\"Physical read depth at start breakpoint\">\n"
        "##FORMAT=<ID=ERD,Number=1,Type=Integer,Description=\"Physical read depth at end breakpoint\">\n"
        "##FORMAT=<ID=SCO,Number=1,Type=Integer,Description=\"Concordant pairs at start breakpoint\">\n"
        "##FORMAT=<ID=ECO,Number=1,Type=Integer,Description=\"Concordant pairs at end breakpoint\">\n"
        "##FORMAT=<ID=SOT,Number=1,Type=Integer,Description=\"Count of distinct SVs with evidence at start breakpoint\">\n"
        "##FORMAT=<ID=EOT,Number=1,Type=Integer,Description=\"Count of distinct SVs with evidence at end breakpoint\">\n"
        "##FORMAT=<ID=SSC,Number=1,Type=Integer,Description=\"Soft-clipped reads at start breakpoint\">\n"
        "##FORMAT=<ID=ESC,Number=1,Type=Integer,Description=\"Soft-clipped at end breakpoint\">\n"
        "##FORMAT=<ID=SFR,Number=1,Type=Integer,Description=\"Position of first read supporting start breakpoint\">\n"
        "##FORMAT=<ID=SLR,Number=1,Type=Integer,Description=\"Position of last read supporting start breakpoint\">\n"
        "##FORMAT=<ID=EFR,Number=1,Type=Integer,Description=\"Position of first read supporting end breakpoint\">\n"
        "##FORMAT=<ID=ELR,Number=1,Type=Integer,Description=\"Position of last read supporting end breakpoint\">\n"
        "##FORMAT=<ID=AF,Number=1,Type=Float,Description=\"Allele frequency (high mapping quality reads)\">\n"
        "##FORMAT=<ID=PR,Number=1,Type=Float,Description=\"Probability of SNV evidence occurring by chance\">\n"
        "##FORMAT=<ID=A,Number=1,Type=Integer,Description=\"A nucleotides (high mapping quality reads)\">\n"
        "##FORMAT=<ID=C,Number=1,Type=Integer,Description=\"C nucleotides (high mapping quality reads)\">\n"
        "##FORMAT=<ID=G,Number=1,Type=Integer,Description=\"G nucleotides (high mapping quality reads)\">\n"
        "##FORMAT=<ID=T,Number=1,Type=Integer,Description=\"T nucleotides (high mapping quality reads)\">\n"
        "##FORMAT=<ID=AL,Number=1,Type=Integer,Description=\"A nucleotides (low mapping quality reads)\">\n"
        "##FORMAT=<ID=CL,Number=1,Type=Integer,Description=\"C nucleotides (low mapping quality reads)\">\n"
        "##FORMAT=<ID=GL,Number=1,Type=Integer,Description=\"G nucleotides (low mapping quality reads)\">\n"
        "##FORMAT=<ID=TL,Number=1,Type=Integer,Description=\"T nucleotides (low mapping quality reads)\">\n"
        "##FORMAT=<ID=BQ,Number=1,Type=Float,Description=\"Average base quality (all reads)\">\n"
        "##FORMAT=<ID=MQ,Number=1,Type=Float,Description=\"Average mapping quality (all reads)\">\n"
        "##FORMAT=<ID=PIR,Number=1,Type=Float,Description=\"Average distance of SNV from DNA fragment end)\">\n"
        "##FORMAT=<ID=FS,Number=1,Type=Integer,Description=\"SNV reads mapped to forward strand)\">\n"
"";
    fputs(rest, f);
    if (!ctx)
        fputs("##FORMAT=<ID=SD,Number=1,Type=Float,Description=\"CNV standard deviation\"\n"
              "##FORMAT=<ID=Z,Number=1,Type=Float,Description=\"CNV probability score\"\n"
              "##FORMAT=<ID=CN,Number=1,Type=Float,Description=\"CNV copy number\"\n"
              "##FORMAT=<ID=CS,Number=1,Type=Float,Description=\"CNV copy number standard deviation\"\n", f);
    fputs("#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\n", f);
}

/* ---------------- driver: main + find_disc_svs ---------------- */
int grom_oracle_main(int argc, char **argv, const char *dump_prefix) {
    g_dump_prefix = dump_prefix;
    const char *bam_file_name = NULL, *fasta_file_name = NULL, *results_file_name = NULL;
    optind = 0; /* GNU getopt: full re-initialisation */
    int opt;
    g_1000gen_window = 0;
    g_fetch_mode = 0;
    /* getopt string of GROM.c:21908 */
    while ((opt = getopt(argc, argv,
                         "Z:W:X:Q:A:Y:B:D:E:K:N:V:U:L:F:SP:c:R:MG:i:r:o:p:q:s:v:g:l:d:b:n:a:y:z:e:fj:k:m:u:w:x:h")) != -1) {
        switch (opt) {
        case 'S': g_splitread = 0; break;
        case 'G': g_sv_list_len = atoi(optarg); break;
        case 'M': g_rmdup = 1; break;
        case 'i': bam_file_name = optarg; break;
        case 'r': fasta_file_name = optarg; break;
        case 'o': results_file_name = optarg; break;
        case 'B': g_max_chr_fasta_len = atol(optarg); break;
        case 'p': g_ploidy = atoi(optarg); break;
        case 'q': g_min_mapq = atoi(optarg); break;
        case 's': g_insert_num_st_devs = atof(optarg); break;
        case 'g': g_gender = atoi(optarg); break;
        case 'l': g_overlap_mult = atoi(optarg); break;
        case 'b': g_min_base_qual = atoi(optarg); break;
        case 'n': g_min_snv = atoi(optarg); break;
        case 'a': g_min_snv_ratio = atof(optarg); break;
        case 'f': g_vcf = 0; break;
        case 'x': g_min_ave_bq = atof(optarg); break;
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
        case 'Z': g_block_min = atol(optarg); break;
        case 'W': g_min_rd_window_len = atol(optarg); break;
        case 'X': g_max_rd_window_len = atol(optarg); break;
        case 'A': g_windows_sampling_factor = atol(optarg); break;
        case 'Y': g_min_blocks = atol(optarg); break;
        case 'D': g_min_repeat = atol(optarg); break;
        case 'E': g_min_repeat_stdev = atof(optarg); break;
        case 'K': g_ranks_stdev = atoi(optarg); break;
        case 'V': g_rd_pval_threshold = atof(optarg); break;
        case 'N': g_1000gen_window = atol(optarg); break;
        case 'U': g_chr_rd_threshold_factor = atoi(optarg); break;
        case 'L': g_dup_threshold_factor = atol(optarg); break;
        case 'F': g_mapq_factor = atof(optarg); break;
        case 'P': { const int n = atoi(optarg); g_fetch_mode = n >= 1 && n <= 256; break; } /* GROM.c:21923 */
        case 'h': return 0;
        case '?': return 1;
        default: break; /* options outside this restatement's scope */
        }
    }
    g_pval_threshold1 = g_pval_threshold; /* GROM.c:22101 */
    g_1000gen_base = results_file_name;
    g_rd_min_mapq = g_min_mapq; /* GROM.c:22102 */
    if (!bam_file_name) { printf("ERROR: No bam file specified.\n"); return 1; }
    stream_t st;
    if (stream_open(&st, bam_file_name) != 0) { printf("\nCould not open %s\n", bam_file_name); return 1; }
    if (!bai_exists(bam_file_name)) { printf("Could not open BAM indexing file\n"); return 1; }
    if (!results_file_name) { printf("ERROR: No output file specified.\n"); return 1; }
    if (!fasta_file_name) { printf("ERROR: No reference file specified.\n"); return 1; }
    FILE *fasta = fopen(fasta_file_name, "r");
    if (!fasta) { printf("\nCould not open %s\n", fasta_file_name); return 1; }

    calculate_normal_binom_constants();
    build_binom_tables();
    g_insert_mean = find_insert_mean(&st, &g_lseq, &g_insert_min_size, &g_insert_max_size);
    stream_close(&st);
    if (g_insert_mean < g_lseq) g_insert_mean = g_lseq;
    g_one_base_window_size = 2 * g_insert_mean - 1;
    g_one_base_window_size_total = g_insert_mean;
    for (long a = 0; a < g_insert_mean - 1; a++) g_one_base_window_size_total += 2 * (a + 1);
    printf("insert mean, insert minimum, insert maximum: %d %d %d\n", g_insert_mean, g_insert_min_size, g_insert_max_size);
    /* window sizes, GROM.c:22282-22290 */
    g_one_base_rd_len = g_overlap_mult * 8 * (2 * g_insert_mean - 1);
    if (g_overlap_mult * 8 * (g_insert_max_size + 1) > g_one_base_rd_len)
        g_one_base_rd_len = g_overlap_mult * 8 * (g_insert_max_size + 1);
    g_half_one_base_rd_len = g_one_base_rd_len;
    g_34_one_base_rd_len = g_half_one_base_rd_len + g_half_one_base_rd_len / 2;
    g_14_one_base_rd_len = g_34_one_base_rd_len - g_half_one_base_rd_len;
    g_one_base_rd_len = 2 * g_one_base_rd_len;

    find_genome_length(fasta);

    FILE *vcf = fopen(results_file_name, "w");
    if (!vcf) { printf("Error opening file %s\n", results_file_name); return 1; }
    char ctx_name[4096];
    size_t rl = strlen(results_file_name);
    if (rl > 4 && strcmp(results_file_name + rl - 4, ".vcf") == 0)
        snprintf(ctx_name, sizeof(ctx_name), "%.*s.ctx.vcf", (int)(rl - 4), results_file_name);
    else
        snprintf(ctx_name, sizeof(ctx_name), "%s.ctx", results_file_name);
    FILE *ctx = fopen(ctx_name, "w");
    if (g_vcf == 1) write_header(vcf, fasta_file_name, 0);
    else write_tab_header(vcf);

    build_pval2sd(); /* GROM.c:20705-20748 */
    /* test hook: a smaller sample-list cap makes the reservoir draws of
     * GROM.c:18292/18393 fire on small inputs (the product reads the same) */
    if (getenv("GROM_SAMPLE_LISTS_LEN") && atol(getenv("GROM_SAMPLE_LISTS_LEN")) > 0 &&
        atol(getenv("GROM_SAMPLE_LISTS_LEN")) < g_sample_lists_len)
        g_sample_lists_len = atol(getenv("GROM_SAMPLE_LISTS_LEN"));
    for (int g = 0; g < G_NUM_GC_BINS; g++) {
        if (!g_sample_hi[g]) g_sample_hi[g] = (int *)malloc(g_sample_lists_len * sizeof(int));
        if (!g_sample_lo[g]) g_sample_lo[g] = (int *)malloc(g_sample_lists_len * sizeof(int));
    }
    for (int g = 0; g < G_REPEAT_SEGMENTS; g++)
        if (!g_sample_rep[g]) g_sample_rep[g] = (int *)malloc(g_sample_lists_len * sizeof(int));

    /* find_disc_svs opens its own stream from the file start, GROM.c:20471 */
    if (stream_open(&st, bam_file_name) != 0) return 1;
    char *chr_fasta = (char *)malloc(g_max_chr_fasta_len + 1);
    memset(chr_fasta, 0, g_max_chr_fasta_len + 1);
    int idx_start = g_one_base_rd_len / 4 + 1;
    cur_t cur;
    memset(&cur, 0, sizeof(cur));
    int line_len = 0, alpha_len = 0;
    for (int t = 0; t < st.hdr.n_ref; t++) {
        char bam_lc[MAX_CHR_NAMES];
        int bl = bam_name_lc(st.hdr.ref_name[t], bam_lc, (int)sizeof(bam_lc));
        int fmatch = -1;
        for (int f = 0; f < g_chr_names_index; f++)
            if (names_match(bam_lc, bl, g_chr_names[f], g_chr_names_len[f])) { fmatch = f; break; }
        if ((bl == 4 && strncmp(bam_lc, "chry", 4) == 0 && g_gender == 0) ||
            (bl == 1 && strncmp(bam_lc, "y", 1) == 0 && g_gender == 0))
            fmatch = -1; /* GROM.c:20979-20988 */
        if (fmatch < 0) continue;
        /* load the chromosome, GROM.c:21009-21045 */
        long chr_len = 0;
        char line[1000];
        fseek(fasta, g_fasta_file_position[fmatch], SEEK_SET);
        while (fgets(line, sizeof(line), fasta) && line[0] != '>') {
            if (chr_len == 0 || (int)strlen(line) != line_len) {
                line_len = (int)strlen(line);
                int w = line_len - 1;
                while (isalpha((unsigned char)line[w]) == 0 && w > 0) w -= 1;
                alpha_len = w + 1;
            }
            if (chr_len + alpha_len <= g_max_chr_fasta_len) memcpy(chr_fasta + chr_len, line, alpha_len);
            else printf("ERROR: Reference chromosome length exceeds maximum allowed chromosome size (%ld)\n",
                        g_max_chr_fasta_len);
            chr_len += alpha_len;
        }
        if (!(chr_len > idx_start + g_overlap_mult * g_insert_max_size)) continue;
        if (!(chr_len > 0 && chr_len <= g_max_chr_fasta_len)) continue;
        /* count_discordant_pairs re-derives the BAM target, GROM.c:1894-1961 */
        int chr_match = -1;
        const char *target_name = NULL;
        for (int a = 0; a < st.hdr.n_ref; a++) {
            char lc[MAX_CHR_NAMES];
            int l2 = bam_name_lc(st.hdr.ref_name[a], lc, (int)sizeof(lc));
            target_name = st.hdr.ref_name[a];
            if (names_match(lc, l2, g_chr_names[fmatch], g_chr_names_len[fmatch])) { chr_match = a; break; }
        }
        FILE *dump_cnt = NULL, *dump_ind = NULL, *dump_sv = NULL;
        char cname[MAX_CHR_NAME_LEN + 1];
        snprintf(cname, sizeof(cname), "%.*s", g_chr_names_len[fmatch], g_chr_names[fmatch]);
        if (g_dump_prefix) {
            char path[4096];
            snprintf(path, sizeof(path), "%s.%s.cnt", g_dump_prefix, cname);
            dump_cnt = fopen(path, "wb");
            snprintf(path, sizeof(path), "%s.%s.ind", g_dump_prefix, cname);
            dump_ind = fopen(path, "wb");
            snprintf(path, sizeof(path), "%s.%s.sv", g_dump_prefix, cname);
            dump_sv = fopen(path, "wb");
        }
        if (g_fetch_mode) {
            /* this chromosome's own stream (bam_fetch), from a fresh record */
            stream_t fst;
            cur_t fcur;
            memset(&fcur, 0, sizeof(fcur));
            if (stream_open(&fst, bam_file_name) != 0) return 1;
            fst.only_tid = chr_match;
            scan_chromosome(&fst, &fcur, target_name, chr_match, chr_fasta, chr_len, cname, vcf, ctx, dump_cnt,
                            dump_ind, dump_sv);
            bam_free_rec(&fcur.b);
            stream_close(&fst);
        } else {
            scan_chromosome(&st, &cur, target_name, chr_match, chr_fasta, chr_len, cname, vcf, ctx, dump_cnt, dump_ind,
                            dump_sv);
        }
        if (dump_cnt) fclose(dump_cnt);
        if (dump_ind) fclose(dump_ind);
        if (dump_sv) fclose(dump_sv);
    }
    /* BAM target names, lower-cased, for main's CTX post-pass (GROM.c:22408-22430) */
    int n_targets = st.hdr.n_ref;
    char **names_lc = (char **)calloc(n_targets > 0 ? n_targets : 1, sizeof(char *));
    for (int a = 0; a < n_targets; a++) {
        size_t L = strlen(st.hdr.ref_name[a]);
        names_lc[a] = (char *)malloc(L + 1);
        for (size_t b = 0; b <= L; b++) names_lc[a][b] = (char)tolower((unsigned char)st.hdr.ref_name[a][b]);
    }
    bam_free_rec(&cur.b);
    stream_close(&st);
    free(chr_fasta);
    fclose(vcf);
    if (ctx) {
        /* CTX post-pass of main (GROM.c:22400-22770): pair the raw CTX rows
         * and rewrite the file with its header */
        fclose(ctx);
        g_hdr_fasta = fasta_file_name;
        sv_ctx_postpass(ctx_name, names_lc, n_targets, g_insert_max_size, g_lseq,
                        g_vcf == 1 ? write_ctx_header : write_ctx_tab_header, g_vcf);
    }
    for (int a = 0; a < n_targets; a++) free(names_lc[a]);
    free(names_lc);
    fclose(fasta);
    return 0;
}

/* test hook: the two binomial tables exactly as a run with -q min_mapq uses them */
/* The SNV acceptance test of one base (GROM.c:11126-11156): a base other
 * than the (upper-cased) reference with float ratio >= -a, at least -n reads
 * and average base quality (all reads) >= -x; of several, the first with the
 * largest ratio.  Returns the base index (ACGT) or -1. */
int grom_oracle_snv_pick(const int snv[4], int ref, long bq_all, long rc_all, int min_snv, double min_ratio,
                         double min_ave_bq) {
    int total = 0;
    for (int a = 0; a < 4; a++) total += snv[a];
    int best = -1;
    float best_ratio = 0;
    for (int a = 0; a < 4; a++) {
        const float ratio = (float)snv[a] / (float)total;
        if (toupper((unsigned char)ref) != g_dna[a] && ratio >= min_ratio && snv[a] >= min_snv &&
            (double)bq_all / (double)rc_all >= min_ave_bq) {
            if (best < 0 || ratio > best_ratio) {
                best = a;
                best_ratio = ratio;
            }
        }
    }
    return best;
}

void grom_oracle_tables(int min_mapq, double *mq_out, double *hez_out) {
    g_min_mapq = min_mapq;
    calculate_normal_binom_constants();
    build_binom_tables();
    memcpy(mq_out, g_mq_table, sizeof(g_mq_table));
    memcpy(hez_out, g_hez_table, sizeof(g_hez_table));
}

#ifdef GROM_ORACLE_MAIN
int main(int argc, char **argv) {
    const char *dump = getenv("GROM_ORACLE_DUMP");
    return grom_oracle_main(argc, argv, dump);
}
#endif

/* ---- test hooks for the library restatements of the CNV path ---- */
/* n outputs of glibc's rand() after srand(seed) (restated TYPE_3 generator) */
void grom_oracle_rand_seq(unsigned int seed, int n, int *out) {
    glibc_rng g;
    glibc_srand(&g, seed);
    for (int i = 0; i < n; i++) out[i] = glibc_rand(&g);
}
/* glibc 2.12 qsort (merge sort) of doubles with the reference's int comparator */
void grom_oracle_msort_lo(double *a, long n) { qsort_dbl_intcmp(a, n); }
/* grom_rand(max) n times after srand(seed), GROM.c:1185 */
void grom_oracle_grom_rand(unsigned int seed, long mx, int n, long *out) {
    glibc_srand(&g_rng, seed);
    for (int i = 0; i < n; i++) out[i] = grom_rand(mx);
}
