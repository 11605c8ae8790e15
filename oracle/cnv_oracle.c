/*
 * cnv_oracle.c -- TEST INFRASTRUCTURE ONLY.  #included by grom_oracle.c.
 *
 * CPU restatement of GROM's read-depth CNV path, SURVEY.md §8 rows A14-A16:
 *   - the GC / ACGT triangular-weighted windows and the dinucleotide repeat
 *     list, computed before the read walk   (GROM.c:1586-1881)
 *   - the chromosome read-depth statistics, 10 kb coverage blocks and
 *     low-variance block list             (GROM.c:16633-16990)
 *   - detect_del_dup                      (GROM.c:18228-20358)
 *   - the CNV p-value filter and VCF rows (GROM.c:17011-17300)
 * It follows the reference statement by statement, in the reference's loop
 * order (every double sum is accumulated in the same order), so it is the
 * bit-level checker for the HIP path in grom_amd/csrc/cnv*.
 *
 * Not restated: the N-block list (GROM.c:1626-1722; it is built but never
 * read, only freed at GROM.c:18100-18101), tumor/normal mode (g_normal is
 * never set from argv, SURVEY.md §2 #18b).
 */

/* ---- parameters (GROM.c:710-979; CLI letters GROM.c:21907-22102) ---- */
static long g_min_repeat = 20;                  /* -D, GROM.c:733 */
static double g_min_repeat_stdev = 1.5;         /* -E, GROM.c:734 */
static int g_chr_rd_threshold_factor = 2;       /* -U, GROM.c:737 */
static long g_block_factor = 4;                 /* GROM.c:738 */
static long g_min_blocks = 4;                   /* -Y, GROM.c:739 */
static long g_block_unit_size = 10000;          /* GROM.c:740 */
static long g_block_min = 10000;                /* -Z, GROM.c:758 */
static int g_insert_min_acgt = 99;              /* GROM.c:926 */
static long g_rd_no_combine_min_windows = 100;  /* GROM.c:929 */
static long g_min_rd_window_len = 100;          /* -W, GROM.c:931 */
static long g_max_rd_window_len = 10000;        /* -X, GROM.c:933 */
/* set from the DEFAULT -X before getopt runs (GROM.c:21898) */
static long g_max_distance_since_last_del_good = 10000 + 500;
static double g_rd_pval_threshold = 0.000000001; /* -V, GROM.c:722 */
static long g_1000gen_window = 0;               /* -N, GROM.c:746 */
static const char *g_1000gen_base;              /* the results file name (-o), GROM.c:21057 */
static const char *g_1000gen_chr;               /* ddd_chr_name */
static int g_rd_max_mapq = 60;                  /* GROM.c:718 */
static double g_mapq_factor = 0.5;              /* -F, GROM.c:719 */
static long g_sample_lists_len = 100000;        /* GROM.c:725 */
static long g_genome_reduction_factor = 1;      /* GROM.c:726 */
static long g_windows_sampling_factor = 2;      /* -A, GROM.c:727 */
static long g_dup_threshold_factor = 2;         /* -L, GROM.c:731 */
#define G_REPEAT_SEGMENTS 10                    /* GROM.c:732 */
static int g_ranks_stdev = 1;                   /* -K, GROM.c:925 */
static long g_rd_min_windows = 20;              /* GROM.c:928 */
static long g_one_base_read_depth_min_rd_low_stdev = 3; /* GROM.c:935 */
static double g_max_rd_low_acgt_or_windows = 2; /* GROM.c:937 */
static double g_ploidy_threshold_numerator = 0.6; /* GROM.c:939 */
static double g_stdev_step = 0.01;              /* GROM.c:940 */
#define G_NUM_GC_BINS 101                       /* GROM.c:947 */
#define MAX_BLOCK_LIST_LEN 10000                /* GROM.c:633 */

/* ---- glibc random()/rand() (TYPE_3 additive feedback, as linked into the
 * reference's static binary) so grom_rand is reproducible for a given seed.
 * srandom_r / random_r of glibc's stdlib/random_r.c, restated. ---- */
typedef struct { int32_t st[31]; int f, r; } glibc_rng;
static glibc_rng g_rng;
static void glibc_srand(glibc_rng *g, unsigned int seed) {
    if (seed == 0) seed = 1;
    g->st[0] = (int32_t)seed;
    int32_t word = (int32_t)seed; /* int32_t in glibc's __srandom_r: seeds >= 2^31 start negative */
    for (int i = 1; i < 31; i++) {
        long hi = word / 127773, lo = word % 127773;
        word = (int32_t)(16807 * lo - 2836 * hi);
        if (word < 0) word += 2147483647;
        g->st[i] = word;
    }
    g->f = 3;
    g->r = 0;
    for (int i = 0; i < 310; i++) {
        uint32_t v = (uint32_t)g->st[g->f] + (uint32_t)g->st[g->r];
        g->st[g->f] = (int32_t)v;
        if (++g->f >= 31) { g->f = 0; ++g->r; } else if (++g->r >= 31) g->r = 0;
    }
}
static int glibc_rand(glibc_rng *g) {
    uint32_t v = (uint32_t)g->st[g->f] + (uint32_t)g->st[g->r];
    g->st[g->f] = (int32_t)v;
    if (++g->f >= 31) { g->f = 0; ++g->r; } else if (++g->r >= 31) g->r = 0;
    return (int)(v >> 1);
}

/* GROM.c:1185-1201 */
static long grom_rand(long gr_max) {
    long gr_rand = 0, gr_counter = 1, gr_temp = 0;
    while (gr_counter < gr_max) {
        gr_temp = (glibc_rand(&g_rng) % 10) * gr_counter;
        while ((gr_temp + gr_rand) >= gr_max) gr_temp = (glibc_rand(&g_rng) % 10) * gr_counter;
        gr_rand += gr_temp;
        gr_counter = gr_counter * 10;
    }
    return gr_rand;
}

/* qsort(int[]) with cmpfunc (GROM.c:1105-1108): on small non-negative ints
 * every correct sort gives the same array. */
static void sort_ints(int *a, long n) { qsort(a, (size_t)n, sizeof(int), cmp_int); }

/* qsort(double[], ..., cmpfunc) (GROM.c:20113, 20186): the int
 * comparator compares the LOW 32 bits of each double (little endian) with a
 * wrapping subtraction.  glibc 2.12's qsort is the top-down merge sort of
 * stdlib/msort.c (n1 = n/2, stable "<= 0 takes left"), restated here. */
static int cmp_dbl_lo(const double *a, const double *b) {
    uint32_t x, y;
    memcpy(&x, a, 4);
    memcpy(&y, b, 4);
    return (int32_t)(x - y);
}
static void msort_dbl_rec(double *b, size_t n, double *t) {
    if (n <= 1) return;
    size_t n1 = n / 2, n2 = n - n1;
    double *b1 = b, *b2 = b + n1;
    msort_dbl_rec(b1, n1, t);
    msort_dbl_rec(b2, n2, t);
    double *tmp = t;
    while (n1 > 0 && n2 > 0) {
        if (cmp_dbl_lo(b1, b2) <= 0) { *tmp++ = *b1++; --n1; }
        else { *tmp++ = *b2++; --n2; }
    }
    if (n1 > 0) memcpy(tmp, b1, n1 * sizeof(double));
    memcpy(b, t, (n - n2) * sizeof(double));
}
static void qsort_dbl_intcmp(double *b, long n) {
    double *t = (double *)malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
    msort_dbl_rec(b, (size_t)n, t);
    free(t);
}

/* GROM.c:21630-21860 (exact, including the off-by-one exits) */
static long bisect_left(const int *l, int rd, long s, long e) {
    int found = 0;
    long i = s + (e - s) / 2, lo = s, hi = e;
    while (found == 0) {
        if (i <= s) { i = (rd <= l[s]) ? s : s + 1; found = 1; }
        else if (i >= e - 1) { i = (rd <= l[e - 1]) ? e - 1 : e; found = 1; }
        else if (rd <= l[i]) { hi = i; i = lo + (i - lo) / 2; if (hi == i) { found = 1; i += 1; } }
        else if (rd > l[i]) { lo = i; i = i + (hi - i) / 2; if (lo == i) { found = 1; i += 1; } }
    }
    return i;
}
static long bisect_right(const int *l, int rd, long s, long e) {
    int found = 0;
    long i = s + (e - s) / 2, lo = s, hi = e;
    while (found == 0) {
        if (i <= s) { i = (rd < l[s]) ? s : s + 1; found = 1; }
        else if (i >= e - 1) { i = (rd < l[e - 1]) ? e - 1 : e; found = 1; }
        else if (rd < l[i]) { hi = i; i = lo + (i - lo) / 2; if (hi == i) { found = 1; i += 1; } }
        else if (rd >= l[i]) { lo = i; i = i + (hi - i) / 2; if (lo == i) { found = 1; i += 1; } }
    }
    return i;
}
static long bisect_right_double(const double *l, double p, long s, long e) {
    int found = 0;
    long i = s + (e - s) / 2, lo = s, hi = e;
    while (found == 0) {
        if (i <= s) { i = (p < l[s]) ? s : s + 1; found = 1; }
        else if (i >= e - 1) { i = (p < l[e - 1]) ? e - 1 : e; found = 1; }
        else if (p < l[i]) { hi = i; i = lo + (i - lo) / 2; if (hi == i) { found = 1; i += 1; } }
        else if (p >= l[i]) { lo = i; i = i + (hi - i) / 2; if (lo == i) { found = 1; i += 1; } }
    }
    return i;
}

/* pval2sd table, find_disc_svs GROM.c:20705-20748 */
static double *g_pval2sd_p, *g_pval2sd_sd;
static int g_pval2sd_len;
static void build_pval2sd(void) {
    double p = 0.3275911, a1 = 0.254829592, a2 = -0.284496736, a3 = 1.421413741, a4 = -1.453152027,
           a5 = 1.061405429;
    double sd_max = 10.0;
    int n = (int)(sd_max / g_stdev_step + 0.5);
    n += 1;
    free(g_pval2sd_p);
    free(g_pval2sd_sd);
    g_pval2sd_p = (double *)malloc(n * sizeof(double));
    g_pval2sd_sd = (double *)malloc(n * sizeof(double));
    for (int k = 0; k < n; k++) {
        double sd = sd_max - k * g_stdev_step;
        if (sd < 0) sd = 0;
        double x = sd / sqrt(2.0);
        double t = 1.0 / (1.0 + p * x);
        double erf_ = 1.0 - ((a1 * t + a2 * pow(t, 2) + a3 * pow(t, 3) + a4 * pow(t, 4) + a5 * pow(t, 5)) *
                             exp(-pow(x, 2)));
        g_pval2sd_p[k] = (1.0 - erf_) / 2.0;
        g_pval2sd_sd[k] = sd;
    }
    g_pval2sd_len = n;
}

/* per-chromosome CNV inputs built before the read walk */
typedef struct {
    int *gc_w, *acgt_w; /* caf_one_base_rd_{gc,acgt}_weighted (0 outside the written range) */
    int *rep_type;
    long *rep_start, *rep_end;
    long rep_n;
} cnv_pre;

/* GC/ACGT triangular windows and repeats, GROM.c:1586-1881 (the rolling form
 * exactly as written; caf_*_count_list entries the reference leaves unwritten
 * are zero here, as they are in the reference's fresh mmap'd allocation). */
static void cnv_prepass(const char *fa, long len, cnv_pre *o) {
    const char *gc_chars = "CGcg", *at_chars = "ATat";
    long gc_count = 0, acgt_count = 0, gc_inc = 0, acgt_inc = 0, gc_dec = 0, acgt_dec = 0;
    int *gcl = (int *)calloc(len + 1, sizeof(int));
    int *acl = (int *)calloc(len + 1, sizeof(int));
    o->gc_w = (int *)calloc(len + 1, sizeof(int));
    o->acgt_w = (int *)calloc(len + 1, sizeof(int));
    long cap = 1 + len / g_min_repeat;
    o->rep_type = (int *)malloc(cap * sizeof(int));
    o->rep_start = (long *)malloc(cap * sizeof(long));
    o->rep_end = (long *)malloc(cap * sizeof(long));
    o->rep_n = 0;
    static const char rc[10][2] = {{'A', 'A'}, {'A', 'C'}, {'A', 'G'}, {'A', 'T'}, {'C', 'C'},
                                   {'C', 'G'}, {'C', 'T'}, {'G', 'G'}, {'G', 'T'}, {'T', 'T'}};
    static const char rl[10][2] = {{'a', 'a'}, {'a', 'c'}, {'a', 'g'}, {'a', 't'}, {'c', 'c'},
                                   {'c', 'g'}, {'c', 't'}, {'g', 'g'}, {'g', 't'}, {'t', 't'}};
    int old_t = 10, new_t = 10;
    long rs = 0, re = 0;
    long m = g_insert_mean, W = g_one_base_window_size;
#define ISIN(set, ch) ((ch) != 0 && strchr(set, (ch)) != NULL)
    for (long p = m - 1; p < len - W; p++) {
        /* repeats, GROM.c:1727-1768 */
        new_t = 10;
        for (int a = 0; a < 10; a++) {
            char x = fa[p], y = fa[p + 1];
            if ((rc[a][0] == x && rc[a][1] == y) || (rc[a][1] == x && rc[a][0] == y) ||
                (rl[a][0] == x && rl[a][1] == y) || (rl[a][1] == x && rl[a][0] == y)) {
                new_t = a;
                break;
            }
        }
        if (new_t != old_t || new_t == 10) {
            if (re > 0 && re - rs >= (g_min_repeat - 1)) {
                o->rep_start[o->rep_n] = rs;
                o->rep_end[o->rep_n] = re + 1;
                o->rep_type[o->rep_n] = old_t;
                o->rep_n += 1;
            }
            if (new_t == 10) { rs = 0; re = 0; }
            else { rs = p; re = p; }
        } else {
            re = p;
        }
        old_t = new_t;
        /* weighted GC / ACGT, GROM.c:1770-1861 */
        if (p == m - 1) {
            for (long a = 0; a < m; a++) {
                if (ISIN(gc_chars, fa[a])) {
                    gcl[a] = 1; acl[a] = 1;
                    gc_count += a + 1; acgt_count += a + 1;
                    gc_dec += 1; acgt_dec += 1;
                } else {
                    gcl[a] = 0;
                    if (ISIN(at_chars, fa[a])) { acl[a] = 1; acgt_count += a + 1; acgt_dec += 1; }
                    else acl[a] = 0;
                }
            }
            for (long a = m; a < W; a++) {
                if (ISIN(gc_chars, fa[a])) {
                    gcl[a] = 1; acl[a] = 1;
                    gc_count += W - a; acgt_count += W - a;
                    gc_inc += 1; acgt_inc += 1;
                } else {
                    gcl[a] = 0;
                    if (ISIN(at_chars, fa[a])) { acl[a] = 1; acgt_count += W - a; acgt_inc += 1; }
                }
            }
        } else {
            long gc_adj = gcl[p - m], acgt_adj = acl[p - m];
            long q = p + m - 1;
            if (ISIN(gc_chars, fa[q])) { gcl[q] = 1; acl[q] = 1; gc_inc += 1; acgt_inc += 1; }
            else if (ISIN(at_chars, fa[q])) { gcl[q] = 0; acl[q] = 1; acgt_inc += 1; }
            else { gcl[q] = 0; acl[q] = 0; }
            gc_count += gc_inc - gc_dec;
            acgt_count += acgt_inc - acgt_dec;
            gc_dec -= gc_adj;
            acgt_dec -= acgt_adj;
            if (gcl[p] == 1) { gc_dec += 1; gc_inc -= 1; acgt_dec += 1; acgt_inc -= 1; }
            else if (acl[p] == 1) { acgt_dec += 1; acgt_inc -= 1; }
        }
        o->gc_w[p] = (int)(100 * gc_count / g_one_base_window_size_total);
        o->acgt_w[p] = (int)(100 * acgt_count / g_one_base_window_size_total);
    }
#undef ISIN
    free(gcl);
    free(acl);
}

static void cnv_pre_free(cnv_pre *o) {
    free(o->gc_w); free(o->acgt_w);
    free(o->rep_type); free(o->rep_start); free(o->rep_end);
}

/* chromosome-level results handed from the stats block to detect_del_dup */
static int g_most_biased_repeat = -1;
static long g_lowvar_block_index, g_lowvar_block_sample_index;
static long g_lowvar_block_start_list[MAX_BLOCK_LIST_LEN + 2], g_lowvar_block_end_list[MAX_BLOCK_LIST_LEN + 2];
static long g_lowvar_block_sample_start_list[MAX_BLOCK_LIST_LEN + 2],
    g_lowvar_block_sample_end_list[MAX_BLOCK_LIST_LEN + 2];
static long g_block_start_list[MAX_BLOCK_LIST_LEN], g_block_end_list[MAX_BLOCK_LIST_LEN];

/* sample buffers of find_disc_svs (GROM.c:20751-20806): allocated once and
 * reused across chromosomes without clearing */
static int *g_sample_hi[G_NUM_GC_BINS], *g_sample_lo[G_NUM_GC_BINS], *g_sample_rep[G_REPEAT_SEGMENTS];

typedef struct {
    long n;
    long *start, *end;
    double *stdev, *cn, *cn_stdev;
} cnv_list;

static void cnv_list_init(cnv_list *l, long cap) {
    l->n = 0;
    l->start = (long *)malloc(cap * sizeof(long));
    l->end = (long *)malloc(cap * sizeof(long));
    l->stdev = (double *)malloc(cap * sizeof(double));
    l->cn = (double *)malloc(cap * sizeof(double));
    l->cn_stdev = (double *)malloc(cap * sizeof(double));
}
static void cnv_list_free(cnv_list *l) { free(l->start); free(l->end); free(l->stdev); free(l->cn); free(l->cn_stdev); }

#define RDT(p) (rd[p] + low[p])

/* detect_del_dup, GROM.c:18228-20358 (g_normal == 0 branch; the CN loop and
 * the 1000gen side file excluded as noted in the header) */
/* test hook: samples that met a full list (the reservoir draws of
 * GROM.c:18292, 18393-18451) and how many replaced a kept sample */
static long g_res_over, g_res_repl;

static void detect_del_dup(long len, const int *gc_w, const int *acgt_w, const int *mql, const int *rd, const int *low,
                           const cnv_pre *pre, int ploidy, cnv_list *del, cnv_list *dup) {
    long pos;
    int last_low_mq = 0;
    long a, b;
    int seg;
    double del_thr_f = (1.0 - g_ploidy_threshold_numerator / ploidy);
    double dup_thr_f = (1.0 + g_ploidy_threshold_numerator / ploidy);
    long lo_idx[G_NUM_GC_BINS], hi_idx[G_NUM_GC_BINS], lo_all[G_NUM_GC_BINS], hi_all[G_NUM_GC_BINS];
    for (a = 0; a < G_NUM_GC_BINS; a++) lo_idx[a] = hi_idx[a] = lo_all[a] = hi_all[a] = 0;
    long mb_idx[G_REPEAT_SEGMENTS], mb_all[G_REPEAT_SEGMENTS];
    for (a = 0; a < G_REPEAT_SEGMENTS; a++) mb_idx[a] = mb_all[a] = 0;
    long half = g_insert_mean / 2;
    /* most-biased repeat samples, GROM.c:18284-18330 */
    if (g_most_biased_repeat != -1) {
        for (long r = 0; r < pre->rep_n; r++) {
            if (pre->rep_type[r] != g_most_biased_repeat) continue;
            for (pos = pre->rep_start[r] - half; pos < pre->rep_end[r] + half; pos++) {
                if (acgt_w[pos] >= g_insert_min_acgt) {
                    if (pos < pre->rep_start[r]) seg = (G_REPEAT_SEGMENTS - 1) * (pos - (pre->rep_start[r] - half)) / half;
                    else if (pos >= pre->rep_end[r]) seg = (G_REPEAT_SEGMENTS - 1) * ((pre->rep_end[r] + half) - pos) / half;
                    else seg = G_REPEAT_SEGMENTS - 1;
                    if (mb_idx[seg] < g_sample_lists_len) {
                        g_sample_rep[seg][mb_idx[seg]] = RDT(pos);
                        mb_idx[seg] += 1;
                        mb_all[seg] += 1;
                    } else {
                        g_res_over++;
                        if (grom_rand(mb_all[seg]) == 0) { g_sample_rep[seg][grom_rand(mb_idx[seg])] = RDT(pos); g_res_repl++; }
                        mb_all[seg] += 1;
                    }
                }
            }
        }
    }
    for (int r = 0; r < G_REPEAT_SEGMENTS; r++)
        if (mb_idx[r] > 1) sort_ints(g_sample_rep[r], mb_idx[r]);
    double rep_ave[G_REPEAT_SEGMENTS], rep_sd[G_REPEAT_SEGMENTS];
    if (g_most_biased_repeat != -1) {
        for (int r = 0; r < G_REPEAT_SEGMENTS; r++) {
            rep_sd[r] = 0.0;
            rep_ave[r] = 0.0;
            if (mb_idx[r] > 0) {
                long s0 = mb_idx[r] / 20, e0 = mb_idx[r] - s0, n0 = e0 - s0;
                for (a = s0; a < e0; a++) rep_ave[r] += g_sample_rep[r][a];
                rep_ave[r] = rep_ave[r] / n0;
                for (a = s0; a < e0; a++) rep_sd[r] += pow((g_sample_rep[r][a] - rep_ave[r]), 2);
                if (n0 > 1) rep_sd[r] = sqrt(rep_sd[r] / (n0 - 1));
            } else {
                rep_ave[r] = 0.0;
            }
        }
    }
    /* GC-bin samples every insert_mean/2 bases, GROM.c:18373-18456 */
#define PUSH_SAMPLE(LIST, IDX, ALL, BIN, VAL)                                     \
    do {                                                                          \
        if (IDX[BIN] < g_sample_lists_len) {                                      \
            LIST[BIN][IDX[BIN]] = (VAL);                                          \
            IDX[BIN] += 1;                                                        \
            ALL[BIN] += 1;                                                        \
        } else {                                                                  \
            g_res_over++;                                                         \
            if (grom_rand(ALL[BIN]) == 0) {                                       \
                LIST[BIN][grom_rand(IDX[BIN])] = (VAL);                           \
                g_res_repl++;                                                     \
            }                                                                     \
            ALL[BIN] += 1;                                                        \
        }                                                                         \
    } while (0)
    for (long bl = 0; bl < g_lowvar_block_sample_index; bl++) {
        for (pos = g_lowvar_block_sample_start_list[bl]; pos < g_lowvar_block_sample_end_list[bl]; pos += half) {
            if (acgt_w[pos] >= g_insert_min_acgt) {
                int bin = gc_w[pos];
                if (rd[pos] == 0 && low[pos] == 0) {
                    if (last_low_mq == 0) PUSH_SAMPLE(g_sample_hi, hi_idx, hi_all, bin, RDT(pos));
                    else PUSH_SAMPLE(g_sample_lo, lo_idx, lo_all, bin, RDT(pos));
                } else if (mql[pos] >= g_rd_min_mapq) {
                    PUSH_SAMPLE(g_sample_hi, hi_idx, hi_all, bin, RDT(pos));
                    last_low_mq = 0;
                } else {
                    PUSH_SAMPLE(g_sample_lo, lo_idx, lo_all, bin, RDT(pos));
                    last_low_mq = 1;
                }
            }
        }
    }
#undef PUSH_SAMPLE
    int g;
    for (g = 0; g < G_NUM_GC_BINS; g++) {
        if (hi_idx[g] > 1) sort_ints(g_sample_hi[g], hi_idx[g]);
        if (lo_idx[g] > 1) sort_ints(g_sample_lo[g], lo_idx[g]);
    }
    /* merge thin bins with their +-2 neighbours, GROM.c:18480-18548 */
    long tlo[G_NUM_GC_BINS], thi[G_NUM_GC_BINS];
    for (a = 0; a < G_NUM_GC_BINS; a++) { tlo[a] = lo_idx[a]; thi[a] = hi_idx[a]; }
#define THIN(IDX, G) ((G) >= 2 && (G) < (G_NUM_GC_BINS - 2) && IDX[G] >= g_rd_min_windows && IDX[G] < g_rd_no_combine_min_windows)
    for (g = 0; g < G_NUM_GC_BINS; g++) {
        if (THIN(hi_idx, g))
            for (a = g - 2; a <= g + 2; a++)
                if (a != g)
                    for (b = 0; b < hi_idx[a]; b++)
                        if (thi[g] < g_sample_lists_len) { g_sample_hi[g][thi[g]] = g_sample_hi[a][b]; thi[g] += 1; }
        if (THIN(lo_idx, g))
            for (a = g - 2; a <= g + 2; a++)
                if (a != g)
                    for (b = 0; b < lo_idx[a]; b++)
                        if (tlo[g] < g_sample_lists_len) { g_sample_lo[g][tlo[g]] = g_sample_lo[a][b]; tlo[g] += 1; }
    }
    for (g = 0; g < G_NUM_GC_BINS; g++) {
        if (THIN(hi_idx, g)) { hi_idx[g] = thi[g]; sort_ints(g_sample_hi[g], hi_idx[g]); }
        if (THIN(lo_idx, g)) { lo_idx[g] = tlo[g]; sort_ints(g_sample_lo[g], lo_idx[g]); }
    }
#undef THIN
    /* per-bin mean / stdev / thresholds, GROM.c:18560-18641 */
    double ave[3][G_NUM_GC_BINS], sdv[3][G_NUM_GC_BINS], del_thr[2][G_NUM_GC_BINS], dup_thr[2][G_NUM_GC_BINS];
    long wins[3][G_NUM_GC_BINS];
    for (g = 0; g < G_NUM_GC_BINS; g++) {
        sdv[0][g] = sdv[1][g] = sdv[2][g] = 0.0;
        ave[2][g] = 0.0;
        for (int k = 0; k < 2; k++) {
            long n = (k == 0) ? hi_idx[g] : lo_idx[g];
            int *list = (k == 0) ? g_sample_hi[g] : g_sample_lo[g];
            if (n > 0) {
                ave[k][g] = 0.0;
                for (a = 0; a < n; a++) ave[k][g] += list[a];
                ave[k][g] = ave[k][g] / n;
                del_thr[k][g] = del_thr_f * ave[k][g];
                dup_thr[k][g] = dup_thr_f * ave[k][g];
                wins[k][g] = n;
                for (a = 0; a < n; a++) sdv[k][g] += pow((list[a] - ave[k][g]), 2);
                if (n > 1) sdv[k][g] = sqrt(sdv[k][g] / (n - 1));
            } else {
                ave[k][g] = 0.0;
                del_thr[k][g] = 0.0;
                dup_thr[k][g] = 0.0;
                wins[k][g] = 0;
            }
        }
    }
    long L = g_max_rd_window_len;
    long *win_count = (long *)calloc(L + 1, sizeof(long));
    long n_win_genome = (g_windows_sampling_factor * len) / (L * g_genome_reduction_factor) + g_windows_sampling_factor;
    double **win_low = (double **)malloc((L + 1) * sizeof(double *));
    for (a = 0; a < L + 1; a++) win_low[a] = (double *)calloc(n_win_genome, sizeof(double));
    /* low-ACGT-or-thin-bin flags, GROM.c:18654-18712 */
    last_low_mq = 0;
    int mqi = 0;
    char *flag = (char *)malloc(len);
    long W = g_one_base_window_size;
    for (pos = 0; pos < g_insert_mean - 1; pos++) flag[pos] = 1;
    for (pos = len - W; pos < len; pos++) flag[pos] = 1;
    for (pos = g_insert_mean - 1; pos < len - W; pos++) {
        if (acgt_w[pos] >= g_insert_min_acgt) {
            if (RDT(pos) == 0) mqi = last_low_mq;
            else if (mql[pos] >= g_rd_min_mapq) { mqi = 0; last_low_mq = 0; }
            else { mqi = 1; last_low_mq = 1; }
            flag[pos] = (wins[mqi][gc_w[pos]] < g_rd_no_combine_min_windows) ? 1 : 0;
        } else {
            flag[pos] = 1;
        }
    }
    /* per-base z score, GROM.c:18740-18963 */
    last_low_mq = 0;
    mqi = 0;
    double *sd = (double *)calloc(len, sizeof(double));
#define GUARD(p) (flag[p] == 0 && ((mql[p] >= g_rd_min_mapq && wins[0][gc_w[p]] > 1) || (mql[p] < g_rd_min_mapq && wins[1][gc_w[p]] > 1)))
#define MQF(p) (g_mapq_factor + (1.0 - g_mapq_factor) * (mql[p] - g_rd_min_mapq) / (double)(g_rd_max_mapq - g_rd_min_mapq))
    for (long bl = 0; bl < g_lowvar_block_index; bl++) {
        for (pos = g_lowvar_block_start_list[bl]; pos < g_lowvar_block_end_list[bl]; pos++) {
            if (!GUARD(pos)) continue;
            if (mql[pos] >= g_rd_min_mapq) { mqi = 0; last_low_mq = 0; }
            else if (RDT(pos) == 0) mqi = last_low_mq;
            else { mqi = 1; last_low_mq = 1; }
            int bin = gc_w[pos];
            long gs = 0, ge = (mqi == 0) ? hi_idx[bin] : lo_idx[bin];
            int *list = (mqi == 0) ? g_sample_hi[bin] : g_sample_lo[bin];
            if (ge <= gs) continue;
            long i1, i2;
            double d1, d2, prob;
            if (RDT(pos) < ave[mqi][bin]) {
                i1 = bisect_right(list, RDT(pos), gs, ge) - gs;
                i2 = bisect_left(list, RDT(pos), gs, ge) - gs;
                d1 = (i1 <= 0) ? 0.5 : (double)i1;
                d2 = (i2 <= 0) ? 0.5 : (double)i2;
                prob = (d1 + d2) / (2 * (ge - gs));
                i1 = bisect_right_double(g_pval2sd_p, prob, 0, g_pval2sd_len);
                if (i1 < 0) i1 = 0;
                else if (i1 >= g_pval2sd_len) i1 = g_pval2sd_len - 1;
                if (g_ranks_stdev == 0) {
                    if (mql[pos] >= g_rd_min_mapq) sd[pos] = MQF(pos) * (ave[mqi][bin] - rd[pos] - low[pos]) / sdv[mqi][bin];
                    else sd[pos] = g_mapq_factor * (ave[mqi][bin] - rd[pos] - low[pos]) / sdv[mqi][bin];
                } else {
                    if (mql[pos] >= g_rd_min_mapq) sd[pos] = MQF(pos) * g_pval2sd_sd[i1];
                    else sd[pos] = g_mapq_factor * g_pval2sd_sd[i1];
                }
            } else {
                if (RDT(pos) > g_dup_threshold_factor * ave[mqi][bin]) {
                    i1 = bisect_left(list, (int)(g_dup_threshold_factor * ave[mqi][bin]), gs, ge); /* Q11 */
                    i2 = bisect_right(list, RDT(pos), gs, ge);
                } else {
                    i1 = bisect_left(list, RDT(pos), gs, ge);
                    i2 = bisect_right(list, RDT(pos), gs, ge);
                }
                i1 = ge - i1;
                i2 = ge - i2;
                d1 = (i1 <= 0) ? 0.5 : (double)i1;
                d2 = (i2 <= 0) ? 0.5 : (double)i2;
                prob = (d1 + d2) / (2 * (ge - gs));
                i1 = bisect_right_double(g_pval2sd_p, prob, 0, g_pval2sd_len);
                if (i1 < 0) i1 = 0;
                else if (i1 >= g_pval2sd_len) i1 = g_pval2sd_len - 1;
                if (g_ranks_stdev == 0) {
                    if (RDT(pos) > (g_dup_threshold_factor * ave[mqi][bin])) {
                        if (mql[pos] >= g_rd_min_mapq)
                            sd[pos] = MQF(pos) * (g_dup_threshold_factor - 1) * (-ave[mqi][bin]) / sdv[mqi][bin];
                        else
                            sd[pos] = g_mapq_factor * (g_dup_threshold_factor - 1) * (-ave[mqi][bin]) / sdv[mqi][bin];
                    } else {
                        if (mql[pos] >= g_rd_min_mapq) sd[pos] = MQF(pos) * (ave[mqi][bin] - rd[pos] - low[pos]) / sdv[mqi][bin];
                        else sd[pos] = g_mapq_factor * (ave[mqi][bin] - rd[pos] - low[pos]) / sdv[mqi][bin];
                    }
                } else {
                    if (mql[pos] >= g_rd_min_mapq) sd[pos] = -MQF(pos) * g_pval2sd_sd[i1];
                    else sd[pos] = -g_mapq_factor * g_pval2sd_sd[i1];
                }
            }
        }
    }
    /* sampled window means by window length, GROM.c:18967-19018.  The window
     * state carries across the sampling passes of a block; temp_win_count
     * carries across blocks. */
    long wlen = 0, temp_win_count = 0, tlc = 0, flag_total = 0;
    double wlen_d, tlc_d, low_total = 0.0;
    for (long bl = 0; bl < g_lowvar_block_sample_index; bl++) {
        wlen = 0;
        low_total = 0;
        flag_total = 0;
        tlc = 0;
        for (long sl = 0; sl < g_windows_sampling_factor; sl++) {
            long adj = sl * L / g_windows_sampling_factor;
            for (pos = g_lowvar_block_sample_start_list[bl] + adj; pos < g_lowvar_block_sample_end_list[bl]; pos++) {
                if (GUARD(pos)) { low_total += sd[pos]; tlc += 1; }
                flag_total += flag[pos];
                wlen += 1;
                if (wlen >= g_min_rd_window_len && temp_win_count == 0) {
                    wlen_d = wlen;
                    if ((flag_total / wlen_d) < g_max_rd_low_acgt_or_windows) {
                        if (tlc > 0) {
                            tlc_d = tlc;
                            win_low[wlen][win_count[wlen]] = low_total / tlc_d;
                            win_count[wlen] += 1;
                        }
                    }
                }
                if (wlen == L) {
                    temp_win_count += 1;
                    if (temp_win_count == g_genome_reduction_factor) temp_win_count = 0;
                    wlen = 0;
                    low_total = 0;
                    flag_total = 0;
                    tlc = 0;
                }
            }
        }
    }
    /* most-biased repeat z scores override, GROM.c:19022-19150 */
    if (g_most_biased_repeat != -1) {
        for (long r = 0; r < pre->rep_n; r++) {
            if (pre->rep_type[r] != g_most_biased_repeat) continue;
            for (pos = pre->rep_start[r] - half; pos < pre->rep_end[r] + half; pos++) {
                if (pos < pre->rep_start[r]) seg = (G_REPEAT_SEGMENTS - 1) * (pos - (pre->rep_start[r] - half)) / half;
                else if (pos >= pre->rep_end[r]) seg = (G_REPEAT_SEGMENTS - 1) * ((pre->rep_end[r] + half) - pos) / half;
                else seg = G_REPEAT_SEGMENTS - 1;
                if (flag[pos] != 0) continue;
                long n = mb_idx[seg];
                int *list = g_sample_rep[seg];
                long i1, i2;
                double d1, d2, prob;
                if (RDT(pos) < rep_ave[seg]) {
                    i1 = bisect_right(list, RDT(pos), 0, n);
                    i2 = bisect_left(list, RDT(pos), 0, n);
                    d1 = (i1 <= 0) ? 0.5 : (double)i1;
                    d2 = (i2 <= 0) ? 0.5 : (double)i2;
                    prob = (d1 + d2) / (2 * n);
                    i1 = bisect_right_double(g_pval2sd_p, prob, 0, g_pval2sd_len);
                    if (i1 < 0) i1 = 0;
                    else if (i1 >= g_pval2sd_len) i1 = g_pval2sd_len - 1;
                    if (g_ranks_stdev == 0) sd[pos] = (rep_ave[seg] - rd[pos] - low[pos]) / rep_sd[seg];
                    else sd[pos] = g_pval2sd_sd[i1];
                } else {
                    if (RDT(pos) > g_dup_threshold_factor * rep_ave[seg]) {
                        i1 = bisect_left(list, (int)(g_dup_threshold_factor * rep_ave[seg]), 0, n);
                        i2 = bisect_right(list, RDT(pos), 0, n);
                    } else {
                        i1 = bisect_left(list, RDT(pos), 0, n);
                        i2 = bisect_right(list, RDT(pos), 0, n);
                    }
                    i1 = n - i1;
                    i2 = n - i2;
                    d1 = (i1 <= 0) ? 0.5 : (double)i1;
                    d2 = (i2 <= 0) ? 0.5 : (double)i2;
                    prob = (d1 + d2) / (2 * n);
                    i1 = bisect_right_double(g_pval2sd_p, prob, 0, g_pval2sd_len);
                    if (i1 < 0) i1 = 0;
                    else if (i1 >= g_pval2sd_len) i1 = g_pval2sd_len - 1;
                    if (g_ranks_stdev == 0) {
                        if (RDT(pos) > g_dup_threshold_factor * rep_ave[seg])
                            sd[pos] = (g_dup_threshold_factor - 1) * (-rep_ave[seg]) / rep_sd[seg];
                        else
                            sd[pos] = (rep_ave[seg] - rd[pos] - low[pos]) / rep_sd[seg];
                    } else {
                        sd[pos] = -g_pval2sd_sd[i1];
                    }
                }
            }
        }
    }
    /* window stdev by length, GROM.c:19156-19179 */
    double *wsd = (double *)calloc(L + 1, sizeof(double));
    for (long w = g_min_rd_window_len; w <= L; w++) {
        double tot = 0.0;
        if (win_count[w] > 1) {
            for (a = 0; a < win_count[w]; a++) tot += win_low[w][a] * win_low[w][a];
            wsd[w] = sqrt(tot / (win_count[w] - 1));
        } else {
            wsd[w] = 0.0;
        }
    }
    for (a = 0; a < L + 1; a++) free(win_low[a]);
    free(win_low);
    free(win_count);

    /* DEL then DUP window search, GROM.c:19359-20020.  sgn = +1 for DEL
     * (low depth, z summed as is), -1 for DUP (high depth, z negated). */
    for (int kind = 0; kind < 2; kind++) {
        cnv_list *out = (kind == 0) ? del : dup;
        double (*thr)[G_NUM_GC_BINS] = (kind == 0) ? del_thr : dup_thr;
        double sgn = (kind == 0) ? 1.0 : -1.0;
#define PASS(p, m) ((kind == 0) ? (RDT(p) <= thr[m][gc_w[p]]) : (RDT(p) >= thr[m][gc_w[p]]))
#define ADD(x, v) ((kind == 0) ? ((x) += (v)) : ((x) -= (v)))
#define SUB(x, v) ((kind == 0) ? ((x) -= (v)) : ((x) += (v)))
        (void)sgn;
        for (long bl = 0; bl < g_lowvar_block_index; bl++) {
            long start = g_lowvar_block_start_list[bl];
            long end = g_lowvar_block_end_list[bl] - g_min_rd_window_len;
            int begin = 0, mqa = 0, mqb = 0;
            long cs = 0, ce = 0, last_good = 0, temp_pos = 0, pa, pb, wl;
            double stdevs = 0.0, tstd, tot;
            long cnt, cnt2, cnt3;
            int stop;
            pos = start;
            mqi = 0;
            last_low_mq = 0;
            while (pos < end) {
                stop = 0;
                if (mql[pos] >= g_rd_min_mapq) { mqi = 0; last_low_mq = 0; }
                else if (RDT(pos) > 0) { mqi = 1; last_low_mq = 1; }
                else mqi = last_low_mq;
                if (PASS(pos, mqi)) {
                    temp_pos = pos;
                    tot = 0;
                    cnt = 0;
                    cnt2 = 0;
                    wl = 0;
                    for (pa = pos; pa < pos + g_min_rd_window_len; pa++) {
                        wl += 1;
                        if (flag[pa] == 0) {
                            if (mql[pa] >= g_rd_min_mapq) mqi = 0;
                            else if (RDT(pa) > 0) mqi = 1;
                            if (PASS(pa, mqi)) cnt2 += 1;
                            else if ((2 * cnt2) < wl) { stop = 1; temp_pos = pa; break; }
                        } else if ((2 * cnt2) < wl) { stop = 1; temp_pos = pa; break; }
                    }
                    if (stop == 0) {
                        cnt = g_min_rd_window_len;
                        tot = 0;
                        for (a = pos; a < pos + g_min_rd_window_len; a++) {
                            if (kind == 0) {
                                /* DEL: flagged bases reduce the count, unflagged z sum (GROM.c:19420-19431) */
                                cnt -= flag[a];
                                tot += sd[a];
                            } else {
                                cnt -= flag[a];
                                tot -= sd[a];
                            }
                        }
                    }
                    if (stop == 0 && cnt > 0 && wsd[g_min_rd_window_len] > 0 &&
                        (tot / (cnt * wsd[g_min_rd_window_len])) >= g_one_base_read_depth_min_rd_low_stdev &&
                        ((g_min_rd_window_len - cnt) / ((double)g_min_rd_window_len)) <= g_max_rd_low_acgt_or_windows) {
                        begin = 1;
                        cs = pos;
                        last_good = pos + g_min_rd_window_len;
                        ce = pos + g_min_rd_window_len;
                        stdevs = tot / (cnt * wsd[g_min_rd_window_len]);
                    }
                    if (stop == 0) {
                        for (pa = pos + g_min_rd_window_len; pa < pos + L; pa++) {
                            wl += 1;
                            if (pa < end) {
                                if (flag[pa] == 0) {
                                    if (mql[pa] >= g_rd_min_mapq) mqi = 0;
                                    else if (RDT(pa) > 0) mqi = 1;
                                    ADD(tot, sd[pa]);
                                    cnt += 1;
                                    if (PASS(pa, mqi)) {
                                        cnt2 += 1;
                                        if (wsd[wl] > 0 && (tot / (cnt * wsd[wl])) >= g_one_base_read_depth_min_rd_low_stdev &&
                                            ((wl - cnt) / ((double)wl)) <= g_max_rd_low_acgt_or_windows) {
                                            last_good = pa;
                                            if (begin == 0) {
                                                begin = 1;
                                                cs = pos;
                                                ce = pa;
                                                stdevs = tot / (cnt * wsd[wl]);
                                            } else {
                                                tstd = tot / (cnt * wsd[wl]);
                                                ce = pa;
                                                if (tstd > stdevs) stdevs = tstd;
                                            }
                                        }
                                    } else if ((2 * cnt2) < wl) { stop = 1; break; }
                                } else if ((2 * cnt2) < wl) { stop = 1; break; }
                            } else { stop = 1; break; }
                        }
                    }
                    if (stop == 0 && begin == 1) {
                        pa = pos + L;
                        tot = 0;
                        cnt = 0;
                        mqb = mqi;
                        while (pa < len && (pa - last_good) <= g_max_distance_since_last_del_good) {
                            if (pa == (pos + L)) {
                                for (pb = (pa - L + 1); pb < (pa + 1); pb++) {
                                    if (mql[pb] >= g_rd_min_mapq) mqb = 0;
                                    else if (RDT(pb) > 0) mqb = 1;
                                    if (flag[pb] == 0 && wins[mqb][gc_w[pb]] > 1) { ADD(tot, sd[pb]); cnt += 1; }
                                }
                            } else {
                                pb = pa - L;
                                if (mql[pb] >= g_rd_min_mapq) mqb = 0;
                                else if (RDT(pb) > 0) mqb = 1;
                                if (flag[pb] == 0 && wins[mqb][gc_w[pb]] > 1) { SUB(tot, sd[pb]); cnt -= 1; }
                                if (mql[pa] >= g_rd_min_mapq) mqi = 0;
                                else if (RDT(pa) > 0) mqi = 1;
                                if (flag[pa] == 0 && wins[mqi][gc_w[pa]] > 1) { ADD(tot, sd[pa]); cnt += 1; }
                            }
                            if (cnt > 0 && wsd[L] > 0 && (tot / (cnt * wsd[L])) >= g_one_base_read_depth_min_rd_low_stdev &&
                                ((L - cnt) / ((double)L)) <= g_max_rd_low_acgt_or_windows) {
                                last_good = pa;
                                ce = pa;
                                tstd = tot / (cnt * wsd[L]);
                                if (tstd > stdevs) stdevs = tstd;
                            }
                            pa += 1;
                        }
                    }
                    if (begin == 1) {
                        /* trim the end back to depth-consistent bases, GROM.c:19550-19600 */
                        pos = ce;
                        while (pos > (cs + g_min_rd_window_len)) {
                            if (mql[pos] >= g_rd_min_mapq) mqi = 0;
                            else if (RDT(pos) > 0) mqi = 1;
                            if (!PASS(pos, mqi)) {
                                pos -= 1;
                                ce = pos;
                            } else {
                                cnt2 = 0;
                                cnt3 = 0;
                                pa = ce;
                                int stop_while = 0;
                                mqa = mqi;
                                while (pa > (cs + g_min_rd_window_len) && stop_while == 0) {
                                    if (flag[pa] == 0) {
                                        if (mql[pa] >= g_rd_min_mapq) mqa = 0;
                                        else if (RDT(pa) > 0) mqa = 1;
                                        cnt3 += 1;
                                        if (PASS(pa, mqa)) cnt2 += 1;
                                    }
                                    if (cnt3 == 0 || (cnt3 > 0 && (cnt2 / ((double)cnt3)) < 0.5) ||
                                        ((ce - pa + 1 - cnt3) / ((double)ce - (double)pa + 1.0)) > g_max_rd_low_acgt_or_windows) {
                                        ce = pa - 1;
                                        stop_while = 1;
                                    }
                                    pa -= 1;
                                }
                                pos = pa;
                            }
                        }
                        pos = ce + 1;
                        out->start[out->n] = cs;
                        out->end[out->n] = ce;
                        out->stdev[out->n] = stdevs;
                        out->n += 1;
                        cs = 0;
                        ce = 0;
                        stdevs = 0;
                        last_good = 0;
                        begin = 0;
                    } else if (stop == 1) {
                        pos = temp_pos;
                    }
                }
                pos += 1;
            }
        }
#undef PASS
#undef ADD
#undef SUB
    }
    /* copy-number estimate, GROM.c:20024-20228 */
    long longest[2] = {0, 0};
    for (a = 0; a < del->n; a++) if (del->end[a] - del->start[a] > longest[0]) longest[0] = del->end[a] - del->start[a];
    for (a = 0; a < dup->n; a++) if (dup->end[a] - dup->start[a] > longest[1]) longest[1] = dup->end[a] - dup->start[a];
    for (int kind = 0; kind < 2; kind++) {
        cnv_list *l = (kind == 0) ? del : dup;
        double *pl = (double *)malloc((longest[kind] + 1) * sizeof(double));
        for (a = 0; a < l->n; a++) {
            double ploidy_sum = 0.0;
            long pc = 0;
            for (b = l->start[a]; b < l->end[a]; b++) {
                if (flag[b] != 0) continue;
                int k = (mql[b] >= g_rd_min_mapq) ? 0 : 1;
                if (ave[k][gc_w[b]] > 0) { pl[pc] = (double)RDT(b) / ave[k][gc_w[b]]; pc += 1; }
            }
            if (pc > 0) {
                qsort_dbl_intcmp(pl, pc);
                long s0 = 0.1 * pc;
                long e0 = pc - s0;
                for (long c = s0; c < e0; c++) ploidy_sum += pl[c];
                if ((e0 - s0) > 0) {
                    l->cn[a] = (ploidy_sum / (e0 - s0)) * ploidy;
                    l->cn_stdev[a] = 0;
                    for (long c = 0; c < pc; c++) l->cn_stdev[a] += pow((ploidy * pl[c] - l->cn[a]), 2);
                    l->cn_stdev[a] = sqrt(l->cn_stdev[a] / pc);
                } else {
                    l->cn[a] = -1;
                    l->cn_stdev[a] = 0;
                }
            } else {
                l->cn[a] = -1;
                l->cn_stdev[a] = 0;
            }
        }
        free(pl);
    }
    /* the -N side file <results>.1000gen.<chr>, GROM.c:20234-20345: per
     * complete window of g_1000gen_window bases, the copy number of the
     * window's qualifying bases and its deviation */
    if (g_1000gen_window > 0 && g_1000gen_base && g_1000gen_chr) {
        char *fn = (char *)malloc(strlen(g_1000gen_base) + strlen(g_1000gen_chr) + 16);
        sprintf(fn, "%s.1000gen.%s", g_1000gen_base, g_1000gen_chr);
        FILE *gf = fopen(fn, "w");
        if (gf == NULL) {
            printf("\nCould not open %s\n", fn);
            exit(1);
        }
        double *gl = (double *)malloc((g_1000gen_window + 1) * sizeof(double));
        double g_sum = 0.0, g_cn, g_sd;
        long g_n = 0, g_nw = 0;
        for (a = 0; a < len; a++) {
            if (flag[a] == 0) {
                int k = (mql[a] >= g_rd_min_mapq) ? 0 : 1;
                if (ave[k][gc_w[a]] > 0) { gl[g_n] = (double)RDT(a) / ave[k][gc_w[a]]; g_n += 1; }
            }
            g_nw += 1;
            if (g_nw == g_1000gen_window) {
                if (g_n > 0) {
                    for (long c = 0; c < g_n; c++) g_sum += gl[c];
                    g_cn = (g_sum / g_n) * ploidy;
                    g_sd = 0;
                    for (long c = 0; c < g_n; c++) g_sd += pow((ploidy * gl[c] - g_cn), 2);
                    g_sd = sqrt(g_sd / g_n);
                } else {
                    g_cn = -1;
                    g_sd = 0;
                }
                fprintf(gf, "%ld\t%e\t%e\n", a - g_1000gen_window + 1, g_cn, g_sd);
                g_n = 0;
                g_nw = 0;
                g_sum = 0;
            }
        }
        fclose(gf);
        free(gl);
        free(fn);
    }
#undef GUARD
#undef MQF
    free(wsd);
    free(sd);
    free(flag);
}

/* Chromosome statistics, blocks, detect_del_dup and the CNV rows
 * (GROM.c:16633-17300).  `mql` is caf_rd_mq_list; it is divided in place. */
static void cnv_chromosome(long len, const char *fa, const cnv_pre *pre, int *mql, const int *rd, const int *low,
                           const char *chr_name, FILE *vcf) {
    long a, b;
    for (a = 0; a < len; a++)
        if ((rd[a] + low[a]) > 0) mql[a] = mql[a] / (rd[a] + low[a]);
    long W = g_one_base_window_size;
    double chr_ave = 0, chr_sd = 0;
    long chr_cnt = 0;
    for (a = g_insert_mean - 1; a < len - W; a++)
        if (pre->acgt_w[a] >= g_insert_min_acgt) { chr_ave += rd[a] + low[a]; chr_cnt += 1; }
    if (chr_cnt > 0) chr_ave = chr_ave / chr_cnt;
    for (a = g_insert_mean - 1; a < len - W; a++) {
        if (pre->acgt_w[a] >= g_insert_min_acgt) {
            if ((rd[a] + low[a]) < 2 * chr_ave) chr_sd += ((rd[a] + low[a]) - chr_ave) * ((rd[a] + low[a]) - chr_ave);
            else chr_sd += chr_ave * chr_ave;
        }
    }
    chr_sd = (chr_cnt > 1) ? sqrt(chr_sd / ((double)chr_cnt - 1.0)) : 0;
    /* repeat-type depth, GROM.c:16693-16775 */
    double rep_ave[10], rep_sd[10];
    long rep_cnt[10];
    for (a = 0; a < 10; a++) { rep_ave[a] = 0; rep_sd[a] = 0; rep_cnt[a] = 0; }
    double *rrl = (double *)malloc((pre->rep_n + 1) * sizeof(double));
    for (a = 0; a < pre->rep_n; a++) {
        long s = 0;
        for (b = pre->rep_start[a]; b < pre->rep_end[a]; b++) s += rd[b] + low[b];
        rrl[a] = (double)s / (pre->rep_end[a] - pre->rep_start[a]);
        if (rrl[a] < 2 * chr_ave) rep_ave[pre->rep_type[a]] += rrl[a];
        else rep_ave[pre->rep_type[a]] += 2 * chr_ave;
        rep_cnt[pre->rep_type[a]] += 1;
    }
    for (a = 0; a < 10; a++) rep_ave[a] = rep_ave[a] / (double)rep_cnt[a];
    for (a = 0; a < pre->rep_n; a++) {
        int t = pre->rep_type[a];
        if (rrl[a] < 2 * chr_ave) rep_sd[t] += (rrl[a] - rep_ave[t]) * (rrl[a] - rep_ave[t]);
        else rep_sd[t] += ((2 * chr_ave) - rep_ave[t]) * ((2 * chr_ave) - rep_ave[t]);
    }
    free(rrl);
    for (a = 0; a < 10; a++) rep_sd[a] = (rep_cnt[a] > 1) ? sqrt(rep_sd[a] / ((double)rep_cnt[a] - 1.0)) : 0;
    g_most_biased_repeat = -1;
    long biased_cnt = 0;
    for (a = 0; a < 10; a++) {
        if (rep_cnt[a] > g_rd_no_combine_min_windows &&
            (rep_ave[a] + (g_min_repeat_stdev * rep_sd[a])) < chr_ave &&
            (chr_ave - (g_min_repeat_stdev * chr_sd)) > rep_ave[a] && rep_cnt[a] > biased_cnt) {
            g_most_biased_repeat = (int)a;
            biased_cnt = rep_cnt[a];
        }
    }
    /* 10 kb coverage blocks, GROM.c:16784-16912 */
    long nblocks = len / g_block_unit_size;
    double *blk = (double *)malloc((nblocks + 1) * sizeof(double));
    long *over = (long *)malloc((nblocks + 1) * sizeof(long));
    long blk_total = 0, chr_blk_total = 0, bin_count = 0, blk_count = 0, nb = 0, nover = 0;
    for (a = 0; a < len; a++) {
        char ch = fa[a];
        if (ch && (strchr("CGcg", ch) || strchr("ATat", ch))) { chr_blk_total += rd[a] + low[a]; blk_count += 1; }
        blk_total += rd[a] + low[a];
        bin_count += 1;
        if (bin_count == g_block_unit_size) {
            blk[nb] = blk_total / (double)bin_count;
            nb += 1;
            bin_count = 0;
            blk_total = 0;
        }
    }
    double chr_rd_ave = chr_blk_total / (double)blk_count;
    double chr_rd_thr = g_chr_rd_threshold_factor * chr_rd_ave;
    for (a = 0; a < nb; a++)
        if (blk[a] > chr_rd_thr) over[nover++] = a;
    long tb = 0, tbs = 0, tbe = 0, block_index = 0;
    if (nover > 1) {
        for (a = 1; a < nover; a++) {
            if (tb == 0) {
                if ((tb + 1) > ((over[a] - over[a - 1]) / g_block_factor)) { tbe = over[a] + 1; tb += 1; }
                else tbe = over[a - 1] + 1;
                tbs = over[a - 1];
                tb += 1;
            } else {
                if ((tb + 1) > ((over[a - 1] - tbs) / g_block_factor)) { tbe = over[a - 1] + 1; tb += 1; }
                else {
                    if (tb >= g_min_blocks) block_index += 1;
                    tb = 0;
                    tbs = over[a - 1];
                    tbe = over[a - 1] + 1;
                    tb += 1;
                }
                if (tb >= g_min_blocks && block_index < MAX_BLOCK_LIST_LEN) {
                    g_block_start_list[block_index] = tbs * g_block_unit_size;
                    g_block_end_list[block_index] = tbe * g_block_unit_size;
                }
            }
        }
    }
    if (tb >= g_min_blocks) block_index += 1;
    free(blk);
    free(over);
    /* low-variance blocks (the complement of high-depth blocks), GROM.c:16913-16993 */
    g_lowvar_block_index = 0;
    g_lowvar_block_start_list[0] = 0; /* GROM.c:21899; later chromosomes keep whatever this slot holds */
    for (a = 0; a < block_index; a++) {
        if ((g_block_end_list[a] - g_block_start_list[a]) >= g_block_min) {
            g_lowvar_block_end_list[g_lowvar_block_index] = g_block_start_list[a];
            g_lowvar_block_start_list[g_lowvar_block_index + 1] = g_block_end_list[a];
            g_lowvar_block_index += 1;
        }
    }
    g_lowvar_block_index += 1;
    g_lowvar_block_end_list[g_lowvar_block_index - 1] = len;
    for (long k = 0; k < g_lowvar_block_index; k++) {
        if (g_lowvar_block_start_list[k] < (g_insert_mean - 1)) g_lowvar_block_start_list[k] = g_insert_mean - 1;
        else if (g_lowvar_block_start_list[k] >= (len - W)) g_lowvar_block_start_list[k] = len - W;
        if (g_lowvar_block_end_list[k] < (g_insert_mean - 1)) g_lowvar_block_end_list[k] = g_insert_mean - 1;
        else if (g_lowvar_block_end_list[k] >= (len - W)) g_lowvar_block_end_list[k] = len - W;
    }
    long k = 0;
    while (k < g_lowvar_block_index) {
        if ((g_lowvar_block_end_list[k] - g_lowvar_block_start_list[k]) < g_min_rd_window_len) {
            for (long k2 = k + 1; k2 < g_lowvar_block_index; k2++) {
                g_lowvar_block_start_list[k2 - 1] = g_lowvar_block_start_list[k2];
                g_lowvar_block_end_list[k2 - 1] = g_lowvar_block_end_list[k2];
            }
            g_lowvar_block_index -= 1;
        } else {
            k += 1;
        }
    }
    for (k = 0; k < g_lowvar_block_index; k++) {
        g_lowvar_block_sample_start_list[k] = g_lowvar_block_start_list[k];
        g_lowvar_block_sample_end_list[k] = g_lowvar_block_end_list[k];
    }
    g_lowvar_block_sample_index = g_lowvar_block_index;

    /* detect_del_dup over one block spanning the chromosome, GROM.c:17122-17135 */
    int ploidy = g_ploidy; /* Q16: caf_bam_name_len never matches, no chrX halving */
    long cap = len / g_min_rd_window_len + 1;
    cnv_list del, dup;
    cnv_list_init(&del, cap);
    cnv_list_init(&dup, cap);
    g_lowvar_block_start_list[0] = g_insert_mean - 1;
    g_lowvar_block_end_list[0] = len - W;
    g_lowvar_block_index = 1;
    g_res_over = g_res_repl = 0;
    g_1000gen_chr = chr_name;
    detect_del_dup(len, pre->gc_w, pre->acgt_w, mql, rd, low, pre, ploidy, &del, &dup);
    if (getenv("GROM_CNV_STATS")) {
        FILE *sf = fopen(getenv("GROM_CNV_STATS"), "a");
        if (sf) { fprintf(sf, "%s over=%ld repl=%ld\n", chr_name, g_res_over, g_res_repl); fclose(sf); }
    }
    /* p value (Q8: t = 1/(1+p+x)) and filter, GROM.c:17139-17236 */
    double p = 0.3275911, a1 = 0.254829592, a2 = -0.284496736, a3 = 1.421413741, a4 = -1.453152027,
           a5 = 1.061405429;
    for (int kind = 0; kind < 2; kind++) {
        cnv_list *l = (kind == 0) ? &del : &dup;
        double *pv = (double *)malloc((l->n + 1) * sizeof(double));
        for (a = 0; a < l->n; a++) {
            double x = fabs(l->stdev[a]) / sqrt(2.0);
            double t = 1.0 / (1.0 + p + x);
            double erf_ = 1.0 - ((a1 * t + a2 * pow(t, 2) + a3 * pow(t, 3) + a4 * pow(t, 4) + a5 * pow(t, 5)) *
                                 exp(-pow(x, 2)));
            pv[a] = (1.0 - erf_) / 2.0;
        }
        /* -f: a column header before each kind's rows, GROM.c:17242-17245, 17378 */
        if (g_vcf == 0) fprintf(vcf, "SV Type\tChromosome\tStart\tEnd\tStdev from mean\tP Value\tCopy Number\n");
        /* caf_old_*_list_index stays 0, so every passing call is written */
        for (a = 0; a < l->n; a++) {
            if (!(pv[a] < g_rd_pval_threshold)) continue;
            if (g_vcf == 1)
                fprintf(vcf, "%s\t%ld\t.\t.\t%s\t.\t.\tEND=%ld\tSD:Z:CN:CS\t%e:%e:%.2f:%e\n", chr_name, l->start[a] + 1,
                        kind == 0 ? "<DEL>" : "<DUP>", l->end[a] + 1, l->stdev[a], pv[a], l->cn[a], l->cn_stdev[a]);
            else /* GROM.c:17340-17343 (caf_del_text / caf_dup_text, GROM.c:1575-1576) */
                fprintf(vcf, "%s\t%s\t%ld\t%ld\t%e\t%e\t%e\t%e\n", kind == 0 ? "DEL RD" : "DUP RD", chr_name, l->start[a],
                        l->end[a], l->stdev[a], pv[a], l->cn[a], l->cn_stdev[a]);
        }
        free(pv);
    }
    cnv_list_free(&del);
    cnv_list_free(&dup);
}
