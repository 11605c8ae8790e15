/*
 * tables.c -- parameters and binomial tables of the scan (host side).
 *
 * grom_build_tables restates read_binom_tables (GROM.c:21134-21586) and
 * calculate_normal_binom_constants (GROM.c:21589-21626).  GROM computes the
 * tables once, writes them next to its executable as "%e" text and from then
 * on parses that text (GROM.c:21343-21355, 21531-21545), so every steady-state
 * run sees 7-significant-digit values; the tables are therefore produced at
 * full precision and passed through the same "%e" round trip here.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "../../include/grom_amd.h"

#define NT (GROM_MAX_TRIALS + 1)

/* Abramowitz-Stegun erf constants used throughout GROM (GROM.c:21157-21162) */
static const double AS_P = 0.3275911, AS_A1 = 0.254829592, AS_A2 = -0.284496736, AS_A3 = 1.421413741,
                    AS_A4 = -1.453152027, AS_A5 = 1.061405429;

static double as_erf(double x) {
    double t = 1.0 / (1.0 + AS_P * x);
    return 1.0 - (AS_A1 * t + AS_A2 * pow(t, 2) + AS_A3 * pow(t, 3) + AS_A4 * pow(t, 4) + AS_A5 * pow(t, 5)) *
                     exp(-pow(x, 2));
}

/* x86-64 `long = double`: cvttsd2si yields 0x8000000000000000 out of range */
static int64_t cvt_long(double v) {
    if (!(v > -9223372036854775808.0 && v < 9223372036854775808.0)) return INT64_MIN;
    return (int64_t)v;
}

/* P(X >= successes) for X ~ Bin(n, prob) the way GROM evaluates it: Poisson
 * when n is large and prob small, normal approximation past `norm_k`
 * successes, exact sum otherwise (GROM.c:21226-21301 / 21401-21476). */
static double upper_tail(int64_t n, int64_t successes, double prob, int64_t norm_k) {
    double cdf = 0;
    if ((n >= 20 && prob <= 0.05) || (n >= 100 && n * prob <= 10)) {
        double lambda = n * prob;
        uint64_t fact = 1; /* a C `long` in GROM: wraps like this past 20! */
        for (int64_t k = 0; k < successes; k++) {
            if (k > 1) fact *= (uint64_t)k;
            cdf += pow(lambda, k) * exp(-lambda) / (double)(int64_t)fact;
        }
    } else if (n * prob * (1 - prob) >= 5 && successes >= norm_k) {
        double sd = sqrt(n * prob * (1.0 - prob));
        double z = (n * prob - successes + 0.5) / sd;
        double e = as_erf(z / sqrt(2.0));
        cdf = (z >= 0) ? (1.0 - e) / 2.0 : 1 - (e + (1.0 - e) / 2.0);
    } else {
        int64_t rem = n, comb = 1;
        for (int64_t k = 0; k < successes; k++) {
            cdf += comb * pow(prob, k) * pow((1 - prob), rem);
            comb = (k > 0) ? cvt_long((comb / (k + 1.0)) * rem) : cvt_long((double)comb * rem);
            rem -= 1;
        }
    }
    if (cdf < 0) cdf = 0;
    if (cdf > 1) cdf = 1;
    return 1.0 - cdf;
}

static double through_text(double v) {
    char b[48];
    snprintf(b, sizeof(b), "%e", v);
    return strtod(b, NULL);
}

/* One row of both tables: the upper tails, GROM's clamps, the mq tails and
 * the text round trip.  Rows depend only on themselves (the clamp reads the
 * row's next tail and its own clamped previous column, the mq stop rule the
 * row's previous columns), so rows are built on threads. */
static void build_row(int r, double p, double *hez, double *mq) {
#define H(r, c) hez[(size_t)(r) * NT + (c)]
#define M(r, c) mq[(size_t)(r) * NT + (c)]
    if (r >= 1)
        for (int64_t s = 0; s <= r; s++) H(r, s) = upper_tail(r, s, 0.5, 17);
    /* turn the upper tail into P(X <= c) with GROM's clamps (GROM.c:21309-21324) */
    if (r < GROM_MAX_TRIALS) {
        for (int c = 0; c < GROM_MAX_TRIALS; c++) {
            double v = 1.0 - H(r, c + 1);
            if (v < 0) v = 0;
            if (c > 0 && H(r, c - 1) == 1) v = 1;
            H(r, c) = v;
        }
        H(r, GROM_MAX_TRIALS) = 1.0;
    }
    if (r >= 1)
        for (int64_t s = 0; s <= r; s++) {
            int stop = (s > 0 && M(r, s - 1) == 0) || (s > 1 && M(r, s - 1) == M(r, s - 2));
            M(r, s) = stop ? 0 : upper_tail(r, s, p, 20);
        }
    for (size_t i = (size_t)r * NT; i < (size_t)(r + 1) * NT; i++) {
        hez[i] = through_text(hez[i]);
        mq[i] = through_text(mq[i]);
    }
#undef H
#undef M
}

typedef struct {
    double p, *hez, *mq;
    int next;
    pthread_mutex_t mu;
} table_job;

static void *table_main(void *arg) {
    table_job *j = (table_job *)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        const int r = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (r >= NT) break;
        /* rows taken longest first (row r costs ~r entries) */
        build_row(NT - 1 - r, j->p, j->hez, j->mq);
    }
    return NULL;
}

void grom_build_tables(int32_t min_mapq, double *hez, double *mq) {
    memset(hez, 0, sizeof(double) * NT * NT);
    memset(mq, 0, sizeof(double) * NT * NT);
    table_job j;
    j.p = pow(10, (-min_mapq / 10.0)); /* g_mq_prob, GROM.c:21616 */
    j.hez = hez;
    j.mq = mq;
    j.next = 0;
    pthread_mutex_init(&j.mu, NULL);
    long nc = sysconf(_SC_NPROCESSORS_ONLN);
    int nt = nc < 1 ? 1 : (nc > 16 ? 16 : (int)nc);
    pthread_t th[16];
    int started = 0;
    for (int t = 1; t < nt; t++) {
        if (pthread_create(&th[started], NULL, table_main, &j) != 0) break;
        started++;
    }
    table_main(&j);
    for (int t = 0; t < started; t++) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&j.mu);
}

void grom_default_params(grom_params *p) {
    memset(p, 0, sizeof(*p));
    p->min_mapq = 20;
    p->rd_min_mapq = 20;
    p->min_base_qual = 20;
    p->min_snv = 3;
    p->ploidy = 2;
    p->gender = 0;
    p->splitread = 1;
    p->rmdup = 0;
    p->vcf = 1;
    p->overlap_mult = 1;
    p->sv_list_len = 1000000;
    p->rmdup_list_len = 10000;
    p->read_name_len = 50;
    p->sc_min = 1;
    p->min_snv_ratio = 0.2;
    p->min_ave_bq = 15;
    p->snv_rd_min_factor = 1.75;
    p->high_cov_min_snv_ratio = 0.4;
    p->ranks_stdev = 1;
    p->chr_rd_threshold_factor = 2;
    p->min_repeat = 20;
    p->min_blocks = 4;
    p->block_min = 10000;
    p->min_rd_window_len = 100;
    p->max_rd_window_len = 10000;
    p->windows_sampling_factor = 2;
    p->dup_threshold_factor = 2;
    p->min_repeat_stdev = 1.5;
    p->rd_pval_threshold = 0.000000001;
    p->mapq_factor = 0.5;
    /* breakpoint path (GROM.c:810-969) */
    p->min_disc = 3;
    p->sc_range = 35;
    p->max_split_loss = 20;
    p->min_sr_len = 30;
    p->max_homopolymer = 10;
    p->max_ins_range = 10;
    p->sv_list2_len = p->sv_list_len / 10;
    p->pval_threshold = 0.001;
    p->pval_threshold1 = 0.001; /* = g_pval_threshold, GROM.c:22101 */
    p->pval_insertion1 = 0.01;
    p->pval_insertion = 0.0000000001;
    p->min_sv_ratio = 0.05;
    p->min_indel_ratio = 0.125;
    p->max_evidence_ratio = 0.25;
    p->range_mult = 0.75;
    p->max_inv_rd_diff = 1.75;
    p->min_overlap_ratio = 0.5;
    p->gen1000_window = 0;
}

void grom_params_set_insert(grom_params *p, int32_t mean, int32_t imin, int32_t imax, int32_t lseq) {
    if (mean < lseq) mean = lseq; /* GROM.c:22260-22263 */
    p->insert_mean = mean;
    p->insert_min_size = imin;
    p->insert_max_size = imax;
    p->lseq = lseq;
    int32_t half = p->overlap_mult * 8 * (2 * mean - 1); /* GROM.c:22282-22290 */
    if (p->overlap_mult * 8 * (imax + 1) > half) half = p->overlap_mult * 8 * (imax + 1);
    p->half_one_base_rd_len = half;
    p->r34_one_base_rd_len = half + half / 2;
    p->r14_one_base_rd_len = p->r34_one_base_rd_len - half;
    p->one_base_rd_len = 2 * half;
}

void grom_out_free(grom_out *o) {
    free(o->vcf);
    free(o->ctx);
    free(o->side);
    memset(o, 0, sizeof(*o));
}
