/*
 * grom_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of GROM v1.0.1's per-chromosome scan (GROM.c), used by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * checker.  It is never linked into, called by or shipped with the product
 * path (grom_amd/).  See oracle/README.md for its pinning status.
 */
#ifndef GROM_ORACLE_H
#define GROM_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Per-position counters, in the order the reference declares them
 * (GROM.c:2923-3680).  `rd` is cdp_one_base_rd. */
typedef struct orc_counts {
    int32_t pos;
    int32_t snv[4], snv_lowmq[4];
    int32_t bq, bq_all, mq, mq_all, bq_rc, mq_rc, rc_all;
    int32_t pir[4], fs[4];
    int32_t rd;
    int32_t sc_left, sc_right, sc_left_rd, sc_right_rd, sc_rd;
    int32_t ctx_sc_left, ctx_sc_right, ctx_sc_left_rd, ctx_sc_right_rd, ctx_sc_rd;
    int32_t indel_sc_left, indel_sc_right, indel_sc_left_rd, indel_sc_right_rd, indel_sc_rd;
} orc_counts;

/* CIGAR indel evidence of one base (row A7, GROM.c:7187-7423): the primary
 * insertion / forward-deletion / reverse-deletion counters with their lengths,
 * the deletion read depths, how many of the base's "other" slots are occupied
 * (the first OTHER_EMPTY index, as GROM.c:11415-11425 computes it) and the
 * 50-byte inserted-sequence buffer (zero-filled when the base enters the
 * window, GROM.c:5634-5636, 6030-6040).  Only indel-typed "other" slots exist
 * here: the discordant-pair and split-read types that share them (A8/A9) are
 * not restated.  Same layout as grom_indel_rec (include/grom_amd.h). */
typedef struct orc_indel {
    int32_t pos;
    int32_t ins, ins_len;
    int32_t del_f, del_f_len, del_f_rd;
    int32_t del_r, del_r_len, del_r_rd;
    int32_t other_len;
    char ins_seq[52];
    int32_t pad;
} orc_indel;

/* Breakpoint cluster state of one evaluated base (rows A8/A9), same layout
 * as grom_sv_rec (include/grom_amd.h): per cluster type (DEL_F, DEL_R,
 * DUP_F, DUP_R, INV_F1, INV_R1, INV_F2, INV_R2, CTX_F, CTX_R) the weighted
 * count, first/last read position and running-mean distance; the CTX mate
 * chromosomes; the occupied "other" slots; the pair binning's depth adds,
 * concordant pairs, short-insert pairs and unmapped-mate reads. */
typedef struct orc_sv_rec {
    int32_t pos, other_len;
    int32_t cnt[10], rs[10], re[10];
    double dist[10];
    int32_t ctx_mchr[2];
    int32_t rd_add, conc, ins, mun_f, mun_r, pad;
} orc_sv_rec;

/* Run the reference CLI semantics: argv as for GROM (-i -r -o ...).
 * If dump_prefix is non-NULL, for every processed chromosome the counters of
 * every evaluated base (p > 2*insert_max, GROM.c:11086) are written to
 * <dump_prefix>.<chrname>.cnt as packed orc_counts records, and the caf read
 * depth arrays to <dump_prefix>.<chrname>.caf (3 x int32 x chr_len), and
 * the indel evidence of every evaluated base that any CIGAR I/D op touched
 * to <dump_prefix>.<chrname>.ind as packed orc_indel records, and the
 * breakpoint state of every evaluated base with any to <dump>.<chr>.sv.
 * Returns the process exit code the reference would return. */
int grom_oracle_main(int argc, char **argv, const char *dump_prefix);

/* The mq and hez binomial tables (1001 x 1001 doubles each, row-major) as a
 * run with `-q min_mapq` uses them, i.e. after the "%e" text round trip. */
void grom_oracle_tables(int min_mapq, double *mq_out, double *hez_out);
/* the SNV acceptance test of one base (GROM.c:11126-11156): the picked alt or -1 */
int grom_oracle_snv_pick(const int snv[4], int ref, long bq_all, long rc_all, int min_snv, double min_ratio,
                         double min_ave_bq);

/* test hooks of the CNV path's library restatements (cnv_oracle.c) */
void grom_oracle_rand_seq(unsigned int seed, int n, int *out);
void grom_oracle_msort_lo(double *a, long n);
void grom_oracle_grom_rand(unsigned int seed, long mx, int n, long *out);

#ifdef __cplusplus
}
#endif
#endif
