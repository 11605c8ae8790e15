/*
 * scan_common.h -- layouts shared by the HIP scan kernels and their host code.
 */
#ifndef GROM_AMD_SCAN_COMMON_H
#define GROM_AMD_SCAN_COMMON_H

#include <stdint.h>

/* positions per tile of the pileup kernel and threads per tile */
#ifndef GROM_TILE
#define GROM_TILE 256
#endif
#define GROM_TILE_THREADS GROM_TILE
/* read-name slots per position supported by the kernel (g_min_snv, -n);
 * the gather kernel is also built with GROM_FEW_NAME_SLOTS for -n up to that */
#define GROM_MAX_NAME_SLOTS 32 /* register builds for 4, 8, 16 and 32 slots */
#define GROM_MEM_SLOT_BLOCKS 2048 /* -n above 32: workgroups of the global-slot kernel */
#define GROM_MEM_SLOT_BUDGET ((size_t)256 << 20) /* at most this much name-slot scratch (bytes) */
#define GROM_FEW_NAME_SLOTS 4

/* order of the GROM_NCOUNT int32 per-base counters exported by
 * grom_debug_counts; it follows the reference's declarations
 * (cdp_one_base_*, GROM.c:2923-3680) */
enum {
    GC_POS = 0,
    GC_SNV = 1,        /* 4: cdp_one_base_snv[A,C,G,T] */
    GC_SNV_LOWMQ = 5,  /* 4 */
    GC_BQ = 9, GC_BQ_ALL, GC_MQ, GC_MQ_ALL, GC_BQ_RC, GC_MQ_RC, GC_RC_ALL,
    GC_PIR = 16,       /* 4: cdp_one_base_pos_in_read */
    GC_FS = 20,        /* 4: cdp_one_base_fstrand */
    GC_RD = 24,        /* cdp_one_base_rd */
    GC_SC_LEFT = 25, GC_SC_RIGHT, GC_SC_LEFT_RD, GC_SC_RIGHT_RD, GC_SC_RD,
    GC_CTX_SC_LEFT = 30, GC_CTX_SC_RIGHT, GC_CTX_SC_LEFT_RD, GC_CTX_SC_RIGHT_RD, GC_CTX_SC_RD,
    GC_INDEL_SC_LEFT = 35, GC_INDEL_SC_RIGHT, GC_INDEL_SC_LEFT_RD, GC_INDEL_SC_RIGHT_RD, GC_INDEL_SC_RD,
    GC_COUNT = 40
};

/* one SNV list entry (cdp_snv_*_list, GROM.c:3714-3790) */
typedef struct grom_snv_cand {
    int32_t pos;
    int32_t base;
    float ratio;
    int32_t ref_base;  /* cdp_chr_fasta[pos] as loaded (the VCF REF column) */
    double binom;
    double hez;
    int32_t snv[4], lowmq[4], pir[4], fs[4];
    int32_t bq, bq_all, mq, mq_all, bq_rc, mq_rc, rc_all;
    int32_t pad1;
} grom_snv_cand;

/* The pileup's counters at a position the breakpoint tests may use (row
 * A10): every position with soft-clip evidence, and the positions the SV
 * fold or the insertion ranges mark (sv.hip). */
typedef struct grom_sv_ctx {
    int32_t pos;
    int32_t rd;            /* physical depth over the read spans (GROM.c:7173-7181) */
    int32_t sc_rd, indel_sc_rd;
    int32_t sc_left, sc_right, sc_left_rd, sc_right_rd;
    int32_t indel_sc_left, indel_sc_right;
    int32_t snv_all;       /* sum of snv[4] + snv_lowmq[4] (GROM.c:11341-11344) */
    int32_t pad;
} grom_sv_ctx;

/* scan-wide scalars handed to the kernels */
typedef struct grom_scan_args {
    int64_t chr_len;
    int64_t n_reads;
    int32_t max_span;       /* longest M/D/N/=/X reference extent of any read */
    int32_t eval_lo;        /* first evaluated base: max(index_start, 2*insert_max+1) */
    int32_t eval_hi;        /* last evaluated base (p_last) or -1 */
    int32_t flush_end;      /* final SNV flush range end (p_end - index_end) */
    int32_t min_mapq, rd_min_mapq, min_base_qual, min_snv;
    int32_t insert_max;
    int32_t sc_min;
    int32_t chr_tid;        /* BAM target id of the scanned chromosome */
    double min_snv_ratio, min_ave_bq;
} grom_scan_args;

#endif
