// sv.h -- internal interface of the breakpoint pass
// between the scan driver (scan.hip), its kernels (sv.hip) and the host list
// logic / SV rows (svcall.cpp).
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/grom_amd.h"
#include "scan_common.h"
#include "devmem.h"

// cluster types in the order of the reference's OTHER_* codes minus one
// (GROM.c:668-681)
enum SvCl { CL_DEL_F, CL_DEL_R, CL_DUP_F, CL_DUP_R, CL_INV_F1, CL_INV_R1, CL_INV_F2, CL_INV_R2, CL_CTX_F, CL_CTX_R, CL_N };

// one cluster test that passed its p-value cut at a base
struct SvClusterHit {
    double dist, binom, hez;
    int32_t cnt, rs, re, pad;
};

// everything the candidate-list logic of GROM.c:11396-13541 reads at a base
// where at least one per-base test passed (mask bit set)
enum : uint32_t {
    HIT_II = 1u << 0,   // CIG insertion, GROM.c:11338-11453
    HIT_DF = 1u << 1,   // deletion start, 11460-11629
    HIT_DR = 1u << 2,   // deletion end, 11631-11745
    HIT_INSL = 1u << 3, // soft-clip insertion start, 11750-11857
    HIT_INSR = 1u << 4, // soft-clip insertion end, 11859-11960
    HIT_CL0 = 1u << 5   // + CL_*: breakpoint clusters, 11966-13541
};

struct SvHit {
    int32_t pos;
    uint32_t mask;
    int32_t conc, rd, ins, other_len;
    double ii_binom, ii_hez;
    int32_t ii_dist, ii_i, ii_rd, ii_sc;
    double df_binom, df_hez;
    int32_t df_f, df_rd, df_sc, pad1;
    double dr_binom, dr_hez;
    int32_t dr_r, dr_rd, dr_sc, dr_rdist;
    double insl_binom, insr_binom;
    SvClusterHit cl[CL_N];
    int32_t ctx_mchr[2];
    char ii_seq[52];
    int32_t pad2;
};

struct SvScratch;
SvScratch *sv_scratch_new();
void sv_scratch_free(SvScratch *s);
// a new pileup/breakpoint phase (scan.hip): with an arena, every buffer is
// carved from its phase (their contents are dead); without one, the buffers
// are the scratch's own and persist
void sv_scratch_phase(SvScratch *s, grom_arena *ar);

// device views of the reads the breakpoint pass walks
struct SvInput {
    int64_t n;
    const int32_t *pos;
    const uint16_t *flag;
    const uint8_t *mapq;
    const int32_t *mtid, *mpos, *isize, *lqseq;
    const uint32_t *cig_off, *cigar;
    const int64_t *base_off;
    const uint8_t *seq;
    const uint8_t *keep;  // nullable (-M off)
    const int32_t *aux_idx;
    const grom_aux *aux;
    int64_t n_drop;
    const int32_t *drop_pos, *drop_lq;
    const int64_t *drop_before;
};

// Phase 1, before the pileup: per-read evidence events (CIGAR indels, split
// reads, read pairs), the order-free range sums, the ordered fold of every
// base's events, and the candidate bitmap the pileup reads.
int sv_prepare(SvScratch *S, hipStream_t st, const grom_params &P, const SvInput &in, const grom_chrom &ch,
               int32_t eval_lo, int32_t eval_hi, bool debug, char *err, size_t errlen);
const uint32_t *sv_bits(const SvScratch *S);
const int32_t *sv_rd_add(const SvScratch *S);
// the buffer the pileup fills with grom_sv_ctx records (grown by sv_prepare)
grom_sv_ctx *sv_ctx_buf(const SvScratch *S);
uint32_t sv_ctx_cap(const SvScratch *S);
// the pileup's context records written (or wanted) in the last pass; a pass
// that wanted more than sv_ctx_cap is run again after sv_ctx_reserve
int sv_ctx_used(SvScratch *S, hipStream_t st, uint32_t *used);
void sv_ctx_reserve(SvScratch *S, uint32_t cap);
uint32_t *sv_ctx_count(const SvScratch *S);

// Phase 2, after the pileup: the per-base tests at every context record;
// the bases where one passed come back in position order.
// the hits come back in base order in a pinned host buffer owned by S
// (valid until the next call on S)
int sv_evaluate(SvScratch *S, hipStream_t st, const grom_params &P, const SvInput &in, const grom_chrom &ch,
                int32_t eval_lo, int32_t eval_hi, const double *d_mq, const double *d_hez, const SvHit **hits,
                size_t *n_hits, double *ms_device, char *err, size_t errlen);

// cdp_lseq at the evaluation of each base h_pos[0..n) (host arrays): the
// length of the stream's next record not yet ingested there
int sv_pending_lseq(hipStream_t st, const grom_params &P, const SvInput &in, const grom_chrom &ch,
                    const int32_t *h_pos, int n, int32_t *h_out, char *err, size_t errlen);

// test hooks: records of the last scan
const grom_indel_rec *sv_indel_records(const SvScratch *S);
int64_t sv_indel_count(const SvScratch *S);
const grom_sv_rec *sv_debug_records(const SvScratch *S);
int64_t sv_debug_count(const SvScratch *S);

// Host: the candidate lists, SV assembly and rows of one chromosome
// (svcall.cpp).  `caf_sum(lo, hi)` returns the sum of caf_rd + caf_low over
// [lo, hi) (the INV depth check, GROM.c:15816-15826).
struct SvRowsInput {
    const grom_params *P;
    const char *chr_name;
    const char *ref;
    int64_t len;
    double (*caf_sum)(void *u, int64_t lo, int64_t hi);
    void *u;
};
void sv_rows(const SvRowsInput &in, const SvHit *hits, size_t n_hits, std::string &vcf, std::string &ctx);

// Test hook (GROM_SV_HITS_DUMP=<prefix>): one chromosome's sv_rows inputs and
// outputs as recorded by a GPU scan -- parameters, reference, hits, every
// caf_sum query with its answer, the VCF and CTX text -- in <prefix>.<chr>.svh.
// sv_rows_record_write writes it; grom_sv_rows_replay (C ABI below) runs
// sv_rows on it again (host only: the sanitizer tests) and compares.
struct SvCafRec {
    int64_t lo, hi;
    double v;
};
int sv_rows_record_write(const char *path, const SvRowsInput &in, const SvHit *hits, size_t n_hits,
                         const std::vector<SvCafRec> &caf, const std::string &vcf, const std::string &ctx);
extern "C" {
// 0: sv_rows on the recorded inputs gives the recorded rows; 1: they differ;
// negative: unreadable record or a caf_sum query that was not recorded
int grom_sv_rows_replay(const char *path);
}

