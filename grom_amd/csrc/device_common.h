// device_common.h -- declarations shared by the scan kernels (scan.hip) and
// the host-side kernel emulator used by the tests (tests/emu/).
#ifndef GROM_AMD_DEVICE_COMMON_H
#define GROM_AMD_DEVICE_COMMON_H

#include <stdint.h>

#include "scan_common.h"

// htslib bam_nt16_rev_table
__constant__ char c_nt16[16] = {'=', 'A', 'C', 'M', 'G', 'R', 'S', 'V', 'T', 'W', 'Y', 'H', 'K', 'D', 'B', 'N'};
// 4-bit code -> index into "ACGT", 4 for anything else
__constant__ int8_t c_nt16_acgt[16] = {4, 0, 1, 4, 2, 4, 4, 4, 3, 4, 4, 4, 4, 4, 4, 4};
__constant__ char c_acgt[4] = {'A', 'C', 'G', 'T'};

__device__ __forceinline__ int64_t floordiv(int64_t a, int64_t b) {
    int64_t q = a / b;
    return (a % b != 0 && ((a < 0) != (b < 0))) ? q - 1 : q;
}

__device__ __forceinline__ char upcase(char c) { return (c >= 'a' && c <= 'z') ? (char)(c - 32) : c; }

// device views of grom_reads (include/grom_amd.h) plus the -M keep flags
struct ReadArrays {
    const int32_t *pos;
    const uint16_t *flag;
    const uint8_t *mapq;
    const int32_t *mtid;
    const int32_t *mpos;
    const int32_t *isize;
    const int32_t *lqseq;
    const uint32_t *cig_off;
    const uint32_t *cigar;
    const int64_t *base_off;
    const uint8_t *seq;
    const uint8_t *qual;
    const uint32_t *name_id;
    const uint8_t *keep;  // nullable (-M off)
};

struct PileOut {
    int32_t *caf_mq, *caf_rd, *caf_low;
    grom_snv_cand *cands;
    uint32_t *n_cands;
    uint32_t cand_cap;
    uint32_t *run_base, *run_cnt;  // per tile: first candidate slot, candidates
    unsigned long long *flush_part;  // per tile: [0] sum of caf rd, [1] non-N bases (k_flush_reduce)
    int32_t *dbg;                   // nullable: GC_COUNT int32 per evaluated base
    uint32_t *status;               // reserved
    uint32_t *n_events;             // reserved
    // breakpoint-test context (sv.hip): positions marked in sv_bits or with
    // soft-clip evidence get a grom_sv_ctx record (unordered; sorted later)
    const uint32_t *sv_bits;
    grom_sv_ctx *sv_ctx;
    uint32_t *n_sv_ctx;
    uint32_t sv_ctx_cap;
    const int32_t *rd_add;          // nullable: breakpoint depth adds, for the debug counters
};

#endif
