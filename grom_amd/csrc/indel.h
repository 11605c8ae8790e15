// indel.h -- internal interface of the CIGAR indel-evidence pass (SURVEY.md
// §8 row A7) between the scan driver (scan.hip) and indel.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/grom_amd.h"

struct IndelScratch;
IndelScratch *indel_scratch_new();
void indel_scratch_free(IndelScratch *s);

// The indel evidence of one chromosome (GROM.c:7187-7423), on stream `st`, from
// the device-resident reads the pileup ingests (`keep` = the -M flags, or
// null).  Writes one grom_indel_rec per evaluated base in [eval_lo, eval_hi]
// that a CIGAR I/D op of an ingested read reaches, in position order, into
// device memory owned by S; *n_out receives the count.  Returns a GROM_E_*
// code (message in err).
int indel_chrom(IndelScratch *S, hipStream_t st, int64_t n_reads, const int32_t *pos, const uint8_t *mapq,
                const uint8_t *keep, const uint32_t *cig_off, const uint32_t *cigar, const int64_t *base_off,
                const int32_t *lqseq, const uint8_t *seq, int32_t min_mapq, int32_t eval_lo, int32_t eval_hi,
                int64_t *n_out, double *ms_device, char *err, size_t errlen);

// device pointer to, and count of, the records of the last indel_chrom
const grom_indel_rec *indel_records(const IndelScratch *S);
int64_t indel_count(const IndelScratch *S);
