// indel_emu.cpp -- TEST INFRASTRUCTURE ONLY.  The CIGAR indel pass (indel.hip)
// is built on hipCUB, which this emulator does not provide; under the emulator
// the pass reports no records.  Its parity is checked on the GPU
// (tests/test_gpu_parity.py) and the oracle by tests/test_oracle_indel.py.
#include "../../grom_amd/csrc/indel.h"

struct IndelScratch {
    int64_t n = 0;
};
IndelScratch *indel_scratch_new() { return new IndelScratch(); }
void indel_scratch_free(IndelScratch *s) { delete s; }
const grom_indel_rec *indel_records(const IndelScratch *) { return nullptr; }
int64_t indel_count(const IndelScratch *S) { return S->n; }
int indel_chrom(IndelScratch *S, hipStream_t, int64_t, const int32_t *, const uint8_t *, const uint8_t *,
                const uint32_t *, const uint32_t *, const int64_t *, const int32_t *, const uint8_t *, int32_t,
                int32_t, int32_t, int64_t *n_out, double *ms, char *, size_t) {
    S->n = 0;
    *n_out = 0;
    if (ms) *ms = 0;
    return GROM_OK;
}
