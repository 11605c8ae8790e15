// cnv.h -- internal interface of the read-depth CNV path (SURVEY.md §8 rows
// A14-A16) between the scan driver (scan.hip) and cnv.hip.
#pragma once
#include "devmem.h"
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>

#include "../../include/grom_amd.h"

struct CnvScratch;
CnvScratch *cnv_scratch_new();
void cnv_scratch_free(CnvScratch *s);
// a new CNV phase (scan.hip): with an arena every buffer but the GC windows is
// carved from the phase; without one the buffers are the scratch's own
void cnv_scratch_phase(CnvScratch *s, grom_arena *ar);
// wait for the CNV path's own streams (before its arena phase is reused)
void cnv_scratch_sync(CnvScratch *s);

// Start the reference-only GC/ACGT window kernel of a chromosome on the CNV
// path's own stream (to overlap the pileup); the next cnv_chrom with the same
// d_ref and len waits for it instead of launching it.  The kernel starts after
// the work already queued on `after` (the reference upload).
int cnv_prelaunch(CnvScratch *S, hipStream_t after, const grom_params &P, const char *d_ref, int64_t len, char *err,
                  size_t errlen);

struct CnvTiming {
    double ms_device;  // device time of the CNV kernels (HIP events)
    double ms_host;    // host wall time of the whole CNV step
    int64_t del_calls, dup_calls, rows;
};

// The CNV path of one chromosome, run after the pileup has written the three
// whole-chromosome read-depth arrays (caf_rd_mq_list, caf_rd_rd_list,
// caf_rd_low_mq_rd_list) on stream `st`:
//   GC/ACGT triangular windows and dinucleotide repeats  GROM.c:1586-1881
//   chromosome depth statistics, 10 kb blocks            GROM.c:16633-16990
//   detect_del_dup                                       GROM.c:18228-20358
//   p-value filter and <DEL>/<DUP> rows                  GROM.c:17139-17300
// d_mq is divided by the depth in place (GROM.c:16637-16643).  The rows are
// appended to `rows`.  `seed` replaces the srand(time()) of GROM.c:1584.
int cnv_chrom(CnvScratch *S, hipStream_t st, const grom_params &P, uint32_t seed, const char *chr_name,
              const char *d_ref, int64_t len, int32_t *d_mq, const int32_t *d_rd, const int32_t *d_low,
              std::string &rows, CnvTiming *timing, char *err, size_t errlen, std::string *side = nullptr);
