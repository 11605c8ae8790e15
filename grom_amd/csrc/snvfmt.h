// snvfmt.h -- host-side VCF text of the SNV rows (GROM.c:11203-11274 mid-scan
// flushes, 15063-15107 final flush), formatted without printf on the hot path.
#ifndef GROM_AMD_SNVFMT_H
#define GROM_AMD_SNVFMT_H

#include <stddef.h>

#include <string>
#include <vector>

#include "../../include/grom_amd.h"
#include "scan_common.h"

// Rows of one SNV list flush: candidates c[0..n) (position order) whose
// rc_all passes the flush's depth limit `lim` (or whose ratio passes
// high_cov_min_snv_ratio).  Large lists are split over up to 16 host threads;
// the text of part t goes to parts[t] (join in order).
void snv_rows_format(const grom_params &P, const char *chr_name, const grom_snv_cand *c, size_t n, double lim,
                     std::vector<std::string> &parts);

// The same rows in the -f tab-separated form (GROM.c:11265-11322,
// 15099-15156): raw counters, 0-based position, the reference context
// (lseq bases up to the site, then lseq-1 bases read backwards from
// pos+lseq-1) and both p-values.  `lseq` is cdp_lseq at the flush.
void snv_rows_format_tab(const grom_params &P, const char *chr_name, const grom_snv_cand *c, size_t n, double lim,
                         const char *ref, int64_t len, int32_t lseq, std::string &out);

// Byte-identical replacement for printf("%.2f", v) (glibc semantics: the
// exact binary value, rounded half to even).  `out` must hold 400 bytes.
// Returns the length written.
int fmt_2f(char *out, double v);

#endif
