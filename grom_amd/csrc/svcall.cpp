// svcall.cpp -- host side of the breakpoint path: the candidate lists the
// per-base tests feed (GROM.c:11338-13541), the SV assembly and the rows
// (row A13, GROM.c:15163-16580).
//
// The device (sv.hip) returns, in base order, only the bases where a test
// passed its p-value cut, with everything the list logic reads there.  The
// lists are order-dependent state machines over a few thousand entries per
// chromosome, so they run here sequentially, exactly in the reference's
// per-base order: indel insertion, deletion start, deletion end, soft-clip
// insertion start and end, then CTX_F, CTX_R, DUP_R, DUP_F, DEL_F, DEL_R,
// INV_F1, INV_F2, INV_R1, INV_R2.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "sv.h"

namespace {

constexpr int AF = 6;          // cdp_add_factor, GROM.c:1548
constexpr int SEQ_MAX = 50;    // g_indel_i_seq_len

// ---- list entries; a fresh entry reads as the reference's initialised
// arrays: start/end -1 (GROM.c:5524-5560), everything else 0 ----
struct InsIEnt {  // indel_i_list
    int32_t start = -1, end = -1, conc_s = 0, conc_e = 0, dist = 0, other_s = 0, other_e = 0, i = 0, rd = 0, sc = 0;
    double binom = 0, hez = 0;
    char seq[SEQ_MAX + 1] = {0};
};
struct DelIEnt {  // indel_d_list
    int32_t start = -1, end = -1, conc_s = 0, conc_e = 0, other_s = 0, other_e = 0, f = 0, r = 0, rd_s = 0, rd_e = 0,
            sc_s = 0, sc_e = 0;
    double binom_s = 0, binom_e = 0, hez_s = 0, hez_e = 0;
};
struct InsEnt {  // ins_list
    int32_t start = -1, end = -1, ins_s = 0, ins_e = 0, rd_s = 0, rd_e = 0, conc_s = 0, conc_e = 0, other_s = 0,
            other_e = 0;
    double binom_s = 0, binom_e = 0;
};
struct PairEnt {  // dup / del / inv_f / inv_r lists
    int32_t start = -1, end = -1, cnt_s = 0, cnt_e = 0, rd_s = 0, rd_e = 0, conc_s = 0, conc_e = 0, other_s = 0,
            other_e = 0, rs_s = 0, re_s = 0, rs_e = 0, re_e = 0;
    double dist = 0, binom_s = 0, binom_e = 0, hez_s = 0, hez_e = 0;
};
struct CtxEnt {  // ctx_f / ctx_r lists
    int32_t pos = -1, cnt = 0, rd = 0, conc = 0, mchr = 0, mpos = 0, other = 0, rs = 0, re = 0;
    double binom = 0, hez = 0;
};

// A list whose entries past the written ones read as fresh entries (the
// reference allocates g_sv_list_len of them up front; this grows on demand).
template <class E>
struct List {
    std::vector<E> v;
    E &at(int64_t k) {
        if ((int64_t)v.size() <= k) v.resize((size_t)k + 1);
        return v[(size_t)k];
    }
};

enum { PR_DUP, PR_DEL, PR_INVF, PR_INVR };

struct Lists {
    int64_t cap;
    List<InsIEnt> ii;
    int64_t n_ii = 0;
    List<DelIEnt> id;
    int64_t n_id = -1;  // cdp_indel_d_list_index
    List<InsEnt> ins;
    int64_t n_ins = -1;  // cdp_ins_list_index
    List<PairEnt> pr[4];
    int64_t n_pr[4] = {0, 0, 0, 0};
    List<CtxEnt> cx[2];
    int64_t n_cx[2] = {0, 0};
};

// the inlined bisect over a start list (GROM.c:12270-12345): interpolated
// first guess from list[end] (the fresh entry past the last, start -1), then
// bisection; type 0 rounds up, type 1 down
static inline int to_int_trunc(double v) {
    return (v != v || v >= 2147483648.0 || v < -2147483648.0) ? (int)0x80000000u : (int)v;
}

static int bisect(List<PairEnt> &L, int pos, int start, int end, int type) {
    int range = end / 64;
    if (range < 4) range = 4;
    else if (range > 64) range = 64;
    const double guess = std::round((double)pos * (double)end / (double)L.at(end).start);
    int lo = to_int_trunc(guess - range), hi = to_int_trunc(guess + range);
    if (lo < start || lo >= end) lo = start;
    else if (L.at(lo).start > pos) { hi = lo; lo = start; }
    if (hi > end || hi < start) hi = end;
    else if (L.at(hi).start < pos) { lo = hi; hi = end; }
    int idx = lo + (hi - lo) / 2;
    for (;;) {
        const int s = L.at(idx).start;
        if (pos < s) {
            hi = idx;
            idx = lo + (idx - lo) / 2;
            if (hi == idx) break;
        } else if (pos > s) {
            lo = idx;
            idx = idx + (hi - idx) / 2;
            if (lo == idx) break;
        } else {
            break;
        }
    }
    if (type == 0 && pos > L.at(idx).start && idx < end) idx += 1;
    else if (type == 1 && pos < L.at(idx).start && idx > start) idx -= 1;
    return idx;
}

static void append_start(Lists &L, int k, const SvHit &h, const SvClusterHit &c) {
    if (L.n_pr[k] >= L.cap - 1) return;
    PairEnt &q = L.pr[k].at(L.n_pr[k]);
    q.start = h.pos;
    q.dist = c.dist;
    q.binom_s = c.binom;
    q.hez_s = c.hez;
    q.conc_s = h.conc;
    q.rd_s = h.rd;
    q.cnt_s = c.cnt;
    q.rs_s = c.rs;
    q.re_s = c.re;
    q.other_s = h.other_len;
    L.n_pr[k] += 1;
}

// end breakpoint matched against the start list (DUP_F GROM.c:12247-12470,
// DEL_R 12595-12844, INV_F2 12969-13193, INV_R2 13316-13541)
static void match_end(const grom_params &P, List<PairEnt> &lst, int n, const SvHit &h, const SvClusterHit &c,
                      double base, int off, bool tie_ge) {
    const double w = P.range_mult * (double)(P.insert_max_size - P.insert_min_size);
    const int mn = (int)((base - w) + 0.5);
    const int mx = (int)((base + w) + 0.5);
    const int p = h.pos;
    int lps = bisect(lst, p + off - mn, 0, n, 0);
    int lpe = bisect(lst, p + off - mx, 0, n, 1);
    if (lpe < lps) std::swap(lps, lpe);
    const int sp = p + off - mx, ep = p + off - mn;
    for (int a = lps; a < lpe; a++) {
        PairEnt &q = lst.at(a);
        if (q.dist >= mn && q.dist <= mx && q.start >= sp && q.start <= ep) {
            const bool better = (q.binom_e > c.binom && c.cnt >= q.cnt_e) || q.end == -1 ||
                                (q.binom_e == c.binom && (tie_ge ? c.cnt >= q.cnt_e : c.cnt > q.cnt_e));
            if (better) {
                q.end = p;
                q.binom_e = c.binom;
                q.hez_e = c.hez;
                q.conc_e = h.conc;
                q.rd_e = h.rd;
                q.cnt_e = c.cnt;
                q.rs_e = c.rs;
                q.re_e = c.re;
                q.other_e = h.other_len;
            }
        }
    }
}

static void ctx_append(Lists &L, int k, const SvHit &h, const SvClusterHit &c) {
    if (L.n_cx[k] >= L.cap - 1) return;
    CtxEnt &q = L.cx[k].at(L.n_cx[k]++);
    q.pos = h.pos;
    q.binom = c.binom;
    q.hez = c.hez;
    q.mchr = h.ctx_mchr[k];
    q.mpos = (int32_t)c.dist;
    q.conc = h.conc;
    q.rd = h.rd;
    q.cnt = c.cnt;
    q.rs = c.rs;
    q.re = c.re;
    q.other = h.other_len;
}

// the list updates of one base (GROM.c:11338-13541, reference order)
static void apply_hit(const grom_params &P, Lists &L, const SvHit &h) {
    const int p = h.pos;
    const int other = h.other_len;
    if (h.mask & HIT_II) {  // GROM.c:11402-11450
        if (L.n_ii < L.cap - 1) {
            InsIEnt &q = L.ii.at(L.n_ii);
            q.start = p;
            q.binom = h.ii_binom;
            q.hez = h.ii_hez;
            q.dist = h.ii_dist;
            q.conc_s = h.conc;
            q.i = h.ii_i;
            q.sc = h.ii_sc;
            q.rd = h.ii_rd;
            if (q.dist <= SEQ_MAX)
                for (int k = 0; k < q.dist; k++) q.seq[k] = h.ii_seq[k];
            q.other_s = other;
            L.n_ii += 1;
        }
    }
    if (h.mask & HIT_DF) {  // GROM.c:11480-11625
        int set = 0;
        if (L.n_id == -1) {
            L.n_id = 0;
            set = 1;
        } else if (L.id.at(L.n_id).start != -1 && L.id.at(L.n_id).end != -1) {
            if (L.n_id < L.cap - 1) {
                L.n_id += 1;
                set = 1;
            }
        } else if ((p - L.id.at(L.n_id).start > P.lseq && L.id.at(L.n_id).end == -1) ||
                   h.df_binom < L.id.at(L.n_id).binom_s) {
            set = 2;
        }
        if (set) {
            DelIEnt &q = L.id.at(L.n_id);
            q.start = p;
            q.binom_s = h.df_binom;
            q.hez_s = h.df_hez;
            q.conc_s = h.conc;
            if (set == 2 && q.end < q.start) q.end = -1;
            q.f = h.df_f;
            q.sc_s = h.df_sc;
            q.rd_s = h.df_rd;
            q.other_s = other;
        }
    }
    if ((h.mask & HIT_DR) && L.n_id >= 0) {  // GROM.c:11650-11742
        DelIEnt &q = L.id.at(L.n_id);
        // the distance test is float arithmetic (GROM.c:11670)
        volatile float fp = (float)p, fs = (float)q.start;
        volatile float d = fp - fs;
        d = d - (float)h.dr_rdist;
        if ((d < 5.0f && q.start != -1 && q.end != -1) || (d < 5.0f && (q.end == -1 || h.dr_binom < q.binom_e))) {
            q.end = p;
            q.binom_e = h.dr_binom;
            q.hez_e = h.dr_hez;
            q.conc_e = h.conc;
            q.r = h.dr_r;
            q.sc_e = h.dr_sc;
            q.rd_e = h.dr_rd;
            q.other_e = other;
        }
    }
    for (int side = 0; side < 2; side++) {  // GROM.c:11770-11855, 11880-11958
        if (!(h.mask & (side == 0 ? HIT_INSL : HIT_INSR))) continue;
        const double binom = side == 0 ? h.insl_binom : h.insr_binom;
        int set = 0;
        if (L.n_ins == -1) {
            L.n_ins = 0;
            set = 1;
        } else {
            InsEnt &c = L.ins.at(L.n_ins);
            if ((p - c.start > P.sc_range && c.start != -1) || (p - c.end > P.sc_range && c.end != -1)) {
                if (L.n_ins < L.cap - 1) {
                    L.n_ins += 1;
                    set = 1;
                }
            } else if (side == 0 ? (c.start == -1 || binom < c.binom_s) : (c.end == -1 || binom < c.binom_e)) {
                set = 1;
            }
        }
        if (set) {
            InsEnt &q = L.ins.at(L.n_ins);
            if (side == 0) {
                q.start = p; q.binom_s = binom; q.ins_s = h.ins; q.rd_s = h.rd; q.conc_s = h.conc; q.other_s = other;
            } else {
                q.end = p; q.binom_e = binom; q.ins_e = h.ins; q.rd_e = h.rd; q.conc_e = h.conc; q.other_e = other;
            }
        }
    }
    auto has = [&](int t) { return (h.mask & (HIT_CL0 << t)) != 0; };
    const int glseq = P.lseq, mean = P.insert_mean;
    if (has(CL_CTX_F)) ctx_append(L, 0, h, h.cl[CL_CTX_F]);   // GROM.c:11966-12045
    if (has(CL_CTX_R)) ctx_append(L, 1, h, h.cl[CL_CTX_R]);   // 12047-12126
    if (has(CL_DUP_R)) append_start(L, PR_DUP, h, h.cl[CL_DUP_R]);  // 12128-12205
    if (has(CL_DUP_F))                                         // 12207-12472
        match_end(P, L.pr[PR_DUP], (int)L.n_pr[PR_DUP], h, h.cl[CL_DUP_F], h.cl[CL_DUP_F].dist + 2 * glseq,
                  -mean + 2 * glseq, false);
    if (has(CL_DEL_F)) append_start(L, PR_DEL, h, h.cl[CL_DEL_F]);  // 12474-12553
    if (has(CL_DEL_R))                                         // 12555-12846
        match_end(P, L.pr[PR_DEL], (int)L.n_pr[PR_DEL], h, h.cl[CL_DEL_R], h.cl[CL_DEL_R].dist, mean, true);
    if (has(CL_INV_F1)) append_start(L, PR_INVF, h, h.cl[CL_INV_F1]);  // 12848-12927
    if (has(CL_INV_F2))                                        // 12929-13195
        match_end(P, L.pr[PR_INVF], (int)L.n_pr[PR_INVF], h, h.cl[CL_INV_F2], h.cl[CL_INV_F2].dist + glseq, glseq,
                  false);
    if (has(CL_INV_R1)) append_start(L, PR_INVR, h, h.cl[CL_INV_R1]);  // 13197-13274
    if (has(CL_INV_R2))                                        // 13276-13543
        match_end(P, L.pr[PR_INVR], (int)L.n_pr[PR_INVR], h, h.cl[CL_INV_R2], h.cl[CL_INV_R2].dist + glseq, glseq,
                  false);
}

// list -> list2 merge of a start/end pair list (DUP GROM.c:15163-15318; DEL,
// INV_F and INV_R run the same code over their lists)
static std::vector<PairEnt> merge_pairs(List<PairEnt> &lst, int64_t n, int64_t cap2, int Mx, int glseq) {
    std::vector<PairEnt> l2;
    bool open = false;
    int first_start = 0, last_start = 0, first_end = 0, last_end = 0;
    double first_dist = 0, last_dist = 0;
    for (int64_t a = 0; a < n; a++) {
        const PairEnt q = lst.at(a);
        if (open) {
            if (q.start > last_start + Mx - 2 * glseq) {
                open = false;
                first_start = last_start = first_end = last_end = 0;
                first_dist = last_dist = 0;
            } else {
                PairEnt &t = l2.back();
                const double mb = q.binom_e > q.binom_s ? q.binom_e : q.binom_s;
                const double mb2 = t.binom_e > t.binom_s ? t.binom_e : t.binom_s;
                if (mb <= mb2 && q.start >= 0 && q.end >= 0 && t.cnt_s <= q.cnt_s && t.cnt_e <= q.cnt_e) {
                    bool replace = false;
                    if (q.binom_s == t.binom_s && q.binom_e == t.binom_e) {
                        if ((t.cnt_s < q.cnt_s && t.cnt_e <= q.cnt_e) || (t.cnt_s <= q.cnt_s && t.cnt_e < q.cnt_e)) {
                            replace = true;
                        } else if (t.cnt_s == q.cnt_s && t.cnt_e == q.cnt_e) {
                            // equal evidence: keep the counts, average the span (GROM.c:15250-15275)
                            last_start = q.start;
                            last_end = q.end;
                            last_dist = q.dist;
                            const int32_t cs = t.cnt_s, ce = t.cnt_e;
                            t = q;
                            t.cnt_s = cs;
                            t.cnt_e = ce;
                            t.start = (first_start + last_start) / 2;
                            t.end = (first_end + last_end) / 2;
                            t.dist = (first_dist + last_dist) / 2.0;
                        }
                    } else {
                        replace = true;
                    }
                    if (replace) {
                        first_start = last_start = q.start;
                        first_end = last_end = q.end;
                        first_dist = last_dist = q.dist;
                        t = q;
                    }
                }
            }
        }
        if (!open && q.start >= 0 && q.end >= 0 && (int64_t)l2.size() < cap2 - 1) {
            open = true;
            first_start = last_start = q.start;
            first_end = last_end = q.end;
            first_dist = last_dist = q.dist;
            l2.push_back(q);
        }
    }
    return l2;
}

struct Out {
    std::string &s;
    void f(const char *fmt, ...) __attribute__((format(printf, 2, 3))) {
        char buf[1024];
        va_list ap;
        va_start(ap, fmt);
        int n = vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        if (n < 0) return;
        if ((size_t)n < sizeof buf) {
            s.append(buf, (size_t)n);
            return;
        }
        std::vector<char> big((size_t)n + 1);
        va_start(ap, fmt);
        vsnprintf(big.data(), big.size(), fmt, ap);
        va_end(ap);
        s.append(big.data(), (size_t)n);
    }
};

// -f rows of the paired classes: DUP (GROM.c:15347), INV_F/INV_R (15947,
// 16003), DEL (16564) -- raw counts, 0-based positions, the hez p-values
static void pair_row_tab(Out &o, const char *chr, const char *type, const PairEnt &q) {
    o.f("%s\t%s\t%d\t%d\t%6.2f\t%e\t%e\t%d\t%d\t%d\t%d\t%d\t%d\t%d\t%d\t%d\t%d\t%d\t%d\t%e\t%e\n", type, chr, q.start,
        q.end, q.dist, q.binom_s, q.binom_e, q.cnt_s, q.cnt_e, q.rd_s, q.rd_e, q.conc_s, q.conc_e, q.other_s, q.other_e,
        q.rs_s, q.re_s, q.rs_e, q.re_e, q.hez_s, q.hez_e);
}

static void pair_row(Out &o, const char *chr, const char *alt, const PairEnt &q) {
    o.f("%s\t%d\t.\t.\t%s\t.\t.\tEND=%d\tSPR:EPR:SEV:EEV:SRD:ERD:SCO:ECO:SOT:EOT:SFR:SLR:EFR:ELR\t"
        "%e:%e:%.1f:%.1f:%d:%d:%d:%d:%d:%d:%d:%d:%d:%d\n",
        chr, q.start + 1, alt, q.end + 1, q.binom_s, q.binom_e, (double)q.cnt_s / (double)AF,
        (double)q.cnt_e / (double)AF, q.rd_s, q.rd_e, q.conc_s, q.conc_e, q.other_s, q.other_e, q.rs_s + 1,
        q.re_s + 1, q.rs_e + 1, q.re_e + 1);
}

// the overlap ratios of an indel deletion q against a <DEL> call o, as the
// INDEL_DEL filter computes them (GROM.c:16350-16380); `quirk_end` is
// del_list2_end[a_loop] read with the indel's index (GROM.c:16366)
static bool indel_del_dropped(const grom_params &P, const DelIEnt &q, const std::vector<PairEnt> &d2, int64_t a,
                              int span) {
    for (size_t b = 0; b < d2.size(); b++) {
        const PairEnt &o = d2[b];
        if (!(std::abs(o.start - q.start) < span && std::abs(o.end - q.end) < span)) continue;
        double r1 = 0, r2 = 0;
        if (o.start >= q.start && o.start <= q.end) {
            if (o.end >= q.end) {
                r1 = (double)(q.end - o.start) / (double)(q.end - q.start);
                r2 = (double)(q.end - o.start) / (double)(o.end - o.start);
            } else {
                r1 = (double)(o.end - o.start) / (double)(q.end - q.start);
                // list2 entries past the merged ones read as zero (fresh calloc of list2)
                const int32_t qe = a < (int64_t)d2.size() ? d2[(size_t)a].end : 0;
                r2 = (double)(qe - o.start) / (double)(o.end - o.start);
            }
        } else if (q.start >= o.start && q.start <= o.end) {
            if (o.end >= q.end) {
                r1 = (double)(q.end - q.start) / (double)(q.end - q.start);
                r2 = (double)(q.end - q.start) / (double)(o.end - o.start);
            } else {
                r1 = (double)(o.end - q.start) / (double)(q.end - q.start);
                r2 = (double)(o.end - q.start) / (double)(o.end - o.start);
            }
        }
        if (r1 >= P.min_overlap_ratio && r2 >= P.min_overlap_ratio && o.binom_s * o.binom_e < q.binom_s * q.binom_e)
            return true;
    }
    return false;
}

static bool del_dropped(const grom_params &P, const PairEnt &q, Lists &L, int span) {
    for (int64_t b = 0; b < L.n_id; b++) {
        const DelIEnt &o = L.id.at(b);
        if (!(o.binom_s <= P.pval_threshold && o.binom_e <= P.pval_threshold &&
              (double)o.f / (double)o.rd_s > P.min_indel_ratio * (double)AF &&
              (double)o.r / (double)o.rd_e > P.min_indel_ratio * (double)AF && std::abs(q.start - o.start) < span &&
              std::abs(q.end - o.end) < span))
            continue;
        double r1 = 0, r2 = 0;
        if (q.start >= o.start && q.start <= o.end) {
            if (q.end >= o.end) {
                r1 = (double)(o.end - q.start) / (double)(o.end - o.start);
                r2 = (double)(o.end - q.start) / (double)(q.end - q.start);
            } else {
                r1 = (double)(q.end - q.start) / (double)(o.end - o.start);
                r2 = (double)(q.end - q.start) / (double)(q.end - q.start);
            }
        } else if (o.start >= q.start && o.start <= q.end) {
            if (q.end >= o.end) {
                r1 = (double)(o.end - o.start) / (double)(o.end - o.start);
                r2 = (double)(o.end - o.start) / (double)(q.end - q.start);
            } else {
                r1 = (double)(q.end - o.start) / (double)(o.end - o.start);
                r2 = (double)(q.end - o.start) / (double)(q.end - q.start);
            }
        }
        if (r1 >= P.min_overlap_ratio && r2 >= P.min_overlap_ratio && o.binom_s * o.binom_e <= q.binom_s * q.binom_e)
            return true;
    }
    return false;
}

}  // namespace

void sv_rows(const SvRowsInput &in, const SvHit *hits, size_t n_hits, std::string &vcf, std::string &ctx) {
    const grom_params &P = *in.P;
    const bool timing = getenv("GROM_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    double tm[8] = {0};
    int ti = 0;
    auto mark = [&]() {
        if (timing) tm[ti++] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    };
    Lists L;
    L.cap = P.sv_list_len;
    for (size_t k = 0; k < n_hits; k++) apply_hit(P, L, hits[k]);
    mark();

    const char *chr = in.chr_name ? in.chr_name : "";
    const char *fasta = in.ref;
    const int64_t chr_len = in.len;
    const int Mx = P.insert_max_size, glseq = P.lseq;
    const int span = Mx - 2 * glseq;
    const int64_t cap2 = P.sv_list2_len > 0 ? P.sv_list2_len : std::max<int64_t>(P.sv_list_len / 10, 1);
    const double pv = P.pval_threshold, ratio = P.min_sv_ratio * (double)AF;
    Out o{vcf};
    const bool tab = P.vcf != 1;  // -f: tab-separated rows (g_vcf == 0)
    std::vector<PairEnt> l2[4];
    for (int k = 0; k < 4; k++) l2[k] = merge_pairs(L.pr[k], L.n_pr[k], cap2, Mx, glseq);
    mark();

    // DUP rows, GROM.c:15320-15334
    for (const PairEnt &q : l2[PR_DUP])
        if ((q.binom_s <= pv || q.hez_s <= pv) && (q.binom_e <= pv || q.hez_e <= pv) &&
            (double)q.cnt_s / (double)q.rd_s >= ratio && (double)q.cnt_e / (double)q.rd_e >= ratio)
            tab ? pair_row_tab(o, chr, "DUP", q) : pair_row(o, chr, "<DUP>", q);

    // INV rows: dropped when the other orientation overlaps with a smaller
    // p-value product, or when the depth at the two ends differs (GROM.c:15795-15890)
    for (int side = 0; side < 2; side++) {
        const std::vector<PairEnt> &A = l2[side == 0 ? PR_INVF : PR_INVR], &B = l2[side == 0 ? PR_INVR : PR_INVF];
        for (const PairEnt &q : A) {
            if (!(q.binom_s <= pv && q.binom_e <= pv && (double)q.cnt_s / (double)q.rd_s >= ratio &&
                  (double)q.cnt_e / (double)q.rd_e >= ratio))
                continue;
            bool overlap = false;
            for (const PairEnt &b : B) {
                if (std::abs(q.start - b.start) < span && std::abs(q.end - b.end) < span &&
                    ((q.start >= b.start && q.start <= b.end) || (b.start >= q.start && b.start <= q.end))) {
                    const bool better = side == 0 ? (b.binom_s * b.binom_e < q.binom_s * q.binom_e)
                                                  : (b.binom_s * b.binom_e <= q.binom_s * q.binom_e);
                    if (better) {
                        overlap = true;
                        break;
                    }
                }
            }
            double r1 = in.caf_sum(in.u, q.rs_s, (int64_t)q.re_s + glseq);
            r1 = r1 / (q.re_s + glseq - q.rs_s);
            double r2 = in.caf_sum(in.u, q.rs_e, (int64_t)q.re_e + glseq);
            r2 = r2 / (q.re_e + glseq - q.rs_e);
            if (!overlap && r1 / r2 <= P.max_inv_rd_diff && r2 / r1 <= P.max_inv_rd_diff)
                tab ? pair_row_tab(o, chr, side == 0 ? "INV_F" : "INV_R", q) : pair_row(o, chr, "<INV>", q);
        }
    }

    mark();
    // INS: start/end merge and rows, GROM.c:15897-15968
    {
        std::vector<InsEnt> i2;
        bool open = false;
        for (int64_t a = 0; a < L.n_ins; a++) {
            const InsEnt q = L.ins.at(a);
            if (open) {
                InsEnt &t = i2.back();
                if (q.start > t.start + span || q.start > t.end + span || q.end > t.start + span || q.end > t.end + span)
                    open = false;
                else if (q.binom_s <= t.binom_s && q.start >= 0 && q.binom_e <= t.binom_e && q.end >= 0)
                    t = q;
            }
            // the capacity guard reads the list index, not the list2 count (GROM.c:15935)
            if (!open && q.start >= 0 && q.end >= 0 && L.n_ins < cap2 - 1) {
                open = true;
                i2.push_back(q);
            }
        }
        for (const InsEnt &q : i2) {
            if (!(q.binom_s <= P.pval_insertion && q.binom_e <= P.pval_insertion &&
                  std::abs(q.end - q.start) <= P.max_ins_range))
                continue;
            if (tab)  // GROM.c:16091
                o.f("INS\t%s\t%d\t%d\t\t%e\t%e\t%d\t%d\t%d\t%d\t%d\t%d\t%d\t%d\n", chr, q.start, q.end, q.binom_s, q.binom_e,
                    q.ins_s, q.ins_e, q.rd_s, q.rd_e, q.conc_s, q.conc_e, q.other_s, q.other_e);
            else
                o.f("%s\t%d\t.\t.\t<INS>\t.\t.\tEND=%d\tSPR:EPR:SEV:EEV:SRD:ERD:SCO:ECO:SOT:EOT\t"
                    "%e:%e:%.1f:%.1f:%d:%d:%d:%d:%d:%d\n",
                    chr, q.start + 1, q.start + 1, q.binom_s, q.binom_e, (double)q.ins_s / (double)AF,
                    (double)q.ins_e / (double)AF, q.rd_s, q.rd_e, q.conc_s, q.conc_e, q.other_s, q.other_e);
        }
    }

    // CTX_F / CTX_R: merged and written raw for the translocation post-pass
    // (GROM.c:15970-16248)
    {
        Out oc{ctx};
        for (int k = 0; k < 2; k++) {
            std::vector<CtxEnt> c2;
            bool open = false;
            for (int64_t a = 0; a < L.n_cx[k]; a++) {
                const CtxEnt q = L.cx[k].at(a);
                if (open) {
                    CtxEnt &t = c2.back();
                    if (q.pos > t.pos + span) open = false;
                    else if (((q.binom < t.binom && t.cnt <= q.cnt) || (q.binom == t.binom && t.cnt < q.cnt)) && q.pos >= 0)
                        t = q;
                }
                if (!open && q.pos >= 0 && (int64_t)c2.size() < cap2 - 1) {
                    open = true;
                    c2.push_back(q);
                }
            }
            for (const CtxEnt &q : c2)
                if ((q.binom <= pv || q.hez <= pv) && (double)q.cnt / (double)q.rd >= ratio)
                    oc.f("%s\t%s\t%d\t%e\t%.1f\t%d\t%d\t%d\t%d\t%d\t%d\t%d\t%e\n", k == 0 ? "CTX_F" : "CTX_R", chr, q.pos,
                         q.binom, (double)q.cnt / (double)AF, q.rd, q.conc, q.other, q.mchr, q.mpos, q.rs, q.re, q.hez);
        }
    }

    mark();
    // INDEL_INS rows, GROM.c:16250-16330
    const double iratio = P.min_indel_ratio * (double)AF;
    for (int64_t a = 0; a < L.n_ii; a++) {
        const InsIEnt &q = L.ii.at(a);
        if (!(q.binom <= pv && (double)q.i / (double)q.rd > iratio)) continue;
        int hp = 1;
        char hc = fasta[q.start];
        for (int b = 1; b < 20 && q.start - b >= 0; b++) {
            if (hc == fasta[q.start - b]) hp += 1;
            else break;
        }
        int hp2 = 1;
        if (fasta[q.start] + 1 < chr_len) {  // sic: the base letter plus one, GROM.c:16282
            hc = (char)(fasta[q.start] + 1);
            for (int b = 1; b < 20 && q.start + b + 1 < chr_len; b++) {
                if (hc == fasta[q.start + b + 1]) hp2 += 1;
                else break;
            }
        }
        if (hp2 > hp) hp = hp2;
        if (hp > P.max_homopolymer) continue;
        if (tab) {  // GROM.c:16342
            o.f("INDEL_INS\t%s\t%d\t%d\t%d\t%e\t%e\t%d\t%d\t%d\t%d\t%d\t%d\t%d\t%d\n", chr, q.start, q.end, q.dist, q.binom,
                q.hez, q.conc_s, q.conc_e, q.other_s, q.other_e, q.i, q.rd, q.sc, hp);
            continue;
        }
        char gts[SEQ_MAX + 8];
        if (q.dist <= SEQ_MAX) {
            memcpy(gts, q.seq, (size_t)std::max(q.dist, 0));
            gts[std::max(q.dist, 0)] = 0;
        } else {
            strcpy(gts, "<INS>");
        }
        o.f("%s\t%d\t.\t.\t%s\t.\t.\tEND=%d\tSPR:SEV:SRD:SCO:ECO:SOT:EOT:SSC:HP\t%e:%.1f:%d:%d:%d:%d:%d:%d:%d\n", chr,
            q.start + 1, gts, q.end + 1, q.binom, (double)q.i / (double)AF, q.rd, q.conc_s, q.conc_e, q.other_s,
            q.other_e, q.sc, hp);
    }

    mark();
    // INDEL_DEL rows, dropped when a <DEL> call overlaps with a smaller
    // p-value product; the loop stops before the open last entry (the list
    // index, not a count: GROM.c:16336-16470)
    for (int64_t a = 0; a < L.n_id; a++) {
        const DelIEnt q = L.id.at(a);
        if (!(q.binom_s <= pv && q.binom_e <= pv && (double)q.f / (double)q.rd_s > iratio &&
              (double)q.r / (double)q.rd_e > iratio))
            continue;
        if (indel_del_dropped(P, q, l2[PR_DEL], a, span)) continue;
        int hp = 1;
        if (fasta[q.start] - 1 >= 0) {
            const char hc = fasta[q.start - 1];
            for (int b = 1; b < 20 && q.start - b - 1 >= 0; b++) {
                if (hc == fasta[q.start - b - 1]) hp += 1;
                else break;
            }
        }
        int hp2 = 1;
        if (fasta[q.end] + 1 < chr_len) {
            const char hc = (char)(fasta[q.end] + 1);
            for (int b = 1; b < 20 && q.end + b + 1 < chr_len; b++) {
                if (hc == fasta[q.end + b + 1]) hp2 += 1;
                else break;
            }
        }
        if (hp2 > hp) hp = hp2;
        if (hp > P.max_homopolymer) continue;
        const int cn = q.end - q.start + 1;
        if (tab) {  // GROM.c:16490
            o.f("INDEL_DEL\t%s\t%d\t%d\t%d\t%e\t%e\t%d\t%d\t%d\t%d\t%d\t%d\t%d\t%d\t%d\t%d\t%e\t%e\t%d\n", chr, q.start,
                q.end, cn, q.binom_s, q.binom_e, q.conc_s, q.conc_e, q.other_s, q.other_e, q.f, q.r, q.rd_s, q.rd_e, q.sc_s,
                q.sc_e, q.hez_s, q.hez_e, hp);
            continue;
        }
        if (cn > 0 && cn < 100 - 1) {
            std::string ref(fasta + q.start, (size_t)cn);
            o.f("%s\t%d\t.\t%s\t.\t.\t.\tEND=%d\tSPR:EPR:SEV:EEV:SRD:ERD:SCO:ECO:SOT:EOT:SSC:ESC:HP\t"
                "%e:%e:%.1f:%.1f:%d:%d:%d:%d:%d:%d:%d:%d:%d\n",
                chr, q.start + 1, ref.c_str(), q.end + 1, q.binom_s, q.binom_e, (double)q.f / (double)AF,
                (double)q.r / (double)AF, q.conc_s, q.conc_e, q.other_s, q.other_e, q.rd_s, q.rd_e, q.sc_s, q.sc_e, hp);
        } else {
            o.f("%s\t%d\t.\t.\t<DEL>\t.\t.\tEND=%d\tSPR:EPR:SEV:EEV:SRD:ERD:SCO:ECO:SOT:EOT:SSC:ESC:HP\t"
                "%e:%e:%.1f:%.1f:%d:%d:%d:%d:%d:%d:%d:%d:%d\n",
                chr, q.start + 1, q.end + 1, q.binom_s, q.binom_e, (double)q.f / (double)AF, (double)q.r / (double)AF,
                q.conc_s, q.conc_e, q.other_s, q.other_e, q.rd_s, q.rd_e, q.sc_s, q.sc_e, hp);
        }
    }

    mark();
    // DEL rows, dropped when an indel deletion overlaps with a smaller or
    // equal p-value product (GROM.c:16474-16580)
    for (const PairEnt &q : l2[PR_DEL]) {
        if (!((q.binom_s <= pv || q.hez_s <= pv) && (q.binom_e <= pv || q.hez_e <= pv) &&
              (double)q.cnt_s / (double)q.rd_s >= ratio && (double)q.cnt_e / (double)q.rd_e >= ratio))
            continue;
        if (!del_dropped(P, q, L, span)) tab ? pair_row_tab(o, chr, "DEL", q) : pair_row(o, chr, "<DEL>", q);
    }
    mark();
    if (timing)
        fprintf(stderr,
                "sv rows ms: lists %.3f merge %.3f dup+inv %.3f ins+ctx %.3f indel_ins %.3f indel_del %.3f del %.3f "
                "(%zu hits; list sizes ii %lld id %lld ins %lld dup %lld del %lld invf %lld invr %lld; "
                "list2 del %zu)\n",
                tm[0], tm[1] - tm[0], tm[2] - tm[1], tm[3] - tm[2], tm[4] - tm[3], tm[5] - tm[4], tm[6] - tm[5],
                n_hits, (long long)L.n_ii, (long long)L.n_id, (long long)L.n_ins, (long long)L.n_pr[0],
                (long long)L.n_pr[1], (long long)L.n_pr[2], (long long)L.n_pr[3], l2[PR_DEL].size());
}

// ---------------- test hook: recorded sv_rows inputs (sv.h) ----------------
namespace {
constexpr char SVH_MAGIC[8] = {'G', 'S', 'V', 'H', '1', 0, 0, 0};

struct Replay {
    const std::vector<SvCafRec> *caf;
    bool missing = false;
    static double call(void *u, int64_t lo, int64_t hi) {
        Replay &r = *(Replay *)u;
        for (const SvCafRec &c : *r.caf)
            if (c.lo == lo && c.hi == hi) return c.v;
        r.missing = true;
        return 0.0;
    }
};

bool put(FILE *f, const void *p, size_t n) { return n == 0 || fwrite(p, 1, n, f) == n; }
bool get(FILE *f, void *p, size_t n) { return n == 0 || fread(p, 1, n, f) == n; }
bool put_blob(FILE *f, const void *p, uint64_t n) { return put(f, &n, 8) && put(f, p, n); }
bool get_blob(FILE *f, std::string &out) {
    uint64_t n;
    if (!get(f, &n, 8) || n > ((uint64_t)1 << 34)) return false;
    out.resize((size_t)n);
    return get(f, out.empty() ? nullptr : &out[0], (size_t)n);
}
}  // namespace

int sv_rows_record_write(const char *path, const SvRowsInput &in, const SvHit *hits, size_t n_hits,
                         const std::vector<SvCafRec> &caf, const std::string &vcf, const std::string &ctx) {
    FILE *f = fopen(path, "wb");
    if (!f) return -1;
    const char *nm = in.chr_name ? in.chr_name : "";
    const uint64_t sz[2] = {sizeof(grom_params), sizeof(SvHit)};
    bool ok = put(f, SVH_MAGIC, 8) && put(f, sz, 16) && put(f, in.P, sizeof(grom_params)) && put(f, &in.len, 8) &&
              put_blob(f, nm, strlen(nm)) && put_blob(f, in.ref, (uint64_t)in.len) &&
              put_blob(f, hits, sizeof(SvHit) * n_hits) && put_blob(f, caf.data(), sizeof(SvCafRec) * caf.size()) &&
              put_blob(f, vcf.data(), vcf.size()) && put_blob(f, ctx.data(), ctx.size());
    ok = (fclose(f) == 0) && ok;
    return ok ? 0 : -1;
}

extern "C" int grom_sv_rows_replay(const char *path) {
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    char magic[8];
    uint64_t sz[2];
    grom_params P;
    int64_t len = 0;
    std::string name, ref, hits, caf, vcf, ctx;
    const bool ok = get(f, magic, 8) && memcmp(magic, SVH_MAGIC, 8) == 0 && get(f, sz, 16) &&
                    sz[0] == sizeof(grom_params) && sz[1] == sizeof(SvHit) && get(f, &P, sizeof(P)) &&
                    get(f, &len, 8) && get_blob(f, name) && get_blob(f, ref) && get_blob(f, hits) &&
                    get_blob(f, caf) && get_blob(f, vcf) && get_blob(f, ctx);
    fclose(f);
    if (!ok || (int64_t)ref.size() != len || hits.size() % sizeof(SvHit) || caf.size() % sizeof(SvCafRec)) return -2;
    std::vector<SvHit> H(hits.size() / sizeof(SvHit));
    if (!H.empty()) memcpy(H.data(), hits.data(), hits.size());
    std::vector<SvCafRec> C(caf.size() / sizeof(SvCafRec));
    if (!C.empty()) memcpy(C.data(), caf.data(), caf.size());
    Replay rp{&C};
    SvRowsInput in{&P, name.c_str(), ref.data(), len, &Replay::call, &rp};
    std::string v, c;
    sv_rows(in, H.data(), H.size(), v, c);
    if (rp.missing) return -3;
    return (v == vcf && c == ctx) ? 0 : 1;
}

