// sv.hip -- breakpoint evidence on MI355X: CIGAR indels (row A7), split reads
// (A8), read-pair binning (A9) and the per-base indel / insertion / breakpoint
// tests (A10).  GROM.c:7187-10953 and 11338-13553.
//
// The reference folds every read into per-base ring state in stream order.
// Two kinds of state come out of that:
//
//   order-free sums  rd (+1 over every range), conc, ins, munmapped_f/r:
//                    difference arrays (two atomics per read and range) and
//                    one inclusive scan per array;
//   ordered clusters the DEL/DUP/INV/CTX running means, the CIGAR indel
//                    primaries and the 50 "other" slots they share with
//                    swap-to-primary: order-dependent, so every read emits its
//                    events in the reference's write order, a stable radix
//                    sort on the base keeps each base's events in stream
//                    order, and one lane per base folds its run sequentially.
//
//   k_sv_count / scan / k_sv_emit   one lane per read: events + range sums
//   radix sort, run-length encode   one run per base
//   k_sv_fold<0>, scan, k_sv_fold<1>  the fold, twice: flags, then compacted
//                    records of the bases a test could fire at (and the
//                    indel records, and the debug records) in base order;
//                    it also marks those bases in the candidate bitmap
//   (pileup)         writes a grom_sv_ctx for every marked base and every
//                    base with soft-clip evidence
//   radix sort       contexts in base order
//   k_sv_eval        one lane per context: the tests; bases where one passes
//                    return to the host as SvHit records
//
// Exactness notes.  An event whose read is ingested after its base was
// evaluated (p_ing > x) changes nothing the reference reads, so it is not
// emitted.  Range ends clip to the ring exactly where the reference does
// (g_one_base_rd_len, GROM.c:8350-8353).  The running means use the
// reference's operation order; this file is built with -ffp-contract=off.
// The reference's ring keeps cluster groups only under "set" flags
// (GROM.c:5868-6392); every write of a group's primary arrays sets that
// group's flags (the split-read DUP_F starts set the DEL and DUP flags,
// GROM.c:8027-8043, 9408-9411), so no evidence is left behind by a shift and
// the ring is exactly the absolute-coordinate state folded here.

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>

#include "sv.h"
#include "ddecode.h"
#include "copystats.h"  // (GROM_COPY_STATS, last: it wraps the runtime copy calls)

namespace {

constexpr int OTHER_LEN = 50;   // g_other_len, GROM.c:837
constexpr int ISEQ_LEN = 50;    // g_indel_i_seq_len, GROM.c:904
constexpr int MAX_CIGAR = 1000; // the reference copies at most 1000 ops, GROM.c:6740-6750
constexpr int AF = 6;           // cdp_add_factor, GROM.c:1548
constexpr int MT = GROM_MAX_TRIALS;
enum : uint8_t { OT_EMPTY = 0, OT_I = 11, OT_DF = 12, OT_DR = 13 };  // GROM.c:668-681
enum { RM_SET = 0, RM_MAX = 1, RM_MINMAX = 2 };
enum { SUM_RD = 0, SUM_CONC, SUM_INS, SUM_MUNF, SUM_MUNR, SUM_N };

__constant__ char c_nt16_sv[16] = {'=', 'A', 'C', 'M', 'G', 'R', 'S', 'V', 'T', 'W', 'Y', 'H', 'K', 'D', 'B', 'N'};

// one ordered evidence event (32 bytes)
struct SvEv {
    double v;      // cluster: the value its running mean averages
    int64_t aux;   // indel I: nibble offset of the inserted bases
    int32_t rp;    // cluster: read position kept in rs/re; indel I: read bases left from aux
    int32_t mchr;  // ctx: mate chromosome
    int32_t len;   // indel: op length; cluster: tolerance (Mx - Mn [+ insert_temp])
    uint8_t type;  // 1..10 cluster (CL_* + 1), 11..13 indel
    uint8_t w;     // count increment (add, or add/2 away from a clipped edge)
    uint8_t add;   // full weight (6 or 0)
    uint8_t fl;    // bits 0-1 rs/re rule, 2-3 ctx kind, 4-5 split DUP_F start (re -> del_f_read_end)
};

struct Geo {
    int32_t Mx, Mn, mean, lseq_g, overlap, s0, n_skip, H, r14, R, sc_min, min_mapq, max_split_loss, min_sr_len;
    int32_t eval_lo, eval_hi, chr_tid, min_disc;
    int32_t splitread;
};

struct View {
    SvInput in;
    Geo g;
};

// ring index after k increments of cdp_one_base_index (GROM.c:5845-5847, 6392)
__device__ __forceinline__ int64_t ring_idx(const Geo &g, int64_t k) { return g.r14 + ((k + 1) % g.H); }

// Walk one read as the ingest body does (GROM.c:6418-10953) and hand
//   ev(x, SvEv)          every ordered event at base x, in write order
//   rg(kind, lo, hi, v)  every order-free range sum [lo, hi) += v
// Only what the evaluation can still see is handed over: bases in the
// evaluated range at or after the read's ingest iteration.
template <class EV, class RG>
__device__ void sv_walk(const View &V, int64_t i, EV &&ev, RG &&rg) {
    const SvInput &in = V.in;
    const Geo &g = V.g;
    const uint16_t flag = in.flag[i];
    if (in.keep && in.keep[i] == 0) return;  // -M drop (GROM.c:6588)
    const int32_t pos = in.pos[i], mpos = in.mpos[i], tlen = in.isize[i], mtid = in.mtid[i];
    const int32_t mq = in.mapq[i];
    const int add = mq >= g.min_mapq ? AF : 0;
    // the iteration that ingests this read, and the ring index then
    const int64_t p_ing = max((int64_t)g.s0, (int64_t)pos - (int64_t)g.overlap * g.Mx);
    const int64_t k_ing = (int64_t)g.n_skip + (p_ing - g.s0) + 1;
    const int64_t idx = ring_idx(g, k_ing);
    const int64_t ring_lo = p_ing - idx, ring_hi = p_ing - idx + g.R;  // positions of ring index 0 and R
    const int64_t vis_lo = max(p_ing, (int64_t)g.eval_lo), vis_hi = g.eval_hi;  // inclusive
    auto event = [&](int64_t x, SvEv e) {
        if (x >= vis_lo && x <= vis_hi) ev((int32_t)x, e);
    };
    auto range = [&](int kind, int64_t lo, int64_t hi, int32_t v) {
        lo = max(lo, vis_lo);
        hi = min(hi, vis_hi + 1);
        if (lo < hi) rg(kind, (int32_t)lo, (int32_t)hi, v);
    };

    // CIGAR (GROM.c:6740-7100): clip lengths, hard clips into cdp_lseq, I-D
    // balance, and the I/D events (GROM.c:7187-7423)
    const uint32_t cb = in.cig_off[i];
    uint32_t ce = in.cig_off[i + 1];
    if (ce - cb > (uint32_t)MAX_CIGAR) ce = cb + MAX_CIGAR;
    int32_t lseq = in.lqseq[i];
    const int32_t lq_raw = lseq;
    int sa = 0, ea = 0, eai = 0;
    {
        int64_t tp = pos;
        int32_t sb = 0;
        for (uint32_t k = cb; k < ce; k++) {
            const uint32_t cw = in.cigar[k];
            const int op = cw & 15;
            const int32_t len = (int32_t)(cw >> 4);
            if (k == cb && (op == 4 || op == 5)) sa = len;
            if (k == ce - 1 && (op == 4 || op == 5)) ea = len;
            if (op == 5) lseq += len;
            if (op == 1) eai += len;
            else if (op == 2) eai -= len;
            if (op == 4) {
                sb += len;
            } else if (op == 0 || op == 3 || op == 7 || op == 8) {
                tp += len;
                if (op != 3) sb += len;
            } else if (op == 1) {
                SvEv e{};
                e.type = OT_I;
                e.add = (uint8_t)add;
                e.w = (uint8_t)add;
                e.len = len;
                e.aux = in.base_off[i] + sb;
                e.rp = lq_raw - sb;
                event(tp, e);
                sb += len;
            } else if (op == 2) {
                SvEv e{};
                e.add = (uint8_t)add;
                e.w = (uint8_t)add;
                e.len = len;
                e.type = OT_DF;
                event(tp, e);
                e.type = OT_DR;
                event(tp + len - 1, e);
                tp += len;
            }
        }
    }
    const bool rev = flag & 0x10, mrev = flag & 0x20, paired = flag & 0x1, munmap = flag & 0x8;
    const int64_t E = (int64_t)pos - sa + lseq - ea - eai;
    const int32_t Mx = g.Mx, Mn = g.Mn;
    const int32_t tol = Mx - Mn;

    // an order-dependent cluster event
    auto clus = [&](int64_t x, int t, int w, double v, int32_t tl, int32_t rp, int rmode, int ctx, int quirk) {
        SvEv e{};
        e.v = v;
        e.rp = rp;
        e.mchr = mtid;
        e.len = tl;
        e.type = (uint8_t)(t + 1);
        e.w = (uint8_t)w;
        e.add = (uint8_t)add;
        e.fl = (uint8_t)(rmode | (ctx << 2) | (quirk << 4));
        event(x, e);
    };
    // a range block: rd += 1 and the cluster event at every base of [lo, hi)
    // (GROM.c:8388-8525); half 1: full weight only at lo when end-clipped,
    // half 2: only at hi-1 when start-clipped
    auto crange = [&](int64_t lo, int64_t hi, int t, double v, int32_t tl, int ctx, int half) {
        range(SUM_RD, lo, hi, 1);
        const bool clipped = (half == 1) ? (ea >= g.sc_min) : (sa >= g.sc_min);
        const int64_t edge = (half == 1) ? lo : hi - 1;
        for (int64_t x = max(lo, vis_lo); x < min(hi, vis_hi + 1); x++) {
            const bool full = !clipped || x == edge;
            clus(x, t, full ? add : add / 2, v, tl, pos, RM_SET, ctx, 0);
        }
    };

    // aux alignment (GROM.c:6683-6733)
    const int ai = in.aux_idx ? in.aux_idx[i] : -1;
    grom_aux A{};
    A.pos = -1;
    if (ai >= 0) A = in.aux[ai];
    const bool has_aux = ai >= 0 && A.pos >= 0;
    const int asa = A.start_adj, aea = A.end_adj, aeai = A.end_adj_indel;

    // ---- split-read deletion, GROM.c:7431-7945 ----
    if (has_aux && A.same_chr) {
        if (A.mq >= g.min_mapq && mq >= g.min_mapq) {
            bool sr = false;
            int64_t lps = 0, lpe = 0;
            if ((!rev && A.strand == 0) || (rev && A.strand == 1)) {
                if (paired && !munmap && in.mtid[i] == g.chr_tid) {
                    if (!rev && A.strand == 0) {
                        if (pos < A.pos && tlen <= Mx && A.pos < mpos && A.pos - E < Mx && A.pos - E > 0 &&
                            abs(lseq - ea - asa) <= g.max_split_loss && lseq - sa - ea - eai >= g.min_sr_len &&
                            lseq - asa - aea - aeai >= g.min_sr_len) {
                            sr = true;
                            lps = E;
                            lpe = A.pos;
                        }
                    } else if (rev && A.strand == 1) {
                        if (A.pos < pos && abs(tlen) < Mx && mpos < A.pos && abs(lseq - sa - aea) <= g.max_split_loss &&
                            lseq - sa - ea - eai >= g.min_sr_len && lseq - asa - aea - aeai >= g.min_sr_len) {
                            lps = (int64_t)A.pos - asa + lseq - aea - aeai;
                            lpe = pos;
                            sr = lps < lpe;
                        }
                    }
                } else {
                    if (!rev && A.strand == 0) {
                        if (pos < A.pos && A.pos - E < Mx && A.pos - E > 0) {
                            sr = true;
                            lps = E;
                            lpe = A.pos;
                        }
                    } else if (rev && A.strand == 1) {
                        if (A.pos < pos && pos - ((int64_t)A.pos - asa + lseq - aea - aeai) < Mx) {
                            lps = (int64_t)A.pos - asa + lseq - aea - aeai;
                            lpe = pos;
                            sr = lps < lpe;
                        }
                    }
                }
            }
            if (sr) {
                const int32_t d = (int32_t)(lpe - lps);
                if (d < g.lseq_g && d < Mx - g.mean) {  // also CIGAR-style indel evidence, GROM.c:7514-7640
                    SvEv e{};
                    e.add = (uint8_t)add;
                    e.w = (uint8_t)add;
                    e.len = d;
                    e.type = OT_DF;
                    event(lps, e);
                    e.type = OT_DR;
                    event(lpe - 1, e);
                }
                const double v = (double)(d + g.mean);
                range(SUM_RD, lps, lps + 1, 1);
                clus(lps, CL_DEL_F, add, v, tol, pos < A.pos ? pos : A.pos, RM_MAX, 0, 0);
                range(SUM_RD, lpe - 1, lpe, 1);
                clus(lpe - 1, CL_DEL_R, add, v, tol, pos < A.pos ? A.pos : pos, RM_MINMAX, 0, 0);
            }
        }
    }

    const int32_t insert_temp = (g.mean - 2 * lseq > 0) ? g.mean - 2 * lseq : 0;  // GROM.c:7954-7958
    const int32_t tol_inv = Mx - Mn + insert_temp;
    const int64_t fwd_end = (int64_t)pos - sa - eai + Mx - lseq;  // F-read range end before clips
    const int64_t rev_start = (int64_t)pos - sa - Mx + 2 * lseq;  // R-read range start

    // ---- pair classification, GROM.c:7960-10953 ----
    if (paired && !munmap) {
        if (g.chr_tid == mtid) {
            if (mpos > pos) {
                if (!rev && mrev) {
                    if (tlen >= Mn && tlen <= Mx) {
                        bool sr_dup = false;
                        int64_t lps = 0, lpe = 0;
                        if (has_aux && A.same_chr && A.mq >= g.min_mapq && mq >= g.min_mapq && A.strand == 0 &&
                            pos < A.pos && A.pos < mpos) {
                            const int eai_t = eai > 0 ? eai : 0;
                            const int aeai_t = aeai > 0 ? eai : 0;  // sic: cdp_end_adj_indel, GROM.c:7995
                            if (abs(lseq - sa - aea) <= g.max_split_loss && lseq - sa - ea - eai_t >= g.min_sr_len &&
                                lseq - asa - aea - aeai_t >= g.min_sr_len) {
                                sr_dup = true;
                                lps = pos;
                                lpe = (int64_t)A.pos - asa + lseq - aea - aeai;
                            }
                        }
                        if (sr_dup) {
                            const double v = (double)(lpe - lps - g.mean);
                            range(SUM_RD, lpe, lpe + 1, 1);
                            clus(lpe, CL_DUP_F, add, v, tol, pos < A.pos ? A.pos : pos, RM_MINMAX, 0, 1);
                            range(SUM_RD, lps - 1, lps, 1);
                            clus(lps - 1, CL_DUP_R, add, v, tol, pos < A.pos ? pos : A.pos, RM_MINMAX, 0, 0);
                        } else {
                            // concordant gap, GROM.c:8342-8365
                            const int64_t hi = min((int64_t)mpos, ring_hi);
                            range(SUM_RD, E, hi, 1);
                            range(SUM_CONC, E, hi, 1);
                        }
                    } else if (tlen > 2 * Mx) {
                        const int64_t hi = min(min(fwd_end, ring_hi), (int64_t)mpos);  // GROM.c:8370-8386
                        crange(E, hi, CL_DEL_F, (double)tlen, tol, 0, 1);
                    } else if (tlen > Mx) {
                        // GROM.c:8531-8825
                        const int64_t lo = E, hi = min((int64_t)mpos, ring_hi);
                        range(SUM_RD, lo, hi, 1);
                        const int64_t dr_after = (int64_t)pos - sa + tlen - Mx + lseq;
                        for (int64_t x = max(lo, vis_lo); x < min(hi, vis_hi + 1); x++) {
                            if (x < fwd_end) {
                                const bool full = ea < g.sc_min || x == lo;
                                clus(x, CL_DEL_F, full ? add : add / 2, (double)tlen, tol, pos, RM_SET, 0, 0);
                            }
                            if (abs(tlen) <= 2 * Mx && x > dr_after) {
                                const bool full = sa < g.sc_min || x == hi - 1;
                                clus(x, CL_DEL_R, full ? add : add / 2, (double)tlen, tol, mpos, RM_MINMAX, 0, 0);
                            }
                        }
                    } else if (tlen < Mn) {
                        // GROM.c:8826-8873 (the reverse-strand veto is nested unreachably)
                        const bool no_ins = has_aux && A.same_chr && A.strand == 0 && A.pos < pos && pos < mpos;
                        if (!no_ins) {
                            const int64_t hi = min((int64_t)mpos, ring_hi);
                            range(SUM_RD, E, hi, 1);
                            range(SUM_INS, E, hi, add);
                        }
                    }
                } else if (!rev && !mrev) {
                    if (mpos - pos >= 10) {  // GROM.c:8875-9044
                        const int64_t hi = min(min(fwd_end, ring_hi), (int64_t)mpos);
                        crange(E, hi, CL_INV_F1, (double)tlen, tol_inv, 0, 1);
                    }
                } else if (rev) {
                    if (mpos - pos >= 10) {  // GROM.c:9045-9351
                        const int64_t lo = max(rev_start, ring_lo);
                        if (mrev) crange(lo, pos, CL_INV_R1, (double)tlen, tol_inv, 0, 2);
                        else crange(lo, pos, CL_DUP_R, (double)tlen, tol, 0, 2);
                    }
                }
            } else {
                if (rev && !mrev) {
                    if (abs(tlen) >= Mn && abs(tlen) <= Mx) {
                        // split read over a tandem duplication, GROM.c:9359-9727
                        if (has_aux && A.same_chr && A.mq >= g.min_mapq && mq >= g.min_mapq && A.strand == 1 &&
                            A.pos < pos && mpos < A.pos) {
                            const int eai_t = eai > 0 ? eai : 0;
                            const int aeai_t = aeai > 0 ? eai : 0;  // sic, GROM.c:9381
                            if (abs(lseq - asa - ea) <= g.max_split_loss && lseq - sa - ea - eai_t >= g.min_sr_len &&
                                lseq - asa - aea - aeai_t >= g.min_sr_len) {
                                const int64_t lps = A.pos, lpe = E;
                                if (lps < lpe) {
                                    const double v = (double)(lpe - lps - g.mean);
                                    range(SUM_RD, lpe, lpe + 1, 1);
                                    clus(lpe, CL_DUP_F, add, v, tol, pos < A.pos ? A.pos : pos, RM_MINMAX, 0, 2);
                                    range(SUM_RD, lps - 1, lps, 1);
                                    clus(lps - 1, CL_DUP_R, add, v, tol, pos < A.pos ? pos : A.pos, RM_MINMAX, 0, 0);
                                }
                            }
                        }
                    } else if (abs(tlen) > 2 * Mx) {
                        // GROM.c:9730-9867
                        crange(max(rev_start, ring_lo), pos, CL_DEL_R, (double)abs(tlen), tol, 0, 2);
                    }
                } else if (!rev && !mrev) {
                    if (pos - mpos >= 10)  // GROM.c:9876-10019
                        crange(E, min(fwd_end, ring_hi), CL_INV_F2, (double)abs(tlen), tol_inv, 0, 1);
                } else if (mrev) {
                    if (pos - mpos >= 10) {  // GROM.c:10023-10312
                        if (!rev) crange(E, min(fwd_end, ring_hi), CL_DUP_F, (double)abs(tlen), tol, 0, 1);
                        else crange(max(rev_start, (int64_t)mpos + lseq), pos, CL_INV_R2, (double)abs(tlen), tol_inv, 0, 2);
                    }
                }
            }
        } else {
            // mate on another chromosome, GROM.c:10321-10903
            if (!rev) {
                if (!mrev) crange(E, min(fwd_end, ring_hi), CL_CTX_F, (double)mpos, tol, 1, 1);
                else crange(E, min(fwd_end, ring_hi), CL_CTX_F, (double)(-mpos), tol, 2, 1);
            } else {
                const int64_t lo = max((int64_t)pos - sa + lseq - Mx + lseq, ring_lo);
                if (!mrev) crange(lo, pos, CL_CTX_R, (double)mpos, tol, 1, 2);
                else crange(lo, pos, CL_CTX_R, (double)(-mpos), tol, 2, 2);
            }
        }
    } else if (paired && munmap) {
        // mate unmapped, GROM.c:10908-10952
        if (!rev) {
            const int64_t hi = min(fwd_end, ring_hi);
            range(SUM_RD, E, hi, 1);
            range(SUM_MUNF, E, hi, add);
        } else {
            const int64_t lo = max((int64_t)pos - sa + lseq + eai - Mx + lseq, ring_lo);
            range(SUM_RD, lo, pos, 1);
            range(SUM_MUNR, lo, pos, add);
        }
    }
}

__global__ void k_sv_count(View V, uint32_t *__restrict__ cnt, int32_t *__restrict__ sums, int64_t len) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < V.in.n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t c = 0;
        sv_walk(V, i, [&](int32_t, const SvEv &) { c++; },
                [&](int kind, int32_t lo, int32_t hi, int32_t v) {
                    int32_t *d = sums + (size_t)kind * (size_t)(len + 1);
                    atomicAdd(&d[lo], v);
                    atomicAdd(&d[hi], -v);
                });
        cnt[i] = c;
    }
}

__global__ void k_sv_emit(View V, const uint32_t *__restrict__ off, uint32_t *__restrict__ keys,
                          uint32_t *__restrict__ vals, SvEv *__restrict__ ev) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < V.in.n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t o = off[i];
        sv_walk(V, i,
                [&](int32_t x, const SvEv &e) {
                    ev[o] = e;
                    keys[o] = (uint32_t)x;
                    vals[o] = o;
                    o++;
                },
                [&](int, int32_t, int32_t, int32_t) {});
    }
}

// abs() of a double in the reference truncates to int first (cvttsd2si:
// NaN or out of range gives INT_MIN), SURVEY Q4
__device__ __forceinline__ int abs_trunc(double x) {
    const int i = (x != x || x >= 2147483648.0 || x < -2147483648.0) ? (int)0x80000000u : (int)x;
    return i < 0 ? (int)(0u - (uint32_t)i) : i;
}

struct Clus {
    int32_t cnt, rs, re;
    double dist;
};

struct FoldOut {
    // pass 1: per-run flags; pass 2: compacted outputs at the scanned offsets
    uint32_t *f_cand, *f_ind, *f_dbg;
    const uint32_t *o_cand, *o_ind, *o_dbg;
    grom_sv_rec *rec;         // candidate bases: cluster state
    grom_indel_rec *irec_c;   // candidate bases: indel state (parallel to rec)
    grom_indel_rec *irec;     // every base an indel event reached (test hook)
    grom_sv_rec *drec;        // debug: every base with cluster state
    uint32_t *bits;
    int32_t min_disc;
    const uint8_t *seq;
};

__device__ __forceinline__ bool compat(const SvEv &e, double dist, int32_t cnt, int32_t mchr) {
    const double lim = (double)e.len * (1.0 + (1.0 / (double)cnt));
    const int ctx = (e.fl >> 2) & 3;
    if (ctx == 0) return (double)abs_trunc(dist - e.v) <= lim;
    if (ctx == 1) return mchr == e.mchr && (double)abs_trunc(dist - e.v) <= lim && dist > 0;
    return mchr == e.mchr && (double)abs_trunc((double)abs_trunc(dist) - (-e.v)) <= lim && dist < 0;
}

__device__ __forceinline__ void rsre(int32_t &rs, int32_t &re, int32_t rp, int mode) {
    if (mode == RM_SET) re = rp;
    else if (mode == RM_MAX) re = max(re, rp);
    else { rs = min(rs, rp); re = max(re, rp); }
}

// One lane per base: the reference's fold over the base's events in stream
// order (GROM.c:7209-7420 indel primaries, and the 22 cluster blocks such as
// GROM.c:8403-8523), with the 50 shared "other" slots in scratch.
template <int WRITE>
__global__ __launch_bounds__(64) void k_sv_fold(uint32_t n_runs, const uint32_t *__restrict__ run_pos,
                                                const uint32_t *__restrict__ run_len,
                                                const uint32_t *__restrict__ run_off,
                                                const uint32_t *__restrict__ order, const SvEv *__restrict__ ev,
                                                FoldOut O) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_runs) return;
    const int32_t x = (int32_t)run_pos[r];
    Clus cl[CL_N];
    int32_t mchr[2] = {0, 0};
    for (int t = 0; t < CL_N; t++) cl[t] = Clus{0, 0, 0, 0.0};
    grom_indel_rec d;
    memset(&d, 0, sizeof(d));
    d.pos = x;
    bool any_indel = false;
    // the "other" slots in use are a prefix [0, n_used) (a slot is never
    // emptied again), so none is initialised until it is first taken: the
    // 300 scratch stores per base of round 5 were most of the fold's time
    int32_t ocnt[OTHER_LEN], omchr[OTHER_LEN], ors[OTHER_LEN], ore[OTHER_LEN];
    double odist[OTHER_LEN];
    uint8_t otype[OTHER_LEN];
    int n_used = 0;
    const uint32_t b = run_off[r], e_end = b + run_len[r];
    for (uint32_t j = b; j < e_end; j++) {
        const SvEv E = ev[order[j]];
        const int add = E.add;
        if (E.type >= OT_I) {
            // CIGAR-style indel evidence (GROM.c:7209-7420, split reads 7514-7640)
            any_indel = true;
            int32_t *cnt, *dist;
            if (E.type == OT_I) { cnt = &d.ins; dist = &d.ins_len; }
            else if (E.type == OT_DF) { cnt = &d.del_f; dist = &d.del_f_len; d.del_f_rd += 1; }
            else { cnt = &d.del_r; dist = &d.del_r_len; d.del_r_rd += 1; }
            if (*cnt == 0) {
                *cnt = add;
                *dist = E.len;
                if (E.type == OT_I && E.len <= ISEQ_LEN) {
                    for (int q = 0; q < E.len; q++) {
                        const int64_t nb = E.aux + q;
                        const uint8_t byte = O.seq[nb >> 1];
                        d.ins_seq[q] = q < E.rp ? c_nt16_sv[(nb & 1) ? (byte & 15) : (byte >> 4)] : 0;
                    }
                }
            } else if ((uint32_t)E.len == (uint32_t)*dist) {
                *cnt += add;
            } else {
                bool found = false;
                for (int o = 0; o < n_used; o++) {
                    if (otype[o] == E.type) {
                        if ((uint32_t)E.len == (uint32_t)(odist[o] + 0.5)) {
                            found = true;
                            ocnt[o] += add;
                            if (ocnt[o] > *cnt) {  // the slot overtakes the primary: swap (count, length)
                                const int32_t tc = ocnt[o];
                                const double td = odist[o];
                                ocnt[o] = *cnt;
                                odist[o] = (double)*dist;
                                *cnt = tc;
                                *dist = (int32_t)(uint32_t)(td + 0.5);
                            }
                            break;
                        }
                    }
                }
                if (!found && n_used < OTHER_LEN) {  // the first empty slot
                    const int o = n_used++;
                    found = true;
                    ocnt[o] = add;
                    otype[o] = E.type;
                    odist[o] = (double)E.len;
                    omchr[o] = 0;
                    ors[o] = ore[o] = 0;
                }
                if (!found) {
                    for (int o = 0; o < OTHER_LEN; o++) {
                        if (ocnt[o] <= add) {
                            ocnt[o] = add;
                            otype[o] = E.type;
                            odist[o] = (double)E.len;
                            ors[o] = 0;
                            ore[o] = 0;
                            break;
                        }
                    }
                }
            }
            continue;
        }
        // breakpoint cluster (the block of GROM.c:8403-8523 and its siblings)
        const int t = E.type - 1;
        const int rmode = E.fl & 3, quirk = (E.fl >> 4) & 3;
        const bool is_ctx = t >= CL_CTX_F;
        Clus &c = cl[t];
        int32_t *pm = is_ctx ? &mchr[t - CL_CTX_F] : nullptr;
        if (c.cnt == 0) {
            c.cnt = E.w;
            c.dist = E.v;
            if (pm) *pm = E.mchr;
            c.rs = E.rp;
            // sic: del_f_read_end (GROM.c:8036, 9419); both starts set the DEL
            // and DUP ring flags (GROM.c:8027-8036, 9408-9411), so the ring
            // shifts this evidence like any other
            if (quirk) cl[CL_DEL_F].re = E.rp;
            else c.re = E.rp;
        } else if (compat(E, c.dist, c.cnt, pm ? *pm : 0)) {
            c.cnt += E.w;
            c.dist += (double)E.w * (E.v - c.dist) / (double)c.cnt;
            rsre(c.rs, c.re, E.rp, rmode);
        } else {
            // an "other" slot write leaves the group's flags alone but moves no
            // primary data, so it cannot strand DUP evidence
            bool found = false;
            for (int o = 0; o < n_used; o++) {
                if (otype[o] == (uint8_t)E.type) {
                    if (compat(E, odist[o], ocnt[o], omchr[o])) {
                        found = true;
                        ocnt[o] += E.w;
                        odist[o] += (double)E.w * (E.v - odist[o]) / (double)ocnt[o];
                        rsre(ors[o], ore[o], E.rp, rmode);
                        if (ocnt[o] > c.cnt) {
                            const Clus tmp{ocnt[o], ors[o], ore[o], odist[o]};
                            ocnt[o] = c.cnt;
                            odist[o] = c.dist;
                            ors[o] = c.rs;
                            ore[o] = c.re;
                            c = tmp;
                            if (pm) { const int32_t tm = omchr[o]; omchr[o] = *pm; *pm = tm; }
                        }
                        break;
                    }
                }
            }
            if (!found && n_used < OTHER_LEN) {  // the first empty slot
                const int o = n_used++;
                found = true;
                ocnt[o] = E.w;
                otype[o] = E.type;
                odist[o] = E.v;
                omchr[o] = pm ? E.mchr : 0;
                ors[o] = ore[o] = E.rp;
            }
            if (!found) {
                for (int o = 0; o < OTHER_LEN; o++) {
                    if (ocnt[o] <= add) {
                        ocnt[o] = E.w;
                        otype[o] = E.type;
                        odist[o] = E.v;
                        if (pm) omchr[o] = E.mchr;
                        ors[o] = ore[o] = E.rp;
                        break;
                    }
                }
            }
        }
    }
    const int other_len = n_used;  // the first empty slot, GROM.c:11415-11425
    d.other_len = other_len;
    const int32_t thr = AF * O.min_disc;  // count / 6 >= g_min_disc
    bool cand = d.ins >= thr || d.del_f >= thr || d.del_r >= thr;
    bool dbg = other_len > 0;
    for (int t = 0; t < CL_N; t++) {
        cand = cand || cl[t].cnt >= thr;
        dbg = dbg || cl[t].cnt != 0;
    }
    if (!WRITE) {
        O.f_cand[r] = cand;
        O.f_ind[r] = any_indel;
        O.f_dbg[r] = dbg;
        if (cand) {
            atomicOr(&O.bits[x >> 5], 1u << (x & 31));
            if (d.ins >= thr) atomicOr(&O.bits[(x + 1) >> 5], 1u << ((x + 1) & 31));  // sc_left(p+1), GROM.c:11409
        }
        return;
    }
    grom_sv_rec s;
    memset(&s, 0, sizeof(s));
    s.pos = x;
    s.other_len = other_len;
    for (int t = 0; t < CL_N; t++) {
        s.cnt[t] = cl[t].cnt;
        s.rs[t] = cl[t].rs;
        s.re[t] = cl[t].re;
        s.dist[t] = cl[t].dist;
    }
    s.ctx_mchr[0] = mchr[0];
    s.ctx_mchr[1] = mchr[1];
    if (cand) {
        O.rec[O.o_cand[r]] = s;
        O.irec_c[O.o_cand[r]] = d;
    }
    if (any_indel && O.irec) O.irec[O.o_ind[r]] = d;
    if (dbg && O.drec) O.drec[O.o_dbg[r]] = s;
}

// the debug records get the range sums at their base
__global__ void k_sv_dbg_sums(int64_t n, grom_sv_rec *__restrict__ rec, const int32_t *__restrict__ sums, int64_t len) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t x = rec[i].pos;
    const size_t L = (size_t)(len + 1);
    rec[i].rd_add = sums[x];
    rec[i].conc = sums[L + x];
    rec[i].ins = sums[2 * L + x];
    rec[i].mun_f = sums[3 * L + x];
    rec[i].mun_r = sums[4 * L + x];
}

// bases with an insertion-range sum that alone reaches g_min_disc reads
__global__ void k_sv_ins_bits(int32_t lo, int32_t hi, const int32_t *__restrict__ ins, int32_t thr,
                              uint32_t *__restrict__ bits) {
    const int64_t x = lo + blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (x > hi) return;
    if (ins[x] >= thr) atomicOr(&bits[x >> 5], 1u << (x & 31));
}

struct EvalIn {
    const grom_sv_ctx *ctx;
    uint32_t n_ctx;
    const grom_sv_rec *rec;
    const grom_indel_rec *irec;
    uint32_t n_rec;
    const int32_t *sums;
    int64_t len;
    const double *mq, *hez;
    int32_t eval_lo, eval_hi, lseq_tail;
    int32_t Mx, overlap;
    int32_t min_disc, mean, glseq;
    double pval1, pval_ins1, max_ev_ratio;
    SvInput in;
    SvHit *hits;
    uint32_t *n_hits;
    uint32_t hit_cap;
};

__device__ __forceinline__ double T(const double *t, int64_t n, int64_t k) { return t[n * (MT + 1) + k]; }

// binomial test of a breakpoint count (GROM.c:11968-12006 and nine copies);
// the evidence-ratio check reads (rn_hi, rden_hi) above g_max_trials and
// (rn_lo, rden_lo) otherwise -- they differ only for CTX_R
__device__ void sv_test(const EvalIn &I, int cnt, int rd, int scmu, int rn_hi, int rden_hi, int rn_lo, int rden_lo,
                        double &binom, double &hez) {
    hez = 2.0;
    if (rd > MT) {
        binom = T(I.mq, MT, cnt * MT / (AF * rd));
        if ((double)((float)rn_hi / (float)rden_hi) <= I.max_ev_ratio) {
            if ((cnt + scmu) / AF < rd) hez = T(I.hez, MT, (cnt + scmu) * MT / (AF * rd));
            else hez = T(I.hez, MT, MT);
        }
    } else {
        binom = T(I.mq, rd, cnt / AF);
        if ((double)((float)rn_lo / (float)rden_lo) <= I.max_ev_ratio) {
            if ((cnt + scmu) / AF < rd) hez = T(I.hez, rd, (cnt + scmu) / AF);
            else hez = T(I.hez, rd, rd);
        }
    }
}

// cdp_lseq at the evaluation of p: the length of the stream's next record
// not yet ingested (pos - l*Mx > p), kept or dropped, else the tail record's
__device__ int32_t pending_lseq(const EvalIn &I, int32_t p) {
    const int64_t t = (int64_t)p + (int64_t)I.overlap * I.Mx;
    int64_t lo = 0, hi = I.in.n;  // first kept read with pos > t
    while (lo < hi) {
        const int64_t m = (lo + hi) >> 1;
        if ((int64_t)I.in.pos[m] > t) hi = m;
        else lo = m + 1;
    }
    const int64_t ik = lo;
    lo = 0;
    hi = I.in.n_drop;
    while (lo < hi) {
        const int64_t m = (lo + hi) >> 1;
        if ((int64_t)I.in.drop_pos[m] > t) hi = m;
        else lo = m + 1;
    }
    const int64_t id = lo;
    if (id < I.in.n_drop && (ik >= I.in.n || I.in.drop_before[id] <= ik)) return I.in.drop_lq[id];
    if (ik < I.in.n) return I.in.lqseq[ik];
    return I.lseq_tail;
}

// cdp_lseq at the evaluation of each base in pos[] (the -f SNV rows print
// that many bases of context at a mid-scan flush, GROM.c:11296-11316)
__global__ void k_pending_lseq(EvalIn I, const int32_t *__restrict__ pos, int n, int32_t *__restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = pending_lseq(I, pos[i]);
}

__global__ void k_sv_eval(EvalIn I) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= I.n_ctx) return;
    const grom_sv_ctx c = I.ctx[j];
    const int32_t p = c.pos;
    if (p < I.eval_lo || p > I.eval_hi) return;
    // the fold record of this base, if any
    uint32_t lo = 0, hi = I.n_rec;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (I.rec[m].pos < p) lo = m + 1;
        else hi = m;
    }
    const bool has = lo < I.n_rec && I.rec[lo].pos == p;
    grom_sv_rec s;
    grom_indel_rec d;
    if (has) {
        s = I.rec[lo];
        d = I.irec[lo];
    } else {
        memset(&s, 0, sizeof(s));
        memset(&d, 0, sizeof(d));
    }
    // sc_left at p + 1: its context record follows, or there is no clip evidence there
    int32_t scl_next = 0;
    if (j + 1 < I.n_ctx && I.ctx[j + 1].pos == p + 1) scl_next = I.ctx[j + 1].sc_left;
    const size_t L = (size_t)(I.len + 1);
    const int32_t rd = c.rd + I.sums[p];
    const int32_t conc = I.sums[L + p], ins = I.sums[2 * L + p], munf = I.sums[3 * L + p], munr = I.sums[4 * L + p];
    SvHit h;
    memset(&h, 0, sizeof(h));
    h.pos = p;
    h.conc = conc;
    h.rd = rd;
    h.ins = ins;
    h.other_len = s.other_len;
    h.ctx_mchr[0] = s.ctx_mchr[0];
    h.ctx_mchr[1] = s.ctx_mchr[1];
    uint32_t mask = 0;
    double binom, hez;
    if (rd + c.indel_sc_rd > 0) {
        // CIGAR insertion, GROM.c:11338-11453
        int irt = c.snv_all;
        int it = d.ins;
        if (it / AF > irt) it = irt * AF;
        if (it / AF >= I.min_disc && irt <= MT) {
            binom = T(I.mq, irt, it / AF);
            if ((it + c.indel_sc_left) / AF < irt) {
                hez = T(I.hez, irt, (it + c.indel_sc_left) / AF);
                if ((it + c.indel_sc_right) / AF < irt) {
                    const double h2 = T(I.hez, irt, (it + c.indel_sc_right) / AF);
                    if (h2 > hez) hez = h2;
                } else {
                    hez = T(I.hez, irt, irt);
                }
            } else {
                hez = T(I.hez, irt, irt);
            }
            if (binom <= I.pval1) {
                mask |= HIT_II;
                h.ii_binom = binom;
                h.ii_hez = hez;
                h.ii_dist = d.ins_len;
                h.ii_i = it;
                h.ii_rd = irt;
                h.ii_sc = scl_next + c.sc_right;
                for (int q = 0; q < 52; q++) h.ii_seq[q] = d.ins_seq[q];
            }
        }
        // deletion start, GROM.c:11460-11629
        irt = d.del_f / AF + c.snv_all;
        const int dft = d.del_f;
        if (dft / AF >= I.min_disc && irt <= MT) {
            binom = T(I.mq, irt, dft / AF);
            hez = ((dft + c.indel_sc_right) / AF < irt) ? T(I.hez, irt, (dft + c.indel_sc_right) / AF) : T(I.hez, irt, irt);
            if (binom <= I.pval1) {
                mask |= HIT_DF;
                h.df_binom = binom;
                h.df_hez = hez;
                h.df_f = dft;
                h.df_rd = irt;
                h.df_sc = c.sc_right;
            }
        }
        // deletion end, GROM.c:11631-11745 (the list-index gate is applied on the host)
        irt = d.del_r / AF + c.snv_all;
        const int drt = d.del_r;
        if (drt / AF >= I.min_disc && irt <= MT) {
            binom = T(I.mq, irt, drt / AF);
            hez = ((drt + c.indel_sc_left) / AF < irt) ? T(I.hez, irt, (drt + c.indel_sc_left) / AF) : T(I.hez, irt, irt);
            if (binom <= I.pval1) {
                mask |= HIT_DR;
                h.dr_binom = binom;
                h.dr_hez = hez;
                h.dr_r = drt;
                h.dr_rd = irt;
                h.dr_sc = c.sc_left;
                h.dr_rdist = d.del_r_len;
            }
        }
    }
    if (rd + c.sc_rd > 0) {
        // soft-clip insertion start / end, GROM.c:11750-11960
        for (int side = 0; side < 2; side++) {
            const int sc = side == 0 ? c.sc_left : c.sc_right;
            const int mu = side == 0 ? munr : munf;
            const int rdt = rd + (side == 0 ? c.sc_left_rd : c.sc_right_rd);
            if ((sc + ins) / AF >= I.min_disc && rdt <= MT) {
                binom = ((mu + sc + ins) / AF < rdt) ? T(I.mq, rdt, (mu + sc + ins) / AF) : T(I.mq, rdt, rdt);
                if (binom <= I.pval_ins1) {
                    mask |= side == 0 ? HIT_INSL : HIT_INSR;
                    if (side == 0) h.insl_binom = binom;
                    else h.insr_binom = binom;
                }
            }
        }
    }
    if (rd > 0) {
        const int scr_muf = c.sc_right + munf, scl_mur = c.sc_left + munr;
        const int32_t cur_lseq = pending_lseq(I, p);
        for (int t = 0; t < CL_N; t++) {
            const int cnt = s.cnt[t];
            if (cnt / AF < I.min_disc) continue;
            // F clusters end near their last read, R clusters start near their first (GROM.c:11966, 12047)
            const bool f_side = t == CL_CTX_F || t == CL_DUP_F || t == CL_DEL_F || t == CL_INV_F1 || t == CL_INV_F2;
            if (f_side ? !(p - s.re[t] < I.mean) : !(s.rs[t] + cur_lseq - p < I.mean)) continue;
            const int scmu = f_side ? scr_muf : scl_mur;
            if (t == CL_CTX_R) sv_test(I, cnt, rd, scmu, scl_mur, cnt, scr_muf, s.cnt[CL_CTX_F], binom, hez);
            else sv_test(I, cnt, rd, scmu, scmu, cnt, scmu, cnt, binom, hez);
            if (binom <= I.pval1) {
                mask |= HIT_CL0 << t;
                h.cl[t].dist = s.dist[t];
                h.cl[t].binom = binom;
                h.cl[t].hez = hez;
                h.cl[t].cnt = cnt;
                h.cl[t].rs = s.rs[t];
                h.cl[t].re = s.re[t];
            }
        }
    }
    if (!mask) return;
    h.mask = mask;
    const uint32_t k = atomicAdd(I.n_hits, 1u);
    if (k < I.hit_cap) I.hits[k] = h;
}

__global__ void k_ctx_keys(const grom_sv_ctx *__restrict__ c, uint32_t n, uint32_t *__restrict__ k,
                           uint32_t *__restrict__ v) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        k[i] = (uint32_t)c[i].pos;
        v[i] = i;
    }
}

__global__ void k_ctx_gather(const grom_sv_ctx *__restrict__ src, const uint32_t *__restrict__ ord, uint32_t n,
                             grom_sv_ctx *__restrict__ dst) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[ord[i]];
}

struct Buf {
    void *p = nullptr;
    size_t cap = 0;
    bool own = false;          // p is this buffer's own allocation (else a piece of `ar`'s phase)
    grom_arena *ar = nullptr;  // the context's phase arena (sv_scratch_phase), or none
};

}  // namespace

struct SvScratch {
    Buf cnt, off, keys, vals, keys2, vals2, ev, run_pos, run_len, run_off, n_runs, tmp, sums, bits;
    Buf f_cand, f_ind, f_dbg, o_cand, o_ind, o_dbg, rec, irec_c, irec, drec;
    Buf ctx, ctx2, ckeys, ckeys2, cvals, cvals2, n_ctx, hits, n_hits, hits2;
    SvHit *h_hits = nullptr;  // pinned: the hits of the last evaluation, in base order
    size_t h_hits_cap = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int64_t len = 0;
    uint32_t n_rec = 0, n_irec = 0, n_drec = 0, ctx_cap = 0;
    uint32_t ctx_min = 0;  // a retry's capacity for the pileup's context records
};

static int sbuf(Buf &b, size_t bytes, char *err, size_t errlen) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return GROM_OK;
    if (b.p && b.own) grom_dev_free(b.p, b.cap, GROM_DEVCAT_SV);
    b.p = nullptr;
    b.cap = 0;
    b.own = false;
    const size_t want = bytes + bytes / 8 + 64;
    if (b.ar && (b.p = grom_arena_take(b.ar, want)) != nullptr) {
        b.cap = want;
        return GROM_OK;
    }
    if (grom_dev_malloc(&b.p, want, GROM_DEVCAT_SV)) {
        snprintf(err, errlen, "breakpoint pass: hipMalloc(%zu) failed", want);
        return GROM_E_NOMEM;
    }
    b.cap = want;
    b.own = true;
    return GROM_OK;
}

SvScratch *sv_scratch_new() { return new SvScratch(); }

#define SV_ALL_BUFS(s)                                                                                                \
    {&s->cnt, &s->off, &s->keys, &s->vals, &s->keys2, &s->vals2, &s->ev, &s->run_pos, &s->run_len, &s->run_off,       \
     &s->n_runs, &s->tmp, &s->sums, &s->bits, &s->f_cand, &s->f_ind, &s->f_dbg, &s->o_cand, &s->o_ind, &s->o_dbg,      \
     &s->rec, &s->irec_c, &s->irec, &s->drec, &s->ctx, &s->ctx2, &s->ckeys, &s->ckeys2, &s->cvals, &s->cvals2,         \
     &s->n_ctx, &s->hits, &s->n_hits, &s->hits2}

void sv_scratch_phase(SvScratch *s, grom_arena *ar) {
    Buf *all[] = SV_ALL_BUFS(s);
    for (Buf *b : all) {
        if (b->own && ar) grom_dev_free(b->p, b->cap, GROM_DEVCAT_SV);  // (an overflow of the last phase)
        if (!b->own || ar) {
            b->p = nullptr;
            b->cap = 0;
            b->own = false;
        }
        b->ar = ar;
    }
}

void sv_scratch_free(SvScratch *s) {
    if (!s) return;
    Buf *all[] = SV_ALL_BUFS(s);
    for (Buf *b : all)
        if (b->p && b->own) grom_dev_free(b->p, b->cap, GROM_DEVCAT_SV);
    if (s->h_hits) (void)hipHostFree(s->h_hits);
    if (s->e0) (void)hipEventDestroy(s->e0);
    if (s->e1) (void)hipEventDestroy(s->e1);
    delete s;
}

const uint32_t *sv_bits(const SvScratch *S) { return (const uint32_t *)S->bits.p; }
const int32_t *sv_rd_add(const SvScratch *S) { return (const int32_t *)S->sums.p; }
grom_sv_ctx *sv_ctx_buf(const SvScratch *S) { return (grom_sv_ctx *)S->ctx.p; }
uint32_t sv_ctx_cap(const SvScratch *S) { return S->ctx_cap; }
int sv_ctx_used(SvScratch *S, hipStream_t st, uint32_t *used) {
    *used = 0;
    if (!S || !S->n_ctx.p) return GROM_OK;
    if (hipMemcpyAsync(used, S->n_ctx.p, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return GROM_E_HIP;
    return GROM_OK;
}
void sv_ctx_reserve(SvScratch *S, uint32_t cap) {
    if (S) S->ctx_min = std::max(S->ctx_min, cap);
}
uint32_t *sv_ctx_count(const SvScratch *S) { return (uint32_t *)S->n_ctx.p; }
const grom_indel_rec *sv_indel_records(const SvScratch *S) { return (const grom_indel_rec *)S->irec.p; }
int64_t sv_indel_count(const SvScratch *S) { return S->n_irec; }
const grom_sv_rec *sv_debug_records(const SvScratch *S) { return (const grom_sv_rec *)S->drec.p; }
int64_t sv_debug_count(const SvScratch *S) { return S->n_drec; }

#define SCHK(x)                                                                          \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            snprintf(err, errlen, "breakpoint pass: %s: %s", #x, hipGetErrorString(e_)); \
            return GROM_E_HIP;                                                           \
        }                                                                                \
    } while (0)

static Geo make_geo(const grom_params &P, const grom_chrom &ch, int32_t eval_lo, int32_t eval_hi) {
    Geo g{};
    g.Mx = P.insert_max_size;
    g.Mn = P.insert_min_size;
    g.mean = P.insert_mean;
    g.lseq_g = P.lseq;
    g.overlap = P.overlap_mult;
    g.s0 = P.one_base_rd_len / 4 + 1;  // GROM.c:2918
    g.n_skip = ch.n_skip;
    g.H = P.half_one_base_rd_len;
    g.r14 = P.r14_one_base_rd_len;
    g.R = P.one_base_rd_len;
    g.sc_min = P.sc_min;
    g.min_mapq = P.min_mapq;
    g.max_split_loss = P.max_split_loss;
    g.min_sr_len = P.min_sr_len;
    g.eval_lo = eval_lo;
    g.eval_hi = eval_hi;
    g.chr_tid = ch.tid;
    g.min_disc = P.min_disc;
    g.splitread = P.splitread;
    return g;
}

int sv_prepare(SvScratch *S, hipStream_t st, const grom_params &P, const SvInput &in, const grom_chrom &ch,
               int32_t eval_lo, int32_t eval_hi, bool debug, char *err, size_t errlen) {
    int rc;
    const int64_t n = in.n, len = ch.len;
    S->len = len;
    S->n_rec = S->n_irec = S->n_drec = 0;
    if (n >= (int64_t)UINT32_MAX) {
        snprintf(err, errlen, "breakpoint pass: %lld reads exceed the 32-bit event index", (long long)n);
        return GROM_E_ARG;
    }
    if (!S->e0) {
        SCHK(hipEventCreate(&S->e0));
        SCHK(hipEventCreate(&S->e1));
    }
    SCHK(hipEventRecord(S->e0, st));
    const size_t L = (size_t)(len + 1);
    const int64_t n_words = (len + 64) / 32 + 1;
    if ((rc = sbuf(S->sums, sizeof(int32_t) * SUM_N * L, err, errlen)) ||
        (rc = sbuf(S->bits, sizeof(uint32_t) * n_words, err, errlen)) ||
        (rc = sbuf(S->cnt, sizeof(uint32_t) * (n + 1), err, errlen)) ||
        (rc = sbuf(S->off, sizeof(uint32_t) * (n + 1), err, errlen)) ||
        (rc = sbuf(S->n_ctx, 16, err, errlen)))
        return rc;
    int32_t *sums = (int32_t *)S->sums.p;
    SCHK(hipMemsetAsync(sums, 0, sizeof(int32_t) * SUM_N * L, st));
    SCHK(hipMemsetAsync(S->bits.p, 0, sizeof(uint32_t) * n_words, st));
    SCHK(hipMemsetAsync(S->n_ctx.p, 0, 16, st));
    // room for the pileup's context records: every clipped base and every marked one
    S->ctx_cap = (uint32_t)std::min<int64_t>(std::max<int64_t>(1 << 16, len / 64 + 2 * n / 16), (int64_t)1 << 28);
    if (const char *e = getenv("GROM_SV_CTX_CAP")) {  // test hook: a small first guess forces the retry
        if (atol(e) > 0) S->ctx_cap = (uint32_t)atol(e);
    }
    if (S->ctx_min > S->ctx_cap) S->ctx_cap = S->ctx_min;
    if ((rc = sbuf(S->ctx, sizeof(grom_sv_ctx) * S->ctx_cap, err, errlen))) return rc;
    if (eval_hi < eval_lo || n <= 0) return GROM_OK;

    View V{in, make_geo(P, ch, eval_lo, eval_hi)};
    const int g = (int)std::min<int64_t>((n + 255) / 256, 8192);
    uint32_t *cnt = (uint32_t *)S->cnt.p, *off = (uint32_t *)S->off.p;
    SCHK(hipMemsetAsync(cnt + n, 0, sizeof(uint32_t), st));
    hipLaunchKernelGGL(k_sv_count, dim3(g), dim3(256), 0, st, V, cnt, sums, len);
    SCHK(hipGetLastError());
    // order-free range sums: inclusive scans of the difference arrays
    {
        size_t tb = 0;
        SCHK(hipcub::DeviceScan::InclusiveSum(nullptr, tb, sums, sums, (int)L, st));
        if ((rc = sbuf(S->tmp, tb, err, errlen))) return rc;
        for (int k = 0; k < SUM_N; k++)
            SCHK(hipcub::DeviceScan::InclusiveSum(S->tmp.p, tb, sums + k * L, sums + k * L, (int)L, st));
    }
    {
        const int64_t m = (int64_t)eval_hi - eval_lo + 1;
        hipLaunchKernelGGL(k_sv_ins_bits, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, eval_lo, eval_hi,
                           (const int32_t *)(sums + 2 * L), AF * P.min_disc, (uint32_t *)S->bits.p);
        SCHK(hipGetLastError());
    }
    size_t tmp_bytes = 0;
    SCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, cnt, off, (int)(n + 1), st));
    if ((rc = sbuf(S->tmp, tmp_bytes, err, errlen))) return rc;
    SCHK(hipcub::DeviceScan::ExclusiveSum(S->tmp.p, tmp_bytes, cnt, off, (int)(n + 1), st));
    uint32_t n_ev = 0;
    SCHK(hipMemcpyAsync(&n_ev, off + n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    SCHK(hipStreamSynchronize(st));
    if (n_ev == 0) return GROM_OK;
    if ((rc = sbuf(S->keys, sizeof(uint32_t) * n_ev, err, errlen)) ||
        (rc = sbuf(S->vals, sizeof(uint32_t) * n_ev, err, errlen)) ||
        (rc = sbuf(S->keys2, sizeof(uint32_t) * n_ev, err, errlen)) ||
        (rc = sbuf(S->vals2, sizeof(uint32_t) * n_ev, err, errlen)) ||
        (rc = sbuf(S->ev, sizeof(SvEv) * n_ev, err, errlen)) ||
        (rc = sbuf(S->run_pos, sizeof(uint32_t) * n_ev, err, errlen)) ||
        (rc = sbuf(S->run_len, sizeof(uint32_t) * n_ev, err, errlen)) ||
        (rc = sbuf(S->run_off, sizeof(uint32_t) * (n_ev + 1), err, errlen)) ||
        (rc = sbuf(S->n_runs, sizeof(uint32_t) * 2, err, errlen)))
        return rc;
    uint32_t *keys = (uint32_t *)S->keys.p, *vals = (uint32_t *)S->vals.p;
    uint32_t *keys2 = (uint32_t *)S->keys2.p, *vals2 = (uint32_t *)S->vals2.p;
    hipLaunchKernelGGL(k_sv_emit, dim3(g), dim3(256), 0, st, V, off, keys, vals, (SvEv *)S->ev.p);
    SCHK(hipGetLastError());
    // stable LSD radix sort on the base: each base's events stay in stream order
    int bit_hi = 1;
    while (bit_hi < 32 && ((int64_t)1 << bit_hi) <= len + 1) bit_hi++;
    size_t t_sort = 0, t_rle = 0, t_scan = 0;
    SCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, t_sort, keys, keys2, vals, vals2, (int)n_ev, 0, bit_hi, st));
    SCHK(hipcub::DeviceRunLengthEncode::Encode(nullptr, t_rle, keys2, (uint32_t *)S->run_pos.p,
                                               (uint32_t *)S->run_len.p, (uint32_t *)S->n_runs.p, (int)n_ev, st));
    SCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, t_scan, (uint32_t *)S->run_len.p, (uint32_t *)S->run_off.p,
                                          (int)n_ev + 1, st));
    if ((rc = sbuf(S->tmp, std::max(t_sort, std::max(t_rle, t_scan)), err, errlen))) return rc;
    SCHK(hipcub::DeviceRadixSort::SortPairs(S->tmp.p, t_sort, keys, keys2, vals, vals2, (int)n_ev, 0, bit_hi, st));
    SCHK(hipcub::DeviceRunLengthEncode::Encode(S->tmp.p, t_rle, keys2, (uint32_t *)S->run_pos.p,
                                               (uint32_t *)S->run_len.p, (uint32_t *)S->n_runs.p, (int)n_ev, st));
    uint32_t n_runs = 0;
    SCHK(hipMemcpyAsync(&n_runs, S->n_runs.p, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    SCHK(hipStreamSynchronize(st));
    if (n_runs == 0 || n_runs > n_ev) {
        snprintf(err, errlen, "breakpoint pass: %u position runs for %u events", n_runs, n_ev);
        return GROM_E_HIP;
    }
    SCHK(hipcub::DeviceScan::ExclusiveSum(S->tmp.p, t_scan, (uint32_t *)S->run_len.p, (uint32_t *)S->run_off.p,
                                          (int)n_runs, st));
    // the fold, pass 1: flags and candidate bits
    if ((rc = sbuf(S->f_cand, sizeof(uint32_t) * (n_runs + 1), err, errlen)) ||
        (rc = sbuf(S->f_ind, sizeof(uint32_t) * (n_runs + 1), err, errlen)) ||
        (rc = sbuf(S->f_dbg, sizeof(uint32_t) * (n_runs + 1), err, errlen)) ||
        (rc = sbuf(S->o_cand, sizeof(uint32_t) * (n_runs + 1), err, errlen)) ||
        (rc = sbuf(S->o_ind, sizeof(uint32_t) * (n_runs + 1), err, errlen)) ||
        (rc = sbuf(S->o_dbg, sizeof(uint32_t) * (n_runs + 1), err, errlen)))
        return rc;
    FoldOut O{};
    O.f_cand = (uint32_t *)S->f_cand.p;
    O.f_ind = (uint32_t *)S->f_ind.p;
    O.f_dbg = (uint32_t *)S->f_dbg.p;
    O.o_cand = (const uint32_t *)S->o_cand.p;
    O.o_ind = (const uint32_t *)S->o_ind.p;
    O.o_dbg = (const uint32_t *)S->o_dbg.p;
    O.bits = (uint32_t *)S->bits.p;
    O.min_disc = P.min_disc;
    O.seq = in.seq;
    SCHK(hipMemsetAsync(O.f_cand + n_runs, 0, 4, st));
    SCHK(hipMemsetAsync(O.f_ind + n_runs, 0, 4, st));
    SCHK(hipMemsetAsync(O.f_dbg + n_runs, 0, 4, st));
    const dim3 fg((n_runs + 63) / 64), fb(64);
    hipLaunchKernelGGL(k_sv_fold<0>, fg, fb, 0, st, n_runs, (const uint32_t *)S->run_pos.p,
                       (const uint32_t *)S->run_len.p, (const uint32_t *)S->run_off.p, (const uint32_t *)vals2,
                       (const SvEv *)S->ev.p, O);
    SCHK(hipGetLastError());
    for (int k = 0; k < 3; k++) {
        uint32_t *f = k == 0 ? O.f_cand : k == 1 ? O.f_ind : O.f_dbg;
        uint32_t *o = (uint32_t *)(k == 0 ? S->o_cand.p : k == 1 ? S->o_ind.p : S->o_dbg.p);
        size_t tb = 0;
        SCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, f, o, (int)n_runs + 1, st));
        if ((rc = sbuf(S->tmp, tb, err, errlen))) return rc;
        SCHK(hipcub::DeviceScan::ExclusiveSum(S->tmp.p, tb, f, o, (int)n_runs + 1, st));
    }
    uint32_t cnts[3];
    SCHK(hipMemcpyAsync(&cnts[0], (uint32_t *)S->o_cand.p + n_runs, 4, hipMemcpyDeviceToHost, st));
    SCHK(hipMemcpyAsync(&cnts[1], (uint32_t *)S->o_ind.p + n_runs, 4, hipMemcpyDeviceToHost, st));
    SCHK(hipMemcpyAsync(&cnts[2], (uint32_t *)S->o_dbg.p + n_runs, 4, hipMemcpyDeviceToHost, st));
    SCHK(hipStreamSynchronize(st));
    S->n_rec = cnts[0];
    S->n_irec = cnts[1];
    S->n_drec = debug ? cnts[2] : 0;
    if ((rc = sbuf(S->rec, sizeof(grom_sv_rec) * (S->n_rec + 1), err, errlen)) ||
        (rc = sbuf(S->irec_c, sizeof(grom_indel_rec) * (S->n_rec + 1), err, errlen)) ||
        (rc = sbuf(S->irec, sizeof(grom_indel_rec) * (S->n_irec + 1), err, errlen)) ||
        (debug && (rc = sbuf(S->drec, sizeof(grom_sv_rec) * (S->n_drec + 1), err, errlen))))
        return rc;
    O.rec = (grom_sv_rec *)S->rec.p;
    O.irec_c = (grom_indel_rec *)S->irec_c.p;
    O.irec = (grom_indel_rec *)S->irec.p;
    O.drec = debug ? (grom_sv_rec *)S->drec.p : nullptr;
    hipLaunchKernelGGL(k_sv_fold<1>, fg, fb, 0, st, n_runs, (const uint32_t *)S->run_pos.p,
                       (const uint32_t *)S->run_len.p, (const uint32_t *)S->run_off.p, (const uint32_t *)vals2,
                       (const SvEv *)S->ev.p, O);
    SCHK(hipGetLastError());
    if (debug && S->n_drec) {
        hipLaunchKernelGGL(k_sv_dbg_sums, dim3((S->n_drec + 255) / 256), dim3(256), 0, st, (int64_t)S->n_drec,
                           (grom_sv_rec *)S->drec.p, (const int32_t *)sums, len);
        SCHK(hipGetLastError());
    }
    return GROM_OK;
}

// (pos, slot) of each hit, and the hits gathered into base order
__global__ void k_hit_keys(const SvHit *__restrict__ h, uint32_t n, uint32_t *__restrict__ keys,
                           uint32_t *__restrict__ vals) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        keys[i] = (uint32_t)h[i].pos;
        vals[i] = i;
    }
}
__global__ void k_hit_gather(const SvHit *__restrict__ h, const uint32_t *__restrict__ idx, uint32_t n,
                             SvHit *__restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = h[idx[i]];
}

int sv_pending_lseq(hipStream_t st, const grom_params &P, const SvInput &in, const grom_chrom &ch,
                    const int32_t *h_pos, int n, int32_t *h_out, char *err, size_t errlen) {
    if (n <= 0) return GROM_OK;
    EvalIn I{};
    I.in = in;
    I.lseq_tail = ch.lseq_tail;
    I.Mx = P.insert_max_size;
    I.overlap = P.overlap_mult;
    int32_t *d = nullptr;
    SCHK(hipMallocAsync((void **)&d, sizeof(int32_t) * 2 * (size_t)n, st));
    SCHK(hipMemcpyAsync(d, h_pos, sizeof(int32_t) * n, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_pending_lseq, dim3((n + 63) / 64), dim3(64), 0, st, I, (const int32_t *)d, n, d + n);
    SCHK(hipGetLastError());
    SCHK(hipMemcpyAsync(h_out, d + n, sizeof(int32_t) * n, hipMemcpyDeviceToHost, st));
    SCHK(hipFreeAsync(d, st));
    SCHK(hipStreamSynchronize(st));
    return GROM_OK;
}

int sv_evaluate(SvScratch *S, hipStream_t st, const grom_params &P, const SvInput &in, const grom_chrom &ch,
                int32_t eval_lo, int32_t eval_hi, const double *d_mq, const double *d_hez, const SvHit **hits_out,
                size_t *n_hits_out, double *ms_device, char *err, size_t errlen) {
    int rc;
    *hits_out = S->h_hits;
    *n_hits_out = 0;
    uint32_t n_ctx = 0;
    SCHK(hipMemcpyAsync(&n_ctx, S->n_ctx.p, 4, hipMemcpyDeviceToHost, st));
    SCHK(hipStreamSynchronize(st));
    if (n_ctx > S->ctx_cap) {
        snprintf(err, errlen, "breakpoint pass: %u context records exceed the buffer (%u)", n_ctx, S->ctx_cap);
        return GROM_E_OVERFLOW;
    }
    if (n_ctx && eval_hi >= eval_lo) {
        // contexts in base order: sort (pos, index) and gather
        if ((rc = sbuf(S->ckeys, 4 * n_ctx, err, errlen)) || (rc = sbuf(S->ckeys2, 4 * n_ctx, err, errlen)) ||
            (rc = sbuf(S->cvals, 4 * n_ctx, err, errlen)) || (rc = sbuf(S->cvals2, 4 * n_ctx, err, errlen)) ||
            (rc = sbuf(S->ctx2, sizeof(grom_sv_ctx) * n_ctx, err, errlen)) ||
            (rc = sbuf(S->n_hits, 16, err, errlen)))
            return rc;
        const grom_sv_ctx *ctx = (const grom_sv_ctx *)S->ctx.p;
        uint32_t *ck = (uint32_t *)S->ckeys.p, *cv = (uint32_t *)S->cvals.p;
        uint32_t *ck2 = (uint32_t *)S->ckeys2.p, *cv2 = (uint32_t *)S->cvals2.p;
        grom_sv_ctx *ctx2 = (grom_sv_ctx *)S->ctx2.p;
        hipLaunchKernelGGL(k_ctx_keys, dim3((n_ctx + 255) / 256), dim3(256), 0, st, ctx, n_ctx, ck, cv);
        SCHK(hipGetLastError());
        int bit_hi = 1;
        while (bit_hi < 32 && ((int64_t)1 << bit_hi) <= S->len + 1) bit_hi++;
        size_t tb = 0;
        SCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, ck, ck2, cv, cv2, (int)n_ctx, 0, bit_hi, st));
        if ((rc = sbuf(S->tmp, tb, err, errlen))) return rc;
        SCHK(hipcub::DeviceRadixSort::SortPairs(S->tmp.p, tb, ck, ck2, cv, cv2, (int)n_ctx, 0, bit_hi, st));
        hipLaunchKernelGGL(k_ctx_gather, dim3((n_ctx + 255) / 256), dim3(256), 0, st, ctx, (const uint32_t *)cv2,
                           n_ctx, ctx2);
        SCHK(hipGetLastError());
        uint32_t hit_cap = std::max<uint32_t>(4096, n_ctx / 16);
        for (int attempt = 0; attempt < 2; attempt++) {
            if ((rc = sbuf(S->hits, sizeof(SvHit) * hit_cap, err, errlen))) return rc;
            SCHK(hipMemsetAsync(S->n_hits.p, 0, 4, st));
            EvalIn I{};
            I.ctx = ctx2;
            I.n_ctx = n_ctx;
            I.rec = (const grom_sv_rec *)S->rec.p;
            I.irec = (const grom_indel_rec *)S->irec_c.p;
            I.n_rec = S->n_rec;
            I.sums = (const int32_t *)S->sums.p;
            I.len = S->len;
            I.mq = d_mq;
            I.hez = d_hez;
            I.eval_lo = eval_lo;
            I.eval_hi = eval_hi;
            I.lseq_tail = ch.lseq_tail;
            I.Mx = P.insert_max_size;
            I.overlap = P.overlap_mult;
            I.min_disc = P.min_disc;
            I.mean = P.insert_mean;
            I.glseq = P.lseq;
            I.pval1 = P.pval_threshold1;
            I.pval_ins1 = P.pval_insertion1;
            I.max_ev_ratio = P.max_evidence_ratio;
            I.in = in;
            I.hits = (SvHit *)S->hits.p;
            I.n_hits = (uint32_t *)S->n_hits.p;
            I.hit_cap = hit_cap;
            hipLaunchKernelGGL(k_sv_eval, dim3((n_ctx + 63) / 64), dim3(64), 0, st, I);
            SCHK(hipGetLastError());
            uint32_t nh = 0;
            SCHK(hipMemcpyAsync(&nh, S->n_hits.p, 4, hipMemcpyDeviceToHost, st));
            SCHK(hipStreamSynchronize(st));
            if (nh > hit_cap) {
                hit_cap = nh + nh / 4 + 64;
                continue;
            }
            if (nh) {
                // base order on the device (the lanes append in any order):
                // sort (pos, slot) and gather, then one copy to pinned memory
                if ((rc = sbuf(S->hits2, sizeof(SvHit) * nh, err, errlen))) return rc;
                uint32_t *hk = (uint32_t *)S->ckeys.p, *hv = (uint32_t *)S->cvals.p;
                uint32_t *hk2 = (uint32_t *)S->ckeys2.p, *hv2 = (uint32_t *)S->cvals2.p;  // n_ctx >= nh entries
                hipLaunchKernelGGL(k_hit_keys, dim3((nh + 255) / 256), dim3(256), 0, st, (const SvHit *)S->hits.p, nh, hk,
                                   hv);
                size_t tb = 0;
                SCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, hk, hk2, hv, hv2, (int)nh, 0, bit_hi, st));
                if ((rc = sbuf(S->tmp, tb, err, errlen))) return rc;
                SCHK(hipcub::DeviceRadixSort::SortPairs(S->tmp.p, tb, hk, hk2, hv, hv2, (int)nh, 0, bit_hi, st));
                hipLaunchKernelGGL(k_hit_gather, dim3((nh + 255) / 256), dim3(256), 0, st, (const SvHit *)S->hits.p, hv2,
                                   nh, (SvHit *)S->hits2.p);
                SCHK(hipGetLastError());
                if (nh > S->h_hits_cap) {
                    if (S->h_hits) (void)hipHostFree(S->h_hits);
                    S->h_hits = nullptr;
                    S->h_hits_cap = 0;
                    const size_t want = nh + nh / 4 + 1024;
                    SCHK(hipHostMalloc((void **)&S->h_hits, sizeof(SvHit) * want, 0));
                    S->h_hits_cap = want;
                }
                SCHK(hipMemcpyAsync(S->h_hits, S->hits2.p, sizeof(SvHit) * nh, hipMemcpyDeviceToHost, st));
                SCHK(hipStreamSynchronize(st));
            }
            *hits_out = S->h_hits;
            *n_hits_out = nh;
            break;
        }
    }
    SCHK(hipEventRecord(S->e1, st));
    SCHK(hipEventSynchronize(S->e1));
    float ms = 0;
    SCHK(hipEventElapsedTime(&ms, S->e0, S->e1));
    if (ms_device) *ms_device = ms;
    return GROM_OK;
}
