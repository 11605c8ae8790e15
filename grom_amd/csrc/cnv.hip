// cnv.hip -- MI355X (gfx950) implementation of GROM's read-depth CNV path,
// SURVEY.md §8 rows A14-A16, run per chromosome after the pileup
// (scan.hip) has filled the three whole-chromosome depth arrays.
//
//   reference step                              here
//   GC/ACGT triangular windows   GROM.c:1770    k_cnv_gc: two LDS prefix scans per
//                                               4096-base tile give the weighted
//                                               window sum in closed form
//   dinucleotide repeat runs     GROM.c:1727    k_cnv_gc (pair type) + k_cnv_repeats
//   mapq/depth division, 10 kb   GROM.c:16637,  k_cnv_blocks (one workgroup per
//   blocks, chromosome depth     16651, 16811   10 kb block, exact integer sums)
//   GC-bin sampling, sort/merge  GROM.c:18373   host (≈G/250 samples), gathered
//   bins, bin statistics         -18641         by k_cnv_gather
//   low-ACGT/thin-bin flags      GROM.c:18654   k_cnv_tile_last + k_cnv_carry +
//                                               k_cnv_flags: the "last high/low
//                                               MAPQ class" state is a last-value
//                                               scan (tile summary, carry, apply)
//   per-base z score             GROM.c:18740   k_cnv_z (same scan for its own
//                                               state, then bisect + pval2sd)
//   window means per length      GROM.c:18967   k_cnv_windows (one lane per
//                                               10 kb window, sequential double
//                                               sums in reference order) +
//                                               k_cnv_window_sq (one lane per
//                                               window length)
//   DEL/DUP window search        GROM.c:19359   k_cnv_walk: the data-dependent
//                                               walk, chunked and run
//                                               speculatively (one lane per
//                                               chunk), then reconciled
//   copy number, p value, rows   GROM.c:20024,  host, on gathered call ranges
//                                17139
//
// Exactness: every double the VCF depends on is produced with the reference's
// operation order (sequential sums stay sequential, one lane each; this file
// is compiled with -ffp-contract=off so no multiply-add is fused).  The
// chromosome depth variance of GROM.c:16664-16677 only feeds the repeat-bias
// comparison (GROM.c:16765): it is bounded from an exact depth histogram, and
// redone in base order on the host when the bound cannot decide.

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <thread>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "cnv.h"
#include "ddecode.h"
#include "copystats.h"  // (GROM_COPY_STATS, last: it wraps the runtime copy calls)

namespace {

// ---- fixed parameters of the reference (not on its command line) ----
constexpr int NBINS = 101;                 // g_num_gc_bins, GROM.c:947
constexpr int REP_SEGS = 10;               // g_repeat_segments, GROM.c:732
// g_sample_lists_len, GROM.c:725; GROM_SAMPLE_LISTS_LEN lowers it (test hook:
// the reservoir draws of GROM.c:18292/18393 then fire on small inputs, and
// the oracle reads the same variable)
static long sample_len() {
    const char *e = getenv("GROM_SAMPLE_LISTS_LEN");
    const long x = e ? atol(e) : 0;
    return (x > 0 && x < 100000) ? x : 100000L;
}
constexpr long REDUCTION = 1;              // g_genome_reduction_factor, GROM.c:726
constexpr long BLOCK_FACTOR = 4;           // g_block_factor, GROM.c:738
constexpr long BLOCK_UNIT = 10000;         // g_block_unit_size, GROM.c:740
constexpr int MIN_ACGT = 99;               // g_insert_min_acgt, GROM.c:926
constexpr long NO_COMBINE = 100;           // g_rd_no_combine_min_windows, GROM.c:929
constexpr long RD_MIN_WINDOWS = 20;        // g_rd_min_windows, GROM.c:928
constexpr int RD_MAX_MAPQ = 60;            // g_rd_max_mapq, GROM.c:718
constexpr long MIN_RD_LOW_STDEV = 3;       // g_one_base_read_depth_min_rd_low_stdev, GROM.c:935
constexpr double MAX_LOW_ACGT = 2;         // g_max_rd_low_acgt_or_windows, GROM.c:937
constexpr double PLOIDY_NUM = 0.6;         // g_ploidy_threshold_numerator, GROM.c:939
constexpr double STDEV_STEP = 0.01;        // g_stdev_step, GROM.c:940
constexpr long MAX_DIST_LAST_GOOD = 10500; // default -X + 500, set before getopt (GROM.c:21898)
constexpr int MAX_BLOCK_LIST = 10000;      // max_block_list_len, GROM.c:633

constexpr int GC_TP = 16384;               // positions per k_cnv_gc tile
constexpr int GC_MMAX_S = 1536;            // k_cnv_gc<GC_MMAX_S>: 32-bit window arithmetic
constexpr int GC_MMAX = 16384;             // k_cnv_gc<GC_MMAX>: 64-bit, a 25 KB LDS halo; above, k_cnv_gc_global
template <int MMAX>
constexpr int gc_nw() { return (GC_TP + 2 * MMAX + 1 + 63) / 64; }  // 64-bit class words per tile (with halo)
constexpr int SEG_W = 4096;                // positions per wave in the state scans
constexpr int ZT_MAX = 1024;               // depths with a precomputed z rank index
constexpr int HIST_MAX = 4096;             // exact depth histogram for the chromosome variance
constexpr int64_t WALK_CHUNK = 16384;      // positions per speculative walk lane

// flag byte per position
constexpr uint8_t F_LOW = 1;    // ddd_rd_low_acgt_or_windows_list != 0
constexpr uint8_t F_GUARD = 2;  // z-scored / windowed base (GROM.c:18765 condition)

struct Tables {  // device copy of the per-chromosome bin statistics
    int32_t off[2][NBINS], cnt[2][NBINS];
    int64_t wins[2][NBINS];
    double ave[2][NBINS], sdv[2][NBINS], thr[2][2][NBINS];  // thr[0]=del, thr[1]=dup
    double p2s_p[1001], p2s_sd[1001];
    int32_t n_p2s;
};

struct Args {
    int64_t len, lo, hi;  // [lo, hi) = [insert_mean-1, len - window_size)
    int32_t min_mapq, ranks_stdev;
    double mapq_factor, dup_factor;
};

__device__ __forceinline__ int gc_class(char ch) {  // bit0 GC, bit1 ACGT (GROM.c:1591-1592)
    switch (ch) {
    case 'C': case 'G': case 'c': case 'g': return 3;
    case 'A': case 'T': case 'a': case 't': return 2;
    default: return 0;
    }
}

// dinucleotide class of (x, y), GROM.c:1656-1657, 1729-1737: unordered pair of
// two upper-case or two lower-case ACGT bases, 10 for anything else
__device__ __forceinline__ int pair_type(char x, char y) {
    auto code = [](char c, int lower) -> int {
        char u = lower ? (char)(c - 32) : c;
        return u == 'A' ? 0 : u == 'C' ? 1 : u == 'G' ? 2 : u == 'T' ? 3 : -1;
    };
    int lx = (x >= 'a' && x <= 'z'), ly = (y >= 'a' && y <= 'z');
    if (lx != ly) return 10;
    int a = code(x, lx), b = code(y, ly);
    if (a < 0 || b < 0) return 10;
    if (a > b) { int t = a; a = b; b = t; }
    const int base[4] = {0, 4, 7, 9};
    return base[a] + (b - a);
}

// sum of the bit indices set in w: bit b of each index, weighted 2^b
__device__ __forceinline__ int bit_index_sum(uint64_t w) {
    return __popcll(w & 0xAAAAAAAAAAAAAAAAull) + 2 * __popcll(w & 0xCCCCCCCCCCCCCCCCull) +
           4 * __popcll(w & 0xF0F0F0F0F0F0F0F0ull) + 8 * __popcll(w & 0xFF00FF00FF00FF00ull) +
           16 * __popcll(w & 0xFFFF0000FFFF0000ull) + 32 * __popcll(w & 0xFFFFFFFF00000000ull);
}

// Weighted GC / ACGT percent and dinucleotide class per base (GROM.c:1684-1861).
// The reference's rolling sums equal, for p in [m-1, len-2m+1),
//   T(p) = sum_{|q-p|<m} g(q) (m - |q-p|) = Q[p+m+1] - 2 Q[p+1] + Q[p-m+1]
// with P[x] = #{q < x : g(q)} and Q[x] = sum_{y<x} P[y] = (x-1) P[x] - R[x],
// R[x] = sum_{q<x} q g(q) (exact integers; tile-local coordinates, so linear
// offsets cancel in the second difference). The tile's classes are two bit
// planes built by wave ballots; P and R at any x are a per-word prefix plus
// popcounts of the masked word, so the kernel reads each reference byte once
// (plus the 2m halo) and writes 3 bytes per base.
// MMAX: the largest insert mean m the instance takes; above GC_MMAX_S the
// window sums (up to m^2 * 100) need 64-bit arithmetic, as the reference's
// longs give them (GROM.c:1602, 1860)
template <int MMAX>
__global__ __launch_bounds__(256) void k_cnv_gc(const char *__restrict__ ref, Args A, int m, int64_t total,
                                                uint8_t *__restrict__ gcw, uint8_t *__restrict__ acw,
                                                uint8_t *__restrict__ rtype) {
    constexpr int GC_NW = gc_nw<MMAX>();
    using acc_t = typename std::conditional<(MMAX > GC_MMAX_S), int64_t, int>::type;
    using uacc_t = typename std::conditional<(MMAX > GC_MMAX_S), uint64_t, uint32_t>::type;
    __shared__ uint64_t bits[2][GC_NW];  // plane 0: GC, plane 1: ACGT
    __shared__ acc_t pw[2][GC_NW];       // exclusive prefix of the set-bit counts
    __shared__ acc_t rw[2][GC_NW];       // exclusive prefix of the set-bit local indices
    const int64_t t0 = (int64_t)blockIdx.x * GC_TP;
    const int64_t base = t0 - m;
    const int L = GC_TP + 2 * m + 1;
    const int nw = (L + 63) >> 6;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int wi = wv; wi < nw; wi += 4) {
        const int k = wi * 64 + lane;
        const int64_t q = base + k;
        const int c = (k < L && q >= 0 && q < A.len) ? gc_class(ref[q]) : 0;
        const uint64_t g = __ballot(c & 1), a = __ballot(c & 2);
        if (lane == 0) {
            bits[0][wi] = g;
            bits[1][wi] = a;
        }
    }
    __syncthreads();
    {  // wave w scans array w: counts / index sums of plane w & 1
        const int pl = wv & 1, isr = wv >> 1;
        acc_t carry = 0;
        for (int c0 = 0; c0 < nw; c0 += 64) {
            const int wi = c0 + lane;
            acc_t v = 0;
            if (wi < nw) {
                const uint64_t w = bits[pl][wi];
                v = isr ? (acc_t)wi * 64 * (acc_t)__popcll(w) + (acc_t)bit_index_sum(w) : (acc_t)__popcll(w);
            }
            acc_t x = v;
            for (int d = 1; d < 64; d <<= 1) {
                const acc_t y = __shfl_up(x, d);
                if (lane >= d) x += y;
            }
            if (wi < nw) (isr ? rw : pw)[pl][wi] = carry + x - v;
            carry += __shfl(x, 63);
        }
    }
    __syncthreads();
    const uacc_t tot = (uacc_t)total;  // m*m
    // four consecutive positions per thread, stored as one 32-bit word per
    // output (t0 is a multiple of GC_TP, so the words are aligned)
    for (int j0 = 4 * threadIdx.x; j0 < GC_TP; j0 += 4 * 256) {
        const int64_t p0 = t0 + j0;
        if (p0 >= A.len) break;
        uint32_t o[3] = {0, 0, 0};  // gcw, acw, rtype
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int j = j0 + u;
            const int64_t p = p0 + u;
            uint32_t w2[2] = {0, 0}, rt = 10;
            if (p >= A.lo && p < A.hi) {
                const int xs[3] = {j + 2 * m + 1, j + m + 1, j + 1};
#pragma unroll
                for (int pl = 0; pl < 2; pl++) {
                    acc_t Qv[3];
#pragma unroll
                    for (int t = 0; t < 3; t++) {
                        const int x = xs[t], wi = x >> 6, b = x & 63;
                        const uint64_t wd = bits[pl][wi] & ((1ull << b) - 1ull);
                        const acc_t c = (acc_t)__popcll(wd);
                        const acc_t Pv = pw[pl][wi] + c;
                        const acc_t Rv = rw[pl][wi] + (acc_t)wi * 64 * c + (acc_t)bit_index_sum(wd);
                        Qv[t] = (acc_t)(x - 1) * Pv - Rv;
                    }
                    const uacc_t Tv = (uacc_t)(Qv[0] - 2 * Qv[1] + Qv[2]);
                    w2[pl] = (uint32_t)((100u * Tv / tot) & 255u);
                }
                rt = (uint32_t)pair_type(ref[p], ref[p + 1]);
            }
            o[0] |= w2[0] << (8 * u);
            o[1] |= w2[1] << (8 * u);
            o[2] |= rt << (8 * u);
        }
        if (p0 + 4 <= A.len) {
            *reinterpret_cast<uint32_t *>(gcw + p0) = o[0];
            *reinterpret_cast<uint32_t *>(acw + p0) = o[1];
            *reinterpret_cast<uint32_t *>(rtype + p0) = o[2];
        } else {  // the chromosome's last partial word
            for (int u = 0; p0 + u < A.len; u++) {
                gcw[p0 + u] = (uint8_t)(o[0] >> (8 * u));
                acw[p0 + u] = (uint8_t)(o[1] >> (8 * u));
                rtype[p0 + u] = (uint8_t)(o[2] >> (8 * u));
            }
        }
    }
}

struct RepeatRec {
    int64_t start, end, rd;  // [start, end), depth sum over it
    int32_t type, pad;
};

// Repeat runs (GROM.c:1727-1768): a maximal run of one class, closed before
// the last scanned base, of at least g_min_repeat bases.
__global__ void k_cnv_repeats(const uint8_t *__restrict__ rtype, const int32_t *__restrict__ rd,
                              const int32_t *__restrict__ low, Args A, int64_t min_repeat, RepeatRec *out,
                              uint32_t *n_out, uint32_t cap) {
    int64_t p = A.lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= A.hi) return;
    int t = rtype[p];
    if (t == 10 || (p > A.lo && rtype[p - 1] == t)) return;
    int64_t e = p;
    while (e + 1 < A.hi && rtype[e + 1] == t) e++;
    if (e + 1 >= A.hi) return;  // still open when the scan loop ends: never written
    if (e - p < min_repeat - 1) return;
    int64_t s = 0;
    for (int64_t q = p; q <= e; q++) s += rd[q] + low[q];
    uint32_t k = atomicAdd(n_out, 1u);
    if (k < cap) out[k] = RepeatRec{p, e + 1, s, t, 0};
}

struct BlockSums {
    unsigned long long blk_total[1];  // placeholder for alignment
};

// One workgroup per 10 kb block (plus one for the tail): divides the mapq sum
// by the depth in place (GROM.c:16637-16643), the block depth sums of
// GROM.c:16811-16829 and the chromosome depth sums of GROM.c:16651-16662.
__global__ __launch_bounds__(256) void k_cnv_blocks(const char *__restrict__ ref, Args A,
                                                    int32_t *__restrict__ mq, const int32_t *__restrict__ rd,
                                                    const int32_t *__restrict__ low,
                                                    const uint8_t *__restrict__ acw, int64_t *blk_total,
                                                    unsigned long long *acc, unsigned int *hist) {
    __shared__ unsigned int h[HIST_MAX + 1];
    __shared__ unsigned long long s_tot, s_acgt_tot, s_acgt_n, s_chr_tot, s_chr_n;
    for (int i = threadIdx.x; i <= HIST_MAX; i += 256) h[i] = 0;
    if (threadIdx.x == 0) s_tot = s_acgt_tot = s_acgt_n = s_chr_tot = s_chr_n = 0;
    __syncthreads();
    const int64_t b0 = (int64_t)blockIdx.x * BLOCK_UNIT;
    const int64_t b1 = min<int64_t>(b0 + BLOCK_UNIT, A.len);
    unsigned long long tot = 0, at = 0, an = 0, ct = 0, cn = 0;
    for (int64_t p = b0 + threadIdx.x; p < b1; p += 256) {
        int r = rd[p] + low[p];
        if (r > 0) mq[p] = mq[p] / r;
        tot += r;
        if (gc_class(ref[p])) { at += r; an += 1; }
        if (p >= A.lo && p < A.hi && acw[p] >= MIN_ACGT) {
            ct += r;
            cn += 1;
            atomicAdd(&h[min(r, HIST_MAX)], 1u);
        }
    }
    atomicAdd(&s_tot, tot);
    atomicAdd(&s_acgt_tot, at);
    atomicAdd(&s_acgt_n, an);
    atomicAdd(&s_chr_tot, ct);
    atomicAdd(&s_chr_n, cn);
    __syncthreads();
    if (threadIdx.x == 0) {
        blk_total[blockIdx.x] = (int64_t)s_tot;
        if (s_acgt_tot) atomicAdd(&acc[0], s_acgt_tot);
        if (s_acgt_n) atomicAdd(&acc[1], s_acgt_n);
        if (s_chr_tot) atomicAdd(&acc[2], s_chr_tot);
        if (s_chr_n) atomicAdd(&acc[3], s_chr_n);
    }
    for (int i = threadIdx.x; i <= HIST_MAX; i += 256)
        if (h[i]) atomicAdd(&hist[i], h[i]);
}

struct GatherRange {
    int64_t start, count, stride, out;
};

// per-position values for host-side steps (sampling, copy number)
__global__ void k_cnv_gather(const GatherRange *__restrict__ rg, int n_rg, const uint8_t *__restrict__ gcw,
                             const uint8_t *__restrict__ acw, const int32_t *__restrict__ mq,
                             const int32_t *__restrict__ rd, const int32_t *__restrict__ low,
                             const uint8_t *__restrict__ flag, int64_t total, uint8_t *o_gc, uint8_t *o_ac,
                             int32_t *o_mq, int32_t *o_rd, int32_t *o_low, int32_t *o_rt, uint8_t *o_flag) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        int lo = 0, hi = n_rg - 1;
        while (lo < hi) {  // range holding output slot i
            int mid = (lo + hi + 1) / 2;
            if (rg[mid].out <= i) lo = mid; else hi = mid - 1;
        }
        const GatherRange r = rg[lo];
        int64_t p = r.start + (i - r.out) * r.stride;
        o_gc[i] = gcw[p];
        o_ac[i] = acw[p];
        o_mq[i] = mq[p];
        o_rd[i] = rd[p];
        o_low[i] = low[p];
        o_rt[i] = rd[p] + low[p];
        o_flag[i] = flag ? flag[p] : 0;
    }
}

// The copy number's per-base ratios (GROM.c:20100-20160) for output slot i
// of the kept calls' ranges: rt / ave[mapq class][gc], or +inf for a base
// the reference leaves out (a low base or an empty bin).  8 bytes per base
// to the host instead of the six gathered arrays' 15 (and their host split).
__global__ void k_cnv_cn_ratio(const GatherRange *__restrict__ rg, int n_rg, const uint8_t *__restrict__ gcw,
                               const int32_t *__restrict__ mq, const int32_t *__restrict__ rd,
                               const int32_t *__restrict__ low, const uint8_t *__restrict__ flag,
                               const Tables *__restrict__ T, int32_t min_mapq, int64_t total, double *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        int lo = 0, hi = n_rg - 1;
        while (lo < hi) {  // range holding output slot i
            int mid = (lo + hi + 1) / 2;
            if (rg[mid].out <= i) lo = mid; else hi = mid - 1;
        }
        const GatherRange r = rg[lo];
        const int64_t p = r.start + (i - r.out) * r.stride;
        double v = HUGE_VAL;
        if (!(flag[p] & F_LOW)) {
            const int k = mq[p] >= min_mapq ? 0 : 1;
            const double a = T->ave[k][gcw[p]];
            if (a > 0) v = (double)(rd[p] + low[p]) / a;
        }
        out[i] = v;
    }
}

// ---- the "last MAPQ class" state scans ----
// e1(p): GROM.c:18662-18677 -- ACGT-rich base with depth: its class
__device__ __forceinline__ int ev1(const Args &A, int64_t p, const uint8_t *acw, const int32_t *mq,
                                   const int32_t *rd, const int32_t *low) {
    if (p < A.lo || p >= A.hi || acw[p] < MIN_ACGT) return -1;
    int r = rd[p] + low[p];
    if (r == 0) return -1;
    return mq[p] >= A.min_mapq ? 0 : 1;
}
// e2(p): GROM.c:18765-18784 -- guarded base that sets the class
__device__ __forceinline__ int ev2(const Args &A, int64_t p, const uint8_t *flag, const int32_t *mq,
                                   const int32_t *rd, const int32_t *low) {
    if (!(flag[p] & F_GUARD)) return -1;
    if (mq[p] >= A.min_mapq) return 0;
    if (rd[p] + low[p] == 0) return -1;
    return 1;
}

// "last defined value at or before me" across the 64 lanes of a wave, with
// `c` for lanes that have none before them
__device__ __forceinline__ int wave_last_incl(int e, int c) {
    const int lane = threadIdx.x & 63;
    const unsigned long long m = __ballot(e != -1);
    const unsigned long long mine = m & (lane == 63 ? ~0ull : ((2ull << lane) - 1));
    const int src = mine ? 63 - __clzll(mine) : 0;
    const int v = __shfl(e, src);
    return mine ? v : c;
}

// Each wave owns SEG_W consecutive positions, read 64 at a time (coalesced).
template <int WHICH>
__global__ __launch_bounds__(256) void k_cnv_seg_last(Args A, const uint8_t *acw, const uint8_t *flag,
                                                      const int32_t *mq, const int32_t *rd, const int32_t *low,
                                                      int8_t *seg_last) {
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    const int64_t p0 = wave * SEG_W;
    int c = -1;
    for (int r = 0; r < SEG_W / 64; r++) {
        const int64_t p = p0 + r * 64 + lane;
        int e = -1;
        if (p < A.len) e = WHICH == 1 ? ev1(A, p, acw, mq, rd, low) : ev2(A, p, flag, mq, rd, low);
        c = __builtin_amdgcn_readlane(wave_last_incl(e, c), 63);
    }
    if (lane == 0 && p0 < A.len) seg_last[wave] = (int8_t)c;
}

// carry[t] = last defined tile value before tile t (0 before the first)
__global__ __launch_bounds__(1024) void k_cnv_carry(const int8_t *tile_last, int64_t n, int8_t *carry) {
    __shared__ int seg[1024];
    const int tid = threadIdx.x;
    const int64_t per = (n + 1023) / 1024, lo = min<int64_t>(n, tid * per), hi = min<int64_t>(n, lo + per);
    int l = -1;
    for (int64_t i = lo; i < hi; i++) if (tile_last[i] != -1) l = tile_last[i];
    seg[tid] = l;
    __syncthreads();
    if (tid == 0) {
        int c = 0;  // ddd_last_low_mq = 0 at the start (GROM.c:18650, 18740)
        for (int t = 0; t < 1024; t++) { int v = seg[t]; seg[t] = c; if (v != -1) c = v; }
    }
    __syncthreads();
    int c = seg[tid];
    for (int64_t i = lo; i < hi; i++) { carry[i] = (int8_t)c; if (tile_last[i] != -1) c = tile_last[i]; }
}


// flags (GROM.c:18654-18712) and the guard bit of GROM.c:18765
__global__ __launch_bounds__(256) void k_cnv_flags(Args A, const uint8_t *__restrict__ acw,
                                                   const uint8_t *__restrict__ gcw, const int32_t *__restrict__ mq,
                                                   const int32_t *__restrict__ rd, const int32_t *__restrict__ low,
                                                   const int8_t *__restrict__ carry, const Tables *__restrict__ T,
                                                   uint8_t *__restrict__ flag) {
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    const int64_t p0 = wave * SEG_W;
    if (p0 >= A.len) return;
    int c = carry[wave];
    for (int r = 0; r < SEG_W / 64; r++) {
        const int64_t p = p0 + r * 64 + lane;
        const bool in = p < A.len;
        const int e = in ? ev1(A, p, acw, mq, rd, low) : -1;
        const int mqi = wave_last_incl(e, c);  // own class, or the last one before (depth 0)
        c = __builtin_amdgcn_readlane(mqi, 63);
        if (!in) continue;
        uint8_t f = F_LOW;
        if (p >= A.lo && p < A.hi && acw[p] >= MIN_ACGT) f = (T->wins[mqi][gcw[p]] < NO_COMBINE) ? F_LOW : 0;
        if (f == 0) {
            const int g = gcw[p];
            if ((mq[p] >= A.min_mapq && T->wins[0][g] > 1) || (mq[p] < A.min_mapq && T->wins[1][g] > 1)) f |= F_GUARD;
        }
        flag[p] = f;
    }
}

// GROM.c:21630-21860, exact
__device__ long d_bisect_left(const int *l, int rd, long s, long e) {
    int found = 0;
    long i = s + (e - s) / 2, lo = s, hi = e;
    while (found == 0) {
        if (i <= s) { i = (rd <= l[s]) ? s : s + 1; found = 1; }
        else if (i >= e - 1) { i = (rd <= l[e - 1]) ? e - 1 : e; found = 1; }
        else if (rd <= l[i]) { hi = i; i = lo + (i - lo) / 2; if (hi == i) { found = 1; i += 1; } }
        else { lo = i; i = i + (hi - i) / 2; if (lo == i) { found = 1; i += 1; } }
    }
    return i;
}
__device__ long d_bisect_right(const int *l, int rd, long s, long e) {
    int found = 0;
    long i = s + (e - s) / 2, lo = s, hi = e;
    while (found == 0) {
        if (i <= s) { i = (rd < l[s]) ? s : s + 1; found = 1; }
        else if (i >= e - 1) { i = (rd < l[e - 1]) ? e - 1 : e; found = 1; }
        else if (rd < l[i]) { hi = i; i = lo + (i - lo) / 2; if (hi == i) { found = 1; i += 1; } }
        else { lo = i; i = i + (hi - i) / 2; if (lo == i) { found = 1; i += 1; } }
    }
    return i;
}
__device__ long d_bisect_right_double(const double *l, double p, long s, long e) {
    int found = 0;
    long i = s + (e - s) / 2, lo = s, hi = e;
    while (found == 0) {
        if (i <= s) { i = (p < l[s]) ? s : s + 1; found = 1; }
        else if (i >= e - 1) { i = (p < l[e - 1]) ? e - 1 : e; found = 1; }
        else if (p < l[i]) { hi = i; i = lo + (i - lo) / 2; if (hi == i) { found = 1; i += 1; } }
        else { lo = i; i = i + (hi - i) / 2; if (lo == i) { found = 1; i += 1; } }
    }
    return i;
}

// z-score rank index for every (class, bin, depth < ZT_MAX) (ranks mode):
// the two bisects into the sorted bin sample and the pval2sd bisect of
// GROM.c:18800-18940 depend on nothing else.  Entry: +/-(pval2sd index + 1)
// (sign: the depth-above-mean branch), 0: no z (empty bin).
__device__ int z_rank_index(const Tables *T, const int32_t *samples, int mqi, int bin, int r, double dup_factor) {
    const long ge = T->cnt[mqi][bin];
    if (ge <= 0) return 0;
    const int *list = samples + T->off[mqi][bin];
    const double ave = T->ave[mqi][bin];
    long i1, i2;
    double d1, d2, prob;
    int sign = 1;
    if (r < ave) {
        i1 = d_bisect_right(list, r, 0, ge);
        i2 = d_bisect_left(list, r, 0, ge);
    } else {
        sign = -1;
        if (r > dup_factor * ave) {
            i1 = d_bisect_left(list, (int)(dup_factor * ave), 0, ge);  // Q11 truncation
            i2 = d_bisect_right(list, r, 0, ge);
        } else {
            i1 = d_bisect_left(list, r, 0, ge);
            i2 = d_bisect_right(list, r, 0, ge);
        }
        i1 = ge - i1;
        i2 = ge - i2;
    }
    d1 = (i1 <= 0) ? 0.5 : (double)i1;
    d2 = (i2 <= 0) ? 0.5 : (double)i2;
    prob = (d1 + d2) / (2 * ge);
    i1 = d_bisect_right_double(T->p2s_p, prob, 0, T->n_p2s);
    if (i1 < 0) i1 = 0;
    else if (i1 >= T->n_p2s) i1 = T->n_p2s - 1;
    return sign * (int)(i1 + 1);
}

__global__ void k_cnv_ztab(const Tables *__restrict__ T, const int32_t *__restrict__ samples, double dup_factor,
                           int16_t *__restrict__ ztab) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 2 * NBINS * ZT_MAX) return;
    const int r = i % ZT_MAX, bin = (i / ZT_MAX) % NBINS, mqi = i / (ZT_MAX * NBINS);
    ztab[i] = (int16_t)z_rank_index(T, samples, mqi, bin, r, dup_factor);
}

// per-base z score, GROM.c:18740-18963 (g_normal == 0)
__global__ __launch_bounds__(256) void k_cnv_z(Args A, const uint8_t *__restrict__ gcw,
                                               const int32_t *__restrict__ mq, const int32_t *__restrict__ rd,
                                               const int32_t *__restrict__ low, const uint8_t *__restrict__ flag,
                                               const int8_t *__restrict__ carry, const Tables *__restrict__ T,
                                               const int32_t *__restrict__ samples, const int16_t *__restrict__ ztab,
                                               double *__restrict__ sd) {
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    const int64_t p0 = wave * SEG_W;
    if (p0 >= A.len) return;
    int c = carry[wave];
    for (int r0 = 0; r0 < SEG_W / 64; r0++) {
        const int64_t p = p0 + r0 * 64 + lane;
        const bool in = p < A.len;
        const int e = in ? ev2(A, p, flag, mq, rd, low) : -1;
        const int mqi = wave_last_incl(e, c);
        c = __builtin_amdgcn_readlane(mqi, 63);
        if (!in) continue;
        double z = 0.0;
        if (flag[p] & F_GUARD) {
            const int r = rd[p] + low[p], q = mq[p];
            const int bin = gcw[p];
            const double f = q >= A.min_mapq
                                 ? A.mapq_factor + (1.0 - A.mapq_factor) * (q - A.min_mapq) / (double)(RD_MAX_MAPQ - A.min_mapq)
                                 : A.mapq_factor;
            if (A.ranks_stdev == 0) {
                if (T->cnt[mqi][bin] > 0) {
                    const double ave = T->ave[mqi][bin], sdv = T->sdv[mqi][bin];
                    if (r < ave || !(r > A.dup_factor * ave)) z = f * (ave - rd[p] - low[p]) / sdv;
                    else z = f * (A.dup_factor - 1) * (-ave) / sdv;
                }
            } else {
                const int zi = r < ZT_MAX ? ztab[(mqi * NBINS + bin) * ZT_MAX + r]
                                          : z_rank_index(T, samples, mqi, bin, r, A.dup_factor);
                if (zi > 0) z = f * T->p2s_sd[zi - 1];
                else if (zi < 0) z = -f * T->p2s_sd[-zi - 1];
            }
        }
        sd[p] = z;
    }
}

// Window means for every length of one sampled window (GROM.c:18967-19018):
// one lane per window, its sum accumulated in the reference's order.  A
// window is a run of pieces of consecutive bases (it straddles the sampling
// passes of a block: as many as -A when a block is short for -X).  out row:
// [min_len..len] means, NaN = none.
struct WinPiece {
    int64_t start, count;
};
struct WinDesc {
    int64_t p0, n0, p1, n1, p2, n2;  // the first three pieces inline (the common case)
    int64_t piece0, n_pieces, ntot;  // all pieces: [piece0, piece0 + n_pieces) of the piece list, ntot bases
    int64_t row;
};
// Window means for every length (GROM.c:18967-19018).  Each window's running
// sums are one sequential chain in the reference's order, so one lane owns a
// window; what made the one-lane form slow was everything else per base (two
// f64 divisions and a store) on a grid of only ~n_win/64 waves.  Here a
// 256-thread block owns 64 windows: wave 0 runs the 64 chains over chunks of
// WCH bases and leaves (tot, cnt, ftot) per base in LDS; waves 1-3 turn the
// previous chunk into means (the divisions spread over three waves) and store
// them length-major, so each store of a wave covers 64 adjacent windows.
constexpr int WCH = 32;
__global__ __launch_bounds__(256) void k_cnv_windows(const WinDesc *__restrict__ wd, const WinPiece *__restrict__ pcs,
                                                     int64_t n_win, const uint8_t *__restrict__ flag,
                                                     const double *__restrict__ sd, int64_t L, int64_t min_len,
                                                     double *__restrict__ out) {
    __shared__ double s_tot[2][WCH][64];
    __shared__ int32_t s_cnt[2][WCH][64], s_ft[2][WCH][64];
    __shared__ int64_t s_nmax;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t w = (int64_t)blockIdx.x * 64 + lane;
    WinDesc d{};
    int64_t ntot = 0;
    if (w < n_win) {
        d = wd[w];
        ntot = d.ntot;
    }
    // the lane's cursor in its window's pieces (the bases are taken in order)
    int64_t pi = d.piece0, po = 0;
    if (threadIdx.x == 0) s_nmax = 0;
    __syncthreads();
    if (wave == 0) {
        int64_t mx = ntot;
        for (int o = 32; o > 0; o >>= 1) mx = max(mx, (int64_t)__shfl_xor(mx, o, 64));
        if (lane == 0) s_nmax = mx;
    }
    __syncthreads();
    const int64_t nch = (s_nmax + WCH - 1) / WCH;
    double tot = 0.0;
    int32_t cnt = 0, ftot = 0;
    for (int64_t c = 0; c <= nch; c++) {
        if (wave == 0 && c < nch) {
            // the chain over bases [c*WCH, c*WCH + WCH) of this lane's window
            uint8_t f[WCH];
            double v[WCH];
#pragma unroll
            for (int j = 0; j < WCH; j++) {
                const int64_t g = c * WCH + j;
                int64_t a = -1;
                if (d.n_pieces <= 3) {
                    if (g < d.n0) a = d.p0 + g;
                    else if (g < d.n0 + d.n1) a = d.p1 + (g - d.n0);
                    else if (g < ntot) a = d.p2 + (g - d.n0 - d.n1);
                } else if (g < ntot) {  // more pieces (a block short for -X and -A): walk the list
                    while (po >= pcs[pi].count) { pi++; po = 0; }
                    a = pcs[pi].start + po;
                    po++;
                }
                f[j] = a >= 0 ? flag[a] : (uint8_t)0;
                v[j] = a >= 0 ? sd[a] : 0.0;
            }
            const int b = (int)(c & 1);
#pragma unroll
            for (int j = 0; j < WCH; j++) {
                if (f[j] & F_GUARD) { tot += v[j]; cnt += 1; }
                ftot += (f[j] & F_LOW);
                s_tot[b][j][lane] = tot;
                s_cnt[b][j][lane] = cnt;
                s_ft[b][j][lane] = ftot;
            }
        } else if (wave > 0 && c > 0) {
            const int b = (int)((c - 1) & 1);
            for (int j = wave - 1; j < WCH; j += 3) {
                const int64_t g = (c - 1) * WCH + j, wl = g + 1;
                if (g < ntot && wl >= min_len) {
                    const int32_t cn = s_cnt[b][j][lane];
                    double x = __builtin_nan("");
                    if (((int64_t)s_ft[b][j][lane] / (double)wl) < MAX_LOW_ACGT && cn > 0)
                        x = s_tot[b][j][lane] / (double)cn;
                    out[wl * n_win + d.row] = x;
                }
            }
        }
        __syncthreads();
    }
}

// per window length: the sum of squared window means in window order
// (GROM.c:19162-19170).  A block owns 64 lengths: all four waves stage a
// 64-length x 64-window tile (each row segment a coalesced 512-byte load, the
// next tile in flight while the current one is summed), and wave 0 sums its
// lane's length over the tile in window order.
__global__ __launch_bounds__(256) void k_cnv_window_sq(const double *__restrict__ rows, int64_t n_rows,
                                                       const int64_t *__restrict__ row_len, int64_t L,
                                                       int64_t min_len, double *__restrict__ tot,
                                                       int64_t *__restrict__ cnt) {
    __shared__ double tile[64][65];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t l0 = min_len + (int64_t)blockIdx.x * 64;
    const int64_t n_t = (n_rows + 63) / 64;
    double reg[16];
    auto load = [&](int64_t t) {
        const int64_t r = t * 64 + lane;
        const int64_t rl = r < n_rows ? row_len[r] : -1;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int64_t l = l0 + wave * 16 + i;
            reg[i] = (l <= L && rl >= l) ? rows[l * n_rows + r] : __builtin_nan("");
        }
    };
    double s = 0.0;
    int64_t c = 0;
    if (n_t > 0) load(0);
    for (int64_t t = 0; t < n_t; t++) {
#pragma unroll
        for (int i = 0; i < 16; i++) tile[wave * 16 + i][lane] = reg[i];
        __syncthreads();
        if (t + 1 < n_t) load(t + 1);
        if (wave == 0) {
            for (int j = 0; j < 64; j++) {
                const double v = tile[lane][j];
                if (v == v) {
                    s += v * v;
                    c += 1;
                }
            }
        }
        __syncthreads();
    }
    const int64_t l = l0 + lane;
    if (wave == 0 && l <= L) {
        tot[l] = s;
        cnt[l] = c;
    }
}

// ---- the -N side file (GROM.c:20234-20345): per g_1000gen_window bases, the
// copy number of the ratios depth / GC-bin average over the window's
// qualifying bases.  One lane per window; each lane adds its window's terms in
// the reference's order (sum, then the squared deviations), so cn and the
// deviation sum are the reference's doubles; the host takes the sqrt.
__global__ __launch_bounds__(256) void k_cnv_gen1000(const uint8_t *__restrict__ flag, const int32_t *__restrict__ mq,
                                                     const int32_t *__restrict__ rd, const int32_t *__restrict__ low,
                                                     const uint8_t *__restrict__ gcw, const Tables *__restrict__ T,
                                                     int64_t win, int64_t n_win, int min_mapq, int ploidy,
                                                     double *__restrict__ out_cn, double *__restrict__ out_s2,
                                                     int64_t *__restrict__ out_n) {
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= n_win) return;
    const int64_t b0 = w * win;
    double sum = 0.0;
    int64_t n = 0;
    for (int64_t a = b0; a < b0 + win; a++) {
        if (flag[a] & F_LOW) continue;
        const double ave = T->ave[mq[a] >= min_mapq ? 0 : 1][gcw[a]];
        if (ave > 0) {
            sum += (double)(rd[a] + low[a]) / ave;
            n += 1;
        }
    }
    double cn = -1.0, s2 = 0.0;
    if (n > 0) {
        cn = (sum / (double)n) * (double)ploidy;
        for (int64_t a = b0; a < b0 + win; a++) {
            if (flag[a] & F_LOW) continue;
            const double ave = T->ave[mq[a] >= min_mapq ? 0 : 1][gcw[a]];
            if (ave > 0) {
                const double t = (double)ploidy * ((double)(rd[a] + low[a]) / ave) - cn;
                s2 += t * t;  // pow(t, 2): both correctly rounded
            }
        }
    }
    out_cn[w] = cn;
    out_s2[w] = s2;
    out_n[w] = n;
}

// ---------------- DEL / DUP window search (GROM.c:19359-20020) ----------------
struct CallRec {
    int64_t p, ce;
    double stdevs;
    int32_t m, pad;
};

// per-position bit word the walk reads (one uint16 instead of five arrays)
constexpr uint32_t B_LOW = 1, B_HI = 2, B_RTP = 4, B_DEL0 = 8, B_DUP0 = 32, B_W0 = 128;

__global__ void k_cnv_wbits(Args A, const uint8_t *__restrict__ gcw, const int32_t *__restrict__ mq,
                            const int32_t *__restrict__ rd, const int32_t *__restrict__ low,
                            const uint8_t *__restrict__ flag, const Tables *__restrict__ T, uint16_t *__restrict__ wb) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < A.len; p += (int64_t)gridDim.x * blockDim.x) {
        const int r = rd[p] + low[p], g = gcw[p];
        uint32_t b = (flag[p] & F_LOW) ? B_LOW : 0;
        if (mq[p] >= A.min_mapq) b |= B_HI;
        if (r > 0) b |= B_RTP;
        for (int m = 0; m < 2; m++) {
            if (r <= T->thr[0][m][g]) b |= B_DEL0 << m;  // GROM.c:19373 (DEL), 19688 (DUP)
            if (r >= T->thr[1][m][g]) b |= B_DUP0 << m;
            if (T->wins[m][g] > 1) b |= B_W0 << m;
        }
        wb[p] = (uint16_t)b;
    }
}

struct WalkIn {
    const uint16_t *wb;
    const double *sd, *wsd;
    int64_t len, start, end, L, min_len;
    unsigned long long *stats;  // GROM_TIMING: walk counters (ab/cd wave calls and rounds), else null
    unsigned long long *prof;   // GROM_TIMING: slide clock counters (not moved per walk mode), else null
    // per 64-base word bit masks for the trim (phase D), this kind: defining
    // bases and their class-1 bits over every base (the outer scan) and over
    // nonlow bases (the inner scan), nonlow bases, and the pass bits under
    // class 0 / 1 over every base and over nonlow bases
    const uint64_t *t_defa, *t_c1a, *t_defn, *t_c1n, *t_nl, *t_pa0, *t_pa1, *t_pn0, *t_pn1;
};

__device__ __forceinline__ uint64_t low_bits(int n) { return n >= 64 ? ~0ull : ((1ull << n) - 1); }

__device__ __forceinline__ double dbl_of(uint32_t lo, uint32_t hi) {
    uint64_t u = ((uint64_t)hi << 32) | lo;
    double d;
    __builtin_memcpy(&d, &u, 8);
    return d;
}

// RN(tot / d) >= MIN_RD_LOW_STDEV for d > 0, as the reference's division and
// compare decide it, without the division on the common path.  RN(x) >= 3
// iff x >= 3 - 2^-52 (the midpoint below 3 rounds to 3, whose significand is
// even), i.e. iff tot - 3d >= -2^-52 d.  e = fma(-3, d, tot) is that
// difference rounded once, and rounding is monotonic, so e != t decides it;
// e == t is settled by the division itself.
static_assert(MIN_RD_LOW_STDEV == 3, "ratio_ge_min assumes the threshold 3");
__device__ __forceinline__ bool ratio_ge_min(double tot, double d) {
    const double t = -0x1p-52 * d;
    const double e = __builtin_fma(-3.0, d, tot);
    if (e != t) return e > t;
    return tot / d >= (double)MIN_RD_LOW_STDEV;
}
// The low-base fraction tests compare a sub-count over its window (a ratio
// in [0, 1]) with MAX_LOW_ACGT = 2: they never decide anything, so they are
// kept only as this compile-time constant.
static_assert(MAX_LOW_ACGT >= 1.0, "the low-fraction tests are dropped only while MAX_LOW_ACGT >= 1");
constexpr bool LOW_FRAC_OK = true;

// The walk is one serial computation.  A wave runs it with every lane
// executing the same uniform statements; per-position inputs come from a
// 64-position register window (lane i holds position base+i) that is refilled
// by one coalesced load whenever the walk leaves it, and read with readlane.
struct WinRegs {
    uint32_t b, s_lo, s_hi, v;
    int32_t n0, n1;  // nxt[0][p], nxt[1][p]
};

struct Win {
    const uint16_t *wb;
    const double *sd;
    const uint8_t *vis;
    const int32_t *nxt;
    int64_t len;
    int64_t base;
    WinRegs r, nx;  // the window [base, base+64) and, already in flight, [base+64, base+128)
    // unconditional loads from a clamped index (vis and nxt are never null):
    // a load under a branch would be waited for at the join, so the
    // prefetched window would not be in flight while the walk works
    __device__ void load(int64_t b, WinRegs &o) const {
        const int64_t q0 = b + (int64_t)(threadIdx.x & 63);
        const bool ok = q0 >= 0 && q0 < len;
        const int64_t q = q0 < 0 ? 0 : q0 >= len ? len - 1 : q0;
        const uint32_t bb = wb[q], vv = vis[q];
        const double v = sd[q];
        const int32_t n0 = nxt[q], n1 = nxt[len + q];
        uint64_t u;
        __builtin_memcpy(&u, &v, 8);
        o.b = ok ? bb : 0u;
        o.s_lo = ok ? (uint32_t)u : 0u;
        o.s_hi = ok ? (uint32_t)(u >> 32) : 0u;
        o.v = ok ? vv : 0u;
        o.n0 = ok ? n0 : 0;
        o.n1 = ok ? n1 : 0;
    }
    __device__ void fill(int64_t b) {
        base = b;
        load(b, r);
        load(b + 64, nx);  // prefetch: the walk mostly moves forward
    }
    __device__ __forceinline__ int slot(int64_t p) {
        if (p >= base + 64) {
            if (p < base + 128) {
                base += 64;
                r = nx;
                load(base + 64, nx);
            } else {
                fill(p);
            }
        } else if (p < base) {
            fill(p - 63);
        }
        return (int)(p - base);
    }
    __device__ __forceinline__ uint32_t bits(int64_t p) {
        int i = slot(p);
        return (uint32_t)__builtin_amdgcn_readlane((int)r.b, i);
    }
    __device__ __forceinline__ double z(int64_t p) {
        int i = slot(p);
        return dbl_of((uint32_t)__builtin_amdgcn_readlane((int)r.s_lo, i), (uint32_t)__builtin_amdgcn_readlane((int)r.s_hi, i));
    }
};

// state after the first two phases of the window search at one base
struct PreAB {
    int64_t temp_pos, ce, last_good;
    double stdevs;
    int32_t stop, begin, mqi, done;  // done: ce/stdevs below are the finished call
    int64_t ce_final;
    double stdevs_final;
};

// phases A (first min-window) and B (extension to L) of the window search at
// a base that passes the threshold (GROM.c:19370-19470 DEL, 19685-19785 DUP);
// Acc provides bits(p) and z(p)
template <int KIND, class Acc>
__device__ PreAB phase_ab(Acc &c, const WalkIn &W, int64_t pos, int mqi, int64_t max_steps = INT64_MAX,
                          bool *capped = nullptr) {
    const int64_t L = W.L, ML = W.min_len, end = W.end;
    const double *wsd = W.wsd;
    int begin = 0, stop = 0;
    int64_t ce = 0, last_good = 0, temp_pos = pos, pa, wl = 0, cnt = 0, cnt2 = 0;
    double stdevs = 0.0, tot = 0.0;
    const uint32_t pb0 = KIND == 0 ? B_DEL0 : B_DUP0;
    auto cls = [](uint32_t b, int m) { return (b & B_HI) ? 0 : (b & B_RTP) ? 1 : m; };
    for (pa = pos; pa < pos + ML; pa++) {
        wl += 1;
        const uint32_t b = c.bits(pa);
        if (!(b & B_LOW)) {
            mqi = cls(b, mqi);
            if (b & (pb0 << mqi)) cnt2 += 1;
            else if ((2 * cnt2) < wl) { stop = 1; temp_pos = pa; break; }
        } else if ((2 * cnt2) < wl) { stop = 1; temp_pos = pa; break; }
    }
    if (stop == 0) {
        cnt = ML;
        tot = 0;
        for (int64_t a = pos; a < pos + ML; a++) {
            cnt -= (c.bits(a) & B_LOW);
            if (KIND == 0) tot += c.z(a); else tot -= c.z(a);
        }
    }
    if (stop == 0 && cnt > 0 && wsd[ML] > 0 && ratio_ge_min(tot, cnt * wsd[ML]) && LOW_FRAC_OK) {
        begin = 1;
        last_good = pos + ML;
        ce = pos + ML;
        stdevs = tot / (cnt * wsd[ML]);
    }
    if (stop == 0) {
        for (pa = pos + ML; pa < pos + L; pa++) {
            if (capped && pa - pos >= max_steps) { *capped = true; break; }  // the walk decides this base
            wl += 1;
            if (pa < end) {
                const uint32_t b = c.bits(pa);
                if (!(b & B_LOW)) {
                    mqi = cls(b, mqi);
                    if (KIND == 0) tot += c.z(pa); else tot -= c.z(pa);
                    cnt += 1;
                    if (b & (pb0 << mqi)) {
                        cnt2 += 1;
                        if (wsd[wl] > 0 && ratio_ge_min(tot, cnt * wsd[wl]) && LOW_FRAC_OK) {
                            last_good = pa;
                            if (begin == 0) {
                                begin = 1;
                                ce = pa;
                                stdevs = tot / (cnt * wsd[wl]);
                            } else {
                                double ts = tot / (cnt * wsd[wl]);
                                ce = pa;
                                if (ts > stdevs) stdevs = ts;
                            }
                        }
                    } else if ((2 * cnt2) < wl) { stop = 1; break; }
                } else if ((2 * cnt2) < wl) { stop = 1; break; }
            } else { stop = 1; break; }
        }
    }
    PreAB r;
    r.temp_pos = temp_pos;
    r.ce = ce;
    r.last_good = last_good;
    r.stdevs = stdevs;
    r.stop = stop;
    r.begin = begin;
    r.mqi = mqi;
    r.done = 0;
    r.ce_final = 0;
    r.stdevs_final = 0.0;
    return r;
}

// phases C (sliding extension past L, GROM.c:19476-19545) and D (trimming
// the call's end, GROM.c:19550-19600) of a call found at `pos` with phase
// A/B state r.  `a` serves the leading edge and the trim, `t` the trailing
// edge of the slide.  Gives up (returns false) after max_steps steps.
template <int KIND, class Acc>
__device__ bool phase_cd(Acc &a, Acc &t, const WalkIn &W, int64_t pos, const PreAB &r, int64_t max_steps,
                         int64_t &ce_out, double &stdevs_out) {
    const int64_t L = W.L, ML = W.min_len, cs = pos;
    const double *wsd = W.wsd;
    const uint32_t pb0 = KIND == 0 ? B_DEL0 : B_DUP0;
    auto cls = [](uint32_t b, int m) { return (b & B_HI) ? 0 : (b & B_RTP) ? 1 : m; };
    int64_t ce = r.ce, last_good = r.last_good, pa, pb, cnt = 0, steps = 0;
    double stdevs = r.stdevs, tot = 0.0;
    int mqi = r.mqi;
    if (r.stop == 0) {
        pa = pos + L;
        int mqb = mqi;
        while (pa < W.len && (pa - last_good) <= MAX_DIST_LAST_GOOD) {
            if (++steps > max_steps) return false;
            if (pa == pos + L) {
                for (pb = pa - L + 1; pb < pa + 1; pb++) {
                    const uint32_t b = t.bits(pb);
                    mqb = cls(b, mqb);
                    if (!(b & B_LOW) && (b & (B_W0 << mqb))) {
                        if (KIND == 0) tot += t.z(pb); else tot -= t.z(pb);
                        cnt += 1;
                    }
                }
                steps += L;
            } else {
                pb = pa - L;
                const uint32_t bb = t.bits(pb);
                mqb = cls(bb, mqb);
                if (!(bb & B_LOW) && (bb & (B_W0 << mqb))) {
                    if (KIND == 0) tot -= t.z(pb); else tot += t.z(pb);
                    cnt -= 1;
                }
                const uint32_t ba = a.bits(pa);
                mqi = cls(ba, mqi);
                if (!(ba & B_LOW) && (ba & (B_W0 << mqi))) {
                    if (KIND == 0) tot += a.z(pa); else tot -= a.z(pa);
                    cnt += 1;
                }
            }
            if (cnt > 0 && wsd[L] > 0 && ratio_ge_min(tot, cnt * wsd[L]) && LOW_FRAC_OK) {
                last_good = pa;
                ce = pa;
                double ts = tot / (cnt * wsd[L]);
                if (ts > stdevs) stdevs = ts;
            }
            pa += 1;
        }
    }
    int64_t p = ce;
    while (p > cs + ML) {
        if (++steps > max_steps) return false;
        const uint32_t b = a.bits(p);
        mqi = cls(b, mqi);
        if (!(b & (pb0 << mqi))) {
            p -= 1;
            ce = p;
        } else {
            int64_t c2 = 0, c3 = 0;
            pa = ce;
            int stop_while = 0, mqa = mqi;
            while (pa > cs + ML && stop_while == 0) {
                if (++steps > max_steps) return false;
                const uint32_t ba = a.bits(pa);
                if (!(ba & B_LOW)) {
                    mqa = cls(ba, mqa);
                    c3 += 1;
                    if (ba & (pb0 << mqa)) c2 += 1;
                }
                if (c3 == 0 || (c3 > 0 && 2 * c2 < c3) || !LOW_FRAC_OK) {  // c2/(double)c3 < 0.5 exactly, for counts < 2^26
                    ce = pa - 1;
                    stop_while = 1;
                }
                pa -= 1;
            }
            p = pa;
        }
    }
    ce_out = ce;
    stdevs_out = stdevs;
    return true;
}

// ---- wave-cooperative window search (the walk's long calls) ----
//
// A call inside a long copy-number region slides its window across the whole
// region (phase C) and trims it back (phase D), and phase B extends every
// candidate up to L bases: serial loops that one lane runs at ~0.5 us per
// step.  The versions below keep the serial parts serial -- the running
// double sum `tot` is added in the reference's order, one IEEE operation per
// step -- and spread everything else over the 64 lanes, 64 steps at a time:
// coalesced loads, the class state as a last-value scan, integer counts as
// prefix sums, each step's window test on its own lane, the first stopping
// step by ballot.  The results are those of phase_ab / phase_cd exactly.

__device__ __forceinline__ int cdef(uint32_t b) { return (b & B_HI) ? 0 : (b & B_RTP) ? 1 : -1; }

// wave_last_incl for classes e in {-1, 0, 1}: the latest defined lane at or
// below this one, found from two ballots (highest set bit of the defined
// lanes up to this one) -- no cross-lane chain
__device__ __forceinline__ int dpp_last_incl(int e, int c) {
    const int lane = threadIdx.x & 63;
    const unsigned long long d = __ballot(e >= 0) & (~0ull >> (63 - lane));
    const unsigned long long c1 = __ballot(e == 1);
    const int j = 63 - __clzll(d);
    return d ? (int)((c1 >> j) & 1ull) : c;
}

// max of non-negative doubles over the wave (their bit patterns order as
// unsigned integers), returned to every lane
template <int CTL, int RM>
__device__ __forceinline__ void dpp_max_step_u64(int &hi, int &lo) {
    const int h2 = __builtin_amdgcn_update_dpp(hi, hi, CTL, RM, 0xf, false);
    const int l2 = __builtin_amdgcn_update_dpp(lo, lo, CTL, RM, 0xf, false);
    const bool gt = (uint32_t)h2 > (uint32_t)hi || ((uint32_t)h2 == (uint32_t)hi && (uint32_t)l2 > (uint32_t)lo);
    hi = gt ? h2 : hi;
    lo = gt ? l2 : lo;
}

__device__ __forceinline__ double dpp_max_pos(double d) {
    uint64_t u;
    __builtin_memcpy(&u, &d, 8);
    int hi = (int)(uint32_t)(u >> 32), lo = (int)(uint32_t)u;
    dpp_max_step_u64<0x111, 0xf>(hi, lo);
    dpp_max_step_u64<0x112, 0xf>(hi, lo);
    dpp_max_step_u64<0x114, 0xf>(hi, lo);
    dpp_max_step_u64<0x118, 0xf>(hi, lo);
    dpp_max_step_u64<0x142, 0xa>(hi, lo);
    dpp_max_step_u64<0x143, 0xc>(hi, lo);
    return dbl_of((uint32_t)__builtin_amdgcn_readlane(lo, 63), (uint32_t)__builtin_amdgcn_readlane(hi, 63));
}

// inclusive count of the lanes at or below this one whose flag is set
// (mbcnt over the ballot: no cross-lane data movement)
__device__ __forceinline__ int wave_incl_count(bool f) {
    const unsigned long long m = __ballot(f);
    const int below = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    return below + (f ? 1 : 0);
}

__device__ __forceinline__ double rl_d(double v, int k) {
    uint64_t u;
    __builtin_memcpy(&u, &v, 8);
    return dbl_of((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, k),
                  (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), k));
}

__device__ __forceinline__ int64_t rl_i64(int64_t v, int k) {
    return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, k)) |
                     ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), k) << 32));
}

[[maybe_unused]] __device__ __forceinline__ double wave_max_d(double v) {
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}

// `tot` advanced over the lanes in order: at lane k, tot + a then (two-op
// form) + b, where a lane without an operation contributes 0.0.  Adding 0.0
// is exact here: tot starts at +0.0 and a sum of doubles is -0.0 only when
// both terms are, so tot is never -0.0 and x + (+-0.0) == x.
//
// The chain stays one IEEE operation per step in the reference's order, and
// runs in registers: each of 63 rounds shifts the partial sums one lane up
// (DPP wave_shr:1, lane 0 refilled with the incoming tot) and adds the lane's
// own addend, so after round k lanes 0..k hold their exact prefix
// ((tot + a_0) + a_1) + ... + a_lane.  No LDS, no barrier.
// Lane 0 reads +0.0 from the shift (bound_ctrl) and its first addend is
// tot + a_0, the chain's own first operation: +0.0 + x == x for x != -0.0,
// and tot + a_0 is -0.0 only if tot is.
__device__ __forceinline__ double dpp_wave_shr1(double v) {
    uint64_t u;
    __builtin_memcpy(&u, &v, 8);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, 0x138, 0xf, 0xf, true);  // wave_shr:1
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), 0x138, 0xf, 0xf, true);
    return dbl_of((uint32_t)lo, (uint32_t)hi);
}

// The same chain through LDS, for the walk kernels (one wave per block): the
// lanes store their addends, then every lane runs the whole chain on the
// broadcast values -- two dependent f64 adds per step, with no cross-lane move
// on the dependency path -- and lane 0 stores each step's sum for its lane to
// pick up.  Bit-identical to the DPP form (same operations, same order).
struct ChainLds {
    double2 ad[64];
    double to[64];
};

[[maybe_unused]] __device__ __forceinline__ ChainLds &chain_lds() {
    __shared__ ChainLds c;
    return c;
}

// LDS ordering inside the one wave: the wave's LDS instructions execute in
// order, so only the compiler has to be kept from moving them; unlike
// __syncthreads this does not wait for the wave's global loads in flight
// (the next round's inputs)
[[maybe_unused]] __device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0) only (vmcnt, expcnt at their maximum)
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

template <bool TWO>
[[maybe_unused]] __device__ __forceinline__ double lds_chain(double &tot, double a, double b) {
    ChainLds &c = chain_lds();
    const int lane = threadIdx.x & 63;
    c.ad[lane] = make_double2(a, b);
    wave_lds_sync();
    double t = tot;
    // software pipeline: group g+1's addends are read while group g's eight
    // steps run, so the LDS latency stays off the chain
    double2 cur[8], nxt[8];
#pragma unroll
    for (int k = 0; k < 8; k++) cur[k] = c.ad[k];
#pragma unroll
    for (int g = 0; g < 8; g++) {
        if (g < 7) {
#pragma unroll
            for (int k = 0; k < 8; k++) nxt[k] = c.ad[(g + 1) * 8 + k];
        }
        double tt[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            t = t + cur[k].x;
            if (TWO) t = t + cur[k].y;
            tt[k] = t;
        }
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < 8; k++) c.to[g * 8 + k] = tt[k];
        }
#pragma unroll
        for (int k = 0; k < 8; k++) cur[k] = nxt[k];
    }
    wave_lds_sync();
    const double r = c.to[lane];
    wave_lds_sync();  // every lane has read `to` before a next call's lane 0 rewrites it
    tot = t;
    return r;
}

// the register-only form: each round shifts the partial sums one lane up
[[maybe_unused]] __device__ __forceinline__ double dpp_chain1(double &tot, double a) {
    const double a0 = (threadIdx.x & 63) == 0 ? tot + a : a;
    double t = a0;
#pragma unroll
    for (int k = 1; k < 64; k++) t = dpp_wave_shr1(t) + a0;
    tot = rl_d(t, 63);
    return t;
}

[[maybe_unused]] __device__ __forceinline__ double dpp_chain2(double &tot, double a, double b) {
    const double a0 = (threadIdx.x & 63) == 0 ? tot + a : a;
    double t = a0 + b;
#pragma unroll
    for (int k = 1; k < 64; k++) t = (dpp_wave_shr1(t) + a0) + b;
    tot = rl_d(t, 63);
    return t;
}

// measured (tools/chain_bench.hip, and the walk's slide clocks): the DPP form
// 24.7 cycles per step with every lane's sum in place, the LDS form 20.8 for
// the chain alone but 31-35 once the sums are handed back to the lanes
#ifdef GROM_CHAIN_LDS
__device__ __forceinline__ double wave_chain1(double &tot, double a) { return lds_chain<false>(tot, a, 0.0); }
[[maybe_unused]] __device__ __forceinline__ double wave_chain2(double &tot, double a, double b) { return lds_chain<true>(tot, a, b); }
#else
__device__ __forceinline__ double wave_chain1(double &tot, double a) { return dpp_chain1(tot, a); }
[[maybe_unused]] __device__ __forceinline__ double wave_chain2(double &tot, double a, double b) { return dpp_chain2(tot, a, b); }
#endif

// the round-by-round loops below read the next round's inputs before the
// current round's serial work: unconditional loads from a clamped index (a
// load under a branch would be waited for at the join)
__device__ __forceinline__ int64_t clamp_pos(const WalkIn &W, int64_t q) { return q < 0 ? 0 : q >= W.len ? W.len - 1 : q; }

// phases A and B (phase_ab) for the wave; every lane returns the same record
template <int KIND>
__device__ PreAB phase_ab_wave(const WalkIn &W, int64_t pos, int mqi) {
    const int lane = threadIdx.x & 63;
    const int64_t L = W.L, ML = W.min_len, end = W.end;
    const uint32_t pb0 = KIND == 0 ? B_DEL0 : B_DUP0;
    const double sgn = KIND == 0 ? 1.0 : -1.0;  // tot -= z is tot + (-z), exactly
    int begin = 0, stop = 0;
    int64_t ce = 0, last_good = 0, temp_pos = pos, wl = 0, cnt = 0, cnt2 = 0;
    double stdevs = 0.0, tot = 0.0;
    // phase A: the first ML bases (GROM.c:19370-19400)
    uint32_t nb = W.wb[clamp_pos(W, pos + lane)];
    for (int64_t p0 = pos; p0 < pos + ML && !stop; p0 += 64) {
        const int64_t p = p0 + lane;
        const bool in = p < pos + ML;
        const uint32_t b = in ? nb : 0u;
        nb = W.wb[clamp_pos(W, p + 64)];
        const bool nl = in && !(b & B_LOW);
        const int m = dpp_last_incl(nl ? cdef(b) : -1, mqi);
        const bool ps = nl && (b & (pb0 << m));
        const int64_t c2 = cnt2 + wave_incl_count(ps);
        const int64_t w = wl + lane + 1;
        const bool st = in && !ps && (2 * c2) < w;
        const unsigned long long sm = __ballot(st);
        const int n_in = (int)min<int64_t>(64, pos + ML - p0);
        const int last = sm ? __ffsll((long long)sm) - 1 : n_in - 1;
        mqi = __builtin_amdgcn_readlane(m, last);
        cnt2 = rl_i64(c2, last);
        wl += last + 1;
        if (sm) {
            stop = 1;
            temp_pos = p0 + last;
        }
    }
    if (stop == 0) {
        cnt = ML;
        uint32_t nb2 = W.wb[clamp_pos(W, pos + lane)];
        double nz2 = W.sd[clamp_pos(W, pos + lane)];
        for (int64_t p0 = pos; p0 < pos + ML; p0 += 64) {
            const int64_t p = p0 + lane;
            const bool in = p < pos + ML;
            const uint32_t b = in ? nb2 : 0u;
            const double z = nz2;
            nb2 = W.wb[clamp_pos(W, p + 64)];
            nz2 = W.sd[clamp_pos(W, p + 64)];
            cnt -= __popcll(__ballot(in && (b & B_LOW)));
            const double v = in ? sgn * z : 0.0;
            wave_chain1(tot, v);
        }
    }
    if (stop == 0 && cnt > 0 && W.wsd[ML] > 0 && ratio_ge_min(tot, cnt * W.wsd[ML]) && LOW_FRAC_OK) {
        begin = 1;
        last_good = pos + ML;
        ce = pos + ML;
        stdevs = tot / (cnt * W.wsd[ML]);
    }
    // phase B: extension to L (GROM.c:19405-19470); the next round's wsd
    // index assumes this round does not stop (if it does, the loop ends)
    uint32_t nb3 = W.wb[clamp_pos(W, pos + ML + lane)];
    double nz3 = W.sd[clamp_pos(W, pos + ML + lane)];
    double nw3 = W.wsd[min<int64_t>(wl + lane + 1, L)];
    for (int64_t p0 = pos + ML; p0 < pos + L && !stop; p0 += 64) {
        const int64_t p = p0 + lane;
        const bool in = p < pos + L;
        const bool inend = in && p < end;
        const uint32_t b = inend ? nb3 : 0u;
        const double z = nz3, wsdn = nw3;
        nb3 = W.wb[clamp_pos(W, p + 64)];
        nz3 = W.sd[clamp_pos(W, p + 64)];
        nw3 = W.wsd[min<int64_t>(wl + 64 + lane + 1, L)];
        const bool nl = inend && !(b & B_LOW);
        const int m = dpp_last_incl(nl ? cdef(b) : -1, mqi);
        const bool ps = nl && (b & (pb0 << m));
        const int64_t c = cnt + wave_incl_count(nl);
        const int64_t c2 = cnt2 + wave_incl_count(ps);
        const int64_t w = wl + lane + 1;
        const double v = nl ? sgn * z : 0.0;
        const double tj = wave_chain1(tot, v);
        const double wsdw = in ? wsdn : 0.0;
        const bool good = ps && wsdw > 0 && ratio_ge_min(tj, c * wsdw) && LOW_FRAC_OK;
        const double ts = good ? tj / (c * wsdw) : 0.0;
        const bool st = in && (!inend || (!ps && (2 * c2) < w));
        const unsigned long long sm = __ballot(st);
        const int n_in = (int)min<int64_t>(64, pos + L - p0);
        const int js = sm ? __ffsll((long long)sm) - 1 : n_in;  // steps before the stopping one
        const bool eg = good && lane < js;
        const unsigned long long gm = __ballot(eg);
        if (gm) {
            const int jl = 63 - __clzll(gm);
            last_good = ce = p0 + jl;
            const double mx = dpp_max_pos(eg ? ts : 0.0);
            if (begin == 0) { begin = 1; stdevs = mx; }
            else if (mx > stdevs) stdevs = mx;
        }
        const int last = sm ? js : n_in - 1;  // the stopping step still updates the state
        mqi = __builtin_amdgcn_readlane(m, last);
        cnt = rl_i64(c, last);
        cnt2 = rl_i64(c2, last);
        tot = rl_d(tj, last);
        wl += last + 1;
        if (sm) stop = 1;
    }
    PreAB r;
    r.temp_pos = temp_pos;
    r.ce = ce;
    r.last_good = last_good;
    r.stdevs = stdevs;
    r.stop = stop;
    r.begin = begin;
    r.mqi = mqi;
    r.done = 0;
    r.ce_final = 0;
    r.stdevs_final = 0.0;
    return r;
}

// phases C and D (phase_cd) for the wave, in three parts so that the walk can
// pause a long slide (SlideState holds everything the slide carries) and
// resume it later, possibly from another kernel
struct SlideState {
    int64_t pos, pa, cnt, last_good, ce;
    double tot, stdevs;
    int32_t mqi, mqb, m, sliding;  // m: the walk's class at the call base; sliding: phase C not finished
};

// phase C's first window [pos+1, pos+L] (GROM.c:19480-19490)
template <int KIND>
__device__ SlideState slide_begin(const WalkIn &W, int64_t pos, const PreAB &r, int m) {
    const int lane = threadIdx.x & 63;
    const int64_t L = W.L;
    const double sgn = KIND == 0 ? 1.0 : -1.0;
    const double wsdL = W.wsd[L];
    SlideState s;
    s.pos = pos;
    s.ce = r.ce;
    s.last_good = r.last_good;
    s.cnt = 0;
    s.stdevs = r.stdevs;
    s.tot = 0.0;
    s.mqi = r.mqi;
    s.mqb = r.mqi;
    s.m = m;
    s.sliding = 0;
    s.pa = pos + L;
    if (r.stop != 0 || !(s.pa < W.len && (s.pa - s.last_good) <= MAX_DIST_LAST_GOOD)) return s;
    uint32_t nb = W.wb[clamp_pos(W, pos + 1 + lane)];
    double nz = W.sd[clamp_pos(W, pos + 1 + lane)];
    for (int64_t p0 = pos + 1; p0 <= pos + L; p0 += 64) {
        const int64_t p = p0 + lane;
        const bool in = p <= pos + L;
        const uint32_t b = in ? nb : 0u;
        const double z = nz;
        nb = W.wb[clamp_pos(W, p + 64)];
        nz = W.sd[clamp_pos(W, p + 64)];
        const int mm = dpp_last_incl(in ? cdef(b) : -1, s.mqb);
        const bool q = in && !(b & B_LOW) && (b & (B_W0 << mm));
        const double v = q ? sgn * z : 0.0;
        s.cnt += __popcll(__ballot(q));
        wave_chain1(s.tot, v);
        s.mqb = __builtin_amdgcn_readlane(mm, (int)min<int64_t>(63, pos + L - p0));
    }
    if (s.cnt > 0 && wsdL > 0 && ratio_ge_min(s.tot, s.cnt * wsdL) && LOW_FRAC_OK) {
        s.last_good = s.pa;
        s.ce = s.pa;
        const double ts = s.tot / (s.cnt * wsdL);
        if (ts > s.stdevs) s.stdevs = ts;
    }
    s.pa += 1;
    s.sliding = 1;
    return s;
}

// the slide (GROM.c:19492-19545), 64 steps per round; the next round's
// inputs are loaded while this one runs (the rounds are a serial chain, so
// load latency would otherwise add up).  Stops before a round that would
// start at or past `cap` and returns false (s then resumes exactly there).
template <int KIND>
[[maybe_unused]] __device__ bool slide_run64(const WalkIn &W, SlideState &s, int64_t cap) {
    if (!s.sliding) return true;
    const int lane = threadIdx.x & 63;
    const int64_t L = W.L;
    const double sgn = KIND == 0 ? 1.0 : -1.0;
    const double wsdL = W.wsd[L];
    int64_t pa = s.pa, cnt = s.cnt, last_good = s.last_good, ce = s.ce;
    double tot = s.tot;
    // the largest good ratio per lane; max is exact and order-free, so the
    // wave's maximum is taken once, when the slide ends or pauses
    double lmax = 0.0;
    int mqi = s.mqi, mqb = s.mqb;
    // the inputs of one round: lane j holds the leading and trailing bases of step j
    struct In {
        uint32_t ba, bb;
        double za, zb;
    };
    // unconditional loads from a clamped index (q - L >= 0 here): a load
    // under a branch makes the compiler wait for it at the join, which
    // would put a memory latency into every round
    // (no select on the loaded values here: that would wait for them; the
    // round masks lanes past the end itself, inl below)
    auto load = [&](int64_t at, In &o) {
        const int64_t q0 = at + lane;
        const int64_t q = q0 < W.len ? q0 : W.len - 1;
        o.ba = W.wb[q];
        o.bb = W.wb[q - L];
        o.za = W.sd[q];
        o.zb = W.sd[q - L];
    };
    bool finished = true;
    const long long ck_start = W.stats ? clock64() : 0;
    // GROM_TIMING counters, kept in registers (an atomic per round would put
    // its round trip into the next round's load wait)
    long long pc_chain = 0, pc_before = 0, pc_after = 0, pc_rounds = 0;
    // one round (64 steps) from pa with its inputs; false when the slide
    // stops or pauses in it
    auto round = [&](const In &in) -> bool {
        if (pa >= cap) { finished = false; return false; }
        const long long ckt = W.stats ? clock64() : 0;
        const int64_t p = pa + lane;
        const bool inl = p < W.len;
        const uint32_t ba = in.ba, bb = in.bb;
        const double za = in.za, zb = in.zb;
        const int mt = dpp_last_incl(inl ? cdef(bb) : -1, mqb);
        const int ml = dpp_last_incl(inl ? cdef(ba) : -1, mqi);
        const bool qt = inl && !(bb & B_LOW) && (bb & (B_W0 << mt));
        const bool ql = inl && !(ba & B_LOW) && (ba & (B_W0 << ml));
        const double vt = qt ? -sgn * zb : 0.0;
        const double vl = ql ? sgn * za : 0.0;
        const int64_t cj = cnt + wave_incl_count(ql) - wave_incl_count(qt);
        double t = tot;
        const long long ck0 = W.stats ? clock64() : 0;
        const double tj = wave_chain2(t, vt, vl);
        const long long ck1 = W.stats ? clock64() : 0;
        pc_chain += ck1 - ck0;
        pc_before += ck0 - ckt;
        const bool good = inl && cj > 0 && wsdL > 0 && ratio_ge_min(tj, cj * wsdL) && LOW_FRAC_OK;
        const double ts = good ? tj / (cj * wsdL) : 0.0;
        // the loop test of step j sees the last good step before it; no
        // step of the round can fail it while pa + 63 is within MAX_DIST of
        // last_good (the common case: skip the scan)
        bool cont = inl;
        if (pa + 63 - last_good > MAX_DIST_LAST_GOOD) {
            int gi = wave_last_incl(good ? lane : -1, -1);
            int ge = __shfl_up(gi, 1);
            if (lane == 0) ge = -1;
            const int64_t lgb = ge >= 0 ? pa + ge : last_good;
            cont = inl && (p - lgb) <= MAX_DIST_LAST_GOOD;
        }
        const unsigned long long sm = __ballot(!cont);
        const int js = sm ? __ffsll((long long)sm) - 1 : 64;
        const bool eg = good && lane < js;
        const unsigned long long gm = __ballot(eg);
        if (gm) last_good = ce = pa + (63 - __clzll(gm));
        lmax = (eg && ts > lmax) ? ts : lmax;
        if (js == 64) {
            tot = t;  // the chain's last sum (== tj of lane 63), without a cross-lane read
            cnt = rl_i64(cj, 63);
            mqi = __builtin_amdgcn_readlane(ml, 63);
            mqb = __builtin_amdgcn_readlane(mt, 63);
        } else if (js > 0) {
            tot = rl_d(tj, js - 1);
            cnt = rl_i64(cj, js - 1);
            mqi = __builtin_amdgcn_readlane(ml, js - 1);
            mqb = __builtin_amdgcn_readlane(mt, js - 1);
        }
        pa += js;
        pc_rounds++;
        if (W.stats) pc_after += clock64() - ck1;
        return js == 64;
    };
    // four rounds of inputs in flight: a round's loads are issued three
    // rounds before it runs (one round's work does not cover an HBM miss)
    In b0, b1, b2, b3;
    load(pa, b0);
    load(pa + 64, b1);
    load(pa + 128, b2);
    load(pa + 192, b3);
    for (;;) {
        if (!round(b0)) break;
        load(pa + 192, b0);
        if (!round(b1)) break;
        load(pa + 192, b1);
        if (!round(b2)) break;
        load(pa + 192, b2);
        if (!round(b3)) break;
        load(pa + 192, b3);
    }
    if (W.stats && lane == 0) {
        atomicAdd(W.prof + 1, (unsigned long long)(clock64() - ck_start));
        atomicAdd(W.prof + 0, (unsigned long long)pc_chain);
        atomicAdd(W.prof + 2, (unsigned long long)pc_before);
        atomicAdd(W.prof + 3, (unsigned long long)pc_after);
        atomicAdd(W.stats + 2, (unsigned long long)pc_rounds);
    }
    s.pa = pa;
    s.cnt = cnt;
    s.last_good = last_good;
    s.ce = ce;
    s.tot = tot;
    const double mx = dpp_max_pos(lmax);  // ratios are >= 3 > 0; lanes without one hold 0
    if (mx > s.stdevs) s.stdevs = mx;
    s.mqi = mqi;
    s.mqb = mqb;
    s.sliding = finished ? 0 : 1;
    return finished;
}

// ---- the slide, 256 steps per round (4 per lane) ----
//
// The window sum `tot` is one chain of f64 adds in the reference's order.
// Instead of running it across the lanes (one DPP hop per step, ~25 cycles),
// every lane runs its own four steps from a GUESSED start value, and the
// guesses are then checked: lane l's start must equal lane l-1's end, bit for
// bit.  Lane 0 starts from the exact `tot`, so if every check holds, every
// start -- and so every step's sum -- is the reference's exact value (by
// induction over the lanes); the first lane that fails restarts the guessing
// from the exact end of the lane before it.
//
// The guess: while a sum stays in one binade [2^e, 2^(e+1)), every value is an
// integer multiple of u = 2^(e-52), and fl(t + x) = t + RN(x / u) u with the
// rounding independent of t except for exact ties.  So per lane the integer
// increment D = sum of RN(x / u) over its eight adds is computed in parallel,
// a prefix sum over the lanes gives each lane's start, and only a tie or a
// binade change can make a guess wrong -- which the check catches.
__device__ __forceinline__ double dpp_sum_step(double v, int ctl_sel) {
    uint64_t u;
    __builtin_memcpy(&u, &v, 8);
    int lo = (int)(uint32_t)u, hi = (int)(uint32_t)(u >> 32);
    switch (ctl_sel) {  // (constant after unrolling)
    case 0: lo = __builtin_amdgcn_update_dpp(0, lo, 0x111, 0xf, 0xf, true); hi = __builtin_amdgcn_update_dpp(0, hi, 0x111, 0xf, 0xf, true); break;
    case 1: lo = __builtin_amdgcn_update_dpp(0, lo, 0x112, 0xf, 0xf, true); hi = __builtin_amdgcn_update_dpp(0, hi, 0x112, 0xf, 0xf, true); break;
    case 2: lo = __builtin_amdgcn_update_dpp(0, lo, 0x114, 0xf, 0xf, true); hi = __builtin_amdgcn_update_dpp(0, hi, 0x114, 0xf, 0xf, true); break;
    case 3: lo = __builtin_amdgcn_update_dpp(0, lo, 0x118, 0xf, 0xf, true); hi = __builtin_amdgcn_update_dpp(0, hi, 0x118, 0xf, 0xf, true); break;
    case 4: lo = __builtin_amdgcn_update_dpp(0, lo, 0x142, 0xa, 0xf, false); hi = __builtin_amdgcn_update_dpp(0, hi, 0x142, 0xa, 0xf, false); break;
    default: lo = __builtin_amdgcn_update_dpp(0, lo, 0x143, 0xc, 0xf, false); hi = __builtin_amdgcn_update_dpp(0, hi, 0x143, 0xc, 0xf, false); break;
    }
    return dbl_of((uint32_t)lo, (uint32_t)hi);
}

// inclusive prefix sum over the lanes (exact for integer-valued doubles
// whose partial sums stay below 2^53, which is all the guess needs)
__device__ __forceinline__ double wave_incl_sum(double v) {
#pragma unroll
    for (int k = 0; k < 6; k++) v += dpp_sum_step(v, k);
    return v;
}

__device__ __forceinline__ uint64_t dbits(double v) {
    uint64_t u;
    __builtin_memcpy(&u, &v, 8);
    return u;
}

// the class at the start of each lane: the last class-defining step (e: the
// lane's own last, -1 none) among the lanes below, else the carry c
__device__ __forceinline__ int lane_last_excl(int e, int c) {
    const int lane = threadIdx.x & 63;
    const unsigned long long d = __ballot(e >= 0) & ((1ull << lane) - 1);
    const unsigned long long c1 = __ballot(e == 1);
    return d ? (int)((c1 >> (63 - __clzll(d))) & 1ull) : c;
}

// exclusive prefix over the lanes of small counts n in [0, 7], and the total
__device__ __forceinline__ int excl_small(int n, int &total) {
    const int lane = threadIdx.x & 63;
    const unsigned long long b0 = __ballot(n & 1), b1 = __ballot(n & 2), b2 = __ballot(n & 4);
    const unsigned long long below = (1ull << lane) - 1;
    total = __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
    return (int)(__popcll(b0 & below) + 2 * __popcll(b1 & below) + 4 * __popcll(b2 & below));
}

// the chain over the round: tj[i] = the sum after step 4*lane + i, exact
// (see above); `tot` is the sum before the round
__device__ __forceinline__ void chain_round4(double tot, const double (&vt)[4], const double (&vl)[4], double (&tj)[4],
                                             unsigned long long &n_fix) {
    const int lane = threadIdx.x & 63;
    int b = 0;         // lanes below b are checked
    double T = tot;    // the exact start of lane b
    double tin = 0.0;  // this lane's start
    bool ok = false;
    for (int it = 0; it < 4; it++) {
        int E;
        (void)frexp(T, &E);  // |T| in [2^(E-1), 2^E)
        const double inv_u = ldexp(1.0, 53 - E), u = ldexp(1.0, E - 53);
        const double sT = T < 0.0 ? -1.0 : 1.0, scale = sT * inv_u;
        double D = 0.0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const double ya = vt[i] * scale, qa = floor(ya);
            const double yb = vl[i] * scale, qb = floor(yb);
            D += (qa + (ya - qa > 0.5 ? 1.0 : 0.0)) + (qb + (yb - qb > 0.5 ? 1.0 : 0.0));
        }
        if (lane < b) D = 0.0;
        const double ex = wave_incl_sum(D) - D;
        if (lane >= b) tin = lane == b ? T : sT * ((fabs(T) * inv_u + ex) * u);
        double t = tin;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            t = t + vt[i];
            t = t + vl[i];
            tj[i] = t;
        }
        const double prev = dpp_wave_shr1(t);
        const unsigned long long bm = __ballot(lane > b && dbits(tin) != dbits(prev));
        if (!bm) {
            ok = true;
            break;
        }
        n_fix++;
        b = __ffsll((long long)bm) - 1;
        T = rl_d(t, b - 1);
    }
    if (!ok) {  // lane by lane from lane b (rare: repeated ties or binade changes)
        for (int l = b; l < 64; l++) {
            if (lane == l) {
                double t = T;
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    t = t + vt[i];
                    t = t + vl[i];
                    tj[i] = t;
                }
            }
            T = rl_d(tj[3], l);
        }
    }
}

__device__ __forceinline__ double pick4(const double (&v)[4], int k) {
    return k == 0 ? v[0] : k == 1 ? v[1] : k == 2 ? v[2] : v[3];
}
__device__ __forceinline__ int64_t pick4(const int64_t (&v)[4], int k) {
    return k == 0 ? v[0] : k == 1 ? v[1] : k == 2 ? v[2] : v[3];
}
__device__ __forceinline__ int pick4(const int (&v)[4], int k) {
    return k == 0 ? v[0] : k == 1 ? v[1] : k == 2 ? v[2] : v[3];
}

// the slide (GROM.c:19492-19545), 256 steps per round (lane l: steps 4l..4l+3);
// the inputs are loaded three rounds ahead.  Stops before a round that would
// start at or past `cap` and returns false (s then resumes exactly there).
template <int KIND>
__device__ bool slide_run(const WalkIn &W, SlideState &s, int64_t cap) {
    if (!s.sliding) return true;
    const int lane = threadIdx.x & 63;
    const int64_t L = W.L;
    const double sgn = KIND == 0 ? 1.0 : -1.0;
    const double wsdL = W.wsd[L];
    int64_t pa = s.pa, cnt = s.cnt, last_good = s.last_good, ce = s.ce;
    double tot = s.tot;
    // the largest good ratio per lane; max is exact and order-free, so the
    // wave's maximum is taken once, when the slide ends or pauses.  Kept as
    // the step's (tot, divisor) with the largest exact quotient (compared by
    // exact cross products, two-product FMAs) and divided once at the end:
    // rounding is monotonic, so RN of the largest quotient is the largest of
    // the reference's RN(tot / divisor), without a division per good step
    // (the division was most of the slide's work after the sum chain)
    double bt = 0.0, bd = 1.0;
    bool bany = false;
    int mqi = s.mqi, mqb = s.mqb;
    bool finished = true;
    const long long ck_start = W.stats ? clock64() : 0;
    long long pc_chain = 0, pc_before = 0, pc_after = 0, pc_rounds = 0;
    unsigned long long n_fix = 0;
    struct In {
        uint32_t ba[4], bb[4];
        double za[4], zb[4];
    };
    // unconditional loads from a clamped index (q - L >= 0 here); no select
    // on the loaded values (that would wait for them): the round masks steps
    // past the end itself
    auto load = [&](int64_t at, In &o) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int64_t q0 = at + 4 * lane + i;
            const int64_t q = q0 < W.len ? q0 : W.len - 1;
            o.ba[i] = W.wb[q];
            o.bb[i] = W.wb[q - L];
            o.za[i] = W.sd[q];
            o.zb[i] = W.sd[q - L];
        }
    };
    auto round = [&](const In &in) -> bool {
        if (pa >= cap) { finished = false; return false; }
        const long long ckt = W.stats ? clock64() : 0;
        const int64_t p0 = pa + 4 * lane;
        bool inl[4];
        int ct[4], cl[4], lt = -1, ll = -1;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            inl[i] = p0 + i < W.len;
            ct[i] = inl[i] ? cdef(in.bb[i]) : -1;
            cl[i] = inl[i] ? cdef(in.ba[i]) : -1;
            lt = ct[i] >= 0 ? ct[i] : lt;
            ll = cl[i] >= 0 ? cl[i] : ll;
        }
        int mt_c = lane_last_excl(lt, mqb), ml_c = lane_last_excl(ll, mqi);
        int mt[4], ml[4], nqt = 0, nql = 0;
        bool qt[4], ql[4];
        double vt[4], vl[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            mt_c = ct[i] >= 0 ? ct[i] : mt_c;
            ml_c = cl[i] >= 0 ? cl[i] : ml_c;
            mt[i] = mt_c;
            ml[i] = ml_c;
            qt[i] = inl[i] && !(in.bb[i] & B_LOW) && (in.bb[i] & (B_W0 << mt_c));
            ql[i] = inl[i] && !(in.ba[i] & B_LOW) && (in.ba[i] & (B_W0 << ml_c));
            vt[i] = qt[i] ? -sgn * in.zb[i] : 0.0;
            vl[i] = ql[i] ? sgn * in.za[i] : 0.0;
            nqt += qt[i];
            nql += ql[i];
        }
        int tot_l, tot_t;
        int64_t run = cnt + excl_small(nql, tot_l) - excl_small(nqt, tot_t);
        int64_t cj[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            run += (int)ql[i] - (int)qt[i];
            cj[i] = run;
        }
        const long long ck0 = W.stats ? clock64() : 0;
        double tj[4];
        chain_round4(tot, vt, vl, tj, n_fix);
        const long long ck1 = W.stats ? clock64() : 0;
        pc_chain += ck1 - ck0;
        pc_before += ck0 - ckt;
        bool good[4];
        double dv[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            dv[i] = cj[i] * wsdL;  // (the reference's divisor, rounded as it is)
            good[i] = inl[i] && cj[i] > 0 && wsdL > 0 && ratio_ge_min(tj[i], dv[i]) && LOW_FRAC_OK;
        }
        // the loop test of step j (GROM.c:19492) sees the last good step
        // before it; no step of the round can fail it while pa + 255 is
        // within MAX_DIST of last_good (the common case: skip the scan)
        int fi = 4;  // this lane's first step that fails the loop test
        if (pa + 255 - last_good > MAX_DIST_LAST_GOOD) {
            int lg = -1;
#pragma unroll
            for (int i = 0; i < 4; i++) lg = good[i] ? 4 * lane + i : lg;
            const unsigned long long d = __ballot(lg >= 0) & ((1ull << lane) - 1);
            const int src = d ? 63 - __clzll(d) : 0;
            const int lgv = __shfl(lg, src);
            int64_t lgb = d ? pa + lgv : last_good;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                if (fi == 4 && !(inl[i] && (p0 + i - lgb) <= MAX_DIST_LAST_GOOD)) fi = i;
                if (good[i]) lgb = p0 + i;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 4; i++)
                if (fi == 4 && !inl[i]) fi = i;
        }
        const unsigned long long sm = __ballot(fi < 4);
        const int fl_ = sm ? __ffsll((long long)sm) - 1 : 64;
        const int js = sm ? 4 * fl_ + __builtin_amdgcn_readlane(fi, fl_) : 256;
        int eg_last = -1;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const bool eg = good[i] && 4 * lane + i < js;
            eg_last = eg ? 4 * lane + i : eg_last;
            // tj / dv > bt / bd  <=>  tj * bd > bt * dv (both divisors > 0), exactly
            const double p1 = tj[i] * bd, e1 = fma(tj[i], bd, -p1);
            const double p2 = bt * dv[i], e2 = fma(bt, dv[i], -p2);
            const bool gt = !bany || p1 > p2 || (p1 == p2 && e1 > e2);
            if (eg && gt) {
                bt = tj[i];
                bd = dv[i];
                bany = true;
            }
        }
        const unsigned long long gm = __ballot(eg_last >= 0);
        if (gm) last_good = ce = pa + __builtin_amdgcn_readlane(eg_last, 63 - __clzll(gm));
        if (js > 0) {
            const int l = (js - 1) >> 2, k = (js - 1) & 3;
            tot = rl_d(pick4(tj, k), l);
            cnt = rl_i64(pick4(cj, k), l);
            mqi = __builtin_amdgcn_readlane(pick4(ml, k), l);
            mqb = __builtin_amdgcn_readlane(pick4(mt, k), l);
        }
        pa += js;
        pc_rounds++;
        if (W.stats) pc_after += clock64() - ck1;
        return js == 256;
    };
    // three rounds of inputs in flight
    In b0, b1, b2;
    load(pa, b0);
    load(pa + 256, b1);
    load(pa + 512, b2);
    for (;;) {
        if (!round(b0)) break;
        load(pa + 512, b0);
        if (!round(b1)) break;
        load(pa + 512, b1);
        if (!round(b2)) break;
        load(pa + 512, b2);
    }
    if (W.stats && lane == 0) {
        atomicAdd(W.prof + 1, (unsigned long long)(clock64() - ck_start));
        atomicAdd(W.prof + 0, (unsigned long long)pc_chain);
        atomicAdd(W.prof + 2, (unsigned long long)pc_before);
        atomicAdd(W.prof + 3, (unsigned long long)pc_after);
        atomicAdd(W.prof + 5, n_fix);
        atomicAdd(W.stats + 2, (unsigned long long)pc_rounds);
    }
    s.pa = pa;
    s.cnt = cnt;
    s.last_good = last_good;
    s.ce = ce;
    s.tot = tot;
    const double lmax = bany ? bt / bd : 0.0;
    const double mx = dpp_max_pos(lmax);  // ratios are >= 3 > 0; lanes without one hold 0
    if (mx > s.stdevs) s.stdevs = mx;
    s.mqi = mqi;
    s.mqb = mqb;
    s.sliding = finished ? 0 : 1;
    return finished;
}

// phase D: trim the end back (GROM.c:19550-19600), 64 words (4096 bases) per
// round, one word per lane (lane i: the i-th word below the top).  Its two
// scans are searches over bit masks:
//  - the outer one steps down from the end while a base does not pass; the
//    class it tests with is carried down over EVERY base (low ones included)
//    and a low base may pass;
//  - the inner one, from a passing base q, counts nonlow bases (c3) and
//    passing ones (c2) downward -- the class carried over nonlow bases only --
//    and stops at the first base where c3 == 0 or 2*c2 < c3: the first passage
//    of the walk +1 (pass) / -1 (nonlow, not passing) to -1, or q itself when
//    q is low.  The outer class carry does not follow the inner scan: after a
//    stop the outer scan resumes with the class it had at q (as the
//    reference's separate mqi/mqa variables do).
__device__ __forceinline__ uint64_t word_range_mask(int64_t w, int64_t lo, int64_t hi) {
    const int64_t a = max(lo, w * 64), b = min(hi, w * 64 + 63);
    if (a > b) return 0;
    return low_bits((int)(b - a + 1)) << (a - w * 64);
}

// class-1 mask of a word: each base takes the class of the nearest defining
// base at or above it (def/c1: defining bases and their class-1 bits, within
// the valid mask), else the carry from above
__device__ __forceinline__ uint64_t class1_fill_down(uint64_t def, uint64_t c1, int carry) {
    uint64_t have = def, val = c1 & def;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        val |= (val >> d) & ~have;
        have |= have >> d;
    }
    return val | (carry == 1 ? ~have : 0ull);
}

// the class each lane's word starts from (the carry from the words above it
// in this round) and the carry below the round; e: the class of the lane's
// lowest defining base, -1 none
__device__ __forceinline__ int round_carry(int e, int carry_in, int &carry_out) {
    const unsigned long long d = __ballot(e >= 0), c1 = __ballot(e == 1);
    carry_out = d ? (int)((c1 >> (63 - __clzll(d))) & 1ull) : carry_in;
    return lane_last_excl(e, carry_in);
}

template <int KIND>
__device__ void trim_end(const WalkIn &W, const SlideState &s, int64_t &ce_out, double &stdevs_out) {
    const int lane = threadIdx.x & 63;
    const int64_t lim = s.pos + W.min_len;  // both scans run while the position is > lim
    int64_t ce = s.ce, p = ce;
    int mq = s.mqi;
    int64_t rounds = 0;
    while (p > lim) {
        // outer scan: the first base q <= p (q > lim) that passes
        int64_t q = lim;
        int cq = mq;
        {
            int64_t top = p;
            int carry = mq;
            while (top > lim) {
                rounds++;
                const int64_t w = (top >> 6) - lane;
                const uint64_t vm = w >= 0 ? word_range_mask(w, lim + 1, top) : 0ull;
                const uint64_t dfa = vm ? W.t_defa[w] & vm : 0ull, c1a = vm ? W.t_c1a[w] : 0ull;
                const int e = dfa ? (int)((c1a >> (__ffsll((long long)dfa) - 1)) & 1ull) : -1;
                int cout;
                const int cl = round_carry(e, carry, cout);
                const uint64_t cm = class1_fill_down(dfa, c1a, cl);
                const uint64_t pass = vm ? ((W.t_pa0[w] & ~cm) | (W.t_pa1[w] & cm)) & vm : 0ull;
                const unsigned long long fm = __ballot(pass != 0);
                if (fm) {
                    const int f = __ffsll((long long)fm) - 1;
                    const int bit = 63 - __clzll(pass);
                    const int64_t qq = w * 64 + bit;
                    q = __builtin_amdgcn_readlane((int)(uint32_t)qq, f) |
                        ((int64_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)qq >> 32), f) << 32);
                    cq = __builtin_amdgcn_readlane((int)((cm >> bit) & 1ull), f);
                    break;
                }
                carry = cout;
                top = ((top >> 6) - 63) * 64 - 1;
            }
        }
        if (q <= lim) {  // nothing passes down to the limit: the end steps all the way down
            ce = lim;
            break;
        }
        ce = q;
        mq = cq;
        // inner scan from q
        int64_t x = lim;  // the stop base, lim: none
        if (!(W.t_nl[q >> 6] >> (q & 63) & 1ull)) {
            x = q;  // q is low: c3 == 0 at once
        } else {
            int64_t top = q;
            int carry = cq, level = 0;
            while (top > lim) {
                rounds++;
                const int64_t w = (top >> 6) - lane;
                const uint64_t vm = w >= 0 ? word_range_mask(w, lim + 1, top) : 0ull;
                const uint64_t dfn = vm ? W.t_defn[w] & vm : 0ull, c1n = vm ? W.t_c1n[w] : 0ull;
                const int e = dfn ? (int)((c1n >> (__ffsll((long long)dfn) - 1)) & 1ull) : -1;
                int cout;
                const int cl = round_carry(e, carry, cout);
                const uint64_t cm = class1_fill_down(dfn, c1n, cl);
                const uint64_t nl = vm ? W.t_nl[w] & vm : 0ull;
                const uint64_t up = vm ? ((W.t_pn0[w] & ~cm) | (W.t_pn1[w] & cm)) & vm : 0ull;
                const uint64_t down = nl & ~up;
                // this word's walk from its top bit down: net change and lowest prefix
                int rel = 0, mn = 0;
                for (uint64_t m = up | down; m; ) {
                    const int bit = 63 - __clzll(m);
                    m &= ~(1ull << bit);
                    rel += (up >> bit) & 1ull ? 1 : -1;
                    mn = min(mn, rel);
                }
                // each lane's starting level: the levels of the words above it
                int ex = rel;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const int t = __shfl_up(ex, d);
                    if (lane >= d) ex += t;
                }
                ex -= rel;
                const int start = level + ex;
                const unsigned long long hit = __ballot(vm != 0 && start + mn <= -1);
                if (hit) {
                    const int f = __ffsll((long long)hit) - 1;
                    int64_t xx = 0;
                    if (lane == f) {  // the first base of this word where the level reaches -1
                        int lv = start;
                        for (uint64_t m = up | down; m; ) {
                            const int bit = 63 - __clzll(m);
                            m &= ~(1ull << bit);
                            lv += (up >> bit) & 1ull ? 1 : -1;
                            if (lv <= -1) { xx = w * 64 + bit; break; }
                        }
                    }
                    x = __builtin_amdgcn_readlane((int)(uint32_t)xx, f) |
                        ((int64_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)xx >> 32), f) << 32);
                    break;
                }
                int tot_rel = rel;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) tot_rel += __shfl_xor(tot_rel, o);
                level += tot_rel;
                carry = cout;
                top = ((top >> 6) - 63) * 64 - 1;
            }
        }
        if (x > lim) {
            ce = x - 1;
            p = x - 1;
        } else {
            p = lim;
        }
    }
    if (W.stats && lane == 0) atomicAdd(W.stats + 3, (unsigned long long)rounds);
    ce_out = ce;
    stdevs_out = s.stdevs;
}

template <int KIND>
__device__ void phase_cd_wave(const WalkIn &W, int64_t pos, const PreAB &r, int64_t &ce_out, double &stdevs_out) {
    SlideState s = slide_begin<KIND>(W, pos, r, 0);
    slide_run<KIND>(W, s, INT64_MAX);
    trim_end<KIND>(W, s, ce_out, stdevs_out);
}

struct GAcc {  // direct loads (one lane per base)
    const uint16_t *wb;
    const double *sd;
    __device__ __forceinline__ uint32_t bits(int64_t p) const { return wb[p]; }
    __device__ __forceinline__ double z(int64_t p) const { return sd[p]; }
};

// The bases (and classes) the walk can meet that pass the threshold,
// compacted (wave-aggregated append); nxt[m][p] = p (no-op) everywhere else.
template <int KIND>
__global__ __launch_bounds__(256) void k_cnv_cand(WalkIn W, int32_t *__restrict__ nxt, int64_t *__restrict__ cand,
                                                  uint32_t *n_cand, uint32_t cap) {
    __shared__ uint32_t wcnt[8], wbase[8], gbase;
    const int64_t p = W.start + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = p < W.end;
    const uint32_t b = in ? (uint32_t)W.wb[p] : 0u;
    const uint32_t pb0 = KIND == 0 ? B_DEL0 : B_DUP0;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    bool want[2];
    for (int m = 0; m < 2; m++) {
        const bool reach = (b & B_HI) ? m == 0 : (b & B_RTP) ? m == 1 : true;  // classes the walk can be in here
        want[m] = in && reach && (b & (pb0 << m));
        if (in) nxt[m * W.len + p] = (int32_t)p;
    }
    // one global atomic per block: wave ballots, then the block's 8 (wave, m) counts
    const unsigned long long m0 = __ballot(want[0]), m1 = __ballot(want[1]);
    if (lane == 0) {
        wcnt[wv * 2] = (uint32_t)__popcll(m0);
        wcnt[wv * 2 + 1] = (uint32_t)__popcll(m1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int i = 0; i < 8; i++) { wbase[i] = t; t += wcnt[i]; }
        gbase = t ? atomicAdd(n_cand, t) : 0;
    }
    __syncthreads();
    const unsigned long long below = (1ull << lane) - 1;
    if (want[0]) {
        const uint32_t k = gbase + wbase[wv * 2] + (uint32_t)__popcll(m0 & below);
        if (k < cap) cand[k] = (p << 1);
    }
    if (want[1]) {
        const uint32_t k = gbase + wbase[wv * 2 + 1] + (uint32_t)__popcll(m1 & below);
        if (k < cap) cand[k] = (p << 1) | 1;
    }
}

// a candidate's first two phases: nxt[m][p] = the position the walk continues
// from (before its +1), or -(k+2) for a call whose record pre[k] the walk
// completes (phases C, D)
// nxt value of a candidate whose phase B ran past the precompute budget: the
// walk computes it (phase_ab_wave) if it gets there
constexpr int32_t NXT_UNDECIDED = INT32_MIN;

template <int KIND>
__global__ void k_cnv_pre(WalkIn W, const int64_t *__restrict__ cand, uint32_t n_cand, int32_t *__restrict__ nxt,
                          PreAB *__restrict__ pre, uint32_t *n_pre, uint32_t cap, int64_t *__restrict__ pre_pos,
                          int64_t max_steps) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_cand) return;
    const int64_t p = cand[i] >> 1;
    const int m = (int)(cand[i] & 1);
    GAcc c{W.wb, W.sd};
    bool capped = false;
    PreAB r = phase_ab<KIND>(c, W, p, m, max_steps, &capped);
    int32_t out = (int32_t)p;
    if (capped) {
        out = NXT_UNDECIDED;
    } else if (r.begin == 1) {
        uint32_t k = atomicAdd(n_pre, 1u);
        if (k < cap) {
            r.done = 0;
            pre[k] = r;
            pre_pos[k] = p;
            out = -(int32_t)k - 2;
        }  // else: overflow, the host re-runs with a larger buffer
    } else if (r.stop == 1) {
        out = (int32_t)r.temp_pos;
    }
    nxt[m * W.len + p] = out;
}

// phases C and D for every call start found by k_cnv_pre, one lane each,
// capped so that long copy-number regions leave their few visited calls to
// the walk
template <int KIND>
__global__ void k_cnv_post(WalkIn W, PreAB *__restrict__ pre, const uint32_t *n_pre, uint32_t cap,
                           const int64_t *__restrict__ pre_pos, int64_t max_steps, uint32_t *n_left) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= min(*n_pre, cap)) return;
    GAcc a{W.wb, W.sd}, t{W.wb, W.sd};
    PreAB r = pre[i];
    int64_t ce;
    double sdv;
    if (phase_cd<KIND>(a, t, W, pre_pos[i], r, max_steps, ce, sdv)) {
        pre[i].ce_final = ce;
        pre[i].stdevs_final = sdv;
        pre[i].done = 1;
    } else {
        atomicAdd(n_left, 1u);
    }
}

template <int KIND>
struct Walk {
    WalkIn W;
    Win c;
    const int32_t *nxt;
    const PreAB *pre;
    // vis: the marks an earlier walk left (merge checks), or null; the window
    // then reads the bit words in its place (any readable bytes: the marks
    // are only looked at with merge checks on)
    __device__ Walk(const WalkIn &w, const uint8_t *vis, const int32_t *nx, const PreAB *pr) : W(w), nxt(nx), pre(pr) {
        c.wb = w.wb;
        c.sd = w.sd;
        c.vis = vis ? vis : (const uint8_t *)w.wb;
        c.nxt = nx;
        c.len = w.len;
        c.base = INT64_MIN / 4;
    }
    __device__ __forceinline__ bool pass(uint32_t b, int m) const {
        return (b & ((KIND == 0 ? B_DEL0 : B_DUP0) << m)) != 0;
    }
    __device__ __forceinline__ void add(double &x, double v) const { if (KIND == 0) x += v; else x -= v; }
    __device__ __forceinline__ void sub(double &x, double v) const { if (KIND == 0) x -= v; else x += v; }
    // mq >= -q -> class 0, else depth > 0 -> class 1, else unchanged
    __device__ __forceinline__ static int cls(uint32_t b, int m) { return (b & B_HI) ? 0 : (b & B_RTP) ? 1 : m; }
    // update at a visited base; returns the class (== the state after it)
    __device__ __forceinline__ int visit(int64_t pos, int &last) {
        last = cls(c.bits(pos), last);
        return last;
    }
    // the reference's `if` body at a base that passes the threshold: phases A
    // and B come precomputed; a call is completed here (phase C: the sliding
    // extension past L, phase D: trimming the end).  Returns the position the
    // walk continues from (before its `pos += 1`), or -1 when the slide
    // reached `cap` and paused (its state in *ps).
    __device__ int64_t block(int64_t pos, int mqi, int32_t n, CallRec &call, bool &is_call, int64_t cap,
                             SlideState *ps) {
        PreAB r;
        if (n == NXT_UNDECIDED) {  // phases A/B were not precomputed (long region): the wave runs them
            if (W.stats && (threadIdx.x & 63) == 0) atomicAdd(W.stats + 0, 1ull);
            r = phase_ab_wave<KIND>(W, pos, mqi);
            is_call = r.begin == 1;
            if (!is_call) return r.stop == 1 ? r.temp_pos : pos;
        } else {
            is_call = n < -1;
            if (!is_call) return n;
            r = pre[-n - 2];
        }
        int64_t ce;
        double sdv;
        if (r.done == 1) {
            ce = r.ce_final;
            sdv = r.stdevs_final;
        } else {
            if (W.stats && (threadIdx.x & 63) == 0) atomicAdd(W.stats + 1, 1ull);
            SlideState s = slide_begin<KIND>(W, pos, r, mqi);
            if (!slide_run<KIND>(W, s, cap)) {
                *ps = s;
                is_call = false;
                return -1;
            }
            trim_end<KIND>(W, s, ce, sdv);
        }
        call.p = pos;
        call.ce = ce;
        call.stdevs = sdv;
        return ce + 1;
    }
};

struct ChunkState {
    int64_t x1;  // W1 exit position
    int64_t x2;  // W2/W3 exit position (NOMERGE / redone chunks)
    int32_t l1, l2, status, pad;
};
enum { ST_MERGED = 0, ST_NOMERGE = 1, ST_PASSTHRU = 2, ST_FIRST = 3, ST_PENDING = 4 };

__device__ __forceinline__ void emit_call(const CallRec &c, int m, CallRec *calls, uint32_t *n_calls, uint32_t cap) {
    if ((threadIdx.x & 63) == 0) {
        uint32_t k = atomicAdd(n_calls, 1u);
        if (k < cap) {
            calls[k] = c;
            calls[k].m = m;
        }
    }
}

// The walk from (pos, last) while pos < lim.  Bases that do not pass the
// threshold only update the class state, so the wave fast-forwards over them
// 64 at a time: lane i takes base+i, the class each base sees is a
// last-value scan over the window, and a ballot finds the first base that
// passes (or, with merge_check, whose mark from an earlier walk equals its
// class -- from there both walks are identical).  Marks are stored
// coalesced; calls are completed serially (Walk::block).  Returns the exit
// position; *merge = the merge base or -1.  With a `pend` record, a call
// whose slide reaches `slide_cap` pauses the walk: the slide state goes to
// *pend, *paused is set and the call base is returned.
template <int KIND>
__device__ int64_t walk_run(Walk<KIND> &w, int64_t pos, int &last, int64_t lim, uint8_t *vis_out, bool merge_check,
                            int64_t *merge, CallRec *calls, uint32_t *n_calls, uint32_t cap, bool emit,
                            int64_t slide_cap = INT64_MAX, SlideState *pend = nullptr, bool *paused = nullptr) {
    const int lane = threadIdx.x & 63;
    *merge = -1;
    while (pos < lim) {
        const int i0 = w.c.slot(pos);
        const int64_t base = w.c.base;
        const int limi = (int)min<int64_t>(64, lim - base);
        const bool in = lane >= i0 && lane < limi;
        const uint32_t b = w.c.r.b;
        const int e = in ? ((b & B_HI) ? 0 : (b & B_RTP) ? 1 : -1) : -1;
        const int mi = wave_last_incl(e, last);
        // a base that passes but whose window search neither jumps nor calls
        // (nxt == p) continues the walk exactly like one that does not pass
        const int32_t nmi = mi == 0 ? w.c.r.n0 : w.c.r.n1;
        const bool ps = in && w.pass(b, mi) && (int64_t)nmi != base + lane;
        const bool mg = merge_check && in && w.c.r.v == (uint32_t)(1 + mi);
        const unsigned long long stop_m = __ballot(ps || mg);
        const unsigned long long mg_m = __ballot(mg);
        const int j = stop_m ? __ffsll((long long)stop_m) - 1 : limi - 1;
        const bool merged_here = stop_m && ((mg_m >> j) & 1ull);
        if (vis_out && in && lane <= j && !(merged_here && lane == j)) vis_out[base + lane] = (uint8_t)(1 + mi);
        last = __builtin_amdgcn_readlane(mi, j);
        if (!stop_m) {
            pos = base + limi;
            continue;
        }
        pos = base + j;
        if (merged_here) {
            *merge = pos;
            return pos;
        }
        const int32_t n = __builtin_amdgcn_readlane(last == 0 ? w.c.r.n0 : w.c.r.n1, j);
        if (w.W.stats && lane == 0) atomicAdd(w.W.stats + 4, 1ull);
        CallRec c;
        bool is_call = false;
        SlideState sst;
        const int64_t nx = w.block(pos, last, n, c, is_call, pend ? slide_cap : INT64_MAX, &sst);
        if (nx < 0) {
            if (lane == 0) *pend = sst;
            *paused = true;
            return pos;
        }
        pos = nx;
        if (is_call && emit) emit_call(c, last, calls, n_calls, cap);
        pos += 1;
    }
    return pos;
}

// One wave per chunk.  mode 0: speculative first pass from (chunk start,
// class 0) -- exact for chunk 0 -- leaving marks vis[p] = 1 + class at every
// visited base and the calls it finds; mode 1: reconciliation of chunk k from
// chunk k-1's speculative exit up to the first base both walks visit in the
// same state (from there the walks are identical).
template <int KIND>
__global__ __launch_bounds__(64) void k_cnv_walk(WalkIn W, const int32_t *nxt, const PreAB *pre, int mode,
                                                 int64_t n_chunks, int64_t chunk, uint8_t *__restrict__ vis,
                                                 ChunkState *__restrict__ cs, SlideState *pend, CallRec *calls,
                                                 uint32_t *n_calls, uint32_t cap) {
    const int64_t k = blockIdx.x;
    if (k >= n_chunks) return;
    if (mode == 1 && W.stats) W.stats += 5;  // counters per mode (GROM_TIMING)
    const int64_t c0 = W.start + k * chunk, c1 = min(W.end, c0 + chunk);
    int64_t merge;
    if (mode == 0) {
        Walk<KIND> w(W, nullptr, nxt, pre);
        int last = 0;  // exact for chunk 0 (GROM.c:19366-19367), a guess elsewhere
        bool paused = false;
        const int64_t pos = walk_run<KIND>(w, c0, last, c1, vis, false, &merge, calls, n_calls, cap, true,
                                           c1 + chunk, pend + k, &paused);
        if ((threadIdx.x & 63) == 0) {
            cs[k].x1 = pos;
            cs[k].l1 = last;
            cs[k].status = paused ? ST_PENDING : k == 0 ? ST_FIRST : ST_MERGED;
        }
        return;
    }
    if (k == 0) return;
    const int64_t x = cs[k - 1].x1;
    const int l = cs[k - 1].l1;
    if (x >= c1) {  // chunk k lies inside a jump of chunk k-1
        for (int64_t p = c0 + (threadIdx.x & 63); p < c1; p += 64) vis[p] = 0;
        if ((threadIdx.x & 63) == 0) cs[k].status = ST_PASSTHRU;
        return;
    }
    {  // pass 1: find the merge base
        Walk<KIND> w(W, vis, nxt, pre);
        int last = l;
        walk_run<KIND>(w, x, last, c1, nullptr, true, &merge, calls, n_calls, cap, false);
    }
    const int64_t stop_at = merge >= 0 ? merge : c1;
    for (int64_t p = c0 + (threadIdx.x & 63); p < stop_at; p += 64) vis[p] = 0;
    __syncthreads();
    // pass 2: the true walk up to the merge base, with marks and calls
    Walk<KIND> w(W, nullptr, nxt, pre);
    int last = l;
    int64_t m2;
    const int64_t pos = walk_run<KIND>(w, x, last, stop_at, vis, false, &m2, calls, n_calls, cap, true);
    if ((threadIdx.x & 63) == 0) {
        if (merge >= 0) {
            cs[k].status = ST_MERGED;
        } else {
            cs[k].status = ST_NOMERGE;
            cs[k].x2 = pos;
            cs[k].l2 = last;
        }
    }
}

// Paused slides.  A speculative chunk that starts inside a long copy-number
// region finds a call there whose slide runs to the region's end; every chunk
// of the region would slide to the same end, of which only the first one's
// walk is on the true path.  So mode 0 pauses a slide that passes the next
// chunk (ST_PENDING, state in pend[k]), and the host resumes, round by round,
// only the pending chunks whose predecessor has a known exit that does not
// jump over them (the others take that exit: the true walk passes them).
// The resumed walk finishes the call, emits it and walks on to the chunk's
// end as mode 0 would (it may pause again at a later call).
template <int KIND>
__global__ __launch_bounds__(64) void k_cnv_walk_resume(WalkIn W, const int32_t *nxt, const PreAB *pre,
                                                        const int32_t *__restrict__ list, int64_t chunk,
                                                        uint8_t *__restrict__ vis, ChunkState *__restrict__ cs,
                                                        SlideState *pend, CallRec *calls, uint32_t *n_calls,
                                                        uint32_t cap) {
    const int64_t k = list[blockIdx.x];
    const int64_t c0 = W.start + k * chunk, c1 = min(W.end, c0 + chunk);
    if (W.stats) W.stats += 15;  // the resumed walks' own counters (GROM_TIMING)
    const long long kk0 = W.stats ? clock64() : 0;
    SlideState s = pend[k];
    __syncthreads();  // every lane has read the record before lane 0 may write a new one
    const int64_t pa0 = s.pa;
    const uint64_t t0 = W.stats ? wall_clock64() : 0;
    const long long k0 = W.stats ? clock64() : 0;
    slide_run<KIND>(W, s, INT64_MAX);
    if (W.stats && (threadIdx.x & 63) == 0) {  // the longest resumed slide: steps, wall-clock ticks, clocks
        atomicMax(W.stats + 5, (unsigned long long)(s.pa - pa0));  // slots 20, 21 of the counters
        atomicMax(W.stats + 6, (unsigned long long)(wall_clock64() - t0));
        atomicMax(W.prof + 4, (unsigned long long)(clock64() - k0));
    }
    int64_t ce;
    double sdv;
    const long long kk1 = W.stats ? clock64() : 0;
    trim_end<KIND>(W, s, ce, sdv);
    CallRec c;
    c.p = s.pos;
    c.ce = ce;
    c.stdevs = sdv;
    emit_call(c, s.m, calls, n_calls, cap);
    Walk<KIND> w(W, nullptr, nxt, pre);
    int last = s.m;
    int64_t merge;
    bool paused = false;
    const long long kk2 = W.stats ? clock64() : 0;
    const int64_t pos = walk_run<KIND>(w, ce + 1, last, c1, vis, false, &merge, calls, n_calls, cap, true,
                                       c1 + chunk, pend + k, &paused);
    if (W.stats && (threadIdx.x & 63) == 0) {  // the longest resumed wave: whole, trim, walk on
        const long long kk3 = clock64();
        atomicMax(W.prof + 6, (unsigned long long)(kk3 - kk0));
        atomicMax(W.prof + 7, (unsigned long long)(kk2 - kk1));
        atomicMax(W.prof + 8, (unsigned long long)(kk3 - kk2));
    }
    if ((threadIdx.x & 63) == 0) {
        cs[k].x1 = pos;
        cs[k].l1 = last;
        cs[k].status = paused ? ST_PENDING : k == 0 ? ST_FIRST : ST_MERGED;
    }
}

// repair of one chunk from a known-true entry (x, l): like mode 1, it walks
// until it meets a base that an earlier walk of this chunk visited in the
// same state (from there that walk's marks, calls and exit hold) and reports
// in cs[k].status whether it met one (ST_MERGED) or walked the chunk to its
// end (ST_NOMERGE, exit in x2/l2)
template <int KIND>
__device__ __forceinline__ void walk_fix(WalkIn W, const int32_t *nxt, const PreAB *pre, int64_t k, int64_t chunk,
                                         int64_t x, int l, uint8_t *__restrict__ vis, ChunkState *__restrict__ cs,
                                         CallRec *calls, uint32_t *n_calls, uint32_t cap);

template <int KIND>
__global__ __launch_bounds__(64) void k_cnv_walk_fix(WalkIn W, const int32_t *nxt, const PreAB *pre, int64_t k,
                                                     int64_t chunk, int64_t x, int l, uint8_t *__restrict__ vis,
                                                     ChunkState *__restrict__ cs, CallRec *calls, uint32_t *n_calls,
                                                     uint32_t cap) {
    walk_fix<KIND>(W, nxt, pre, k, chunk, x, l, vis, cs, calls, n_calls, cap);
}

// The reconcile of the chunked walk on the device (one wave): the true exit
// of each chunk in order -- GROM.c's walk is one pass -- repairing (walk_fix)
// a chunk whose speculative entry was wrong and marking the chunks the true
// walk jumps over (skipped[k] = 1).  The host reconcile it replaces read every
// chunk state back and waited for each repair; here one launch does them all.
template <int KIND>
__global__ __launch_bounds__(64) void k_cnv_reconcile(WalkIn W, const int32_t *nxt, const PreAB *pre, int64_t n_ch,
                                                      int64_t chunk, uint8_t *__restrict__ vis,
                                                      ChunkState *__restrict__ cs, CallRec *calls, uint32_t *n_calls,
                                                      uint32_t cap, uint8_t *__restrict__ skipped,
                                                      uint32_t *__restrict__ n_fix) {
    // the chunk states come in batches of 64, one load per lane (a serial
    // load per chunk made the launch ~6 ms on a 250 Mb chromosome); a repair
    // rewrites only its own chunk's state, which is read again after it
    __shared__ ChunkState s_prev, s_cur, s_bat[64];
    if (threadIdx.x == 0) s_prev = cs[0];
    for (int64_t k = threadIdx.x; k < n_ch; k += 64) skipped[k] = 0;
    __syncthreads();
    ChunkState prev = s_prev;
    int64_t tx = prev.x1;
    int tl = prev.l1;
    uint32_t fixes = 0;
    for (int64_t k = 1; k < n_ch; k++) {
        if (((k - 1) & 63) == 0) {  // the next batch: chunks k .. k + 63
            __syncthreads();
            if (k + threadIdx.x < n_ch) s_bat[threadIdx.x] = cs[k + threadIdx.x];
            __syncthreads();
        }
        const ChunkState h = s_bat[(k - 1) & 63], hp = prev;
        prev = h;  // (chunk k's state before any repair of it)
        const bool entry_ok = tx == hp.x1 && tl == hp.l1;
        const int64_t c0 = W.start + k * chunk, c1 = min(W.end, c0 + chunk);
        const int64_t ex = h.status == ST_NOMERGE ? h.x2 : h.x1;
        const int el = h.status == ST_NOMERGE ? h.l2 : h.l1;
        if (entry_ok && h.status != ST_PASSTHRU) { tx = ex; tl = el; continue; }
        if (tx >= c1) {  // the true walk jumps over this chunk
            if (threadIdx.x == 0) skipped[k] = 1;
            continue;
        }
        walk_fix<KIND>(W, nxt, pre, k, chunk, tx, tl, vis, cs, calls, n_calls, cap);
        fixes++;
        __threadfence_block();
        __syncthreads();
        if (threadIdx.x == 0) s_cur = cs[k];
        __syncthreads();
        const ChunkState one = s_cur;
        __syncthreads();
        if (one.status == ST_MERGED && h.status != ST_PASSTHRU) { tx = ex; tl = el; }
        else { tx = one.x2; tl = one.l2; }
    }
    if (threadIdx.x == 0) *n_fix = fixes;
}

template <int KIND>
__device__ __forceinline__ void walk_fix(WalkIn W, const int32_t *nxt, const PreAB *pre, int64_t k, int64_t chunk,
                                         int64_t x, int l, uint8_t *__restrict__ vis, ChunkState *__restrict__ cs,
                                         CallRec *calls, uint32_t *n_calls, uint32_t cap) {
    if (W.stats) W.stats += 10;  // the repair walks' own counters (GROM_TIMING)
    const int64_t c0 = W.start + k * chunk, c1 = min(W.end, c0 + chunk);
    int64_t merge;
    {
        Walk<KIND> w(W, vis, nxt, pre);
        int last = l;
        walk_run<KIND>(w, x, last, c1, nullptr, true, &merge, calls, n_calls, cap, false);
    }
    const int64_t stop_at = merge >= 0 ? merge : c1;
    for (int64_t p = c0 + (threadIdx.x & 63); p < stop_at; p += 64) vis[p] = 0;
    __syncthreads();
    Walk<KIND> w(W, nullptr, nxt, pre);
    int last = l;
    int64_t m2;
    const int64_t pos = walk_run<KIND>(w, x, last, stop_at, vis, false, &m2, calls, n_calls, cap, true);
    if ((threadIdx.x & 63) == 0) {
        cs[k].status = merge >= 0 ? ST_MERGED : ST_NOMERGE;
        cs[k].x2 = pos;
        cs[k].l2 = last;
    }
}

// repeat z overrides (GROM.c:19022-19150): positions are unique here (the
// host keeps the last write of each), so a plain scatter
__global__ void k_cnv_zscatter(const int64_t *__restrict__ pos, const double *__restrict__ z, int64_t n,
                               double *__restrict__ sd) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) sd[pos[i]] = z[i];
}

// ---- candidate classification: phases A and B without the serial sum ----
//
// Inside a long copy-number region every base is a candidate whose phase B
// runs to L = 10,000 bases.  The walk needs, per candidate, only: does phase A
// stop (a jump), does any window pass the z test (a call -- rare, and the
// walk then leaves the region), or neither (a no-op, the walk steps on).
// The integer parts (class state, pass counts, the 2*cnt2 < wl stop) are
// exact from per-64-base bit words and popcounts; the z test needs the
// reference's sequential double sum only near its threshold: with the sum
// approximated from per-block sums (error far below 1e-9 of sum |z|), a
// window whose bound stays below 3 * cnt * wsd by that margin is certainly
// not a pass, and a whole 64-base block is skipped when no step in it can
// stop or pass.  Everything else -- phase A's own exact sum decides the first
// window -- is UNDECIDED and computed exactly (k_cnv_pre, or the walk).
constexpr int CW_SEG = 64;  // words per wave segment in the word kernels

struct CandWords {
    uint64_t *nl, *def;  // nonlow; nonlow and class-defining (HI or depth > 0)
    uint64_t *pm;        // [kind][class][word]: nonlow and passing with the class fixed
    uint64_t *pk;        // [kind][word]: nonlow and passing under the last defining base's class
    double *bsum, *bmax, *bmin, *babs;  // per word: sum z (nonlow), max/min running sum, sum |z|
    int8_t *kend;        // per word: the last defining class at its end
    double *rsn, *rsa;   // per base: running sum of z inside its word, nonlow bases / all bases
    double *bmax4, *bmin4;  // per word and quarter (16 bases): max/min of rsn (the classification's finer bound)
    uint64_t *defa, *c1a, *c1n;  // class-defining bases (any / their class-1 bits), class-1 bits of `def`
    uint64_t *pa;        // [kind][class][word]: passing with the class fixed, low bases included
    int64_t n_words;
    struct SuperW *sup;        // per 8 words (k_cnv_super): phase B's block skip
    const double *wsdmin512;   // min wsd over 512 window lengths from each length
    int64_t n_sup;
};

// Per CW_SUP words (512 bases), for phase B of the classification: a
// candidate whose class is defined (pass bits pk) at a block's start skips
// the block in one step when its walk cannot reach -1 inside it (level +
// the block's lowest walk prefix >= 0) and the block's z bound (largest
// running sum, at least one more nonlow base, the smallest wsd over the
// block's lengths) is settled -- the same bound as a word's, over 8 words.
#define CW_SUP 8
struct SuperW {
    // per kind and pass-bit source (0: pk, the class defined; 1 + m: pm with
    // class m fixed, for a candidate whose class is not defined yet): the pass
    // walk's change over the block and its lowest prefix
    int32_t d[2][3], mp[2][3];
    int32_t nlc, hasdef;      // nonlow bases; any class-defining base (a candidate not yet defined becomes defined inside)
    double zs, zmx, zmn, za;  // z over nonlow bases: sum, largest/smallest running sum from the block's start; sum |z|
};

// last defining class per segment of CW_SEG words (for the carry scan)
__global__ __launch_bounds__(256) void k_cnv_cls_seg(const uint16_t *__restrict__ wb, int64_t len, int64_t n_seg,
                                                     int8_t *__restrict__ seg_last) {
    const int64_t sg = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (sg >= n_seg) return;
    int c = -1;
    for (int w = 0; w < CW_SEG; w++) {
        const int64_t p = (sg * CW_SEG + w) * 64 + lane;
        const uint32_t b = p < len ? (uint32_t)wb[p] : (uint32_t)B_LOW;
        const int e = !(b & B_LOW) ? cdef(b) : -1;
        c = __builtin_amdgcn_readlane(wave_last_incl(e, c), 63);
    }
    if (lane == 0) seg_last[sg] = (int8_t)c;
}

__global__ __launch_bounds__(256) void k_cnv_words(const uint16_t *__restrict__ wb, const double *__restrict__ sd,
                                                   int64_t len, int64_t n_seg, const int8_t *__restrict__ carry,
                                                   CandWords C) {
    const int64_t sg = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (sg >= n_seg) return;
    int c = carry[sg];
    for (int w = 0; w < CW_SEG; w++) {
        const int64_t wi = sg * CW_SEG + w;
        if (wi >= C.n_words) return;
        const int64_t p = wi * 64 + lane;
        const bool in = p < len;
        const uint32_t b = in ? (uint32_t)wb[p] : 0u;
        const bool nl = in && !(b & B_LOW);
        const int e = nl ? cdef(b) : -1;
        const int K = wave_last_incl(e, c);
        c = __builtin_amdgcn_readlane(K, 63);
        const unsigned long long wnl = __ballot(nl), wdef = __ballot(e >= 0), wc1n = __ballot(e == 1);
        const int ea = in ? cdef(b) : -1;
        const unsigned long long wdefa = __ballot(ea >= 0), wc1a = __ballot(ea == 1);
        unsigned long long wpm[2][2], wpk[2], wpa[2][2];
        for (int k = 0; k < 2; k++) {
            const uint32_t pb0 = k == 0 ? B_DEL0 : B_DUP0;
            wpm[k][0] = __ballot(nl && (b & pb0));
            wpm[k][1] = __ballot(nl && (b & (pb0 << 1)));
            wpk[k] = __ballot(nl && K >= 0 && (b & (pb0 << K)));
            wpa[k][0] = __ballot(in && (b & pb0));
            wpa[k][1] = __ballot(in && (b & (pb0 << 1)));
        }
        // running sum of z over the word's nonlow bases (any association: a bound input)
        double z = nl ? sd[p] : 0.0, ps = z;
        for (int d = 1; d < 64; d <<= 1) {
            const double t = __shfl_up(ps, d);
            if (lane >= d) ps += t;
        }
        double mx = ps, mn = ps, ab = fabs(in ? sd[p] : 0.0);  // |z| of every base: a slack bound for both phases
        // (per quarter first: lanes 16q..16q+15)
        for (int o = 8; o > 0; o >>= 1) {
            mx = fmax(mx, __shfl_xor(mx, o));
            mn = fmin(mn, __shfl_xor(mn, o));
        }
        if ((lane & 15) == 0) {
            C.bmax4[wi * 4 + (lane >> 4)] = mx;
            C.bmin4[wi * 4 + (lane >> 4)] = mn;
        }
        for (int o = 32; o > 0; o >>= 1) {
            mx = fmax(mx, __shfl_xor(mx, o));
            mn = fmin(mn, __shfl_xor(mn, o));
            ab += __shfl_xor(ab, o);
        }
        const double tot = __shfl(ps, 63);
        // the same running sums per base, and over all bases (phase A's first
        // window adds every base's z)
        double pa = in ? sd[p] : 0.0;
        for (int d = 1; d < 64; d <<= 1) {
            const double t = __shfl_up(pa, d);
            if (lane >= d) pa += t;
        }
        if (in) {
            C.rsn[p] = ps;
            C.rsa[p] = pa;
        }
        if (lane == 0) {
            C.nl[wi] = wnl;
            C.def[wi] = wdef;
            C.defa[wi] = wdefa;
            C.c1a[wi] = wc1a;
            C.c1n[wi] = wc1n;
            for (int k = 0; k < 2; k++) {
                C.pa[(k * 2 + 0) * C.n_words + wi] = wpa[k][0];
                C.pa[(k * 2 + 1) * C.n_words + wi] = wpa[k][1];
            }
            for (int k = 0; k < 2; k++) {
                C.pm[(k * 2 + 0) * C.n_words + wi] = wpm[k][0];
                C.pm[(k * 2 + 1) * C.n_words + wi] = wpm[k][1];
                C.pk[k * C.n_words + wi] = wpk[k];
            }
            C.kend[wi] = (int8_t)c;
            C.bsum[wi] = tot;
            C.bmax[wi] = mx;
            C.bmin[wi] = mn;
            C.babs[wi] = ab;
        }
    }
}

// First-passage tables for the 2*cnt2 - wl walk (+1 at a passing base, -1 at
// any other): per byte of pass bits, the lowest prefix level and, for a
// starting level e in 0..7, the first step that reaches -1 (8: none).
struct ClsTabs {
    int8_t minp[256];
    uint8_t first[256][8];
};

__device__ __forceinline__ void cls_tabs_build(ClsTabs &T) {
    for (int by = threadIdx.x; by < 256; by += blockDim.x) {
        int lvl = 0, mn = 8;
        uint8_t f[8] = {8, 8, 8, 8, 8, 8, 8, 8};
        for (int j = 0; j < 8; j++) {
            lvl += ((by >> j) & 1) ? 1 : -1;
            mn = min(mn, lvl);
            if (lvl < 0 && f[-lvl - 1] == 8) f[-lvl - 1] = (uint8_t)j;
        }
        T.minp[by] = (int8_t)mn;
        for (int e = 0; e < 8; e++) T.first[by][e] = f[e];
    }
}

__global__ __launch_bounds__(256) void k_cnv_super(CandWords C) {
    __shared__ ClsTabs T;
    cls_tabs_build(T);
    __syncthreads();
    const int64_t sg = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (sg >= C.n_sup) return;
    const int64_t nw = C.n_words, w0 = sg * CW_SUP;
    SuperW o;
    if (w0 + CW_SUP > nw) {  // a partial block is never skipped
        for (int k = 0; k < 2; k++)
            for (int v = 0; v < 3; v++) {
                o.d[k][v] = 0;
                o.mp[k][v] = -(1 << 30);
            }
        o.nlc = 0;
        o.hasdef = 1;
        o.zs = o.zmx = o.zmn = o.za = 0.0;
        C.sup[sg] = o;
        return;
    }
    int lv[2][3] = {}, mn[2][3], nlc = 0;
    uint64_t anydef = 0;
    for (int k = 0; k < 2; k++)
        for (int v = 0; v < 3; v++) mn[k][v] = 1 << 30;
    double z = 0.0, mx = -HUGE_VAL, mnz = HUGE_VAL, a = 0.0;
    for (int64_t w = w0; w < w0 + CW_SUP; w++) {
        for (int k = 0; k < 2; k++)
            for (int v = 0; v < 3; v++) {
                const uint64_t P = v == 0 ? C.pk[k * nw + w] : C.pm[(k * 2 + (v - 1)) * nw + w];
                for (int b = 0; b < 64; b += 8) {
                    const uint32_t by = (uint32_t)(P >> b) & 0xffu;
                    mn[k][v] = min(mn[k][v], lv[k][v] + (int)T.minp[by]);
                    lv[k][v] += 2 * (int)__popc(by) - 8;
                }
            }
        anydef |= C.def[w];
        nlc += (int)__popcll(C.nl[w]);
        mx = fmax(mx, z + C.bmax[w]);
        mnz = fmin(mnz, z + C.bmin[w]);
        z += C.bsum[w];
        a += C.babs[w];
    }
    for (int k = 0; k < 2; k++)
        for (int v = 0; v < 3; v++) {
            o.d[k][v] = lv[k][v];
            o.mp[k][v] = mn[k][v];
        }
    o.nlc = nlc;
    o.hasdef = anydef != 0;
    o.zs = z;
    o.zmx = mx;
    o.zmn = mnz;
    o.za = a;
    C.sup[sg] = o;
}

// the first step j in [0, n) at which the walk from level e >= 0 (+1 on a set
// bit of P, -1 otherwise) reaches -1, or n
__device__ __forceinline__ int first_passage(uint64_t P, int n, int e, const ClsTabs &T) {
    // (__popcll is unsigned: keep the arithmetic signed)
    const int nonpass = n - (int)__popcll(P & low_bits(n));
    if (nonpass <= e) return n;  // even every non-passing base cannot get there
    for (int b = 0; b < n; b += 8) {
        uint32_t by = (uint32_t)(P >> b) & 0xffu;
        if (n - b < 8) by |= (0xffu << (n - b)) & 0xffu;  // steps past the end count as +1 (never a new low)
        if (e + T.minp[by] <= -1) return b + T.first[by][e];  // e <= 7 here
        e += 2 * (int)__popc(by) - 8;
    }
    return n;
}

// One lane per candidate, a 64-base word at a time.  nxt[m][p] gets the
// no-op (p) or phase A's jump; the rest are listed in und[] (and get
// NXT_UNDECIDED).  Per word segment the pass bits follow the class rule
// (the candidate's class until the first class-defining base, the running
// class from there), the stop is the first passage of 2*cnt2 - wl to -1
// (exact, from the bits), and the z test is bounded from the word's running
// sums: only a segment whose bound reaches the threshold tests its passing
// bases one by one (from the in-word running sums).  The sums here are not
// the reference's order; any base whose window could pass within a margin
// far above that difference is UNDECIDED and computed exactly (k_cnv_pre or
// the walk), so the jumps and no-ops written are exact.
//
// The work per candidate ranges from one word (a jump near its start) to
// L/64 = 157 words (a no-op window), so the lanes do not stay with one
// candidate: each takes one segment per step and, when its candidate is
// decided, the next candidate from the wave's share of a global queue (one
// atomic per CLS_GRAB candidates).  A wave runs until the queue
// is empty and its lanes are idle, instead of waiting at every candidate for
// its slowest lane.

// candidates a wave takes from the global queue at a time
constexpr uint32_t CLS_GRAB = 128;

template <int KIND>
__global__ __launch_bounds__(256) void k_cnv_classify(WalkIn W, const int64_t *__restrict__ cand, uint32_t n_cand,
                                                      CandWords C, const double *__restrict__ wsdmin,
                                                      int32_t *__restrict__ nxt, int64_t *__restrict__ und,
                                                      uint32_t *n_und, uint32_t und_cap, uint32_t *__restrict__ qhead) {
    __shared__ ClsTabs T;
    // GROM_TIMING counters (W.stats + 24): candidates, phase-A jumps, first
    // window undecided, passing bases tested one by one, segments settled by
    // the bound, phase-B undecided, no-ops, segments tested base by base
    __shared__ unsigned long long cst[8];
    cls_tabs_build(T);
    if (W.stats && threadIdx.x < 8) cst[threadIdx.x] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t L = W.L, ML = W.min_len, end = W.end, nw = C.n_words;
    const double sgn = KIND == 0 ? 1.0 : -1.0;
    unsigned long long c_steps = 0, c_skip = 0, c_wstep = 0, c_n[4] = {0, 0, 0, 0};  // jump, first undecided, B undecided, no-op
    // the lane's candidate
    uint32_t ci = 0;
    bool busy = false;
    int64_t p = 0, lo = 0, wl = 0, cnt = 0;
    int m = 0, E = 0, phase = 0;  // phase 0: A, 1: B
    bool defined = false;
    double R = 0.0, A = 0.0;
    bool drained = false;
    uint32_t qb = 0, qe = 0;  // the wave's share of the queue not yet handed to a lane (wave-uniform)
    for (;;) {
        // refill the idle lanes: from the wave's share, then (one atomic per
        // CLS_GRAB candidates) a new share
        unsigned long long idle = __ballot(!busy);
        for (int pass = 0; pass < 2 && idle && !drained; pass++) {
            if (qb >= qe) {
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(qhead, (uint32_t)CLS_GRAB);
                base = (uint32_t)__shfl((int)base, 0);
                if (base >= n_cand) {
                    drained = true;
                    break;
                }
                qb = base;
                qe = min(base + (uint32_t)CLS_GRAB, n_cand);
            }
            const uint32_t avail = qe - qb, n_idle = (uint32_t)__popcll(idle);
            const uint32_t rank = (uint32_t)__popcll(idle & ((1ull << lane) - 1));
            if (!busy && rank < avail) {
                ci = qb + rank;
                busy = true;
                p = cand[ci] >> 1;
                m = (int)(cand[ci] & 1);
                lo = p;
                wl = cnt = 0;
                E = 0;
                phase = 0;
                defined = false;
                R = A = 0.0;
            }
            qb += min(n_idle, avail);
            idle = __ballot(!busy);
        }
        if (!__ballot(busy)) break;
        if (!busy) continue;
        // one segment of the lane's candidate
        const uint64_t *pmw = C.pm + (KIND * 2 + m) * nw, *pkw = C.pk + KIND * nw;
        int outcome = -2;  // -2 running, 0 jump (out set), 1 first-window undecided, 2 B undecided, 3 no-op
        int32_t out = (int32_t)p;
        const int64_t lim = phase == 0 ? p + ML : min(p + L, end);
        if (lo >= lim) {
            outcome = 3;  // phase B reached its end (or an empty window): no stop, no call
        } else {
            const int64_t w = lo >> 6, hi = min(lim, (w + 1) << 6);
            const int s0 = (int)(lo & 63), n = (int)(hi - lo);
            const uint64_t M = low_bits(n) << s0;
            uint64_t P;
            if (defined) {
                P = pkw[w] & M;
            } else {
                const uint64_t dw = C.def[w] & M;
                if (!dw) {
                    P = pmw[w] & M;
                } else {
                    const uint64_t below = (dw & (0 - dw)) - 1;
                    defined = true;
                    P = ((pmw[w] & below) | (pkw[w] & ~below)) & M;
                }
            }
            const int j = first_passage(P >> s0, n, E, T);
            if (phase == 0) {
                if (j < n) {  // the stop: the walk jumps here
                    out = (int32_t)(lo + j);
                    outcome = 0;
                } else {
                    E += 2 * (int)__popcll(P) - n;
                    wl += n;
                    cnt += __popcll(C.nl[w] & M);
                    R += sgn * (C.rsa[hi - 1] - (s0 ? C.rsa[lo - 1] : 0.0));
                    A += C.babs[w];
                    lo = hi;
                    if (lo == p + ML) {
                        // the first window's z test (every base's z, nonlow count)
                        if (cnt > 0 && W.wsd[ML] > 0) {
                            const double d = (double)cnt * W.wsd[ML];
                            if (!(R + 1e-9 * (A + fabs(R)) + 1e-300 < 3.0 * d * (1.0 - 1e-15))) outcome = 1;
                        }
                        phase = 1;
                    }
                }
            } else {
                const uint64_t Pr = (P >> s0) & low_bits(j);  // passing bases before the stop
                const double base = s0 ? C.rsn[lo - 1] : 0.0;
                if (Pr) {
                    const double ub = KIND == 0 ? R + (C.bmax[w] - base) : R - (C.bmin[w] - base);
                    const double dlo = (double)(cnt + 1) * wsdmin[wl + 1];
                    const double slack = 1e-9 * (A + C.babs[w] + fabs(ub)) + 1e-300;
                    if (dlo > 0 && ub + slack < 3.0 * dlo * (1.0 - 1e-15)) {
                        c_skip++;
                    } else {
                        c_wstep++;
                        const uint64_t nlr = C.nl[w] >> s0;
                        for (uint64_t q = Pr; q; q &= q - 1) {
                            const int k = __ffsll((long long)q) - 1;
                            const double Rk = R + sgn * (C.rsn[lo + k] - base);
                            const int64_t ck = cnt + __popcll(nlr & low_bits(k + 1));
                            const double ws = W.wsd[wl + k + 1];
                            c_steps++;
                            if (ws > 0) {
                                const double d = (double)ck * ws;
                                if (!(Rk + 1e-9 * (A + C.babs[w] + fabs(Rk)) + 1e-300 < 3.0 * d * (1.0 - 1e-15))) {
                                    outcome = 2;
                                    break;
                                }
                            }
                        }
                    }
                }
                if (outcome < 0) {
                    if (j < n) {
                        outcome = 3;  // phase B stops without a call: no-op
                    } else {
                        E += 2 * (int)__popcll(P) - n;
                        wl += n;
                        cnt += __popcll(C.nl[w] & M);
                        R += sgn * (C.rsn[hi - 1] - base);
                        A += C.babs[w];
                        lo = hi;
                    }
                }
            }
        }
        if (outcome >= 0) {
            if (outcome == 1 || outcome == 2) {
                out = NXT_UNDECIDED;
                const uint32_t k = atomicAdd(n_und, 1u);
                if (k < und_cap) und[k] = cand[ci];
            }
            nxt[m * W.len + p] = out;
            c_n[outcome]++;
            busy = false;
        }
    }
    if (W.stats) {
        atomicAdd(&cst[0], c_n[0] + c_n[1] + c_n[2] + c_n[3]);
        atomicAdd(&cst[1], c_n[0]);
        atomicAdd(&cst[2], c_n[1]);
        atomicAdd(&cst[5], c_n[2]);
        atomicAdd(&cst[6], c_n[3]);
        atomicAdd(&cst[3], c_steps);
        atomicAdd(&cst[4], c_skip);
        atomicAdd(&cst[7], c_wstep);
        __syncthreads();
        if (threadIdx.x < 8) atomicAdd(W.stats + 24 + threadIdx.x, cst[threadIdx.x]);
    }
}

// The same classification with one lane per candidate for its whole window
// (the default; GROM_CNV_CLS=1 takes the queue kernel above): lanes of a wave
// walk neighbouring candidates in step, so their word loads coalesce, but a
// wave waits for its longest candidate.  Measured faster than the queue.
template <int KIND>
__global__ __launch_bounds__(256) void k_cnv_classify_lane(WalkIn W, const int64_t *__restrict__ cand, uint32_t n_cand,
                                                      CandWords C, const double *__restrict__ wsdmin,
                                                      int32_t *__restrict__ nxt, int64_t *__restrict__ und,
                                                      uint32_t *n_und, uint32_t und_cap) {
    __shared__ ClsTabs T;
    // GROM_TIMING counters (W.stats + 24): candidates, phase-A jumps, first
    // window undecided, passing bases tested one by one, segments settled by
    // the bound, phase-B undecided, no-ops, segments tested base by base
    __shared__ unsigned long long cst[8];
    cls_tabs_build(T);
    if (W.stats && threadIdx.x < 8) cst[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long c_steps = 0, c_skip = 0, c_wstep = 0;
    // GROM_TIMING, slots 32-35: aligned blocks reached, with the class defined, walk clear, skipped
    unsigned long long c_blk[4] = {0, 0, 0, 0};
    int c_out = -1;  // 0 jump, 1 first-window undecided, 2 B undecided, -1 no-op
    if (i < n_cand) {
        const int64_t p = cand[i] >> 1;
        const int m = (int)(cand[i] & 1);
        const int64_t L = W.L, ML = W.min_len, end = W.end, nw = C.n_words;
        const double sgn = KIND == 0 ? 1.0 : -1.0;
        const uint64_t *pmw = C.pm + (KIND * 2 + m) * nw, *pkw = C.pk + KIND * nw;
        bool defined = false;
        // the pass bits of a segment (mask M of word w) under the class rule
        auto pass_bits = [&](int64_t w, uint64_t M) -> uint64_t {
            if (defined) return pkw[w] & M;
            const uint64_t dw = C.def[w] & M;
            if (!dw) return pmw[w] & M;
            const uint64_t below = (dw & (0 - dw)) - 1;
            defined = true;
            return ((pmw[w] & below) | (pkw[w] & ~below)) & M;
        };
        int32_t out = (int32_t)p;
        bool undecided = false;
        int E = 0;  // 2*cnt2 - wl
        int64_t wl = 0, cnt = 0;
        double R = 0.0, A = 0.0;
        // phase A: the first ML bases (GROM.c:19370-19400)
        for (int64_t lo = p; lo < p + ML;) {
            const int64_t w = lo >> 6, hi = min(p + ML, (w + 1) << 6);
            const int s0 = (int)(lo & 63), n = (int)(hi - lo);
            const uint64_t M = low_bits(n) << s0;
            const uint64_t P = pass_bits(w, M);
            const int j = first_passage(P >> s0, n, E, T);
            if (j < n) {  // the stop: the walk jumps here
                out = (int32_t)(lo + j);
                c_out = 0;
                goto done;
            }
            E += 2 * (int)__popcll(P) - n;
            wl += n;
            cnt += __popcll(C.nl[w] & M);
            R += sgn * (C.rsa[hi - 1] - (s0 ? C.rsa[lo - 1] : 0.0));
            A += C.babs[w];
            lo = hi;
        }
        // the first window's z test (every base's z, nonlow count)
        if (cnt > 0 && W.wsd[ML] > 0) {
            const double d = (double)cnt * W.wsd[ML];
            if (!(R + 1e-9 * (A + fabs(R)) + 1e-300 < 3.0 * d * (1.0 - 1e-15))) {
                undecided = true;
                c_out = 1;
                goto done;
            }
        }
        // phase B: extension to L (GROM.c:19405-19470); reaching `end` stops it
        {
            const int64_t xlim = min(p + L, end);
            for (int64_t lo = p + ML; lo < xlim;) {
                if ((lo & (64 * CW_SUP - 1)) == 0 && lo + 64 * CW_SUP <= xlim) {
                    // (the pass bits over the block: pk once defined, else pm of
                    // the candidate's class while the block defines nothing)
                    const SuperW &B = C.sup[lo / (64 * CW_SUP)];
                    const int v = defined ? 0 : B.hasdef ? -1 : 1 + m;
                    c_blk[0]++;
                    if (v >= 0) c_blk[1]++;
                    if (v >= 0 && E + B.mp[KIND][v] >= 0) {
                        c_blk[2]++;
                        const double ub = KIND == 0 ? R + B.zmx : R - B.zmn;
                        const double dlo = (double)(cnt + 1) * C.wsdmin512[wl + 1];
                        const double slack = 1e-9 * (A + B.za + fabs(ub)) + 1e-300;
                        if (dlo > 0 && ub + slack < 3.0 * dlo * (1.0 - 1e-15)) {
                            c_blk[3]++;
                            c_skip += CW_SUP;
                            E += B.d[KIND][v];
                            wl += 64 * CW_SUP;
                            cnt += B.nlc;
                            R += sgn * B.zs;
                            A += B.za;
                            lo += 64 * CW_SUP;
                            continue;
                        }
                    }
                }
                const int64_t w = lo >> 6, hi = min(xlim, (w + 1) << 6);
                const int s0 = (int)(lo & 63), n = (int)(hi - lo);
                const uint64_t M = low_bits(n) << s0;
                const uint64_t P = pass_bits(w, M);
                const int j = first_passage(P >> s0, n, E, T);
                const uint64_t Pr = (P >> s0) & low_bits(j);  // passing bases before the stop
                const double base = s0 ? C.rsn[lo - 1] : 0.0;
                if (Pr) {
                    const double ub = KIND == 0 ? R + (C.bmax[w] - base) : R - (C.bmin[w] - base);
                    const double dlo = (double)(cnt + 1) * wsdmin[wl + 1];
                    const double slack = 1e-9 * (A + C.babs[w] + fabs(ub)) + 1e-300;
                    if (dlo > 0 && ub + slack < 3.0 * dlo * (1.0 - 1e-15)) {
                        c_skip++;
                    } else {
                        c_wstep++;
                        const uint64_t nlr = C.nl[w] >> s0;
                        // the same bound per quarter word (16 bases) before its
                        // passing bases are tested one by one: a quarter's
                        // largest running sum, at least the nonlow bases before
                        // it plus its own first, and the smallest wsd from there
                        uint64_t qdone = 0;  // quarters settled or tested
                        for (uint64_t q = Pr; q; q &= q - 1) {
                            const int k = __ffsll((long long)q) - 1;
                            const int qi = (s0 + k) >> 4;
                            if (!((qdone >> qi) & 1)) {
                                qdone |= 1ull << qi;
                                const int kq = max((qi << 4) - s0, 0);  // the quarter's first step in the segment
                                const double ubq = KIND == 0 ? R + (C.bmax4[w * 4 + qi] - base)
                                                             : R - (C.bmin4[w * 4 + qi] - base);
                                const double dq = (double)(cnt + __popcll(nlr & low_bits(kq)) + 1) * wsdmin[wl + kq + 1];
                                const double sq = 1e-9 * (A + C.babs[w] + fabs(ubq)) + 1e-300;
                                if (dq > 0 && ubq + sq < 3.0 * dq * (1.0 - 1e-15)) {
                                    // settled: skip the quarter's passing bases
                                    const int qe = ((qi + 1) << 4) - s0;
                                    q &= ~low_bits(qe);
                                    q |= 1ull << k;  // (cleared by the loop step)
                                    continue;
                                }
                            }
                            const double Rk = R + sgn * (C.rsn[lo + k] - base);
                            const int64_t ck = cnt + __popcll(nlr & low_bits(k + 1));
                            const double ws = W.wsd[wl + k + 1];
                            c_steps++;
                            if (ws > 0) {
                                const double d = (double)ck * ws;
                                if (!(Rk + 1e-9 * (A + C.babs[w] + fabs(Rk)) + 1e-300 < 3.0 * d * (1.0 - 1e-15))) {
                                    undecided = true;
                                    c_out = 2;
                                    goto done;
                                }
                            }
                        }
                    }
                }
                if (j < n) goto done;  // phase B stops without a call: no-op
                E += 2 * (int)__popcll(P) - n;
                wl += n;
                cnt += __popcll(C.nl[w] & M);
                R += sgn * (C.rsn[hi - 1] - base);
                A += C.babs[w];
                lo = hi;
            }
        }
    done:
        if (undecided) {
            out = NXT_UNDECIDED;
            const uint32_t k = atomicAdd(n_und, 1u);
            if (k < und_cap) und[k] = cand[i];
        }
        nxt[m * W.len + p] = out;
    }
    if (W.stats) {
        if (i < n_cand) {
            atomicAdd(&cst[0], 1ull);
            atomicAdd(&cst[c_out < 0 ? 6 : c_out == 0 ? 1 : c_out == 1 ? 2 : 5], 1ull);
            atomicAdd(&cst[3], c_steps);
            atomicAdd(&cst[4], c_skip);
            atomicAdd(&cst[7], c_wstep);
            for (int q = 0; q < 4; q++)
                if (c_blk[q]) atomicAdd(W.stats + 32 + q, c_blk[q]);
        }
        __syncthreads();
        if (threadIdx.x < 8) atomicAdd(W.stats + 24 + threadIdx.x, cst[threadIdx.x]);
    }
}

// a call is on the true walk iff its start was visited in its class
// (chunks the true walk jumps over entirely are flagged in `skipped`)
__global__ void k_cnv_calls_valid(const CallRec *calls, uint32_t n, const uint8_t *vis, const uint8_t *skipped,
                                  int64_t start, int64_t chunk, uint8_t *ok) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t p = calls[i].p;
    ok[i] = vis[p] == 1 + calls[i].m && !skipped[(p - start) / chunk];
}

// ---------------- host side ----------------
struct Buf {
    void *p = nullptr;
    size_t cap = 0;
    bool own = false;          // p is this buffer's own allocation (else a piece of `ar`'s phase)
    grom_arena *ar = nullptr;  // the context's phase arena (cnv_scratch_phase), or none
};

}  // namespace

// per-class (DEL, DUP) window-search buffers and stream: the two classes are
// independent (GROM.c:19359-20020 runs them one after the other over the same
// inputs), so they run concurrently, each driven by its own host thread
struct KindBufs {
    Buf nxt, pre, prepos, ppos, calls, ok, tiles, vis, cnt, und, skip, pend, plist;
    hipStream_t st = nullptr;
};

struct CnvScratch {
    KindBufs kb[2];
    hipEvent_t walk_in = nullptr;
    // k_cnv_gc launched early on kb[0].st by cnv_prelaunch (overlaps the pileup)
    hipEvent_t gc_done = nullptr;
    const char *gc_ref = nullptr;
    int64_t gc_len = -1, gc_m = -1;
    Buf zover;  // repeat z overrides: positions then values
    Buf cwords, cw_seg, cw_carry, wsdmin;  // candidate classification: bit words, their class carry, min wsd per 64
    Buf gen1000;                           // the -N side file's per-window results
    Buf gpre, gtmp;                        // insert means above GC_MMAX: chromosome-wide GC/ACGT prefixes
    Buf gcw, acw, rtype, flag, sd, vis, wbits, ztab, nxt, pre, prepos, ppos, rep, misc, blk, hist, tiles, carry, tabs, samples, gat_rg, gat, wd, rows,
        rowlen, wtot, wcnt, wsd, calls, ok;
    Buf cn_v;                // the copy number's per-base ratios of the kept calls
    double *h_cn = nullptr;  // pinned: their host copy
    size_t h_cn_cap = 0;
    // pinned host buffers of the gathers (gather(): at most three alive at once)
    struct PinBuf {
        uint8_t *p = nullptr;
        size_t cap = 0;
        bool busy = false;
    } pin[4];
    hipEvent_t e0 = nullptr, e1 = nullptr;
};

namespace {

#define CK(x)                                                                                       \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) {                                                                     \
            snprintf(err, errlen, "%s failed: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            return GROM_E_HIP;                                                                      \
        }                                                                                           \
    } while (0)

static int grow(Buf &b, size_t bytes, char *err, size_t errlen) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return GROM_OK;
    if (b.p && b.own) grom_dev_free(b.p, b.cap, GROM_DEVCAT_CNV);
    b.p = nullptr;
    b.cap = 0;
    b.own = false;
    size_t want = bytes + bytes / 8 + 256;
    if (b.ar && (b.p = grom_arena_take(b.ar, want)) != nullptr) {
        b.cap = want;
        return GROM_OK;
    }
    if (grom_dev_malloc(&b.p, want, GROM_DEVCAT_CNV)) {
        snprintf(err, errlen, "hipMalloc(%zu) failed in the CNV path", want);
        return GROM_E_NOMEM;
    }
    b.cap = want;
    b.own = true;
    return GROM_OK;
}

// glibc random()/rand() (TYPE_3, stdlib/random_r.c) for grom_rand, GROM.c:1185
struct GlibcRand {
    int32_t st[31];
    int f = 3, r = 0;
    explicit GlibcRand(uint32_t seed) {
        if (seed == 0) seed = 1;
        st[0] = (int32_t)seed;
        int32_t word = (int32_t)seed;  // int32_t in glibc's __srandom_r
        for (int i = 1; i < 31; i++) {
            long hi = word / 127773, lo = word % 127773;
            word = (int32_t)(16807 * lo - 2836 * hi);
            if (word < 0) word += 2147483647;
            st[i] = word;
        }
        for (int i = 0; i < 310; i++) next();
    }
    int next() {
        uint32_t v = (uint32_t)st[f] + (uint32_t)st[r];
        st[f] = (int32_t)v;
        if (++f >= 31) { f = 0; ++r; } else if (++r >= 31) r = 0;
        return (int)(v >> 1);
    }
    long grom_rand(long mx) {  // GROM.c:1185-1201
        long v = 0, c = 1, t;
        while (c < mx) {
            t = (next() % 10) * c;
            while (t + v >= mx) t = (next() % 10) * c;
            v += t;
            c *= 10;
        }
        return v;
    }
};

// qsort(double[], cmpfunc) of glibc 2.12 (msort.c) with the reference's int
// comparator reading each double's low 32 bits
static int dcmp_lo(double a, double b) {
    uint32_t x, y;
    memcpy(&x, &a, 4);
    memcpy(&y, &b, 4);
    return (int32_t)(x - y);
}
static void msort_lo(double *b, size_t n, double *t) {
    if (n <= 1) return;
    size_t n1 = n / 2, n2 = n - n1;
    double *b1 = b, *b2 = b + n1;
    msort_lo(b1, n1, t);
    msort_lo(b2, n2, t);
    double *o = t;
    while (n1 > 0 && n2 > 0) {
        if (dcmp_lo(*b1, *b2) <= 0) { *o++ = *b1++; --n1; }
        else { *o++ = *b2++; --n2; }
    }
    if (n1 > 0) memcpy(o, b1, n1 * sizeof(double));
    memcpy(b, t, (n - n2) * sizeof(double));
}

// the same merge sort with the two halves of the top `depth` levels sorted on
// their own threads (each with its own half of the scratch): the same
// operations on the same data, so the same order -- which matters, since the
// reference's comparator (low 32 bits, wrapping difference) is not a total
// order and only this exact merge sequence reproduces its result
static void msort_lo_par(double *b, size_t n, double *t, int depth) {
    if (depth <= 0 || n < (1u << 16)) {
        msort_lo(b, n, t);
        return;
    }
    size_t n1 = n / 2, n2 = n - n1;
    double *b1 = b, *b2 = b + n1;
    std::thread th([=] { msort_lo_par(b1, n1, t, depth - 1); });
    msort_lo_par(b2, n2, t + n1, depth - 1);
    th.join();
    double *o = t;
    while (n1 > 0 && n2 > 0) {
        if (dcmp_lo(*b1, *b2) <= 0) { *o++ = *b1++; --n1; }
        else { *o++ = *b2++; --n2; }
    }
    if (n1 > 0) memcpy(o, b1, n1 * sizeof(double));
    memcpy(b, t, (n - n2) * sizeof(double));
}

// sort of small non-negative ints (read depths): counting sort, same result
// as the reference's qsort with cmpfunc on these values
static void sort_depths(std::vector<int> &v) {
    if (v.size() < 2) return;
    int mx = 0;
    for (int x : v) {
        if (x < 0) { std::sort(v.begin(), v.end()); return; }
        mx = std::max(mx, x);
    }
    if (mx > (1 << 20)) { std::sort(v.begin(), v.end()); return; }
    std::vector<uint32_t> h((size_t)mx + 1, 0);
    for (int x : v) h[x]++;
    size_t k = 0;
    for (int x = 0; x <= mx; x++)
        for (uint32_t c = 0; c < h[x]; c++) v[k++] = x;
}

// Per-position values of gathered ranges on the host, views of one pinned
// buffer the device copy lands in (round 5 copied 15 bytes per position into
// a zero-filled pageable vector and split it into six more: 54-74 ms per
// chromosome for the copy numbers' ~6 M positions); rt = rd + low is made on
// the device.  The buffer goes back to the scratch's pool with the view.
struct Gathered {
    const uint8_t *gc = nullptr, *ac = nullptr, *flag = nullptr;
    const int32_t *mq = nullptr, *rd = nullptr, *low = nullptr, *rt = nullptr;
    CnvScratch::PinBuf *pb = nullptr;
    Gathered() = default;
    Gathered(const Gathered &) = delete;
    Gathered &operator=(const Gathered &) = delete;
    ~Gathered() {
        if (pb) pb->busy = false;
    }
};

static int gather(CnvScratch *S, hipStream_t st, const std::vector<GatherRange> &rg, int64_t total, const uint8_t *gcw,
                  const uint8_t *acw, const int32_t *mq, const int32_t *rd, const int32_t *low, const uint8_t *flag,
                  Gathered &g, char *err, size_t errlen) {
    if (total == 0 || rg.empty()) return GROM_OK;
    int rc;
    const size_t bytes = (size_t)total * 19;
    if ((rc = grow(S->gat_rg, sizeof(GatherRange) * rg.size(), err, errlen)) || (rc = grow(S->gat, bytes, err, errlen)))
        return rc;
    CnvScratch::PinBuf *pb = nullptr;
    for (auto &b : S->pin)
        if (!b.busy) {
            pb = &b;
            break;
        }
    if (!pb) {
        snprintf(err, errlen, "CNV gather: no free pinned buffer");
        return GROM_E_NOMEM;
    }
    if (pb->cap < bytes) {
        if (pb->p) (void)hipHostFree(pb->p);
        pb->p = nullptr;
        pb->cap = 0;
        const size_t want = bytes + bytes / 4 + 4096;
        CK(hipHostMalloc((void **)&pb->p, want, 0));
        pb->cap = want;
    }
    pb->busy = true;
    g.pb = pb;
    CK(hipMemcpyAsync(S->gat_rg.p, rg.data(), sizeof(GatherRange) * rg.size(), hipMemcpyHostToDevice, st));
    uint8_t *o = (uint8_t *)S->gat.p;
    int32_t *o_mq = (int32_t *)o, *o_rd = o_mq + total, *o_low = o_rd + total, *o_rt = o_low + total;
    uint8_t *o_gc = (uint8_t *)(o_rt + total), *o_ac = o_gc + total, *o_f = o_ac + total;
    int g_ = (int)std::min<int64_t>((total + 255) / 256, 16384);
    hipLaunchKernelGGL(k_cnv_gather, dim3(g_), dim3(256), 0, st, (const GatherRange *)S->gat_rg.p, (int)rg.size(), gcw,
                       acw, mq, rd, low, flag, total, o_gc, o_ac, o_mq, o_rd, o_low, o_rt, o_f);
    CK(hipGetLastError());
    // the seven arrays lie back to back: one copy, viewed in place
    CK(hipMemcpyAsync(pb->p, o, bytes, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    const int32_t *h = (const int32_t *)pb->p;
    g.mq = h;
    g.rd = h + total;
    g.low = h + 2 * total;
    g.rt = h + 3 * total;
    g.gc = (const uint8_t *)(h + 4 * total);
    g.ac = g.gc + total;
    g.flag = g.ac + total;
    return GROM_OK;
}

}  // namespace

CnvScratch *cnv_scratch_new() { return new CnvScratch(); }

static int cnv_init(CnvScratch *S, char *err, size_t errlen) {
    if (S->e0) return GROM_OK;
    CK(hipEventCreate(&S->e0));
    CK(hipEventCreate(&S->e1));
    CK(hipEventCreateWithFlags(&S->walk_in, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&S->gc_done, hipEventDisableTiming));
    for (KindBufs &K : S->kb) CK(hipStreamCreateWithFlags(&K.st, hipStreamNonBlocking));
    return GROM_OK;
}

// Insert means above GC_MMAX (the tile kernel's LDS halo): the same closed
// form over chromosome-wide prefixes in global memory.  k_cnv_gc_marks writes
// per base the GC and ACGT class bits and their positions (4 int64 arrays of
// len+1, the last entry 0); exclusive scans turn them into P and R; then
// T(p) = Q[p+m+1] - 2 Q[p+1] + Q[p-m+1], Q[x] = (x-1) P[x] - R[x], with
// positions past either end holding no class bits, as in k_cnv_gc.
__global__ void k_cnv_gc_marks(const char *__restrict__ ref, int64_t len, int64_t *__restrict__ pre) {
    const int64_t n = len + 1;
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
        const int c = q < len ? gc_class(ref[q]) : 0;
        pre[q] = c & 1;
        pre[n + q] = (c & 1) ? q : 0;
        pre[2 * n + q] = (c >> 1) & 1;
        pre[3 * n + q] = (c & 2) ? q : 0;
    }
}

__global__ void k_cnv_gc_global(const char *__restrict__ ref, Args A, int64_t m, int64_t total,
                                const int64_t *__restrict__ pre, uint8_t *__restrict__ gcw,
                                uint8_t *__restrict__ acw, uint8_t *__restrict__ rtype) {
    const int64_t n = A.len + 1;
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < A.len; p += (int64_t)gridDim.x * blockDim.x) {
        uint32_t w2[2] = {0, 0}, rt = 10;
        if (p >= A.lo && p < A.hi) {
            const int64_t xs[3] = {p + m + 1, p + 1, p - m + 1};
#pragma unroll
            for (int pl = 0; pl < 2; pl++) {
                const int64_t *P = pre + (2 * pl) * n, *R = pre + (2 * pl + 1) * n;
                int64_t Qv[3];
#pragma unroll
                for (int t = 0; t < 3; t++) {
                    const int64_t x = xs[t];
                    const int64_t xc = x < 0 ? 0 : (x > A.len ? A.len : x);
                    const int64_t Pv = x < 0 ? 0 : P[xc], Rv = x < 0 ? 0 : R[xc];
                    Qv[t] = (x - 1) * Pv - Rv;
                }
                const uint64_t Tv = (uint64_t)(Qv[0] - 2 * Qv[1] + Qv[2]);
                w2[pl] = (uint32_t)((100u * Tv / (uint64_t)total) & 255u);
            }
            rt = (uint32_t)pair_type(ref[p], ref[p + 1]);
        }
        gcw[p] = (uint8_t)w2[0];
        acw[p] = (uint8_t)w2[1];
        rtype[p] = (uint8_t)rt;
    }
}

// test hook GROM_GC_GLOBAL=1: the prefix form at any insert mean
static bool gc_global_forced() {
    static const bool f = getenv("GROM_GC_GLOBAL") && atoi(getenv("GROM_GC_GLOBAL")) == 1;
    return f;
}

// GC/ACGT weights and dinucleotide classes depend on the reference alone
// (GROM.c:1586-1881), so the scan driver starts them before the pileup on a
// stream of their own; cnv_chrom then only waits for them.
int cnv_prelaunch(CnvScratch *S, hipStream_t after, const grom_params &P, const char *d_ref, int64_t len, char *err,
                  size_t errlen) {
    int rc;
    S->gc_ref = nullptr;
    const int64_t m = P.insert_mean;
    if (m < 1 || m > GC_MMAX || len <= 0 || gc_global_forced()) return GROM_OK;  // cnv_chrom builds these itself
    if ((rc = cnv_init(S, err, errlen))) return rc;
    if ((rc = grow(S->gcw, len, err, errlen)) || (rc = grow(S->acw, len, err, errlen)) ||
        (rc = grow(S->rtype, len, err, errlen)))
        return rc;
    Args A{};  // the fields k_cnv_gc reads, as cnv_chrom sets them
    A.len = len;
    A.lo = m - 1;
    A.hi = std::max<int64_t>(A.lo, len - (2 * m - 1));
    const hipStream_t side = S->kb[0].st;
    CK(hipEventRecord(S->gc_done, after));  // the reference may still be uploading on `after`
    CK(hipStreamWaitEvent(side, S->gc_done, 0));
    hipLaunchKernelGGL(m <= GC_MMAX_S ? k_cnv_gc<GC_MMAX_S> : k_cnv_gc<GC_MMAX>, dim3((unsigned)((len + GC_TP - 1) / GC_TP)), dim3(256), 0, side, d_ref, A, (int)m,
                       (int64_t)m * m, (uint8_t *)S->gcw.p, (uint8_t *)S->acw.p, (uint8_t *)S->rtype.p);
    CK(hipGetLastError());
    CK(hipEventRecord(S->gc_done, side));
    S->gc_ref = d_ref;
    S->gc_len = len;
    S->gc_m = m;
    return GROM_OK;
}

#define CNV_PHASE_BUFS(S)                                                                                             \
    {&S->flag, &S->sd, &S->vis, &S->wbits, &S->ztab, &S->nxt, &S->pre, &S->prepos, &S->ppos, &S->rep, &S->misc,       \
     &S->blk, &S->hist, &S->tiles, &S->carry, &S->tabs, &S->samples, &S->gat_rg, &S->gat, &S->wd, &S->rows,           \
     &S->rowlen, &S->wtot, &S->wcnt, &S->wsd, &S->calls, &S->ok, &S->zover, &S->cwords, &S->cw_seg, &S->cw_carry,      \
     &S->wsdmin, &S->gen1000, &S->gpre, &S->gtmp, &S->cn_v}
#define CNV_KIND_BUFS(K) \
    {&K.nxt, &K.pre, &K.prepos, &K.ppos, &K.calls, &K.ok, &K.tiles, &K.vis, &K.cnt, &K.und, &K.skip, &K.pend, &K.plist}

// a new CNV phase (scan.hip): with an arena every buffer but the GC windows
// (written beside the pileup by cnv_prelaunch) is carved from it
void cnv_scratch_phase(CnvScratch *S, grom_arena *ar) {
    auto reset = [ar](Buf *b) {
        if (b->own && ar) grom_dev_free(b->p, b->cap, GROM_DEVCAT_CNV);  // (an overflow of the last phase)
        if (!b->own || ar) {
            b->p = nullptr;
            b->cap = 0;
            b->own = false;
        }
        b->ar = ar;
    };
    Buf *all[] = CNV_PHASE_BUFS(S);
    for (Buf *b : all) reset(b);
    for (KindBufs &K : S->kb) {
        Buf *kall[] = CNV_KIND_BUFS(K);
        for (Buf *b : kall) reset(b);
    }
}

void cnv_scratch_sync(CnvScratch *S) {
    if (!S) return;
    for (KindBufs &K : S->kb)
        if (K.st) (void)hipStreamSynchronize(K.st);
}

void cnv_scratch_free(CnvScratch *S) {
    if (!S) return;
    if (S->h_cn) (void)hipHostFree(S->h_cn);
    S->h_cn = nullptr;
    for (auto &b : S->pin)
        if (b.p) (void)hipHostFree(b.p);
    Buf *all[] = CNV_PHASE_BUFS(S);
    for (Buf *b : all)
        if (b->p && b->own) grom_dev_free(b->p, b->cap, GROM_DEVCAT_CNV);
    Buf *gc[] = {&S->gcw, &S->acw, &S->rtype};
    for (Buf *b : gc)
        if (b->p && b->own) grom_dev_free(b->p, b->cap, GROM_DEVCAT_CNV);
    for (KindBufs &K : S->kb) {
        Buf *kall[] = CNV_KIND_BUFS(K);
        for (Buf *b : kall)
            if (b->p && b->own) grom_dev_free(b->p, b->cap, GROM_DEVCAT_CNV);
        if (K.st) (void)hipStreamDestroy(K.st);
    }
    if (S->walk_in) (void)hipEventDestroy(S->walk_in);
    if (S->gc_done) (void)hipEventDestroy(S->gc_done);
    if (S->e0) (void)hipEventDestroy(S->e0);
    if (S->e1) (void)hipEventDestroy(S->e1);
    delete S;
}

int cnv_chrom(CnvScratch *S, hipStream_t st, const grom_params &P, uint32_t seed, const char *chr_name,
              const char *d_ref, int64_t len, int32_t *d_mq, const int32_t *d_rd, const int32_t *d_low,
              std::string &rows, CnvTiming *timing, char *err, size_t errlen, std::string *side) {
    const auto t_host0 = std::chrono::steady_clock::now();
    int rc;
    const int64_t m = P.insert_mean, W = 2 * (int64_t)m - 1;
    const int64_t total_w = (int64_t)m * m;  // g_one_base_window_size_total, GROM.c:22265-22269
    if (m < 1) {
        snprintf(err, errlen, "insert mean %lld below 1", (long long)m);
        return GROM_E_ARG;
    }
    // (window lengths index int32 positions in the walk; -X past a chromosome
    // only makes every window search stop at the end)
    if (P.max_rd_window_len < P.min_rd_window_len || P.min_rd_window_len < 1 || P.windows_sampling_factor < 1 ||
        P.max_rd_window_len > ((int64_t)1 << 30)) {
        snprintf(err, errlen, "unsupported CNV window parameters (-W %lld -X %lld -A %lld)",
                 (long long)P.min_rd_window_len, (long long)P.max_rd_window_len, (long long)P.windows_sampling_factor);
        return GROM_E_ARG;
    }
    if ((rc = cnv_init(S, err, errlen))) return rc;
    GlibcRand rng(seed);
    // GROM_TIMING: per-phase wall clock (syncs the stream at each mark)
    const bool tmg = getenv("GROM_TIMING") != nullptr;
    auto t_last = std::chrono::steady_clock::now();
    std::string tlog;
    auto mark = [&](const char *what) {
        if (!tmg) return;
        (void)hipStreamSynchronize(st);
        auto now = std::chrono::steady_clock::now();
        char b[96];
        snprintf(b, sizeof(b), " %s %.2f", what, std::chrono::duration<double, std::milli>(now - t_last).count());
        tlog += b;
        t_last = now;
    };
    Args A{};
    A.len = len;
    A.lo = m - 1;
    A.hi = std::max<int64_t>(A.lo, len - W);
    A.min_mapq = P.rd_min_mapq;
    A.ranks_stdev = P.ranks_stdev;
    A.mapq_factor = P.mapq_factor;
    A.dup_factor = (double)P.dup_threshold_factor;
    const int64_t n_blk = len / BLOCK_UNIT;
    const int64_t n_seg = (len + SEG_W - 1) / SEG_W;
    if ((rc = grow(S->gcw, len, err, errlen)) || (rc = grow(S->acw, len, err, errlen)) ||
        (rc = grow(S->rtype, len, err, errlen)) || (rc = grow(S->flag, len, err, errlen)) ||
        (rc = grow(S->sd, 8 * len, err, errlen)) || (rc = grow(S->vis, len, err, errlen)) ||
        (rc = grow(S->wbits, 2 * len, err, errlen)) ||
        (rc = grow(S->misc, 4096, err, errlen)) || (rc = grow(S->blk, 8 * (n_blk + 1), err, errlen)) ||
        (rc = grow(S->hist, 4 * (HIST_MAX + 1), err, errlen)) || (rc = grow(S->tiles, n_seg, err, errlen)) ||
        (rc = grow(S->carry, n_seg, err, errlen)) || (rc = grow(S->ztab, 2 * 2 * NBINS * ZT_MAX, err, errlen)) || (rc = grow(S->tabs, sizeof(Tables), err, errlen)))
        return rc;
    uint8_t *gcw = (uint8_t *)S->gcw.p, *acw = (uint8_t *)S->acw.p, *rtype = (uint8_t *)S->rtype.p,
            *flag = (uint8_t *)S->flag.p;
    double *sd = (double *)S->sd.p;
    char *misc = (char *)S->misc.p;
    unsigned long long *acc = (unsigned long long *)misc;  // [0..3] block/chromosome sums
    uint32_t *n_rep = (uint32_t *)(misc + 64);
    // misc + 80: candidate count of the window search (n_pre + 1)
    CK(hipEventRecord(S->e0, st));
    CK(hipMemsetAsync(misc, 0, 128, st));
    CK(hipMemsetAsync(S->hist.p, 0, 4 * (HIST_MAX + 1), st));

    // ---- A14: weighted GC / ACGT and repeat classes (already running if the
    // driver prelaunched them for this reference) ----
    if (S->gc_ref == d_ref && S->gc_len == len && S->gc_m == m) {
        CK(hipStreamWaitEvent(st, S->gc_done, 0));
    } else if (m > GC_MMAX || gc_global_forced()) {
        const int64_t n = len + 1;
        size_t tb = 0;
        int64_t *pre = nullptr;
        CK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, pre, pre, (int)n, st));
        if ((rc = grow(S->gpre, sizeof(int64_t) * 4 * (size_t)n, err, errlen)) || (rc = grow(S->gtmp, tb, err, errlen)))
            return rc;
        pre = (int64_t *)S->gpre.p;
        hipLaunchKernelGGL(k_cnv_gc_marks, dim3(8192), dim3(256), 0, st, d_ref, len, pre);
        CK(hipGetLastError());
        for (int k = 0; k < 4; k++) CK(hipcub::DeviceScan::ExclusiveSum(S->gtmp.p, tb, pre + k * n, pre + k * n, (int)n, st));
        hipLaunchKernelGGL(k_cnv_gc_global, dim3(8192), dim3(256), 0, st, d_ref, A, m, total_w, (const int64_t *)pre, gcw,
                           acw, rtype);
        CK(hipGetLastError());
    } else {
        hipLaunchKernelGGL(m <= GC_MMAX_S ? k_cnv_gc<GC_MMAX_S> : k_cnv_gc<GC_MMAX>, dim3((unsigned)((len + GC_TP - 1) / GC_TP)), dim3(256), 0, st, d_ref, A, (int)m,
                           total_w, gcw, acw, rtype);
        CK(hipGetLastError());
    }
    S->gc_ref = nullptr;
    // ---- A15: mapq division, blocks, chromosome depth ----
    hipLaunchKernelGGL(k_cnv_blocks, dim3((unsigned)(n_blk + 1)), dim3(256), 0, st, d_ref, A, d_mq, d_rd, d_low, acw,
                       (int64_t *)S->blk.p, acc, (unsigned int *)S->hist.p);
    CK(hipGetLastError());
    uint32_t rep_cap = (uint32_t)std::min<int64_t>(len / std::max<int64_t>(P.min_repeat, 1) + 1, 1 << 24);
    if ((rc = grow(S->rep, sizeof(RepeatRec) * rep_cap, err, errlen))) return rc;
    if (A.hi > A.lo)
        hipLaunchKernelGGL(k_cnv_repeats, dim3((unsigned)((A.hi - A.lo + 255) / 256)), dim3(256), 0, st, rtype, d_rd,
                           d_low, A, P.min_repeat, (RepeatRec *)S->rep.p, n_rep, rep_cap);
    CK(hipGetLastError());
    unsigned long long hacc[4];
    uint32_t hnrep = 0;
    std::vector<int64_t> blk_total(n_blk + 1);
    std::vector<unsigned int> hist(HIST_MAX + 1);
    CK(hipMemcpyAsync(hacc, acc, 32, hipMemcpyDeviceToHost, st));
    CK(hipMemcpyAsync(&hnrep, n_rep, 4, hipMemcpyDeviceToHost, st));
    CK(hipMemcpyAsync(blk_total.data(), S->blk.p, 8 * (n_blk + 1), hipMemcpyDeviceToHost, st));
    CK(hipMemcpyAsync(hist.data(), S->hist.p, 4 * (HIST_MAX + 1), hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    if (hnrep > rep_cap) {
        snprintf(err, errlen, "repeat list overflow (%u > %u)", hnrep, rep_cap);
        return GROM_E_OVERFLOW;
    }
    std::vector<RepeatRec> reps(hnrep);
    if (hnrep) {
        CK(hipMemcpyAsync(reps.data(), S->rep.p, sizeof(RepeatRec) * hnrep, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
    }
    std::sort(reps.begin(), reps.end(), [](const RepeatRec &a, const RepeatRec &b) { return a.start < b.start; });

    // chromosome depth mean over ACGT-rich bases, GROM.c:16645-16660: a double
    // sum of integers below 2^53, so the exact integer total is the same value
    double chr_ave = 0;
    const long chr_cnt = (long)hacc[3];
    if (chr_cnt > 0) chr_ave = (double)hacc[2] / chr_cnt;
    // repeat-type depth and the most biased repeat, GROM.c:16686-16775
    double rave[10] = {0}, rsd[10] = {0};
    long rcnt[10] = {0};
    std::vector<double> rrl(reps.size());
    for (size_t i = 0; i < reps.size(); i++) {
        rrl[i] = (double)reps[i].rd / (reps[i].end - reps[i].start);
        rave[reps[i].type] += (rrl[i] < 2 * chr_ave) ? rrl[i] : 2 * chr_ave;
        rcnt[reps[i].type] += 1;
    }
    for (int t = 0; t < 10; t++) rave[t] = rave[t] / (double)rcnt[t];
    for (size_t i = 0; i < reps.size(); i++) {
        int t = reps[i].type;
        double v = (rrl[i] < 2 * chr_ave) ? rrl[i] : 2 * chr_ave;
        rsd[t] += (v - rave[t]) * (v - rave[t]);
    }
    for (int t = 0; t < 10; t++) rsd[t] = rcnt[t] > 1 ? sqrt(rsd[t] / ((double)rcnt[t] - 1.0)) : 0;
    // The chromosome depth stdev (GROM.c:16664-16685) is a sequential double
    // sum in base order, and it only feeds the comparison below.  The terms
    // are the reference's own doubles; only their summation order differs, so
    // the reference's sum lies within gamma(n) = n*u/(1-n*u) (relative) of the
    // exact sum of the histogram's terms.  When every comparison comes out the
    // same at both ends of that interval it is decided; otherwise (or when the
    // depth histogram cannot hold twice the mean) the sum is redone on the host
    // in base order.
    auto biased_for = [&](double sd) {
        int b = -1;
        long bc = 0;
        for (int t = 0; t < 10; t++)
            if (rcnt[t] > NO_COMBINE && (rave[t] + (P.min_repeat_stdev * rsd[t])) < chr_ave &&
                (chr_ave - (P.min_repeat_stdev * sd)) > rave[t] && rcnt[t] > bc) {
                b = t;
                bc = rcnt[t];
            }
        return b;
    };
    int biased = -1;
    bool decided = false;
    if (chr_cnt <= 1) {
        biased = biased_for(0.0);
        decided = true;
    } else if (!(2 * chr_ave >= HIST_MAX) && !getenv("GROM_CNV_SERIAL_SD")) {
        long double s = 0;
        for (int v = 0; v < HIST_MAX; v++) {
            if (!hist[v]) continue;
            double term = (v < 2 * chr_ave) ? (v - chr_ave) * (v - chr_ave) : chr_ave * chr_ave;
            s += (long double)term * hist[v];
        }
        s += (long double)hist[HIST_MAX] * (long double)(chr_ave * chr_ave);
        const long double nu = (long double)chr_cnt * 0x1p-53L;
        const long double g = nu / (1.0L - nu) + 1e-15L;  // + histogram rounding and sqrt/div ulps
        const double sd_lo = (double)sqrtl(s * (1.0L - g) / ((long double)chr_cnt - 1.0L));
        const double sd_hi = (double)sqrtl(s * (1.0L + g) / ((long double)chr_cnt - 1.0L));
        const int b_lo = biased_for(nextafter(sd_lo, 0.0)), b_hi = biased_for(nextafter(sd_hi, INFINITY));
        if (b_lo == b_hi) {
            biased = b_lo;
            decided = true;
        }
    }
    if (!decided) {
        const int64_t n = A.hi - A.lo;
        std::vector<int32_t> hrd(n), hlow(n);
        std::vector<uint8_t> hacw(n);
        CK(hipMemcpyAsync(hrd.data(), d_rd + A.lo, 4 * n, hipMemcpyDeviceToHost, st));
        CK(hipMemcpyAsync(hlow.data(), d_low + A.lo, 4 * n, hipMemcpyDeviceToHost, st));
        CK(hipMemcpyAsync(hacw.data(), acw + A.lo, n, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        double sd = 0;
        for (int64_t i = 0; i < n; i++) {
            if (hacw[i] < MIN_ACGT) continue;
            const int r = hrd[i] + hlow[i];
            if (r < 2 * chr_ave) sd += (r - chr_ave) * (r - chr_ave);
            else sd += chr_ave * chr_ave;
        }
        sd = sqrt(sd / ((double)chr_cnt - 1.0));
        biased = biased_for(sd);
    }
    // 10 kb blocks over twice the mean depth -> low-variance sample blocks, GROM.c:16784-16993
    const double chr_rd_ave = (double)hacc[0] / (double)hacc[1];
    const double chr_rd_thr = P.chr_rd_threshold_factor * chr_rd_ave;
    std::vector<long> over;
    for (int64_t b = 0; b < n_blk; b++)
        if (blk_total[b] / (double)BLOCK_UNIT > chr_rd_thr) over.push_back((long)b);
    std::vector<long> bs(MAX_BLOCK_LIST), be(MAX_BLOCK_LIST);
    long tb = 0, tbs = 0, tbe = 0, nbk = 0;
    for (size_t a = 1; a < over.size(); a++) {
        if (tb == 0) {
            if ((tb + 1) > ((over[a] - over[a - 1]) / BLOCK_FACTOR)) { tbe = over[a] + 1; tb += 1; }
            else tbe = over[a - 1] + 1;
            tbs = over[a - 1];
            tb += 1;
        } else {
            if ((tb + 1) > ((over[a - 1] - tbs) / BLOCK_FACTOR)) { tbe = over[a - 1] + 1; tb += 1; }
            else {
                if (tb >= P.min_blocks) nbk += 1;
                tb = 1;
                tbs = over[a - 1];
                tbe = over[a - 1] + 1;
            }
            if (tb >= P.min_blocks && nbk < MAX_BLOCK_LIST) {
                bs[nbk] = tbs * BLOCK_UNIT;
                be[nbk] = tbe * BLOCK_UNIT;
            }
        }
    }
    if (tb >= P.min_blocks) nbk += 1;
    std::vector<long> ls(1, 0), le;
    for (long a = 0; a < nbk && a < MAX_BLOCK_LIST; a++)
        if (be[a] - bs[a] >= P.block_min) { le.push_back(bs[a]); ls.push_back(be[a]); }
    le.push_back(len);
    for (size_t k = 0; k < ls.size(); k++) {
        for (long *v : {&ls[k], &le[k]}) {
            if (*v < m - 1) *v = m - 1;
            else if (*v >= len - W) *v = len - W;
        }
    }
    std::vector<long> ss, se;  // g_lowvar_block_sample_*_list
    for (size_t k = 0; k < ls.size(); k++)
        if (!(le[k] - ls[k] < P.min_rd_window_len)) { ss.push_back(ls[k]); se.push_back(le[k]); }

    mark("pre+stats");
    // ---- A16: GC-bin samples every insert_mean/2 bases, GROM.c:18373-18456 ----
    const long half = m / 2;
    const long SAMPLE_LEN = sample_len();  // read per chromosome
    Tables T{};
    std::vector<std::vector<int>> smp[2];
    smp[0].assign(NBINS, {});
    smp[1].assign(NBINS, {});
    long idx[2][NBINS] = {{0}}, all[2][NBINS] = {{0}};
    {
        std::vector<GatherRange> rg;
        int64_t tot = 0;
        for (size_t b = 0; b < ss.size(); b++) {
            if (se[b] <= ss[b] || half <= 0) continue;
            int64_t c = (se[b] - ss[b] + half - 1) / half;
            rg.push_back(GatherRange{ss[b], c, half, tot});
            tot += c;
        }
        Gathered g;
        if ((rc = gather(S, st, rg, tot, gcw, acw, d_mq, d_rd, d_low, nullptr, g, err, errlen))) return rc;
        int last_low = 0;
        long res_over = 0, res_repl = 0;  // reservoir draws past a full list (GROM_CNV_STATS)
        auto push = [&](int k, int bin, int v) {
            if (idx[k][bin] < SAMPLE_LEN) {
                smp[k][bin].push_back(v);
                idx[k][bin] += 1;
                all[k][bin] += 1;
            } else {
                res_over++;
                if (rng.grom_rand(all[k][bin]) == 0) { smp[k][bin][rng.grom_rand(idx[k][bin])] = v; res_repl++; }
                all[k][bin] += 1;
            }
        };
        // (the most-biased-repeat samples come first in the reference and draw
        // from the same generator, GROM.c:18284-18330)
        std::vector<std::vector<int>> rsmp(REP_SEGS);
        long mb_idx[REP_SEGS] = {0}, mb_all[REP_SEGS] = {0};
        Gathered rgth;
        std::vector<GatherRange> rrg;
        if (biased != -1) {
            int64_t rt_ = 0;
            for (auto &r : reps)
                if (r.type == biased) {
                    rrg.push_back(GatherRange{r.start - half, r.end - r.start + 2 * half, 1, rt_});
                    rt_ += r.end - r.start + 2 * half;
                }
            if ((rc = gather(S, st, rrg, rt_, gcw, acw, d_mq, d_rd, d_low, nullptr, rgth, err, errlen))) return rc;
            for (auto &x : rrg) {
                const int64_t rs = x.start + half, re = x.start + x.count - half;
                for (int64_t i = 0; i < x.count; i++) {
                    const int64_t pos = x.start + i, o = x.out + i;
                    if (rgth.ac[o] < MIN_ACGT) continue;
                    int seg;
                    if (pos < rs) seg = (int)((REP_SEGS - 1) * (pos - (rs - half)) / half);
                    else if (pos >= re) seg = (int)((REP_SEGS - 1) * ((re + half) - pos) / half);
                    else seg = REP_SEGS - 1;
                    if (mb_idx[seg] < SAMPLE_LEN) {
                        rsmp[seg].push_back(rgth.rt[o]);
                        mb_idx[seg]++;
                        mb_all[seg]++;
                    } else {
                        res_over++;
                        if (rng.grom_rand(mb_all[seg]) == 0) { rsmp[seg][rng.grom_rand(mb_idx[seg])] = rgth.rt[o]; res_repl++; }
                        mb_all[seg]++;
                    }
                }
            }
        }
        for (int64_t i = 0; i < tot; i++) {
            if (g.ac[i] < MIN_ACGT) continue;
            const int bin = g.gc[i], v = g.rt[i];
            if (v == 0) push(last_low, bin, v);
            else if (g.mq[i] >= P.rd_min_mapq) { push(0, bin, v); last_low = 0; }
            else { push(1, bin, v); last_low = 1; }
        }
        for (int k = 0; k < 2; k++)
            for (int b = 0; b < NBINS; b++) sort_depths(smp[k][b]);
        if (const char *sp = getenv("GROM_CNV_STATS")) {
            FILE *sf = fopen(sp, "a");
            if (sf) { fprintf(sf, "%s over=%ld repl=%ld\n", chr_name, res_over, res_repl); fclose(sf); }
        }
        // thin bins borrow their +-2 neighbours' samples, GROM.c:18480-18548
        for (int k = 0; k < 2; k++) {
            std::vector<std::vector<int>> add(NBINS);
            bool thin[NBINS];
            for (int b = 0; b < NBINS; b++)
                thin[b] = b >= 2 && b < NBINS - 2 && idx[k][b] >= RD_MIN_WINDOWS && idx[k][b] < NO_COMBINE;
            for (int b = 0; b < NBINS; b++) {
                if (!thin[b]) continue;
                long n = idx[k][b];
                for (int a = b - 2; a <= b + 2; a++)
                    if (a != b)
                        for (long j = 0; j < idx[k][a] && n < SAMPLE_LEN; j++, n++) add[b].push_back(smp[k][a][j]);
            }
            for (int b = 0; b < NBINS; b++)
                if (thin[b]) {
                    smp[k][b].insert(smp[k][b].end(), add[b].begin(), add[b].end());
                    idx[k][b] = (long)smp[k][b].size();
                    sort_depths(smp[k][b]);
                }
        }
        // repeat-segment statistics, GROM.c:18336-18367 (only with a biased repeat)
        double rp_ave[REP_SEGS] = {0}, rp_sd[REP_SEGS] = {0};
        if (biased != -1) {
            for (int r = 0; r < REP_SEGS; r++) {
                std::sort(rsmp[r].begin(), rsmp[r].end());
                if (mb_idx[r] > 0) {
                    long s0 = mb_idx[r] / 20, e0 = mb_idx[r] - s0, n0 = e0 - s0;
                    for (long a = s0; a < e0; a++) rp_ave[r] += rsmp[r][a];
                    rp_ave[r] = rp_ave[r] / n0;
                    for (long a = s0; a < e0; a++) rp_sd[r] += pow((rsmp[r][a] - rp_ave[r]), 2);
                    if (n0 > 1) rp_sd[r] = sqrt(rp_sd[r] / (n0 - 1));
                }
            }
        }
        // bin statistics, GROM.c:18560-18641
        const double del_f = (1.0 - PLOIDY_NUM / P.ploidy), dup_f = (1.0 + PLOIDY_NUM / P.ploidy);
        std::vector<int32_t> flat;
        for (int k = 0; k < 2; k++)
            for (int b = 0; b < NBINS; b++) {
                const long n = idx[k][b];
                const std::vector<int> &l = smp[k][b];
                T.off[k][b] = (int32_t)flat.size();
                T.cnt[k][b] = (int32_t)n;
                flat.insert(flat.end(), l.begin(), l.end());
                if (n > 0) {
                    double a = 0.0;
                    for (long j = 0; j < n; j++) a += l[j];
                    a = a / n;
                    // the same sequential sum; pow() evaluated once per run of equal depths
                    double s = 0.0;
                    for (long j = 0; j < n;) {
                        const int v = l[j];
                        const double term = pow((v - a), 2);
                        for (; j < n && l[j] == v; j++) s += term;
                    }
                    if (n > 1) s = sqrt(s / (n - 1));
                    T.ave[k][b] = a;
                    T.sdv[k][b] = s;
                    T.thr[0][k][b] = del_f * a;
                    T.thr[1][k][b] = dup_f * a;
                    T.wins[k][b] = n;
                }
            }
        // pval2sd, find_disc_svs GROM.c:20705-20748
        {
            const double pp = 0.3275911, a1 = 0.254829592, a2 = -0.284496736, a3 = 1.421413741, a4 = -1.453152027,
                         a5 = 1.061405429, sd_max = 10.0;
            int n = (int)(sd_max / STDEV_STEP + 0.5) + 1;
            T.n_p2s = n;
            for (int k = 0; k < n; k++) {
                double s = sd_max - k * STDEV_STEP;
                if (s < 0) s = 0;
                double x = s / sqrt(2.0), t = 1.0 / (1.0 + pp * x);
                double e = 1.0 - ((a1 * t + a2 * pow(t, 2) + a3 * pow(t, 3) + a4 * pow(t, 4) + a5 * pow(t, 5)) *
                                  exp(-pow(x, 2)));
                T.p2s_p[k] = (1.0 - e) / 2.0;
                T.p2s_sd[k] = s;
            }
        }
        if ((rc = grow(S->samples, 4 * (flat.size() + 1), err, errlen))) return rc;
        if (!flat.empty())
            CK(hipMemcpyAsync(S->samples.p, flat.data(), 4 * flat.size(), hipMemcpyHostToDevice, st));
        CK(hipMemcpyAsync(S->tabs.p, &T, sizeof(Tables), hipMemcpyHostToDevice, st));
        const Tables *dT = (const Tables *)S->tabs.p;

        mark("sampling");
        // ---- flags, z scores ----
        int8_t *tl = (int8_t *)S->tiles.p, *cr = (int8_t *)S->carry.p;
        const unsigned sblk = (unsigned)((n_seg + 3) / 4);  // 4 waves per block
        hipLaunchKernelGGL(k_cnv_seg_last<1>, dim3(sblk), dim3(256), 0, st, A, acw, flag, d_mq, d_rd, d_low, tl);
        hipLaunchKernelGGL(k_cnv_carry, dim3(1), dim3(1024), 0, st, tl, n_seg, cr);
        hipLaunchKernelGGL(k_cnv_flags, dim3(sblk), dim3(256), 0, st, A, acw, gcw, d_mq, d_rd, d_low, cr, dT, flag);
        hipLaunchKernelGGL(k_cnv_seg_last<2>, dim3(sblk), dim3(256), 0, st, A, acw, flag, d_mq, d_rd, d_low, tl);
        hipLaunchKernelGGL(k_cnv_carry, dim3(1), dim3(1024), 0, st, tl, n_seg, cr);
        if (P.ranks_stdev != 0)
            hipLaunchKernelGGL(k_cnv_ztab, dim3((2 * NBINS * ZT_MAX + 255) / 256), dim3(256), 0, st, dT,
                               (const int32_t *)S->samples.p, A.dup_factor, (int16_t *)S->ztab.p);
        hipLaunchKernelGGL(k_cnv_z, dim3(sblk), dim3(256), 0, st, A, gcw, d_mq, d_rd, d_low, flag, cr, dT,
                           (const int32_t *)S->samples.p, (const int16_t *)S->ztab.p, sd);
        CK(hipGetLastError());

        mark("flags+z");
        // ---- the -N side file (its flags are final here; GROM.c:20234-20345) ----
        if (side && P.gen1000_window > 0) {
            const int64_t win = P.gen1000_window, n_win = len / win;
            side->clear();
            if (n_win > 0) {
                if ((rc = grow(S->gen1000, (size_t)n_win * 24, err, errlen))) return rc;
                double *d_cn = (double *)S->gen1000.p, *d_s2 = d_cn + n_win;
                int64_t *d_n = (int64_t *)(d_s2 + n_win);
                hipLaunchKernelGGL(k_cnv_gen1000, dim3((unsigned)((n_win + 255) / 256)), dim3(256), 0, st, flag, d_mq,
                                   d_rd, d_low, gcw, dT, win, n_win, (int)P.rd_min_mapq, (int)P.ploidy, d_cn, d_s2, d_n);
                CK(hipGetLastError());
                std::vector<double> hcn((size_t)n_win), hs2((size_t)n_win);
                std::vector<int64_t> hn((size_t)n_win);
                CK(hipMemcpyAsync(hcn.data(), d_cn, 8 * n_win, hipMemcpyDeviceToHost, st));
                CK(hipMemcpyAsync(hs2.data(), d_s2, 8 * n_win, hipMemcpyDeviceToHost, st));
                CK(hipMemcpyAsync(hn.data(), d_n, 8 * n_win, hipMemcpyDeviceToHost, st));
                CK(hipStreamSynchronize(st));
                side->reserve((size_t)n_win * 40);
                for (int64_t w = 0; w < n_win; w++) {
                    const double sd_w = hn[w] > 0 ? sqrt(hs2[w] / (double)hn[w]) : 0.0;
                    char line[128];
                    const int nl = snprintf(line, sizeof(line), "%ld\t%e\t%e\n", (long)(w * win), hcn[w], sd_w);
                    side->append(line, (size_t)nl);
                }
            }
        }
        // ---- window means by length, GROM.c:18967-19018 ----
        const int64_t L = P.max_rd_window_len, F = P.windows_sampling_factor, ML = P.min_rd_window_len;
        std::vector<WinDesc> wds;
        std::vector<WinPiece> wps;
        std::vector<int64_t> rlen;
        long twc = 0;  // ddd_temp_win_count carries across blocks
        for (size_t b = 0; b < ss.size(); b++) {
            std::vector<std::pair<int64_t, int64_t>> segs;  // (start, count) of each sampling pass
            for (int64_t s = 0; s < F; s++) {
                int64_t a = ss[b] + s * L / F;
                if (a < se[b]) segs.push_back({a, se[b] - a});
            }
            // chop the concatenation into windows of L
            size_t si = 0;
            int64_t so = 0;
            while (si < segs.size()) {
                WinDesc d{};
                int64_t need = L, got = 0;
                d.piece0 = (int64_t)wps.size();
                while (need > 0 && si < segs.size()) {
                    int64_t take = std::min(need, segs[si].second - so);
                    wps.push_back(WinPiece{segs[si].first + so, take});
                    so += take;
                    need -= take;
                    got += take;
                    if (so == segs[si].second) { si++; so = 0; }
                }
                d.n_pieces = (int64_t)wps.size() - d.piece0;
                d.ntot = got;
                {
                    int64_t *pp[3] = {&d.p0, &d.p1, &d.p2}, *nn[3] = {&d.n0, &d.n1, &d.n2};
                    for (int64_t q = 0; q < 3 && q < d.n_pieces; q++) {
                        *pp[q] = wps[(size_t)(d.piece0 + q)].start;
                        *nn[q] = wps[(size_t)(d.piece0 + q)].count;
                    }
                }
                if (twc == 0 && got >= ML) {
                    d.row = (int64_t)wds.size();
                    wds.push_back(d);
                    rlen.push_back(got);
                } else {
                    wps.resize((size_t)d.piece0);  // not sampled: its pieces are not needed
                }
                if (got == L) { twc += 1; if (twc == REDUCTION) twc = 0; }
            }
        }
        const int64_t n_win = (int64_t)wds.size();
        if ((rc = grow(S->wd, sizeof(WinDesc) * (n_win + 1) + sizeof(WinPiece) * (wps.size() + 1), err, errlen)) ||
            (rc = grow(S->rows, 8 * (size_t)std::max<int64_t>(n_win, 1) * (L + 1), err, errlen)) ||
            (rc = grow(S->rowlen, 8 * (n_win + 1), err, errlen)) || (rc = grow(S->wtot, 8 * (L + 1), err, errlen)) ||
            (rc = grow(S->wcnt, 8 * (L + 1), err, errlen)) || (rc = grow(S->wsd, 8 * (L + 1), err, errlen)))
            return rc;
        std::vector<double> wtot(L + 1, 0.0), wsd(L + 1, 0.0);
        std::vector<int64_t> wcnt(L + 1, 0);
        if (n_win > 0) {
            WinPiece *d_pcs = (WinPiece *)((WinDesc *)S->wd.p + n_win);
            CK(hipMemcpyAsync(S->wd.p, wds.data(), sizeof(WinDesc) * n_win, hipMemcpyHostToDevice, st));
            CK(hipMemcpyAsync(d_pcs, wps.data(), sizeof(WinPiece) * wps.size(), hipMemcpyHostToDevice, st));
            CK(hipMemcpyAsync(S->rowlen.p, rlen.data(), 8 * n_win, hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(k_cnv_windows, dim3((unsigned)((n_win + 63) / 64)), dim3(256), 0, st,
                               (const WinDesc *)S->wd.p, (const WinPiece *)d_pcs, n_win, flag, sd, L, ML,
                               (double *)S->rows.p);
            hipLaunchKernelGGL(k_cnv_window_sq, dim3((unsigned)((L - ML + 1 + 63) / 64)), dim3(256), 0, st,
                               (const double *)S->rows.p, n_win, (const int64_t *)S->rowlen.p, L, ML,
                               (double *)S->wtot.p, (int64_t *)S->wcnt.p);
            CK(hipGetLastError());
            CK(hipMemcpyAsync(wtot.data(), S->wtot.p, 8 * (L + 1), hipMemcpyDeviceToHost, st));
            CK(hipMemcpyAsync(wcnt.data(), S->wcnt.p, 8 * (L + 1), hipMemcpyDeviceToHost, st));
            CK(hipStreamSynchronize(st));
        }
        for (int64_t l = ML; l <= L; l++) wsd[l] = wcnt[l] > 1 ? sqrt(wtot[l] / (wcnt[l] - 1)) : 0.0;  // GROM.c:19162

        mark("windows");
        // ---- most-biased repeat z override, GROM.c:19022-19150 ----
        if (biased != -1 && !rrg.empty()) {
            Gathered rg2;
            int64_t rt_ = rrg.back().out + rrg.back().count;
            if ((rc = gather(S, st, rrg, rt_, gcw, acw, d_mq, d_rd, d_low, flag, rg2, err, errlen))) return rc;
            std::vector<double> zv(rt_);
            std::vector<int64_t> zp(rt_);
            int64_t nz = 0;
            for (auto &x : rrg) {
                const int64_t rs = x.start + half, re = x.start + x.count - half;
                for (int64_t i = 0; i < x.count; i++) {
                    const int64_t pos = x.start + i, o = x.out + i;
                    int seg;
                    if (pos < rs) seg = (int)((REP_SEGS - 1) * (pos - (rs - half)) / half);
                    else if (pos >= re) seg = (int)((REP_SEGS - 1) * ((re + half) - pos) / half);
                    else seg = REP_SEGS - 1;
                    if (rg2.flag[o] & F_LOW) continue;
                    const long n = mb_idx[seg];
                    const int *l = rsmp[seg].data();
                    const int r = rg2.rt[o];
                    auto bl = [&](int v) { long s_ = 0, e_ = n; int fd = 0; long i_ = s_ + (e_ - s_) / 2, lo = s_, hi = e_;
                        while (!fd) { if (i_ <= s_) { i_ = (v <= l[s_]) ? s_ : s_ + 1; fd = 1; } else if (i_ >= e_ - 1) { i_ = (v <= l[e_ - 1]) ? e_ - 1 : e_; fd = 1; }
                            else if (v <= l[i_]) { hi = i_; i_ = lo + (i_ - lo) / 2; if (hi == i_) { fd = 1; i_ += 1; } }
                            else { lo = i_; i_ = i_ + (hi - i_) / 2; if (lo == i_) { fd = 1; i_ += 1; } } } return i_; };
                    auto br = [&](int v) { long s_ = 0, e_ = n; int fd = 0; long i_ = s_ + (e_ - s_) / 2, lo = s_, hi = e_;
                        while (!fd) { if (i_ <= s_) { i_ = (v < l[s_]) ? s_ : s_ + 1; fd = 1; } else if (i_ >= e_ - 1) { i_ = (v < l[e_ - 1]) ? e_ - 1 : e_; fd = 1; }
                            else if (v < l[i_]) { hi = i_; i_ = lo + (i_ - lo) / 2; if (hi == i_) { fd = 1; i_ += 1; } }
                            else { lo = i_; i_ = i_ + (hi - i_) / 2; if (lo == i_) { fd = 1; i_ += 1; } } } return i_; };
                    auto brd = [&](double v) { long s_ = 0, e_ = T.n_p2s; int fd = 0; long i_ = s_ + (e_ - s_) / 2, lo = s_, hi = e_; const double *q = T.p2s_p;
                        while (!fd) { if (i_ <= s_) { i_ = (v < q[s_]) ? s_ : s_ + 1; fd = 1; } else if (i_ >= e_ - 1) { i_ = (v < q[e_ - 1]) ? e_ - 1 : e_; fd = 1; }
                            else if (v < q[i_]) { hi = i_; i_ = lo + (i_ - lo) / 2; if (hi == i_) { fd = 1; i_ += 1; } }
                            else { lo = i_; i_ = i_ + (hi - i_) / 2; if (lo == i_) { fd = 1; i_ += 1; } } } return i_; };
                    long i1, i2;
                    double z;
                    if (r < rp_ave[seg]) {
                        i1 = br(r);
                        i2 = bl(r);
                        double d1 = (i1 <= 0) ? 0.5 : (double)i1, d2 = (i2 <= 0) ? 0.5 : (double)i2;
                        i1 = brd((d1 + d2) / (2 * n));
                        if (i1 < 0) i1 = 0; else if (i1 >= T.n_p2s) i1 = T.n_p2s - 1;
                        z = P.ranks_stdev == 0 ? (rp_ave[seg] - rg2.rd[o] - rg2.low[o]) / rp_sd[seg] : T.p2s_sd[i1];
                    } else {
                        const bool ov = r > A.dup_factor * rp_ave[seg];
                        if (ov) { i1 = bl((int)(A.dup_factor * rp_ave[seg])); i2 = br(r); }
                        else { i1 = bl(r); i2 = br(r); }
                        i1 = n - i1;
                        i2 = n - i2;
                        double d1 = (i1 <= 0) ? 0.5 : (double)i1, d2 = (i2 <= 0) ? 0.5 : (double)i2;
                        i1 = brd((d1 + d2) / (2 * n));
                        if (i1 < 0) i1 = 0; else if (i1 >= T.n_p2s) i1 = T.n_p2s - 1;
                        if (P.ranks_stdev == 0)
                            z = ov ? (A.dup_factor - 1) * (-rp_ave[seg]) / rp_sd[seg]
                                   : (rp_ave[seg] - rg2.rd[o] - rg2.low[o]) / rp_sd[seg];
                        else z = -T.p2s_sd[i1];
                    }
                    zp[nz] = pos;
                    zv[nz] = z;
                    nz++;
                }
            }
            // later writes win, as in the reference's loop order: keep each
            // position's last value, then one upload and a scatter
            std::vector<int64_t> ord(nz);
            for (int64_t i = 0; i < nz; i++) ord[i] = i;
            std::stable_sort(ord.begin(), ord.end(), [&](int64_t x, int64_t y) { return zp[x] < zp[y]; });
            std::vector<int64_t> up_p;
            std::vector<double> up_z;
            up_p.reserve(nz);
            up_z.reserve(nz);
            for (int64_t k = 0; k < nz; k++) {
                const int64_t i = ord[k];
                if (k + 1 < nz && zp[ord[k + 1]] == zp[i]) continue;  // a later write to the same base wins
                up_p.push_back(zp[i]);
                up_z.push_back(zv[i]);
            }
            const int64_t nu = (int64_t)up_p.size();
            if (nu > 0) {
                if ((rc = grow(S->zover, 16 * (size_t)nu, err, errlen))) return rc;
                int64_t *dp = (int64_t *)S->zover.p;
                double *dz = (double *)(dp + nu);
                CK(hipMemcpyAsync(dp, up_p.data(), 8 * nu, hipMemcpyHostToDevice, st));
                CK(hipMemcpyAsync(dz, up_z.data(), 8 * nu, hipMemcpyHostToDevice, st));
                hipLaunchKernelGGL(k_cnv_zscatter, dim3((unsigned)((nu + 255) / 256)), dim3(256), 0, st, dp, dz, nu, sd);
                CK(hipGetLastError());
                CK(hipStreamSynchronize(st));  // the host vectors are released on return
            }
        }
        CK(hipMemcpyAsync(S->wsd.p, wsd.data(), 8 * (L + 1), hipMemcpyHostToDevice, st));

        // ---- DEL then DUP walk over the one lowvar block [m-1, len-W) ----
        hipLaunchKernelGGL(k_cnv_wbits, dim3((unsigned)std::min<int64_t>((len + 255) / 256, 65536)), dim3(256), 0, st,
                           A, gcw, d_mq, d_rd, d_low, flag, dT, (uint16_t *)S->wbits.p);
        CK(hipGetLastError());
        WalkIn WI{(const uint16_t *)S->wbits.p, sd, (const double *)S->wsd.p, len, m - 1, (len - W) - ML, L, ML,
                  nullptr};
        // bit words and block sums for the candidate classification (both kinds)
        CandWords CW{};
        {
            const int64_t n_words = (len + 63) / 64 + 1, n_seg = (n_words + CW_SEG - 1) / CW_SEG;
            const int64_t n_sup = (n_words + CW_SUP - 1) / CW_SUP;
            const size_t wbytes = (size_t)n_words * (15 * 8 + 4 * 8 + 8 * 8 + 1) + 256 + 2 * 8 * (size_t)n_words * 64 +
                                  sizeof(SuperW) * (size_t)n_sup + 8 * (size_t)(L + 2) + 64;
            if ((rc = grow(S->cwords, wbytes, err, errlen)) || (rc = grow(S->cw_seg, (size_t)n_seg, err, errlen)) ||
                (rc = grow(S->cw_carry, (size_t)n_seg, err, errlen)) || (rc = grow(S->wsdmin, 8 * (size_t)(L + 2), err, errlen)))
                return rc;
            uint64_t *u = (uint64_t *)S->cwords.p;
            CW.n_words = n_words;
            CW.nl = u;
            CW.def = u + n_words;
            CW.pm = u + 2 * n_words;   // 4 words
            CW.pk = u + 6 * n_words;   // 2 words
            CW.defa = u + 8 * n_words;
            CW.c1a = u + 9 * n_words;
            CW.c1n = u + 10 * n_words;
            CW.pa = u + 11 * n_words;  // 4 words
            double *dd = (double *)(u + 15 * n_words);
            CW.bsum = dd;
            CW.bmax = dd + n_words;
            CW.bmin = dd + 2 * n_words;
            CW.babs = dd + 3 * n_words;
            CW.rsn = dd + 4 * n_words;
            CW.rsa = CW.rsn + n_words * 64;
            CW.bmax4 = CW.rsa + n_words * 64;
            CW.bmin4 = CW.bmax4 + 4 * n_words;
            CW.kend = (int8_t *)(CW.bmin4 + 4 * n_words);
            {
                uintptr_t q = ((uintptr_t)(CW.kend + n_words) + 63) & ~(uintptr_t)63;
                CW.sup = (SuperW *)q;
                CW.n_sup = n_sup;
                CW.wsdmin512 = (const double *)(CW.sup + n_sup);
            }
            const unsigned gs = (unsigned)((n_seg * 64 + 255) / 256);
            hipLaunchKernelGGL(k_cnv_cls_seg, dim3(gs), dim3(256), 0, st, (const uint16_t *)S->wbits.p, len, n_seg,
                               (int8_t *)S->cw_seg.p);
            hipLaunchKernelGGL(k_cnv_carry, dim3(1), dim3(1024), 0, st, (const int8_t *)S->cw_seg.p, n_seg,
                               (int8_t *)S->cw_carry.p);
            hipLaunchKernelGGL(k_cnv_words, dim3(gs), dim3(256), 0, st, (const uint16_t *)S->wbits.p, (const double *)sd,
                               len, n_seg, (const int8_t *)S->cw_carry.p, CW);
            CK(hipGetLastError());
            std::vector<double> wmin((size_t)L + 2, 0.0);
            for (int64_t a = 0; a <= L; a++) {
                double v = wsd[a];
                for (int64_t b2 = a + 1; b2 <= std::min<int64_t>(a + 63, L); b2++) v = std::min(v, wsd[b2]);
                wmin[a] = v;
            }
            wmin[L + 1] = 0.0;
            CK(hipMemcpyAsync(S->wsdmin.p, wmin.data(), 8 * (L + 2), hipMemcpyHostToDevice, st));
            // the same over 512 lengths (phase B's block skip), from the 64-length minima
            std::vector<double> wmin512((size_t)L + 2, 0.0);
            for (int64_t a = 0; a <= L; a++) {
                double v = wmin[a];
                for (int64_t b2 = a + 64; b2 <= std::min<int64_t>(a + 511, L); b2 += 64) v = std::min(v, wmin[b2]);
                wmin512[a] = v;
            }
            CK(hipMemcpyAsync((void *)CW.wsdmin512, wmin512.data(), 8 * (L + 2), hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(k_cnv_super, dim3((unsigned)((n_sup + 255) / 256)), dim3(256), 0, st, CW);
            CK(hipGetLastError());
            CK(hipStreamSynchronize(st));  // wmin is released on scope exit
        }
        const int64_t span = std::max<int64_t>(0, WI.end - WI.start);
        const int64_t n_ch = (span + WALK_CHUNK - 1) / WALK_CHUNK;
        uint32_t call_cap = (uint32_t)std::min<int64_t>(std::max<int64_t>(4096, len / 1000), 1 << 24);
        uint32_t pre_cap = (uint32_t)std::min<int64_t>(std::max<int64_t>(1 << 16, len / 64), 1 << 26);
        uint32_t cand_cap = (uint32_t)std::min<int64_t>(std::max<int64_t>(1 << 16, len / 4), (int64_t)1 << 30);
        std::vector<CallRec> found[2];
        // both threads call this one lambda: the buffer caps are per-call locals
        auto run_kind = [&, call_cap0 = call_cap, pre_cap0 = pre_cap, cand_cap0 = cand_cap](int kind, char *err,
                                                                                          size_t errlen) -> int {
            uint32_t call_cap = call_cap0, pre_cap = pre_cap0, cand_cap = cand_cap0;
            KindBufs &K = S->kb[kind];
            hipStream_t st = K.st;
            int rc = GROM_OK;
            if ((rc = grow(K.cnt, 512, err, errlen)) || (rc = grow(K.vis, (size_t)len, err, errlen))) return rc;
            // n_calls, n_pre, n_cand, capped, n_und; walk counters from byte 64
            uint32_t *n_calls = (uint32_t *)K.cnt.p, *n_pre = n_calls + 1;
            WalkIn WK = WI;
            WK.t_defa = CW.defa;
            WK.t_c1a = CW.c1a;
            WK.t_defn = CW.def;
            WK.t_c1n = CW.c1n;
            WK.t_nl = CW.nl;
            WK.t_pa0 = CW.pa + (kind * 2 + 0) * CW.n_words;
            WK.t_pa1 = CW.pa + (kind * 2 + 1) * CW.n_words;
            WK.t_pn0 = CW.pm + (kind * 2 + 0) * CW.n_words;
            WK.t_pn1 = CW.pm + (kind * 2 + 1) * CW.n_words;
            WK.stats = tmg ? (unsigned long long *)((char *)K.cnt.p + 64) : nullptr;
            WK.prof = tmg ? WK.stats + 40 : nullptr;  // slots 40..48 (the mode offsets reach slot 21)
            CK(hipStreamWaitEvent(st, S->walk_in, 0));
            if (WK.stats) CK(hipMemsetAsync(WK.stats, 0, 448, st));
            bool done = false;
            for (int attempt = 0; attempt < 8 && !done; attempt++) {
                if ((rc = grow(K.nxt, 8 * (size_t)len, err, errlen)) ||
                    (rc = grow(K.pre, sizeof(PreAB) * pre_cap, err, errlen)) ||
                    (rc = grow(K.prepos, 8 * (size_t)cand_cap, err, errlen)) ||
                    (rc = grow(K.ppos, 8 * (size_t)pre_cap, err, errlen)) ||
                    (rc = grow(K.calls, sizeof(CallRec) * call_cap, err, errlen)) ||
                    (rc = grow(K.ok, call_cap, err, errlen)) ||
                    (rc = grow(K.tiles, sizeof(ChunkState) * n_ch, err, errlen)) ||
                    (rc = grow(K.pend, sizeof(SlideState) * n_ch, err, errlen)) ||
                    (rc = grow(K.plist, 4 * (size_t)n_ch, err, errlen)))
                    return rc;
                ChunkState *dcs = (ChunkState *)K.tiles.p;
                CallRec *dcalls = (CallRec *)K.calls.p;
                uint8_t *vis = (uint8_t *)K.vis.p;
                // the kind's counters in one fill: n_calls, n_pre, n_cand, the
                // capped call starts, n_und, the queue head (n_calls[0..5])
                CK(hipMemsetAsync(n_calls, 0, 24, st));
                CK(hipMemsetAsync(vis, 0, len, st));
                int32_t *nxt = (int32_t *)K.nxt.p;
                PreAB *pre = (PreAB *)K.pre.p;
                const unsigned gpre = (unsigned)((span + 255) / 256);
                uint32_t *n_cand = n_pre + 1;
                int64_t *cand = (int64_t *)K.prepos.p;
                if (kind == 0)
                    hipLaunchKernelGGL(k_cnv_cand<0>, dim3(gpre), dim3(256), 0, st, WK, nxt, cand, n_cand, cand_cap);
                else
                    hipLaunchKernelGGL(k_cnv_cand<1>, dim3(gpre), dim3(256), 0, st, WK, nxt, cand, n_cand, cand_cap);
                CK(hipGetLastError());
                uint32_t ncand = 0;
                CK(hipMemcpyAsync(&ncand, n_cand, 4, hipMemcpyDeviceToHost, st));
                CK(hipStreamSynchronize(st));
                if (ncand > cand_cap) {
                    cand_cap = ncand + ncand / 4 + 1024;
                    found[kind].clear();
                    continue;
                }
                if (ncand) {
                    // GROM_CNV_BUDGET (tests) shrinks the precompute budgets so the
                    // walk's wave routines take the long searches; GROM_CNV_CLASSIFY=0
                    // sends every candidate through the exact per-lane phases A/B
                    const char *bud = getenv("GROM_CNV_BUDGET");
                    const int64_t budget = bud ? std::max<int64_t>(atoll(bud), 1) : (int64_t)1 << 27;
                    const char *cl = getenv("GROM_CNV_CLASSIFY");
                    const bool classify = !(cl && strcmp(cl, "0") == 0);
                    // candidates whose phases A/B are computed exactly, one lane each
                    const int64_t *pcand = cand;
                    uint32_t npc = ncand;
                    if (classify) {
                        // no-ops and phase-A jumps settled here; the undecided rest listed
                        if ((rc = grow(K.und, 8 * (size_t)ncand, err, errlen))) return rc;
                        int64_t *und = (int64_t *)K.und.p;
                        uint32_t *n_und = n_pre + 3;
                        uint32_t *qhead = n_pre + 4;  // the classification's work queue
                        // a fixed grid of waves pulling candidates (k_cnv_classify): enough
                        // to fill the chip, never more than the candidates need
                        const unsigned gcls = (unsigned)std::max<int64_t>(1, std::min<int64_t>((ncand + 255) / 256, 2048));
                        static const int cls_queue = [] {
                            // default: lane per candidate (150 Mb chromosome, walks
                            // 32-34 ms against 40-41 ms with the queue)
                            const char *e = getenv("GROM_CNV_CLS");
                            return e ? atoi(e) : 0;
                        }();
                        if (!cls_queue) {
                            const unsigned gl = (unsigned)((ncand + 255) / 256);
                            if (kind == 0)
                                hipLaunchKernelGGL(k_cnv_classify_lane<0>, dim3(gl), dim3(256), 0, st, WK, cand, ncand, CW, (const double *)S->wsdmin.p, nxt, und, n_und, ncand);
                            else
                                hipLaunchKernelGGL(k_cnv_classify_lane<1>, dim3(gl), dim3(256), 0, st, WK, cand, ncand, CW, (const double *)S->wsdmin.p, nxt, und, n_und, ncand);
                        } else if (kind == 0)
                            hipLaunchKernelGGL(k_cnv_classify<0>, dim3(gcls), dim3(256), 0, st, WK, cand, ncand, CW, (const double *)S->wsdmin.p, nxt, und, n_und, ncand, qhead);
                        else
                            hipLaunchKernelGGL(k_cnv_classify<1>, dim3(gcls), dim3(256), 0, st, WK, cand, ncand, CW, (const double *)S->wsdmin.p, nxt, und, n_und, ncand, qhead);
                        CK(hipGetLastError());
                        uint32_t nu = 0;
                        CK(hipMemcpyAsync(&nu, n_und, 4, hipMemcpyDeviceToHost, st));
                        CK(hipStreamSynchronize(st));
                        // few undecided (calls in the noise): exact per-lane precompute;
                        // many (calls inside long regions, of which the walk visits the
                        // first): the walk decides them
                        npc = (int64_t)nu * L <= budget ? nu : 0;
                        pcand = und;
                        if (tmg) {
                            unsigned long long cs8[8];
                            (void)hipMemcpy(cs8, WK.stats + 24, sizeof(cs8), hipMemcpyDeviceToHost);
                            unsigned long long cb4[4];
                            (void)hipMemcpy(cb4, WK.stats + 32, sizeof(cb4), hipMemcpyDeviceToHost);
                            fprintf(stderr, "cnv classify %s blocks: %llu reached, %llu with known pass bits, %llu walk clear, %llu skipped\n",
                                    kind == 0 ? "DEL" : "DUP", cb4[0], cb4[1], cb4[2], cb4[3]);
                            fprintf(stderr, "cnv classify %s: %u candidates, %u undecided (%s); jumps %llu, first-window "
                                    "undecided %llu, B undecided %llu, no-ops %llu, bases tested %llu, segments settled by the bound %llu, "
                                    "segments tested %llu\n", kind == 0 ? "DEL" : "DUP", ncand, nu,
                                    npc ? "precomputed" : "left to the walk", cs8[1], cs8[2], cs8[5], cs8[6], cs8[3],
                                    cs8[4], cs8[7]);
                        }
                    }
                    if (npc > pre_cap) {  // every precomputed candidate may start a call: no re-run
                        pre_cap = npc;
                        if ((rc = grow(K.pre, sizeof(PreAB) * pre_cap, err, errlen)) ||
                            (rc = grow(K.ppos, 8 * (size_t)pre_cap, err, errlen)))
                            return rc;
                        pre = (PreAB *)K.pre.p;
                    }
                    if (npc) {
                        const int64_t ab_cap = bud ? std::max<int64_t>(std::min<int64_t>(L, budget / npc), ML + 256) : L;
                        if (kind == 0)
                            hipLaunchKernelGGL(k_cnv_pre<0>, dim3((npc + 255) / 256), dim3(256), 0, st, WK, pcand, npc, nxt, pre, n_pre, pre_cap, (int64_t *)K.ppos.p, ab_cap);
                        else
                            hipLaunchKernelGGL(k_cnv_pre<1>, dim3((npc + 255) / 256), dim3(256), 0, st, WK, pcand, npc, nxt, pre, n_pre, pre_cap, (int64_t *)K.ppos.p, ab_cap);
                        CK(hipGetLastError());
                        // phases C/D for every call start, within the same kind of budget
                        // (the walk finishes the rest)
                        const int64_t cd_cap = std::max<int64_t>(
                            std::min<int64_t>(4 * L + 4 * MAX_DIST_LAST_GOOD, budget / std::max<uint32_t>(npc / 4, 1)),
                            (int64_t)1024);
                        const unsigned gpost = (unsigned)((std::min<int64_t>(npc, pre_cap) + 255) / 256);
                        if (kind == 0)
                            hipLaunchKernelGGL(k_cnv_post<0>, dim3(gpost), dim3(256), 0, st, WK, pre, n_pre, pre_cap, (const int64_t *)K.ppos.p, cd_cap, n_pre + 2);
                        else
                            hipLaunchKernelGGL(k_cnv_post<1>, dim3(gpost), dim3(256), 0, st, WK, pre, n_pre, pre_cap, (const int64_t *)K.ppos.p, cd_cap, n_pre + 2);
                        CK(hipGetLastError());
                    }
                }
                const unsigned gch = (unsigned)n_ch;  // one wave per chunk
                SlideState *pend = (SlideState *)K.pend.p;
                if (kind == 0)
                    hipLaunchKernelGGL(k_cnv_walk<0>, dim3(gch), dim3(64), 0, st, WK, nxt, pre, 0, n_ch, WALK_CHUNK, vis, dcs, pend, dcalls, n_calls, call_cap);
                else
                    hipLaunchKernelGGL(k_cnv_walk<1>, dim3(gch), dim3(64), 0, st, WK, nxt, pre, 0, n_ch, WALK_CHUNK, vis, dcs, pend, dcalls, n_calls, call_cap);
                CK(hipGetLastError());
                std::vector<ChunkState> hcs(n_ch);
                // paused slides (k_cnv_walk_resume): resume, round by round, the
                // pending chunks whose predecessor's exit is known and lands in
                // them; a pending chunk that exit jumps over takes that exit
                std::vector<int32_t> plist;
                int n_rounds = 0;
                for (;;) {
                    CK(hipMemcpyAsync(hcs.data(), dcs, sizeof(ChunkState) * n_ch, hipMemcpyDeviceToHost, st));
                    CK(hipStreamSynchronize(st));
                    plist.clear();
                    bool covered = false;
                    for (int64_t k = 0; k < n_ch; k++) {
                        if (hcs[k].status != ST_PENDING) continue;
                        if (k > 0 && hcs[k - 1].status == ST_PENDING) continue;
                        const int64_t c1 = std::min<int64_t>(WK.end, WK.start + (k + 1) * WALK_CHUNK);
                        if (k > 0 && hcs[k - 1].x1 >= c1) {
                            hcs[k].x1 = hcs[k - 1].x1;
                            hcs[k].l1 = hcs[k - 1].l1;
                            hcs[k].status = ST_MERGED;
                            covered = true;
                        } else {
                            plist.push_back((int32_t)k);
                        }
                    }
                    if (covered) CK(hipMemcpyAsync(dcs, hcs.data(), sizeof(ChunkState) * n_ch, hipMemcpyHostToDevice, st));
                    if (plist.empty()) break;
                    n_rounds++;
                    CK(hipMemcpyAsync(K.plist.p, plist.data(), 4 * plist.size(), hipMemcpyHostToDevice, st));
                    const int32_t *dl = (const int32_t *)K.plist.p;
                    if (kind == 0)
                        hipLaunchKernelGGL(k_cnv_walk_resume<0>, dim3((unsigned)plist.size()), dim3(64), 0, st, WK, nxt, pre, dl, WALK_CHUNK, vis, dcs, pend, dcalls, n_calls, call_cap);
                    else
                        hipLaunchKernelGGL(k_cnv_walk_resume<1>, dim3((unsigned)plist.size()), dim3(64), 0, st, WK, nxt, pre, dl, WALK_CHUNK, vis, dcs, pend, dcalls, n_calls, call_cap);
                    CK(hipGetLastError());
                }
                if (tmg) fprintf(stderr, "cnv walk %s: %d resume rounds\n", kind == 0 ? "DEL" : "DUP", n_rounds);
                if (kind == 0)
                    hipLaunchKernelGGL(k_cnv_walk<0>, dim3(gch), dim3(64), 0, st, WK, nxt, pre, 1, n_ch, WALK_CHUNK, vis, dcs, pend, dcalls, n_calls, call_cap);
                else
                    hipLaunchKernelGGL(k_cnv_walk<1>, dim3(gch), dim3(64), 0, st, WK, nxt, pre, 1, n_ch, WALK_CHUNK, vis, dcs, pend, dcalls, n_calls, call_cap);
                CK(hipGetLastError());
                // reconcile (k_cnv_reconcile, one wave): the true exit of each
                // chunk in order, repairs, the chunks the walk jumps over
                if ((rc = grow(K.skip, (size_t)n_ch, err, errlen))) return rc;
                uint32_t *d_nfix = n_calls + 8;  // (a free word of the counters, byte 32)
                if (kind == 0)
                    hipLaunchKernelGGL(k_cnv_reconcile<0>, dim3(1), dim3(64), 0, st, WK, nxt, pre, n_ch, WALK_CHUNK, vis, dcs,
                                       dcalls, n_calls, call_cap, (uint8_t *)K.skip.p, d_nfix);
                else
                    hipLaunchKernelGGL(k_cnv_reconcile<1>, dim3(1), dim3(64), 0, st, WK, nxt, pre, n_ch, WALK_CHUNK, vis, dcs,
                                       dcalls, n_calls, call_cap, (uint8_t *)K.skip.p, d_nfix);
                CK(hipGetLastError());
                int64_t n_fix = 0;
                if (tmg) {
                    uint32_t np_[3] = {0, 0, 0};
                    (void)hipMemcpy(np_, n_pre, 12, hipMemcpyDeviceToHost);
                    unsigned long long wsa[22] = {0};
                    (void)hipMemcpy(wsa, WK.stats, sizeof(wsa), hipMemcpyDeviceToHost);
                    for (int mo = 0; mo < 4; mo++)
                        fprintf(stderr, "cnv walk %s %s: stops %llu, wave A/B %llu, wave C/D %llu, slide rounds %llu, trim rounds %llu\n",
                                kind == 0 ? "DEL" : "DUP", mo == 0 ? "mode 0" : mo == 1 ? "mode 1" : mo == 2 ? "repairs" : "resumed",
                                wsa[5 * mo + 4], wsa[5 * mo], wsa[5 * mo + 1], wsa[5 * mo + 2], wsa[5 * mo + 3]);
                    fprintf(stderr, "cnv walk %s: longest resumed slide %llu steps in %llu wall-clock ticks\n",
                            kind == 0 ? "DEL" : "DUP", wsa[20], wsa[21]);
                    unsigned long long ck2[9];
                    (void)hipMemcpy(ck2, WK.stats + 40, sizeof(ck2), hipMemcpyDeviceToHost);
                    fprintf(stderr, "cnv walk %s: slide cycles %llu: before the sum chain %llu, chain %llu, after %llu; "
                            "longest resumed slide %llu clocks; chain guesses repaired %llu; longest resumed wave %llu "
                            "clocks (trim %llu, walk on %llu)\n",
                            kind == 0 ? "DEL" : "DUP", ck2[1], ck2[2], ck2[0], ck2[3], ck2[4], ck2[5], ck2[6], ck2[7],
                            ck2[8]);
                    unsigned long long ws[5];
                    for (int q = 0; q < 5; q++) ws[q] = wsa[q] + wsa[5 + q] + wsa[10 + q] + wsa[15 + q];
                    fprintf(stderr, "cnv walk %s: %lld chunks, %lld repaired, %u candidates, %u call starts (%u left to the walk); "
                            "walk stops %llu, wave A/B %llu, wave C/D %llu (%llu slide rounds, %llu trim rounds)\n",
                            kind == 0 ? "DEL" : "DUP", (long long)n_ch, (long long)n_fix, ncand, np_[0], np_[2], ws[4],
                            ws[0], ws[1], ws[2], ws[3]);
                }
                // n_calls, n_pre (adjacent) and the repairs in one copy
                uint32_t hn[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
                CK(hipMemcpyAsync(hn, n_calls, sizeof(hn), hipMemcpyDeviceToHost, st));
                CK(hipStreamSynchronize(st));
                const uint32_t nc = hn[0], npre = hn[1];
                n_fix = hn[8];
                (void)n_fix;
                if (npre > pre_cap || nc > call_cap) {
                    pre_cap = std::max(pre_cap, npre + npre / 4 + 1024);
                    call_cap = std::max(call_cap, nc + nc / 4 + 1024);
                    found[kind].clear();
                    continue;
                }
                std::vector<CallRec> hc(nc);
                std::vector<uint8_t> ok(nc);
                if (nc) {
                    hipLaunchKernelGGL(k_cnv_calls_valid, dim3((nc + 255) / 256), dim3(256), 0, st, dcalls, nc, vis,
                                       (const uint8_t *)K.skip.p, WK.start, WALK_CHUNK, (uint8_t *)K.ok.p);
                    CK(hipMemcpyAsync(hc.data(), dcalls, sizeof(CallRec) * nc, hipMemcpyDeviceToHost, st));
                    CK(hipMemcpyAsync(ok.data(), K.ok.p, nc, hipMemcpyDeviceToHost, st));
                    CK(hipStreamSynchronize(st));
                }
                for (uint32_t i = 0; i < nc; i++)
                    if (ok[i]) found[kind].push_back(hc[i]);
                std::sort(found[kind].begin(), found[kind].end(),
                          [](const CallRec &a, const CallRec &b) { return a.p < b.p; });
                found[kind].erase(std::unique(found[kind].begin(), found[kind].end(),
                                              [](const CallRec &a, const CallRec &b) { return a.p == b.p; }),
                                  found[kind].end());
                done = true;
            }
            if (!done) {
                snprintf(err, errlen, "CNV window-search buffers could not be sized");
                return GROM_E_NOMEM;
            }
            return GROM_OK;
        };
        if (n_ch > 0) {
            CK(hipEventRecord(S->walk_in, st));
            char kerr[2][512] = {{0}, {0}};
            int krc[2] = {GROM_OK, GROM_OK};
            int dev = 0;
            CK(hipGetDevice(&dev));
            std::thread dup_thread([&] {  // a new host thread starts on device 0: select ours
                if (hipSetDevice(dev) != hipSuccess) {
                    snprintf(kerr[1], sizeof(kerr[1]), "hipSetDevice(%d) failed in the CNV DUP thread", dev);
                    krc[1] = GROM_E_HIP;
                    return;
                }
                krc[1] = run_kind(1, kerr[1], sizeof(kerr[1]));
            });
            krc[0] = run_kind(0, kerr[0], sizeof(kerr[0]));
            dup_thread.join();
            for (int kind = 0; kind < 2; kind++)
                if (krc[kind] != GROM_OK) {
                    snprintf(err, errlen, "%s", kerr[kind]);
                    return krc[kind];
                }
        }
        CK(hipEventRecord(S->e1, st));
        mark("walks");

        // ---- p value (Q8), filter, copy number, rows: GROM.c:17139-17300, 20024-20228 ----
        const double pp = 0.3275911, a1 = 0.254829592, a2 = -0.284496736, a3 = 1.421413741, a4 = -1.453152027,
                     a5 = 1.061405429;
        int64_t n_rows = 0;
        for (int kind = 0; kind < 2; kind++) {
            std::vector<std::pair<size_t, double>> keep;
            for (size_t i = 0; i < found[kind].size(); i++) {
                double x = fabs(found[kind][i].stdevs) / sqrt(2.0);
                double t = 1.0 / (1.0 + pp + x);
                double e = 1.0 - ((a1 * t + a2 * pow(t, 2) + a3 * pow(t, 3) + a4 * pow(t, 4) + a5 * pow(t, 5)) *
                                  exp(-pow(x, 2)));
                double pv = (1.0 - e) / 2.0;
                if (pv < P.rd_pval_threshold) keep.push_back({i, pv});
            }
            std::vector<GatherRange> rg;
            int64_t tot = 0;
            for (auto &kp : keep) {
                const CallRec &c = found[kind][kp.first];
                int64_t n = std::max<int64_t>(0, c.ce - c.p);
                rg.push_back(GatherRange{c.p, n, 1, tot});
                tot += n;
            }
            const auto tg0 = std::chrono::steady_clock::now();
            if (tot > 0) {
                const size_t nb = (size_t)tot;
                if ((rc = grow(S->gat_rg, sizeof(GatherRange) * rg.size(), err, errlen)) ||
                    (rc = grow(S->cn_v, 8 * nb, err, errlen)))
                    return rc;
                if (S->h_cn_cap < nb) {
                    if (S->h_cn) (void)hipHostFree(S->h_cn);
                    S->h_cn = nullptr;
                    S->h_cn_cap = 0;
                    const size_t want = nb + nb / 4 + 4096;
                    CK(hipHostMalloc((void **)&S->h_cn, 8 * want, 0));
                    S->h_cn_cap = want;
                }
                CK(hipMemcpyAsync(S->gat_rg.p, rg.data(), sizeof(GatherRange) * rg.size(), hipMemcpyHostToDevice, st));
                const int g_ = (int)std::min<int64_t>((tot + 255) / 256, 16384);
                hipLaunchKernelGGL(k_cnv_cn_ratio, dim3(g_), dim3(256), 0, st, (const GatherRange *)S->gat_rg.p,
                                   (int)rg.size(), gcw, d_mq, d_rd, d_low, flag, dT, (int32_t)P.rd_min_mapq, tot,
                                   (double *)S->cn_v.p);
                CK(hipGetLastError());
                CK(hipMemcpyAsync(S->h_cn, S->cn_v.p, 8 * nb, hipMemcpyDeviceToHost, st));
                CK(hipStreamSynchronize(st));
            }
            const auto tg1 = std::chrono::steady_clock::now();
            // copy number of every kept call (GROM.c:20100-20160): independent per
            // call, so host threads share them; the rows are then written in order
            std::vector<double> cnv_cn(keep.size(), -1.0), cnv_cs(keep.size(), 0.0);
            auto cn_of = [&](size_t j, std::vector<double> &pl, std::vector<double> &tmp) {
                pl.clear();
                const double *v = S->h_cn + rg[j].out;
                for (int64_t i = 0; i < rg[j].count; i++)
                    if (v[i] < HUGE_VAL) pl.push_back(v[i]);  // (the reference's list, in base order)
                double cn = -1, cns = 0;
                const long pc = (long)pl.size();
                if (pc > 0) {
                    tmp.resize(pc);
                    msort_lo_par(pl.data(), pl.size(), tmp.data(), 3);
                    long s0 = 0.1 * pc, e0 = pc - s0;
                    double sum = 0.0;
                    for (long i = s0; i < e0; i++) sum += pl[i];
                    if (e0 - s0 > 0) {
                        cn = (sum / (e0 - s0)) * P.ploidy;
                        cns = 0;
                        for (long i = 0; i < pc; i++) cns += pow((P.ploidy * pl[i] - cn), 2);
                        cns = sqrt(cns / pc);
                    }
                }
                cnv_cn[j] = cn;
                cnv_cs[j] = cns;
            };
            {
                int64_t work = 0;
                for (size_t j = 0; j < keep.size(); j++) work += rg[j].count;
                const unsigned nt = (unsigned)std::min<int64_t>({(int64_t)8, (int64_t)keep.size(), 1 + work / 200000});
                std::atomic<size_t> next{0};
                auto worker = [&] {
                    std::vector<double> pl, tmp;
                    for (size_t j; (j = next.fetch_add(1)) < keep.size();) cn_of(j, pl, tmp);
                };
                std::vector<std::thread> th;
                for (unsigned t = 1; t < nt; t++) th.emplace_back(worker);
                worker();
                for (auto &t : th) t.join();
                if (tmg) {
                    const auto tg2 = std::chrono::steady_clock::now();
                    int64_t mx = 0;
                    for (size_t j = 0; j < keep.size(); j++) mx = std::max<int64_t>(mx, rg[j].count);
                    fprintf(stderr, "cnv rows %s: %zu calls, %lld bases (largest %lld), %u threads; gather %.1f ms, copy number %.1f ms\n",
                            kind == 0 ? "DEL" : "DUP", keep.size(), (long long)tot, (long long)mx, nt,
                            std::chrono::duration<double, std::milli>(tg1 - tg0).count(),
                            std::chrono::duration<double, std::milli>(tg2 - tg1).count());
                }
            }
            // -f: a column header before each kind's rows (GROM.c:17242-17245,
            // 17378), rows named by caf_del_text / caf_dup_text (GROM.c:1575)
            if (P.vcf != 1) rows += "SV Type\tChromosome\tStart\tEnd\tStdev from mean\tP Value\tCopy Number\n";
            for (size_t j = 0; j < keep.size(); j++) {
                const CallRec &c = found[kind][keep[j].first];
                char line[512];
                int nl;
                if (P.vcf != 1)  // GROM.c:17340-17343
                    nl = snprintf(line, sizeof(line), "%s\t%s\t%lld\t%lld\t%e\t%e\t%e\t%e\n", kind == 0 ? "DEL RD" : "DUP RD",
                                  chr_name, (long long)c.p, (long long)c.ce, c.stdevs, keep[j].second, cnv_cn[j], cnv_cs[j]);
                else
                    nl = snprintf(line, sizeof(line), "%s\t%lld\t.\t.\t%s\t.\t.\tEND=%lld\tSD:Z:CN:CS\t%e:%e:%.2f:%e\n",
                                  chr_name, (long long)c.p + 1, kind == 0 ? "<DEL>" : "<DUP>", (long long)c.ce + 1,
                                  c.stdevs, keep[j].second, cnv_cn[j], cnv_cs[j]);
                rows.append(line, (size_t)nl);
                n_rows++;
            }
        }
        mark("rows");
        if (tmg) fprintf(stderr, "cnv phases ms:%s\n", tlog.c_str());
        if (timing) {
            float ms = 0;
            (void)hipEventElapsedTime(&ms, S->e0, S->e1);
            timing->ms_device = ms;
            timing->del_calls = (int64_t)found[0].size();
            timing->dup_calls = (int64_t)found[1].size();
            timing->rows = n_rows;
        }
    }
    if (timing)
        timing->ms_host =
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_host0).count();
    return GROM_OK;
}
