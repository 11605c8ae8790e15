// scan.hip -- MI355X (gfx950) implementation of GROM's per-chromosome scan
// behind the C ABI of include/grom_amd.h.
//
// The reference walks a chromosome base by base (GROM.c:5842), ingesting each
// read into a sliding ring of per-position counters (GROM.c:6406-10966) and
// evaluating each base once every read that can touch it has been ingested
// (GROM.c:11086-13553).  Here the chromosome is cut into tiles of GROM_TILE
// absolute positions; one workgroup owns a tile and builds every counter of
// its positions in LDS from all reads overlapping it, then evaluates them.
// Counters that are plain sums are accumulated with LDS atomics in any order;
// the order-dependent step -- read-name de-duplication of mismatching bases
// (GROM.c:6805-6824) -- is turned into an event list that is sorted by read
// order per position and folded by the position's owning thread.
//
// Kernels (one launch each per chromosome):
//   k_span        longest reference extent of any read (tile halo)
//   k_tile_ranges per-tile [first,last) read range, from the sorted positions
//   k_rmdup       -M duplicate filter (GROM.c:6432-6588), per start position
//   k_pileup      the tile kernel: caf read depth, SNV tally, soft-clip
//                 evidence, physical read depth, SNV test, flush sums
//   k_flush_sum   read-depth sum for mid-scan SNV list flushes (rare)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/grom_amd.h"
#include "scan_common.h"

#define T GROM_TILE
#define NTHR GROM_TILE_THREADS
#define NWAVES (NTHR / 64)

static char g_err[512];
static void set_err(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

#define HIPCHK(x)                                                                               \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            set_err("HIP error %s at %s:%d (%s)", hipGetErrorString(e_), __FILE__, __LINE__, #x); \
            return GROM_E_HIP;                                                                  \
        }                                                                                       \
    } while (0)

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

// ---------------------------------------------------------------------------
// k_span: reads' M/D/N/=/X extent; the tile halo
// ---------------------------------------------------------------------------
__global__ void k_span(int64_t n, const uint32_t *__restrict__ cig_off, const uint32_t *__restrict__ cigar,
                       const int32_t *__restrict__ lqseq, int32_t *__restrict__ out_max) {
    int32_t best = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        // reference extent of the tally (M/D/N/=/X) and a bound on the end
        // E = pos - start_adj + lseq - end_adj - (I - D) used for clips/depth
        int32_t s = 0, e = lqseq[i];
        for (uint32_t k = cig_off[i]; k < cig_off[i + 1]; k++) {
            uint32_t c = cigar[k];
            int op = c & 15;
            int32_t len = (int32_t)(c >> 4);
            if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) s += len;
            if (op == 2 || op == 5) e += len;
        }
        best = max(best, max(s, e) + 1);
    }
    for (int o = 32; o > 0; o >>= 1) best = max(best, __shfl_xor(best, o, 64));
    if ((threadIdx.x & 63) == 0) atomicMax(out_max, best);
}

// ---------------------------------------------------------------------------
// k_tile_ranges: lo[t] = lower_bound(pos, t*T - halo), hi[t] = lower_bound(pos, t*T + T + 1)
// computed scatter-style from consecutive read positions (no binary search).
// ---------------------------------------------------------------------------
__global__ void k_tile_ranges(int64_t n, const int32_t *__restrict__ pos, const int32_t *__restrict__ halo_p,
                              int64_t n_tiles, int32_t *__restrict__ lo, int32_t *__restrict__ hi) {
    const int64_t halo = *halo_p;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t big = (int64_t)1 << 40;
        int64_t prev = (i == 0) ? -big : (int64_t)pos[i - 1];
        int64_t cur = (i == n) ? big : (int64_t)pos[i];
        // lo: tiles t with prev < t*T - halo <= cur
        int64_t a = floordiv(prev + halo, T) + 1, b = floordiv(cur + halo, T);
        a = max(a, (int64_t)0);
        b = min(b, n_tiles - 1);
        for (int64_t t = a; t <= b; t++) lo[t] = (int32_t)i;
        // hi: tiles t with prev < t*T + T + 1 <= cur
        a = floordiv(prev - T - 1, T) + 1;
        b = floordiv(cur - T - 1, T);
        a = max(a, (int64_t)0);
        b = min(b, n_tiles - 1);
        for (int64_t t = a; t <= b; t++) hi[t] = (int32_t)i;
    }
}

// ---------------------------------------------------------------------------
// k_rmdup: GROM's -M filter.  A paired read with a mapped mate is classed by
// orientation (DEL/INV_F/INV_R/DUP/CTX_xx, GROM.c:6432-6529) and dropped when
// an earlier listed read with the same start has the same (mate chr, mate pos,
// length, isize, class) and the read's MAPQ >= -q (GROM.c:6546-6581).  The list
// is per start position, so each distinct position is one sequential fold.
// keep[i]: 0 dropped, 1 kept, 2 kept and listed.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool rm_eligible(uint16_t f) { return (f & 0x1) && !(f & 0x8); }

__device__ __forceinline__ int rm_svtype(int32_t tid, int32_t mtid, int32_t p, int32_t mp, uint16_t f) {
    bool rev = f & 0x10, mrev = f & 0x20;
    if (tid == mtid) {
        if (mp > p) {
            if (!rev && mrev) return 0;  // DEL
            if (!rev && !mrev) return 8; // INV_F
            return mrev ? 9 : 1;         // INV_R : DUP
        }
        if (rev && !mrev) return 0;
        if (!rev && !mrev) return 8;
        return rev ? 9 : 1;
    }
    if (!rev) return mrev ? 12 : 11;
    return mrev ? 14 : 13;
}

__global__ void k_rmdup(int64_t n, int32_t tid, const int32_t *__restrict__ pos, const uint16_t *__restrict__ flag,
                        const uint8_t *__restrict__ mapq, const int32_t *__restrict__ mtid,
                        const int32_t *__restrict__ mpos, const int32_t *__restrict__ isize,
                        const int32_t *__restrict__ lqseq, int32_t min_mapq, int32_t list_len,
                        uint8_t *__restrict__ keep) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!rm_eligible(flag[i])) { keep[i] = 1; continue; }
        bool leader = true;
        for (int64_t j = i - 1; j >= 0 && pos[j] == pos[i]; j--)
            if (rm_eligible(flag[j])) { leader = false; break; }
        if (!leader) continue;
        int listed = 0;
        for (int64_t j = i; j < n && pos[j] == pos[i]; j++) {
            if (!rm_eligible(flag[j])) continue;
            int sv = rm_svtype(tid, mtid[j], pos[j], mpos[j], flag[j]);
            bool add = true;
            if (j != i && mapq[j] >= min_mapq) {
                for (int64_t r = i; r < j; r++) {
                    if (!rm_eligible(flag[r]) || keep[r] != 2) continue;
                    if (mpos[r] == mpos[j] && mtid[r] == mtid[j] && lqseq[r] == lqseq[j] && isize[r] == isize[j] &&
                        rm_svtype(tid, mtid[r], pos[r], mpos[r], flag[r]) == sv) {
                        add = false;
                        break;
                    }
                }
            }
            if (!add) { keep[j] = 0; continue; }
            if (listed < list_len) { keep[j] = 2; listed++; }
            else keep[j] = 1;
        }
    }
}

// ---------------------------------------------------------------------------
// k_pileup: the tile kernel
// ---------------------------------------------------------------------------
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
    unsigned long long *flush_acc;  // [0] sum of caf rd, [1] non-N bases
    int32_t *dbg;                   // nullable: GC_COUNT int32 per evaluated base
    uint32_t *status;               // [0] event overflow count, [1] first overflowing tile
    uint32_t *n_events;             // total events (stats)
};

// event word x: [0..9] position in tile, [10..12] kind, [13] forward strand,
// [16..23] base quality, [24..31] MAPQ.  kind 0..3: mismatching A/C/G/T,
// 4: mismatching non-ACGT, 5: left soft clip, 6: right soft clip.
// y: read index.  z: read-name id (mismatch) or category bits | add<<8 (clip).
// w: query offset of the base (mismatch).
enum { EV_CLIP_L = 5, EV_CLIP_R = 6 };

struct __align__(16) PileLds {
    unsigned long long snvfs[4][T];  // lo32: cdp_one_base_snv, hi32: fstrand
    unsigned long long bqmq_hi[T];   // lo32: bq, hi32: mq  (MAPQ >= q && BQ >= b)
    unsigned long long bqmq_lo[T];   // lo32: bq, hi32: mq  (the other bases)
    uint32_t lowmq[4][T];
    uint32_t pir[4][T];
    int32_t diff[4][T + 1];          // rd, caf_mq, caf_rd, caf_low difference arrays
    uint4 ev[GROM_EVENT_CAP];
    uint16_t ev_sorted[GROM_EVENT_CAP];
    uint32_t ev_cnt[T];
    uint32_t ev_fill[T];
    char ref[T];
    int32_t wsum[NWAVES][5];
    unsigned long long red[NWAVES][2];
    uint32_t nev;
    int32_t r0, r1;
};

__device__ __forceinline__ void push_event(PileLds &L, uint4 e) {
    uint32_t k = atomicAdd(&L.nev, 1u);
    if (k < GROM_EVENT_CAP) L.ev[k] = e;
}

// inclusive scan of L.diff[0..3][0..T) and exclusive scan of L.ev_cnt,
// 256 threads x 2 consecutive elements
__device__ void tile_scans(PileLds &L) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    int32_t v[5][2], excl[5];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        v[k][0] = L.diff[k][2 * t];
        v[k][1] = L.diff[k][2 * t + 1];
    }
    const int32_t c0 = (int32_t)L.ev_cnt[2 * t], c1 = (int32_t)L.ev_cnt[2 * t + 1];
    v[4][0] = c0;
    v[4][1] = c1;
#pragma unroll
    for (int k = 0; k < 5; k++) {
        v[k][1] += v[k][0];
        int32_t s = v[k][1];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            int32_t u = __shfl_up(s, o, 64);
            if (lane >= o) s += u;
        }
        excl[k] = s - v[k][1];
        if (lane == 63) L.wsum[w][k] = s;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 5; k++) {
        int32_t off = excl[k];
        for (int ww = 0; ww < w; ww++) off += L.wsum[ww][k];
        v[k][0] += off;
        v[k][1] += off;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        L.diff[k][2 * t] = v[k][0];
        L.diff[k][2 * t + 1] = v[k][1];
    }
    L.ev_cnt[2 * t] = (uint32_t)(v[4][0] - c0);
    L.ev_cnt[2 * t + 1] = (uint32_t)(v[4][1] - c1);
    __syncthreads();
}

__global__ __launch_bounds__(NTHR) void k_pileup(grom_scan_args a, const char *__restrict__ ref, ReadArrays R,
                                                  const int32_t *__restrict__ tile_lo,
                                                  const int32_t *__restrict__ tile_hi, PileOut O,
                                                  const double *__restrict__ mq_tab,
                                                  const double *__restrict__ hez_tab) {
    __shared__ PileLds L;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t t0 = (int64_t)blockIdx.x * T;

    // ---- phase 0: clear, stage the reference tile ----
    for (int i = tid; i < T; i += NTHR) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            L.snvfs[k][i] = 0;
            L.lowmq[k][i] = 0;
            L.pir[k][i] = 0;
            L.diff[k][i] = 0;
        }
        L.bqmq_hi[i] = 0;
        L.bqmq_lo[i] = 0;
        L.ev_cnt[i] = 0;
        L.ev_fill[i] = 0;
        int64_t x = t0 + i;
        L.ref[i] = (x < a.chr_len) ? upcase(ref[x]) : 'N';
    }
    if (tid < 4) L.diff[tid][T] = 0;
    if (tid == 0) {
        L.nev = 0;
        L.r0 = tile_lo[blockIdx.x];
        L.r1 = tile_hi[blockIdx.x];
    }
    __syncthreads();
    const int32_t r0 = L.r0, r1 = L.r1;
    // positions of this tile that are evaluated (GROM.c:11086, 5842)
    const int64_t ev_lo = max((int64_t)a.eval_lo, t0), ev_hi = min((int64_t)a.eval_hi, t0 + T - 1);
    const bool tile_evals = ev_lo <= ev_hi;

    // ---- phase 1: every read overlapping the tile, one wave per read ----
    for (int32_t r = r0 + wave; r < r1; r += NWAVES) {
        const int32_t p0 = R.pos[r];
        const uint16_t fl = R.flag[r];
        const int mq = R.mapq[r];
        if (R.keep && R.keep[r] == 0) continue;
        const uint32_t c0 = R.cig_off[r], c1 = R.cig_off[r + 1];
        const int64_t bo = R.base_off[r];
        const int lq = R.lqseq[r];
        const bool fwd = !(fl & 0x10);
        const bool hq_read = mq >= a.min_mapq;
        const int add = hq_read ? 6 : 0;  // cdp_add, GROM.c:5829-5836
        const uint32_t nid = R.name_id[r];
        const bool pos_ok = p0 >= 0 && p0 < a.chr_len;
        int snv_base = 0, snv_ref_base = 0, lseq_mod = lq, end_adj_indel = 0;
        int64_t caf_pos = p0;
        int first_op = -1, first_len = 0, last_op = -1, last_len = 0;
        const uint32_t ncap = (c1 - c0 > 1000u) ? c0 + 1000u : c1;  // cdp_c_type_len, GROM.c:6743
        for (uint32_t k = c0; k < c1; k++) {
            const uint32_t cg = R.cigar[k];
            const int op = cg & 15;
            const int len = (int)(cg >> 4);
            const bool in_cap = k < ncap;
            if (op == 0 || op == 7 || op == 8) {
                // whole-chromosome read depth, GROM.c:6605-6671 (every op)
                if (caf_pos >= 0 && caf_pos + len < a.chr_len) {
                    int64_t lo = max(caf_pos, t0), hi = min(caf_pos + len, t0 + T);
                    if (lo < hi && lane == 0) {
                        atomicAdd(&L.diff[1][lo - t0], mq);
                        atomicSub(&L.diff[1][hi - t0], mq);
                        int which = (mq >= a.rd_min_mapq) ? 2 : 3;
                        atomicAdd(&L.diff[which][lo - t0], 1);
                        atomicSub(&L.diff[which][hi - t0], 1);
                    }
                }
                caf_pos += len;
                if (!in_cap) continue;
                if (pos_ok) {
                    // SNV tally, GROM.c:6769-7059
                    const int64_t xb = (int64_t)p0 + snv_ref_base;
                    const int loop_end = (xb + len >= a.chr_len) ? (int)(a.chr_len - p0) : len;
                    int64_t blo = max((int64_t)0, max(ev_lo, t0) - xb);
                    int64_t bhi = min((int64_t)loop_end, ev_hi + 1 - xb);
                    if (tile_evals)
                        for (int64_t b = blo + lane; b < bhi; b += 64) {
                            const int64_t x = xb + b;
                            const int xl = (int)(x - t0);
                            const int qi = snv_base + (int)b;
                            int q = 0, s4 = 15;
                            if (qi < lq) {
                                const int64_t nib = bo + qi;
                                q = R.qual[nib];
                                s4 = (R.seq[nib >> 1] >> ((~nib & 1) << 2)) & 15;
                            }
                            const char sb = c_nt16[s4];
                            const int code = c_nt16_acgt[s4];
                            const char rb = L.ref[xl];
                            if (hq_read && q >= a.min_base_qual) {
                                if (rb != sb) {
                                    uint4 e;
                                    e.x = (uint32_t)xl | ((uint32_t)code << 10) | ((uint32_t)fwd << 13) |
                                          ((uint32_t)q << 16) | ((uint32_t)mq << 24);
                                    e.y = (uint32_t)r;
                                    e.z = nid;
                                    e.w = (uint32_t)qi;
                                    push_event(L, e);
                                } else if (code < 4) {
                                    atomicAdd(&L.snvfs[code][xl], 1ull | ((unsigned long long)fwd << 32));
                                    atomicAdd(&L.bqmq_hi[xl], (unsigned long long)q | ((unsigned long long)mq << 32));
                                    atomicAdd(&L.pir[code][xl], (uint32_t)(fwd ? qi : lseq_mod - qi));
                                }
                            } else if (code < 4) {
                                atomicAdd(&L.lowmq[code][xl], 1u);
                                atomicAdd(&L.bqmq_lo[xl], (unsigned long long)q | ((unsigned long long)mq << 32));
                            }
                        }
                    snv_base += loop_end;
                    snv_ref_base += loop_end;
                }
            } else if (op == 2) {
                caf_pos += len;
                if (!in_cap) continue;
                snv_ref_base += len;
                end_adj_indel -= len;
            } else if (in_cap) {
                if (op == 4) snv_base += len;
                else if (op == 5) lseq_mod += len;
                else if (op == 1) { snv_base += len; end_adj_indel += len; }
                else if (op == 3) snv_ref_base += len;
            } else {
                continue;
            }
            if (first_op < 0) { first_op = op; first_len = len; }
            last_op = op;
            last_len = len;
        }
        // clip lengths and reference end, GROM.c:7067-7100
        const int start_adj = (first_op == 4 || first_op == 5) ? first_len : 0;
        const int end_adj = (last_op == 4 || last_op == 5) ? last_len : 0;
        const int64_t E = (int64_t)p0 - start_adj + lseq_mod - end_adj - end_adj_indel;
        // physical read depth over [pos, E), GROM.c:7173-7181
        if (lane == 0 && E > p0) {
            int64_t lo = max((int64_t)p0, t0), hi = min(E, t0 + T);
            if (lo < hi) {
                atomicAdd(&L.diff[0][lo - t0], 1);
                atomicSub(&L.diff[0][hi - t0], 1);
            }
        }
        // soft-clip evidence, GROM.c:7105-7169
        if (lane == 0 && tile_evals) {
            const bool paired = fl & 0x1, munmap = fl & 0x8, rev = fl & 0x10;
            const int32_t mtid = R.mtid[r], mp = R.mpos[r], tl = R.isize[r];
            // the read's own chromosome is the scanned one; its mate is on it iff mtid == tid
            if (start_adj >= a.sc_min) {
                const int64_t x = (int64_t)p0 - 1;
                if (x >= ev_lo && x <= ev_hi) {
                    const bool same_chr = (mtid == a.chr_tid);
                    uint32_t cat = 0;
                    if (!paired || (!rev && (munmap || (!munmap && same_chr && mp > p0)))) cat |= 1;
                    if (paired && !munmap && !same_chr && rev) cat |= 2;
                    if (paired && !munmap && same_chr && rev && abs(tl) <= a.insert_max && mp < p0) cat |= 4;
                    if (cat) push_event(L, make_uint4((uint32_t)(x - t0) | ((uint32_t)EV_CLIP_L << 10), (uint32_t)r,
                                                      cat | ((uint32_t)add << 8), 0));
                }
            }
            if (end_adj >= a.sc_min) {
                const int64_t x = E;
                if (x >= ev_lo && x <= ev_hi) {
                    const bool same_chr = (mtid == a.chr_tid);
                    uint32_t cat = 0;
                    if (!paired || (rev && (munmap || (!munmap && same_chr && mp < p0)))) cat |= 1;
                    if (paired && !munmap && !same_chr && !rev) cat |= 2;
                    if (paired && !munmap && same_chr && !rev && abs(tl) <= a.insert_max && mp > p0) cat |= 4;
                    if (cat) push_event(L, make_uint4((uint32_t)(x - t0) | ((uint32_t)EV_CLIP_R << 10), (uint32_t)r,
                                                      cat | ((uint32_t)add << 8), 0));
                }
            }
        }
    }
    __syncthreads();

    // ---- phase 2: bucket events by position ----
    const uint32_t nev = L.nev;
    if (nev > GROM_EVENT_CAP) {
        if (tid == 0) {
            if (atomicAdd(&O.status[0], 1u) == 0) O.status[1] = blockIdx.x;
        }
        return;  // whole block exits together; the host reports the overflow
    }
    if (tid == 0) atomicAdd(O.n_events, nev);
    for (uint32_t e = tid; e < nev; e += NTHR) atomicAdd(&L.ev_cnt[L.ev[e].x & 1023], 1u);
    __syncthreads();
    tile_scans(L);
    for (uint32_t e = tid; e < nev; e += NTHR) {
        const uint32_t xl = L.ev[e].x & 1023;
        const uint32_t s = atomicAdd(&L.ev_fill[xl], 1u);
        L.ev_sorted[L.ev_cnt[xl] + s] = (uint16_t)e;
    }
    __syncthreads();

    // ---- phase 3: per position fold, evaluation, outputs ----
    unsigned long long fsum = 0, fcnt = 0;
    for (int xl = tid; xl < T; xl += NTHR) {
        const int64_t x = t0 + xl;
        if (x >= a.chr_len) break;
        const int32_t rd = L.diff[0][xl];
        O.caf_mq[x] = L.diff[1][xl];
        O.caf_rd[x] = L.diff[2][xl];
        O.caf_low[x] = L.diff[3][xl];
        const char rb = L.ref[xl];
        if (x < a.flush_end && rb != 'N') {
            fsum += (unsigned long long)((int64_t)L.diff[2][xl] + (int64_t)L.diff[3][xl]);
            fcnt += 1;
        }
        if (x < ev_lo || x > ev_hi) continue;
        // fold this position's events in read order
        const uint32_t es = L.ev_cnt[xl], en = L.ev_fill[xl];
        uint16_t *seg = &L.ev_sorted[es];
        for (uint32_t i = 1; i < en; i++) {  // insertion sort by (read, kind)
            uint16_t v = seg[i];
            unsigned long long kv = ((unsigned long long)L.ev[v].y << 8) | ((L.ev[v].x >> 10) & 7);
            uint32_t j = i;
            while (j > 0) {
                uint16_t u = seg[j - 1];
                unsigned long long ku = ((unsigned long long)L.ev[u].y << 8) | ((L.ev[u].x >> 10) & 7);
                if (ku <= kv) break;
                seg[j] = u;
                j--;
            }
            seg[j] = v;
        }
        uint32_t slots[GROM_MAX_NAME_SLOTS];
#pragma unroll
        for (int k = 0; k < GROM_MAX_NAME_SLOTS; k++) slots[k] = 0;
        int32_t sc[15];
#pragma unroll
        for (int k = 0; k < 15; k++) sc[k] = 0;
        for (uint32_t i = 0; i < en; i++) {
            const uint4 e = L.ev[seg[i]];
            const int kind = (e.x >> 10) & 7;
            if (kind <= 4) {
                // read-name slots, GROM.c:6805-6824
                bool found = false;
                for (int k = 0; k < a.min_snv; k++) {
                    if (slots[k] == 0) {
                        if (e.z != 0) slots[k] = e.z;
                        break;
                    } else if (slots[k] == e.z) {
                        found = true;
                        break;
                    }
                }
                if (found || kind == 4) continue;
                const uint32_t fw = (e.x >> 13) & 1, q = (e.x >> 16) & 255, m = e.x >> 24;
                L.snvfs[kind][xl] += 1ull | ((unsigned long long)fw << 32);
                L.bqmq_hi[xl] += (unsigned long long)q | ((unsigned long long)m << 32);
                L.pir[kind][xl] += e.w;  // mismatches add the query offset on both strands (GROM.c:6896)
            } else {
                const uint32_t cat = e.z & 7;
                const int32_t ad = (int32_t)(e.z >> 8);
                const int base = (kind == EV_CLIP_L) ? 0 : 1;  // left / right
                for (int c = 0; c < 3; c++)
                    if (cat & (1u << c)) {
                        sc[c * 5 + base] += ad;       // sc_left / sc_right
                        sc[c * 5 + 2 + base] += 1;    // *_left_rd / *_right_rd
                        sc[c * 5 + 4] += 1;           // *_sc_rd
                    }
            }
        }
        int32_t snv[4], fs[4], low[4], pir[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            snv[k] = (int32_t)(L.snvfs[k][xl] & 0xffffffffu);
            fs[k] = (int32_t)(L.snvfs[k][xl] >> 32);
            low[k] = (int32_t)L.lowmq[k][xl];
            pir[k] = (int32_t)L.pir[k][xl];
        }
        const int32_t bq_hi = (int32_t)(L.bqmq_hi[xl] & 0xffffffffu), mq_hi = (int32_t)(L.bqmq_hi[xl] >> 32);
        const int32_t bq_lo = (int32_t)(L.bqmq_lo[xl] & 0xffffffffu), mq_lo = (int32_t)(L.bqmq_lo[xl] >> 32);
        const int32_t total = snv[0] + snv[1] + snv[2] + snv[3];
        const int32_t rc_all = total + low[0] + low[1] + low[2] + low[3];
        const int32_t bq_all = bq_hi + bq_lo, mq_all = mq_hi + mq_lo;
        if (O.dbg) {
            int32_t *d = O.dbg + (size_t)(x - a.eval_lo) * GC_COUNT;
            d[GC_POS] = (int32_t)x;
            for (int k = 0; k < 4; k++) {
                d[GC_SNV + k] = snv[k];
                d[GC_SNV_LOWMQ + k] = low[k];
                d[GC_PIR + k] = pir[k];
                d[GC_FS + k] = fs[k];
            }
            d[GC_BQ] = bq_hi;
            d[GC_BQ_ALL] = bq_all;
            d[GC_MQ] = mq_hi;
            d[GC_MQ_ALL] = mq_all;
            d[GC_BQ_RC] = total;
            d[GC_MQ_RC] = total;
            d[GC_RC_ALL] = rc_all;
            d[GC_RD] = rd;
            for (int k = 0; k < 15; k++) d[GC_SC_LEFT + k] = sc[k];
        }
        // SNV test, GROM.c:11096-11199
        if (rd + sc[14] <= 0 || rb == 'N') continue;
        int best = -1;
        float best_ratio = 0.f;
        for (int k = 0; k < 4; k++) {
            const float ratio = (float)snv[k] / (float)total;
            if (rb != c_acgt[k] && (double)ratio >= a.min_snv_ratio && snv[k] >= a.min_snv &&
                (double)bq_all / (double)rc_all >= a.min_ave_bq) {
                if (best < 0 || ratio > best_ratio) {
                    best = k;
                    best_ratio = ratio;
                }
            }
        }
        if (best < 0) continue;
        const uint32_t ci = atomicAdd(O.n_cands, 1u);
        if (ci >= O.cand_cap) continue;  // host sees n_cands > cap and re-runs with room
        grom_snv_cand c;
        c.pos = (int32_t)x;
        c.base = best;
        c.ratio = best_ratio;
        c.ref_base = (int32_t)(unsigned char)ref[x];
        size_t ti = (total > GROM_MAX_TRIALS)
                        ? (size_t)GROM_MAX_TRIALS * (GROM_MAX_TRIALS + 1) + snv[best] * GROM_MAX_TRIALS / total
                        : (size_t)total * (GROM_MAX_TRIALS + 1) + snv[best];
        c.binom = mq_tab[ti];
        c.hez = hez_tab[ti];
        for (int k = 0; k < 4; k++) {
            c.snv[k] = snv[k];
            c.lowmq[k] = low[k];
            c.pir[k] = pir[k];
            c.fs[k] = fs[k];
        }
        c.bq = bq_hi;
        c.bq_all = bq_all;
        c.mq = mq_hi;
        c.mq_all = mq_all;
        c.bq_rc = total;
        c.mq_rc = total;
        c.rc_all = rc_all;
        c.pad1 = 0;
        O.cands[ci] = c;
    }
    // flush-range read-depth sums (GROM.c:15066-15073)
    for (int o = 32; o > 0; o >>= 1) {
        fsum += __shfl_xor(fsum, o, 64);
        fcnt += __shfl_xor(fcnt, o, 64);
    }
    if (lane == 0) {
        L.red[wave][0] = fsum;
        L.red[wave][1] = fcnt;
    }
    __syncthreads();
    if (tid == 0) {
        unsigned long long s = 0, c = 0;
        for (int w = 0; w < NWAVES; w++) {
            s += L.red[w][0];
            c += L.red[w][1];
        }
        if (c) {
            atomicAdd(&O.flush_acc[0], s);
            atomicAdd(&O.flush_acc[1], c);
        }
    }
}

// sums of caf_rd + caf_low over non-N bases of [0, e) for mid-scan flushes
__global__ void k_flush_sum(int64_t e, const char *__restrict__ ref, const int32_t *__restrict__ rd,
                            const int32_t *__restrict__ low, unsigned long long *__restrict__ acc) {
    unsigned long long s = 0, c = 0;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < e; x += (int64_t)gridDim.x * blockDim.x) {
        char b = ref[x];
        if (b != 'N' && b != 'n') {
            s += (unsigned long long)((int64_t)rd[x] + low[x]);
            c += 1;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o, 64);
        c += __shfl_xor(c, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&acc[0], s);
        atomicAdd(&acc[1], c);
    }
}

// ===========================================================================
// host side
// ===========================================================================
namespace {

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
};

static int ensure(DevBuf &b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return GROM_OK;
    if (b.p) hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    size_t want = bytes + bytes / 8;
    if (hipMalloc(&b.p, want) != hipSuccess) {
        set_err("hipMalloc(%zu) failed", want);
        return GROM_E_NOMEM;
    }
    b.cap = want;
    return GROM_OK;
}

struct Ctx {
    bool init = false;
    int device = -1;
    hipStream_t st = nullptr;
    grom_params prm{};
    double *d_mq = nullptr, *d_hez = nullptr;
    // reads (used when the caller passes host memory)
    DevBuf r_pos, r_flag, r_mapq, r_mtid, r_mpos, r_isize, r_lq, r_coff, r_cig, r_boff, r_seq, r_qual, r_nid, ref;
    // scan scratch
    DevBuf keep, tlo, thi, caf_mq, caf_rd, caf_low, cands, misc, dbg;
    hipEvent_t e0 = nullptr, e1 = nullptr, ep0 = nullptr, ep1 = nullptr;
};

static Ctx g_ctx[64];

static Ctx *ctx_of(int device) {
    if (device < 0 || device >= 64 || !g_ctx[device].init) {
        set_err("device %d not initialised (call grom_dev_init)", device);
        return nullptr;
    }
    return &g_ctx[device];
}

// ring index of the reference walk after k iterations (GROM.c:5845-5847,
// 6392): starts at index_start = r14 + 1 and wraps r34 -> r14.
static int64_t ring_index(const grom_params &p, int64_t k) {
    int64_t H = p.half_one_base_rd_len;
    return p.r14_one_base_rd_len + ((k + 1) % H);
}

struct Text {
    char **buf;
    size_t *len, *cap;
    void add(const char *s, size_t n) {
        if (*len + n + 1 > *cap) {
            size_t nc = *cap ? *cap * 2 : 1 << 16;
            while (nc < *len + n + 1) nc *= 2;
            *buf = (char *)realloc(*buf, nc);
            *cap = nc;
        }
        memcpy(*buf + *len, s, n);
        *len += n;
        (*buf)[*len] = 0;
    }
};

// SNV rows of one list flush (GROM.c:11203-11274 mid-scan, 15063-15107 final)
static void snv_rows(const grom_params &P, const grom_chrom *ch, const grom_snv_cand *c, size_t n, double ave_rd,
                     Text &out) {
    static const char dna[4] = {'A', 'C', 'G', 'T'};
    char line[1024], gt[128];
    const double lim = round(P.snv_rd_min_factor * ave_rd);
    for (size_t i = 0; i < n; i++) {
        const grom_snv_cand &s = c[i];
        const double ratio = (double)s.ratio;
        if (!(s.rc_all <= lim || ratio >= P.high_cov_min_snv_ratio)) continue;
        int cn = (int)round(ratio * P.ploidy);
        if (cn == 0) cn = 1;
        for (int k = 0; k < P.ploidy; k++) {
            gt[2 * k] = (k < cn) ? '1' : '0';
            gt[2 * k + 1] = (k < P.ploidy - 1) ? '/' : '\0';
        }
        const int b = s.base;
        int w = snprintf(line, sizeof(line),
                         "%s\t%d\t\t%c\t%c\t.\t.\t.\tGT:PR:AF:A:C:G:T:AL:CL:GL:TL:BQ:MQ:PIR:FS\t%s:%e:%e:%d:%d:%d:%d:%d:%d:%d:"
                         "%d:%.2f:%.2f:%.2f:%.2f\n",
                         ch->name, s.pos + 1, (char)s.ref_base, dna[b], gt, s.binom, ratio, s.snv[0], s.snv[1], s.snv[2],
                         s.snv[3], s.lowmq[0], s.lowmq[1], s.lowmq[2], s.lowmq[3],
                         (double)s.bq_all / (double)s.rc_all, (double)s.mq_all / (double)s.rc_all,
                         (double)s.pir[b] / (double)s.snv[b], (double)s.fs[b] / (double)s.snv[b]);
        out.add(line, (size_t)w);
    }
}

static int check_params(const grom_params &p) {
    if (p.min_snv > GROM_MAX_NAME_SLOTS) {
        set_err("-n %d exceeds the %d read-name slots the kernel keeps per base", p.min_snv, GROM_MAX_NAME_SLOTS);
        return GROM_E_ARG;
    }
    if (p.vcf != 1) {
        set_err("-f (tab-separated output) is not supported by this build");
        return GROM_E_ARG;
    }
    if (p.half_one_base_rd_len <= 0) {
        set_err("insert-size parameters not set (grom_params_set_insert)");
        return GROM_E_ARG;
    }
    if (p.ploidy < 1 || p.ploidy > 50) {
        set_err("ploidy %d outside 1..50", p.ploidy);
        return GROM_E_ARG;
    }
    return GROM_OK;
}

// the scan proper on device-resident reads
static int scan_device(Ctx &C, const grom_chrom *ch, const grom_reads *R, grom_out *out, grom_stats *stats,
                       int32_t *dbg_first, int32_t *dbg_counts, int64_t dbg_cap, int32_t *dbg_caf) {
    const grom_params &P = C.prm;
    int rc = check_params(P);
    if (rc) return rc;
    if (ch->len <= 0 || ch->len >= (int64_t)1 << 31) {
        set_err("chromosome length %lld out of range", (long long)ch->len);
        return GROM_E_ARG;
    }
    hipStream_t st = C.st;
    const int64_t n = R->n;
    const int64_t n_tiles = (ch->len + T - 1) / T;
    const int32_t s0 = P.one_base_rd_len / 4 + 1; /* cdp_one_base_index_start, GROM.c:2918 */

    grom_scan_args a{};
    a.chr_len = ch->len;
    a.n_reads = n;
    a.min_mapq = P.min_mapq;
    a.rd_min_mapq = P.rd_min_mapq;
    a.min_base_qual = P.min_base_qual;
    a.min_snv = P.min_snv;
    a.insert_max = P.insert_max_size;
    a.sc_min = P.sc_min;
    a.chr_tid = ch->tid;
    a.min_snv_ratio = P.min_snv_ratio;
    a.min_ave_bq = P.min_ave_bq;
    a.eval_lo = std::max(s0, 2 * P.insert_max_size + 1);
    a.eval_hi = ch->p_last;
    // final flush range end: p_end - index_end (GROM.c:15066)
    int64_t k_end, p_end;
    if (ch->p_last >= 0) {
        k_end = (int64_t)ch->n_skip + (ch->p_last - s0 + 1);
        p_end = ch->p_last + 1;
    } else {
        k_end = ch->n_skip;
        p_end = s0;
    }
    int64_t flush_end = p_end - ring_index(P, k_end);
    if (ch->n_skip == 0 && ch->p_last < 0) flush_end = 0; /* walk never started */
    a.flush_end = (int32_t)std::max<int64_t>(std::min<int64_t>(flush_end, ch->len), (int64_t)INT32_MIN);

    // scratch
    const bool want_dbg = dbg_counts != nullptr;
    int64_t n_eval = (a.eval_hi >= a.eval_lo) ? (int64_t)a.eval_hi - a.eval_lo + 1 : 0;
    if ((rc = ensure(C.tlo, sizeof(int32_t) * n_tiles)) || (rc = ensure(C.thi, sizeof(int32_t) * n_tiles)) ||
        (rc = ensure(C.caf_mq, sizeof(int32_t) * ch->len)) || (rc = ensure(C.caf_rd, sizeof(int32_t) * ch->len)) ||
        (rc = ensure(C.caf_low, sizeof(int32_t) * ch->len)) || (rc = ensure(C.misc, 256)) ||
        (rc = ensure(C.keep, (size_t)std::max<int64_t>(n, 1))))
        return rc;
    if (want_dbg && (rc = ensure(C.dbg, sizeof(int32_t) * GC_COUNT * std::max<int64_t>(n_eval, 1)))) return rc;
    uint32_t cand_cap = (uint32_t)std::min<int64_t>(std::max<int64_t>(1 << 16, ch->len / 256), (int64_t)1 << 26);
    if (C.cands.cap >= sizeof(grom_snv_cand) * 2)
        cand_cap = std::max<uint32_t>(cand_cap, (uint32_t)(C.cands.cap / sizeof(grom_snv_cand)));

    // misc layout: [0] halo (int32), [4..] n_cands, status[2], n_events ; [32..] flush_acc[2] ; [64..] mid acc[2]
    char *misc = (char *)C.misc.p;
    int32_t *d_halo = (int32_t *)misc;
    uint32_t *d_ncand = (uint32_t *)(misc + 4);
    uint32_t *d_status = (uint32_t *)(misc + 8);
    uint32_t *d_nev = (uint32_t *)(misc + 16);
    unsigned long long *d_facc = (unsigned long long *)(misc + 32);
    unsigned long long *d_macc = (unsigned long long *)(misc + 64);

    for (int attempt = 0; attempt < 2; attempt++) {
        if ((rc = ensure(C.cands, sizeof(grom_snv_cand) * (size_t)cand_cap))) return rc;
        HIPCHK(hipMemsetAsync(C.misc.p, 0, 128, st));
        HIPCHK(hipEventRecord(C.e0, st));
        if (n > 0) {
            int g = (int)std::min<int64_t>((n + 255) / 256, 4096);
            hipLaunchKernelGGL(k_span, dim3(g), dim3(256), 0, st, n, R->cigar_off, R->cigar, R->l_qseq, d_halo);
        }
        {
            int g = (int)std::min<int64_t>((n + 1 + 255) / 256, 8192);
            hipLaunchKernelGGL(k_tile_ranges, dim3(g), dim3(256), 0, st, n, R->pos, d_halo, n_tiles,
                               (int32_t *)C.tlo.p, (int32_t *)C.thi.p);
        }
        const uint8_t *keep = nullptr;
        if (P.rmdup && n > 0) {
            int g = (int)std::min<int64_t>((n + 255) / 256, 8192);
            hipLaunchKernelGGL(k_rmdup, dim3(g), dim3(256), 0, st, n, ch->tid, R->pos, R->flag, R->mapq, R->mtid,
                               R->mpos, R->isize, R->l_qseq, P.min_mapq, P.rmdup_list_len, (uint8_t *)C.keep.p);
            keep = (const uint8_t *)C.keep.p;
        }
        ReadArrays ra{R->pos, R->flag, R->mapq, R->mtid, R->mpos, R->isize, R->l_qseq, R->cigar_off, R->cigar,
                      R->base_off, R->seq, R->qual, R->name_id, keep};
        PileOut po{(int32_t *)C.caf_mq.p, (int32_t *)C.caf_rd.p, (int32_t *)C.caf_low.p,
                   (grom_snv_cand *)C.cands.p, d_ncand, cand_cap, d_facc,
                   want_dbg ? (int32_t *)C.dbg.p : nullptr, d_status, d_nev};
        HIPCHK(hipEventRecord(C.ep0, st));
        hipLaunchKernelGGL(k_pileup, dim3((unsigned)n_tiles), dim3(NTHR), 0, st, a, ch->ref, ra,
                           (const int32_t *)C.tlo.p, (const int32_t *)C.thi.p, po, C.d_mq, C.d_hez);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(C.ep1, st));
        uint32_t hdr[4];
        HIPCHK(hipMemcpyAsync(hdr, misc + 4, 16, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (hdr[1] != 0) {
            set_err("per-tile event buffer overflow in %u tile(s), first tile %u (position %lld)", hdr[1], hdr[2],
                    (long long)hdr[2] * T);
            return GROM_E_OVERFLOW;
        }
        if (hdr[0] > cand_cap) {
            cand_cap = hdr[0] + hdr[0] / 4 + 1024;
            continue;
        }
        uint32_t ncand = hdr[0];
        std::vector<grom_snv_cand> cands(ncand);
        unsigned long long facc[2];
        if (ncand) HIPCHK(hipMemcpyAsync(cands.data(), C.cands.p, sizeof(grom_snv_cand) * ncand, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(facc, d_facc, 16, hipMemcpyDeviceToHost, st));
        if (want_dbg) {
            if (n_eval * GC_COUNT > dbg_cap) {
                set_err("debug buffer too small (%lld needed)", (long long)(n_eval * GC_COUNT));
                return GROM_E_ARG;
            }
            if (n_eval)
                HIPCHK(hipMemcpyAsync(dbg_counts, C.dbg.p, sizeof(int32_t) * GC_COUNT * n_eval, hipMemcpyDeviceToHost, st));
            if (dbg_caf) {
                HIPCHK(hipMemcpyAsync(dbg_caf, C.caf_mq.p, sizeof(int32_t) * ch->len, hipMemcpyDeviceToHost, st));
                HIPCHK(hipMemcpyAsync(dbg_caf + ch->len, C.caf_rd.p, sizeof(int32_t) * ch->len, hipMemcpyDeviceToHost, st));
                HIPCHK(hipMemcpyAsync(dbg_caf + 2 * ch->len, C.caf_low.p, sizeof(int32_t) * ch->len, hipMemcpyDeviceToHost, st));
            }
            if (dbg_first) *dbg_first = a.eval_lo;
        }
        HIPCHK(hipStreamSynchronize(st));
        std::sort(cands.begin(), cands.end(),
                  [](const grom_snv_cand &x, const grom_snv_cand &y) { return x.pos < y.pos; });

        // SNV list with its flushes (GROM.c:11201-11326, 15063-15160)
        Text vt{&out->vcf, &out->vcf_len, &out->vcf_cap};
        const int64_t thr = std::max<int64_t>((int64_t)P.sv_list_len - 10, 1);
        size_t done = 0;
        while ((int64_t)(ncand - done) >= thr) {
            const grom_snv_cand &last = cands[done + thr - 1];
            int64_t k = (int64_t)ch->n_skip + (last.pos - s0 + 1);
            int64_t e = (int64_t)last.pos - ring_index(P, k);
            unsigned long long m[2] = {0, 0};
            if (e > 0) {
                HIPCHK(hipMemsetAsync(d_macc, 0, 16, st));
                int g = (int)std::min<int64_t>((std::min<int64_t>(e, ch->len) + 255) / 256, 8192);
                hipLaunchKernelGGL(k_flush_sum, dim3(g), dim3(256), 0, st, std::min<int64_t>(e, ch->len), ch->ref,
                                   (const int32_t *)C.caf_rd.p, (const int32_t *)C.caf_low.p, d_macc);
                HIPCHK(hipMemcpyAsync(m, d_macc, 16, hipMemcpyDeviceToHost, st));
                HIPCHK(hipStreamSynchronize(st));
            }
            snv_rows(P, ch, cands.data() + done, (size_t)thr, (double)(int64_t)m[0] / (double)(int64_t)m[1], vt);
            done += (size_t)thr;
        }
        snv_rows(P, ch, cands.data() + done, ncand - done, (double)(int64_t)facc[0] / (double)(int64_t)facc[1], vt);

        HIPCHK(hipEventRecord(C.e1, st));
        HIPCHK(hipEventSynchronize(C.e1));
        if (stats) {
            float ms = 0, msp = 0;
            hipEventElapsedTime(&ms, C.e0, C.e1);
            hipEventElapsedTime(&msp, C.ep0, C.ep1);
            uint32_t nev = 0;
            hipMemcpy(&nev, d_nev, 4, hipMemcpyDeviceToHost);
            stats->ms_total = ms;
            stats->ms_pileup = msp;
            stats->bases_evaluated = n_eval;
            stats->snv_candidates = ncand;
            stats->mismatch_events = nev;
        }
        return GROM_OK;
    }
    set_err("SNV candidate buffer could not be sized");
    return GROM_E_NOMEM;
}

template <typename TT>
static int up(DevBuf &b, const TT *src, int64_t count, hipStream_t st) {
    int rc = ensure(b, sizeof(TT) * (size_t)std::max<int64_t>(count, 1));
    if (rc) return rc;
    if (count > 0) HIPCHK(hipMemcpyAsync(b.p, src, sizeof(TT) * (size_t)count, hipMemcpyHostToDevice, st));
    return GROM_OK;
}

// copy a host grom_reads + reference to the context's device buffers
static int upload(Ctx &C, const grom_chrom *ch, const grom_reads *h, grom_chrom *dch, grom_reads *d) {
    hipStream_t st = C.st;
    int rc;
    const int64_t n = h->n;
    if ((rc = up(C.r_pos, h->pos, n, st)) || (rc = up(C.r_flag, h->flag, n, st)) ||
        (rc = up(C.r_mapq, h->mapq, n, st)) || (rc = up(C.r_mtid, h->mtid, n, st)) ||
        (rc = up(C.r_mpos, h->mpos, n, st)) || (rc = up(C.r_isize, h->isize, n, st)) ||
        (rc = up(C.r_lq, h->l_qseq, n, st)) || (rc = up(C.r_coff, h->cigar_off, n + 1, st)) ||
        (rc = up(C.r_cig, h->cigar, h->n_cigar_ops, st)) || (rc = up(C.r_boff, h->base_off, n, st)) ||
        (rc = up(C.r_seq, h->seq, (h->n_bases + 1) / 2, st)) || (rc = up(C.r_qual, h->qual, h->n_bases, st)) ||
        (rc = up(C.r_nid, h->name_id, n, st)) || (rc = up(C.ref, ch->ref, ch->len, st)))
        return rc;
    *dch = *ch;
    dch->ref = (const char *)C.ref.p;
    *d = *h;
    d->pos = (const int32_t *)C.r_pos.p;
    d->flag = (const uint16_t *)C.r_flag.p;
    d->mapq = (const uint8_t *)C.r_mapq.p;
    d->mtid = (const int32_t *)C.r_mtid.p;
    d->mpos = (const int32_t *)C.r_mpos.p;
    d->isize = (const int32_t *)C.r_isize.p;
    d->l_qseq = (const int32_t *)C.r_lq.p;
    d->cigar_off = (const uint32_t *)C.r_coff.p;
    d->cigar = (const uint32_t *)C.r_cig.p;
    d->base_off = (const int64_t *)C.r_boff.p;
    d->seq = (const uint8_t *)C.r_seq.p;
    d->qual = (const uint8_t *)C.r_qual.p;
    d->name_id = (const uint32_t *)C.r_nid.p;
    return GROM_OK;
}

}  // namespace

extern "C" {

int grom_abi_version(void) { return GROM_AMD_ABI_VERSION; }
const char *grom_last_error(void) { return g_err; }

int grom_dev_init(int device, const grom_params *params, const double *hez, const double *mq) {
    if (device < 0 || device >= 64 || !params || !hez || !mq) {
        set_err("grom_dev_init: bad argument");
        return GROM_E_ARG;
    }
    Ctx &C = g_ctx[device];
    if (C.init) grom_dev_fini(device);
    HIPCHK(hipSetDevice(device));
    C.device = device;
    C.prm = *params;
    HIPCHK(hipStreamCreateWithFlags(&C.st, hipStreamNonBlocking));
    const size_t tb = sizeof(double) * (GROM_MAX_TRIALS + 1) * (GROM_MAX_TRIALS + 1);
    HIPCHK(hipMalloc(&C.d_mq, tb));
    HIPCHK(hipMalloc(&C.d_hez, tb));
    HIPCHK(hipMemcpy(C.d_mq, mq, tb, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(C.d_hez, hez, tb, hipMemcpyHostToDevice));
    HIPCHK(hipEventCreate(&C.e0));
    HIPCHK(hipEventCreate(&C.e1));
    HIPCHK(hipEventCreate(&C.ep0));
    HIPCHK(hipEventCreate(&C.ep1));
    C.init = true;
    return GROM_OK;
}

void grom_dev_fini(int device) {
    if (device < 0 || device >= 64 || !g_ctx[device].init) return;
    Ctx &C = g_ctx[device];
    (void)hipSetDevice(device);
    (void)hipStreamSynchronize(C.st);
    DevBuf *all[] = {&C.r_pos, &C.r_flag, &C.r_mapq, &C.r_mtid, &C.r_mpos, &C.r_isize, &C.r_lq, &C.r_coff,
                     &C.r_cig, &C.r_boff, &C.r_seq, &C.r_qual, &C.r_nid, &C.ref, &C.keep, &C.tlo, &C.thi,
                     &C.caf_mq, &C.caf_rd, &C.caf_low, &C.cands, &C.misc, &C.dbg};
    for (DevBuf *b : all)
        if (b->p) hipFree(b->p);
    hipFree(C.d_mq);
    hipFree(C.d_hez);
    hipEventDestroy(C.e0);
    hipEventDestroy(C.e1);
    hipEventDestroy(C.ep0);
    hipEventDestroy(C.ep1);
    hipStreamDestroy(C.st);
    g_ctx[device] = Ctx();
}

int grom_scan_chrom(int device, const grom_chrom *chrom, const grom_reads *reads, grom_out *out, grom_stats *stats) {
    Ctx *C = ctx_of(device);
    if (!C) return GROM_E_NODEV;
    if (!chrom || !reads || !out || !chrom->ref) { set_err("grom_scan_chrom: null argument"); return GROM_E_ARG; }
    HIPCHK(hipSetDevice(device));
    grom_chrom dch;
    grom_reads dr;
    int rc = upload(*C, chrom, reads, &dch, &dr);
    if (rc) return rc;
    return scan_device(*C, &dch, &dr, out, stats, nullptr, nullptr, 0, nullptr);
}

int grom_scan_chrom_device(int device, const grom_chrom *chrom, const grom_reads *dev_reads, grom_out *out,
                           grom_stats *stats) {
    Ctx *C = ctx_of(device);
    if (!C) return GROM_E_NODEV;
    if (!chrom || !dev_reads || !out) { set_err("grom_scan_chrom_device: null argument"); return GROM_E_ARG; }
    HIPCHK(hipSetDevice(device));
    return scan_device(*C, chrom, dev_reads, out, stats, nullptr, nullptr, 0, nullptr);
}

int grom_upload(int device, const grom_chrom *chrom, const grom_reads *reads, grom_chrom *dev_chrom,
                grom_reads *dev_reads) {
    Ctx *C = ctx_of(device);
    if (!C) return GROM_E_NODEV;
    if (!chrom || !reads || !dev_chrom || !dev_reads) { set_err("grom_upload: null argument"); return GROM_E_ARG; }
    HIPCHK(hipSetDevice(device));
    int rc = upload(*C, chrom, reads, dev_chrom, dev_reads);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(C->st));
    return GROM_OK;
}

int grom_debug_counts(int device, const grom_chrom *chrom, const grom_reads *reads, int32_t *first_pos,
                      int32_t *counts, int64_t counts_cap, int32_t *caf3) {
    Ctx *C = ctx_of(device);
    if (!C) return GROM_E_NODEV;
    HIPCHK(hipSetDevice(device));
    grom_chrom dch;
    grom_reads dr;
    int rc = upload(*C, chrom, reads, &dch, &dr);
    if (rc) return rc;
    grom_out tmp{};
    rc = scan_device(*C, &dch, &dr, &tmp, nullptr, first_pos, counts, counts_cap, caf3);
    grom_out_free(&tmp);
    return rc;
}

}  // extern "C"
