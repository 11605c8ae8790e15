// scan.hip -- MI355X (gfx950) implementation of GROM's per-chromosome scan
// behind the C ABI of include/grom_amd.h.
//
// The reference walks a chromosome base by base (GROM.c:5842), ingesting each
// read into a sliding ring of per-position counters (GROM.c:6406-10966) and
// evaluating each base once every read that can touch it has been ingested
// (GROM.c:11086-13553).  Here the chromosome is cut into tiles of GROM_TILE
// absolute positions; one workgroup owns a tile, stages the reads overlapping
// it in LDS and evaluates its positions.  Each lane owns one position and folds the tile's reads into registers in
// read order, which is the order the reference's ring sees them, so even the
// order-dependent read-name de-duplication of mismatching bases
// (GROM.c:6805-6824) is a plain sequential fold (k_scan_tile.h).
//
// Kernels (one launch each per chromosome):
//   k_rmdup       -M duplicate filter (GROM.c:6432-6588), per start position
//   k_prep        packs each read's metadata into one 48-byte record and
//                 finds the longest reference extent (tile halo)
//   k_tile_ranges per-tile [first,last) read range, from the sorted positions
//   k_scan_tile   the tile kernel: caf read depth, SNV tally, soft-clip
//                 evidence, physical read depth, SNV test, flush sums
//   k_flush_sum   read-depth sum for mid-scan SNV list flushes (rare)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/grom_amd.h"
#include "cnv.h"
#include "ddecode.h"
#include "sv.h"
#include "scan_common.h"
#include "snvfmt.h"

#define T GROM_TILE
#define NTHR GROM_TILE_THREADS
#define NWAVES (NTHR / 64)

static thread_local char g_err[512];  // per host thread: contexts may run concurrently
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

#include "device_common.h"

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
// k_scan_tile: the tile kernel (k_scan_tile.h)
// ---------------------------------------------------------------------------
#include "k_scan_tile.h"
#include "copystats.h"  // (GROM_COPY_STATS, last: it wraps the runtime copy calls)

// the per-tile flush sums of the pileup kernels into acc[0..1]
__global__ __launch_bounds__(256) void k_flush_reduce(int64_t n_tiles, const unsigned long long *__restrict__ part,
                                                      unsigned long long *__restrict__ acc) {
    unsigned long long s = 0, c = 0;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n_tiles; t += (int64_t)gridDim.x * blockDim.x) {
        s += part[2 * t];
        c += part[2 * t + 1];
    }
    for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o, 64);
        c += __shfl_xor(c, o, 64);
    }
    if ((threadIdx.x & 63) == 0 && (s | c)) {
        atomicAdd(&acc[0], s);
        atomicAdd(&acc[1], c);
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
    bool own = false;          // p is this buffer's own allocation (else a piece of `ar`'s phase)
    grom_arena *ar = nullptr;  // the context's phase arena, for the pileup phase's per-read buffers
};

static int ensure(DevBuf &b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return GROM_OK;
    if (b.p && b.own) grom_dev_free(b.p, b.cap, GROM_DEVCAT_SCAN);
    b.p = nullptr;
    b.cap = 0;
    b.own = false;
    size_t want = bytes + bytes / 8 + 64;  // slack: kernels read whole 16-byte words
    if (b.ar && (b.p = grom_arena_take(b.ar, want)) != nullptr) {
        b.cap = want;
        return GROM_OK;
    }
    if (grom_dev_malloc(&b.p, want, GROM_DEVCAT_SCAN)) {
        set_err("hipMalloc(%zu) failed", want);
        return GROM_E_NOMEM;
    }
    b.cap = want;
    b.own = true;
    return GROM_OK;
}

struct Ctx {
    bool init = false;
    int device = -1;
    grom_arena *ar = nullptr;  // the phase arena (devmem.h): pileup/breakpoint phase, then CNV phase
    hipStream_t st = nullptr;
    grom_params prm{};
    double *d_mq = nullptr, *d_hez = nullptr;
    // reads (used when the caller passes host memory)
    DevBuf r_pos, r_flag, r_mapq, r_mtid, r_mpos, r_isize, r_lq, r_coff, r_cig, r_boff, r_seq, r_qual, r_nid, ref;
    DevBuf r_aidx, r_aux, r_dpos, r_dlq, r_dbef;
    // scan scratch
    DevBuf keep, meta, tlo, thi, caf_mq, caf_rd, caf_low, cands, cands2, runb, runc, segs, misc, dbg, fpart, slots;
    grom_snv_cand *h_cands = nullptr;  // pinned host copy of the ordered candidates
    unsigned long long *h_cafsum = nullptr, *d_cafsum = nullptr;  // mapped pinned word: k_caf_range_sum's result
    const char *host_ref = nullptr;    // the caller's host reference during grom_scan_chrom
    // device-resident scans: the breakpoint rows read reference bases on the
    // host, so the reference is copied into this pinned buffer on a side
    // stream while the pileup runs (ref_ev marks the copy done)
    char *h_ref = nullptr;
    size_t h_ref_cap = 0;
    hipStream_t st_copy = nullptr;
    hipEvent_t ref_ev = nullptr;
    size_t h_cap = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr, ep0 = nullptr, ep1 = nullptr;
    CnvScratch *cnv = nullptr;  // read-depth CNV path (cnv.hip)
    SvScratch *sv = nullptr;        // breakpoint evidence and tests (sv.hip)
};

static Ctx g_ctx[64];

static Ctx *ctx_of(int device) {
    if (device < 0 || device >= 64 || !g_ctx[device].init) {
        set_err("device %d not initialised (call grom_dev_init)", device);
        return nullptr;
    }
    return &g_ctx[device];
}

// sum of caf_rd + caf_low over [lo, hi) of the device arrays, as the INV
// depth check reads them (GROM.c:15816-15826): int per base, double total
// One block sums rd[i] + low[i] over [lo, hi) as int64 into a mapped pinned
// word: the host's double total of int sums is the same number (each partial
// sum is an integer below 2^53)
__global__ __launch_bounds__(1024) void k_caf_range_sum(const int32_t *__restrict__ rd, const int32_t *__restrict__ low,
                                                        int64_t lo, int64_t hi, unsigned long long *out) {
    __shared__ long long part[16];
    long long s = 0;
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) s += (long long)rd[i] + (long long)low[i];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        long long t = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); w++) t += part[w];
        *out = (unsigned long long)t;
    }
}

// sum of caf_rd + caf_low over [lo, hi) of the device arrays, as the INV
// depth check reads them (GROM.c:15816-15826): int per base, double total.
// Summed on the device (round 4 copied both ranges to the host: two blits and
// up to megabytes per query, the largest source of runtime copies)
struct CafSum {
    hipStream_t st;
    const int32_t *rd, *low;
    int64_t len;
    int rc;
    unsigned long long *h, *d;  // mapped pinned result word
    static double call(void *u, int64_t lo, int64_t hi) {
        CafSum &c = *(CafSum *)u;
        const int64_t a = std::max<int64_t>(lo, 0), b = std::min<int64_t>(hi, c.len);
        if (a >= b || c.rc != GROM_OK) return 0.0;
        hipLaunchKernelGGL(k_caf_range_sum, dim3(1), dim3(1024), 0, c.st, c.rd, c.low, a, b, c.d);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(c.st) != hipSuccess) {
            set_err("INV depth check: device sum failed");
            c.rc = GROM_E_HIP;
            return 0.0;
        }
        return (double)(long long)*(volatile unsigned long long *)c.h;
    }
};

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

static int check_params(const grom_params &p) {
    if (p.min_snv < 0) {
        set_err("-n %d is negative", p.min_snv);
        return GROM_E_ARG;
    }
    if (p.half_one_base_rd_len <= 0) {
        set_err("insert-size parameters not set (grom_params_set_insert)");
        return GROM_E_ARG;
    }
    // any -p >= 1, as GROM.c:22003 takes it (the reference's 100-byte GT
    // text, GROM.c:1477, overflows above 50; the rows print the whole string).
    // Below 1 the reference prints an unset GT (undefined), so it is refused.
    if (p.ploidy < 1) {
        set_err("ploidy %d below 1", p.ploidy);
        return GROM_E_ARG;
    }
    return GROM_OK;
}

// the scan proper on device-resident reads
// reads_done (optional): called once the scan no longer reads R or ch->ref
// (after the breakpoint tests; the CNV path then reads the context's own
// copy of the reference), so a stage can take the next chromosome while this
// one's CNV path runs
static int scan_device(Ctx &C, const grom_chrom *ch, const grom_reads *R, grom_out *out, grom_stats *stats,
                       int32_t *dbg_first, int32_t *dbg_counts, int64_t dbg_cap, int32_t *dbg_caf,
                       void (*reads_done)(void *) = nullptr, void *reads_done_arg = nullptr) {
    const grom_params &P = C.prm;
    int rc = check_params(P);
    if (rc) return rc;
    // int32 positions in the kernels, with room for read extents past the end
    if (ch->len <= 0 || ch->len > (int64_t)INT32_MAX - (1 << 24)) {
        set_err("chromosome length %lld out of range", (long long)ch->len);
        return GROM_E_ARG;
    }
    hipStream_t st = C.st;
    const bool timing = getenv("GROM_TIMING") != nullptr;  // per-phase host clock on stderr
    const auto t_start = std::chrono::steady_clock::now();
    auto ms_since = [&](std::chrono::steady_clock::time_point t) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
    };
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
    const bool sv_debug = getenv("GROM_SV_DEBUG") != nullptr;  // keep the breakpoint records for grom_debug_sv
    // The pileup/breakpoint phase: its per-read records and breakpoint
    // buffers are carved from the context's phase arena, which the CNV phase
    // takes over after the breakpoint tests (devmem.h).  Callers that read
    // those buffers after the scan (the debug dumps) keep them separate.
    const bool use_arena = !want_dbg && !sv_debug && !getenv("GROM_DUMP") && !getenv("GROM_NO_ARENA");
    grom_arena *par = nullptr;
    if (use_arena) {
        if (!C.ar) C.ar = grom_arena_new(GROM_DEVCAT_ARENA);
        cnv_scratch_sync(C.cnv);  // (the last CNV phase's streams are done with the arena)
        // Size the arena for this chromosome's phases before the first one,
        // so that the first chromosome (the longest) does not overflow into
        // separate allocations: the pileup/breakpoint phase holds ~34 bytes
        // per base and ~56 per read, the CNV phase ~83 per base (measured on
        // the 30x genome)
        const double p_est = 34.0 * (double)ch->len + 56.0 * (double)n;
        const double c_est = ch->cnv ? 83.0 * (double)ch->len : 0.0;
        grom_arena_hint(C.ar, (size_t)(std::max(p_est, c_est) + (64 << 20)));
        if (grom_arena_begin(C.ar)) {
            set_err("phase arena: device memory allocation failed");
            return GROM_E_NOMEM;
        }
        par = C.ar;
    }
    if (!C.sv) C.sv = sv_scratch_new();
    sv_scratch_phase(C.sv, par);
    for (DevBuf *b : {&C.meta, &C.keep}) {
        if (b->own && par) grom_dev_free(b->p, b->cap, GROM_DEVCAT_SCAN);
        if (!b->own || par) {
            b->p = nullptr;
            b->cap = 0;
            b->own = false;
        }
        b->ar = par;
    }
    int64_t n_eval = (a.eval_hi >= a.eval_lo) ? (int64_t)a.eval_hi - a.eval_lo + 1 : 0;
    if ((rc = ensure(C.tlo, sizeof(int32_t) * n_tiles)) || (rc = ensure(C.thi, sizeof(int32_t) * n_tiles)) ||
        (rc = ensure(C.caf_mq, sizeof(int32_t) * ch->len)) || (rc = ensure(C.caf_rd, sizeof(int32_t) * ch->len)) ||
        (rc = ensure(C.caf_low, sizeof(int32_t) * ch->len)) || (rc = ensure(C.misc, 256)) ||
        (rc = ensure(C.keep, (size_t)std::max<int64_t>(n, 1))) ||
        (rc = ensure(C.meta, sizeof(ReadMeta) * (size_t)std::max<int64_t>(n, 1))) ||
        (rc = ensure(C.runb, sizeof(uint32_t) * n_tiles)) || (rc = ensure(C.runc, sizeof(uint32_t) * n_tiles)) ||
        (rc = ensure(C.fpart, 2 * sizeof(unsigned long long) * n_tiles)) ||
        (rc = ensure(C.segs, sizeof(uint32_t) * (size_t)((n_tiles + RUN_SEG - 1) / RUN_SEG + 1))))
        return rc;
    if (want_dbg && (rc = ensure(C.dbg, sizeof(int32_t) * GC_COUNT * std::max<int64_t>(n_eval, 1)))) return rc;
    uint32_t cand_cap = (uint32_t)std::min<int64_t>(std::max<int64_t>(1 << 16, ch->len / 256), (int64_t)1 << 26);
    if (C.cands.cap >= sizeof(grom_snv_cand) * 2)
        cand_cap = std::max<uint32_t>(cand_cap, (uint32_t)(C.cands.cap / sizeof(grom_snv_cand)));

    // misc layout: [0] halo (int32), [4..] n_cands, status, n_events ; [24] heavy-tile flag ;
    // [32..] flush_acc[2] ; [64..] mid acc[2]
    char *misc = (char *)C.misc.p;
    int32_t *d_halo = (int32_t *)misc;
    uint32_t *d_ncand = (uint32_t *)(misc + 4);
    uint32_t *d_status = (uint32_t *)(misc + 8);
    uint32_t *d_nev = (uint32_t *)(misc + 16);
    unsigned long long *d_facc = (unsigned long long *)(misc + 32);
    unsigned long long *d_macc = (unsigned long long *)(misc + 64);

    // the CNV path's reference: the context's own copy when the caller takes
    // the input back before the CNV path (reads_done)
    const char *cnv_ref = ch->ref;
    if (reads_done && ch->cnv && !want_dbg) {
        if ((rc = ensure(C.ref, (size_t)ch->len))) return rc;
        HIPCHK(hipMemcpyAsync(C.ref.p, ch->ref, (size_t)ch->len, hipMemcpyDeviceToDevice, st));
        cnv_ref = (const char *)C.ref.p;
    }
    // device-resident reference: its host copy for the breakpoint rows,
    // overlapped with the pileup on the copy stream
    bool ref_copy_pending = false;
    if (!C.host_ref) {
        if ((size_t)ch->len > C.h_ref_cap) {
            if (C.h_ref) (void)hipHostFree(C.h_ref);
            C.h_ref = nullptr;
            C.h_ref_cap = 0;
            HIPCHK(hipHostMalloc((void **)&C.h_ref, (size_t)ch->len, 0));
            C.h_ref_cap = (size_t)ch->len;
        }
        HIPCHK(hipMemcpyAsync(C.h_ref, ch->ref, (size_t)ch->len, hipMemcpyDeviceToHost, C.st_copy));
        HIPCHK(hipEventRecord(C.ref_ev, C.st_copy));
        ref_copy_pending = true;
    }
    // the reference-only part of the CNV path runs beside the pileup
    if (ch->cnv && !want_dbg) {
        if (!C.cnv) C.cnv = cnv_scratch_new();
        char cerr[512] = {0};
        if ((rc = cnv_prelaunch(C.cnv, st, P, cnv_ref, ch->len, cerr, sizeof(cerr)))) {
            set_err("%s", cerr);
            return rc;
        }
    }
    for (int attempt = 0; attempt < 4; attempt++) {
        if ((rc = ensure(C.cands, sizeof(grom_snv_cand) * (size_t)cand_cap)) ||
            (rc = ensure(C.cands2, sizeof(grom_snv_cand) * (size_t)cand_cap)))
            return rc;
        (void)hipGetLastError();  // drop any stale error of an earlier, reported failure
        HIPCHK(hipMemsetAsync(C.misc.p, 0, 128, st));
        HIPCHK(hipEventRecord(C.e0, st));
        const uint8_t *keep = nullptr;
        if (P.rmdup && n > 0) {
            int g = (int)std::min<int64_t>((n + 255) / 256, 8192);
            hipLaunchKernelGGL(k_rmdup, dim3(g), dim3(256), 0, st, n, ch->tid, R->pos, R->flag, R->mapq, R->mtid,
                               R->mpos, R->isize, R->l_qseq, P.min_mapq, P.rmdup_list_len, (uint8_t *)C.keep.p);
            keep = (const uint8_t *)C.keep.p;
        }
        ReadArrays ra{R->pos, R->flag, R->mapq, R->mtid, R->mpos, R->isize, R->l_qseq, R->cigar_off, R->cigar,
                      R->base_off, R->seq, R->qual, R->name_id, keep};
        // breakpoint evidence of every read (rows A7-A9): range sums, the
        // ordered cluster fold, and the bases the pileup must describe
        SvInput svin{n, R->pos, R->flag, R->mapq, R->mtid, R->mpos, R->isize, R->l_qseq, R->cigar_off, R->cigar,
                     R->base_off, R->seq, keep, nullptr, nullptr, 0, nullptr, nullptr, nullptr};
        if (R->n_aux > 0 && R->aux_idx && R->aux) {
            svin.aux_idx = R->aux_idx;
            svin.aux = R->aux;
        }
        if (R->n_drop > 0 && R->drop_pos && R->drop_lq && R->drop_before) {
            svin.n_drop = R->n_drop;
            svin.drop_pos = R->drop_pos;
            svin.drop_lq = R->drop_lq;
            svin.drop_before = R->drop_before;
        }
        {
            if (!C.sv) C.sv = sv_scratch_new();
            char serr[512] = {0};
            if ((rc = sv_prepare(C.sv, st, P, svin, *ch, a.eval_lo, a.eval_hi, sv_debug, serr, sizeof(serr)))) {
                set_err("%s", serr);
                return rc;
            }
        }
        if (n > 0) {
            int g = (int)std::min<int64_t>((n + 255) / 256, 8192);
            hipLaunchKernelGGL(k_prep, dim3(g), dim3(256), 0, st, n, ra, (ReadMeta *)C.meta.p, d_halo, (int64_t)ch->len,
                               (int32_t)P.min_mapq);
        }
        {
            int g = (int)std::min<int64_t>((n + 1 + 255) / 256, 8192);
            hipLaunchKernelGGL(k_tile_ranges, dim3(g), dim3(256), 0, st, n, R->pos, d_halo, n_tiles,
                               (int32_t *)C.tlo.p, (int32_t *)C.thi.p);
        }
        PileOut po{(int32_t *)C.caf_mq.p, (int32_t *)C.caf_rd.p, (int32_t *)C.caf_low.p,
                   (grom_snv_cand *)C.cands.p, d_ncand, cand_cap, (uint32_t *)C.runb.p, (uint32_t *)C.runc.p,
                   (unsigned long long *)C.fpart.p,
                   want_dbg ? (int32_t *)C.dbg.p : nullptr, d_status, d_nev, sv_bits(C.sv), sv_ctx_buf(C.sv),
                   sv_ctx_count(C.sv), sv_ctx_cap(C.sv), want_dbg ? sv_rd_add(C.sv) : nullptr};
        HIPCHK(hipEventRecord(C.ep0, st));
        const unsigned grid = (unsigned)(((n_tiles + 7) / 8) * 8);
        // the build with the fewest read-name slots that holds -n (fewer
        // slots, fewer registers: GROM.c keeps -n names per base)
#define GROM_LAUNCH_TILE(NSL)                                                                                    \
    hipLaunchKernelGGL(k_scan_tile<NSL>, dim3(grid), dim3(GROM_TILE), 0, st, a, ch->ref, ra, (const ReadMeta *)C.meta.p, \
                       (const int32_t *)C.tlo.p, (const int32_t *)C.thi.p, po, C.d_mq, C.d_hez, n_tiles, d_heavy, pack_max)
        // (GROM_MEM_SLOTS=1, a test hook: the global-slot kernel for any -n)
        static const bool force_mem_slots = getenv("GROM_MEM_SLOTS") && atoi(getenv("GROM_MEM_SLOTS")) == 1;
        // the register builds first; then the global-slot kernel: every tile
        // when -n exceeds the register builds, else only the tiles with too
        // many reads for the register builds' 16-bit counters (it returns at
        // once when k_scan_tile flagged none)
        uint32_t *d_heavy = (uint32_t *)(misc + 24);
        // (GROM_HEAVY_TILES=1, a test hook: every tile takes the heavy-tile route)
        static const bool all_heavy = getenv("GROM_HEAVY_TILES") && atoi(getenv("GROM_HEAVY_TILES")) == 1;
        const int32_t pack_max = all_heavy ? -1 : PACK_MAX_READS;
        const bool mem_all = P.min_snv > GROM_MAX_NAME_SLOTS || force_mem_slots;
        if (mem_all) {
        } else if (P.min_snv <= GROM_FEW_NAME_SLOTS) GROM_LAUNCH_TILE(GROM_FEW_NAME_SLOTS);
        else if (P.min_snv <= 8) GROM_LAUNCH_TILE(8);
        else if (P.min_snv <= 16) GROM_LAUNCH_TILE(16);
        else GROM_LAUNCH_TILE(GROM_MAX_NAME_SLOTS);
        // (no tile can hold more than pack_max reads when the chromosome has
        // no more: then the heavy-tile pass is not launched at all)
        if (mem_all || pack_max < 0 || n > pack_max) {
            // the grid walks the tiles with a stride, so any grid size is
            // correct: cap its name-slot scratch ([-n][256] words per
            // workgroup) at GROM_MEM_SLOT_BUDGET bytes
            const size_t ns = (size_t)std::max(P.min_snv, 1);
            const int64_t by_mem = std::max<int64_t>(1, (int64_t)(GROM_MEM_SLOT_BUDGET / (sizeof(uint32_t) * ns * GROM_TILE)));
            const unsigned mg = (unsigned)std::max<int64_t>(1, std::min<int64_t>({n_tiles, (int64_t)GROM_MEM_SLOT_BLOCKS, by_mem}));
            if ((rc = ensure(C.slots, sizeof(uint32_t) * (size_t)mg * ns * GROM_TILE))) return rc;
            hipLaunchKernelGGL(k_scan_tile_mem, dim3(mg), dim3(GROM_TILE), 0, st, a, ch->ref, ra,
                               (const ReadMeta *)C.meta.p, (const int32_t *)C.tlo.p, (const int32_t *)C.thi.p, po,
                               C.d_mq, C.d_hez, n_tiles, (uint32_t *)C.slots.p, mem_all ? 0 : 1,
                               (const uint32_t *)d_heavy, pack_max);
        }
#undef GROM_LAUNCH_TILE
        hipLaunchKernelGGL(k_flush_reduce, dim3(256), dim3(256), 0, st, n_tiles,
                           (const unsigned long long *)C.fpart.p, d_facc);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(C.ep1, st));
        uint32_t hdr[4];
        HIPCHK(hipMemcpyAsync(hdr, misc + 4, 16, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        const double t_kernels = ms_since(t_start);
        {
            // the breakpoint context records (every clipped or marked base) have
            // a guessed buffer: a pass that wanted more runs again with room
            uint32_t used = 0;
            if ((rc = sv_ctx_used(C.sv, st, &used))) { set_err("reading the context record count failed"); return rc; }
            const bool ctx_over = used > sv_ctx_cap(C.sv), cand_over = hdr[0] > cand_cap;
            if (ctx_over) sv_ctx_reserve(C.sv, used + used / 4 + 65536);
            if (cand_over) cand_cap = hdr[0] + hdr[0] / 4 + 1024;
            if (ctx_over || cand_over) continue;
        }
        uint32_t ncand = hdr[0];
        if (ncand > C.h_cap) {
            if (C.h_cands) (void)hipHostFree(C.h_cands);
            C.h_cands = nullptr;
            C.h_cap = 0;
            const size_t want = (size_t)ncand + ncand / 4 + 1024;
            HIPCHK(hipHostMalloc((void **)&C.h_cands, sizeof(grom_snv_cand) * want, 0));
            C.h_cap = want;
        }
        const grom_snv_cand *cands = C.h_cands;
        unsigned long long facc[2];
        if (ncand) {
            // tile runs -> position order on the device, then one pinned copy
            const int64_t n_seg = (n_tiles + RUN_SEG - 1) / RUN_SEG;
            uint32_t *segs = (uint32_t *)C.segs.p;
            hipLaunchKernelGGL(k_run_sums, dim3((unsigned)n_seg), dim3(256), 0, st, n_tiles, (const uint32_t *)C.runc.p,
                               segs);
            hipLaunchKernelGGL(k_run_scan, dim3(1), dim3(256), 0, st, n_seg, segs);
            hipLaunchKernelGGL(k_run_gather, dim3((unsigned)n_seg), dim3(256), 0, st, n_tiles,
                               (const uint32_t *)C.runb.p, (const uint32_t *)C.runc.p, (const uint32_t *)segs,
                               (const grom_snv_cand *)C.cands.p, (grom_snv_cand *)C.cands2.p);
            HIPCHK(hipGetLastError());
            HIPCHK(hipMemcpyAsync(C.h_cands, C.cands2.p, sizeof(grom_snv_cand) * ncand, hipMemcpyDeviceToHost, st));
        }
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

        // SNV list with its flushes (GROM.c:11201-11326, 15063-15160).  The flush
        // spans and their depth averages are settled here (a mid-scan flush
        // needs a device sum); the rows are formatted on a host thread while
        // the indel and CNV passes below keep the GPU busy.
        Text vt{&out->vcf, &out->vcf_len, &out->vcf_cap};
        struct FlushSeg { size_t off, n; double ave_rd; };
        std::vector<FlushSeg> fsegs;
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
            fsegs.push_back({done, (size_t)thr, (double)(int64_t)m[0] / (double)(int64_t)m[1]});
            done += (size_t)thr;
        }
        fsegs.push_back({done, ncand - done, (double)(int64_t)facc[0] / (double)(int64_t)facc[1]});
        // -f rows print cdp_lseq bases of reference context: the pending
        // record's length at each mid-scan flush, the tail record's at the end
        std::vector<int32_t> flush_lseq(fsegs.size(), ch->lseq_tail);
        const char *tab_ref = nullptr;
        if (P.vcf != 1) {
            std::vector<int32_t> fpos;
            for (size_t k = 0; k + 1 < fsegs.size(); k++) fpos.push_back(cands[fsegs[k].off + fsegs[k].n - 1].pos);
            char serr[512] = {0};
            if ((rc = sv_pending_lseq(st, P, svin, *ch, fpos.data(), (int)fpos.size(), flush_lseq.data(), serr,
                                      sizeof(serr)))) {
                set_err("%s", serr);
                return rc;
            }
            tab_ref = C.host_ref;
            if (!tab_ref) {
                HIPCHK(hipEventSynchronize(C.ref_ev));
                ref_copy_pending = false;
                tab_ref = C.h_ref;
            }
        }
        std::string snv_text;
        std::thread fmt([&P, ch, cands, &fsegs, &snv_text, &flush_lseq, tab_ref] {
            for (size_t k = 0; k < fsegs.size(); k++) {
                const FlushSeg &f = fsegs[k];
                const double lim = round(P.snv_rd_min_factor * f.ave_rd);
                if (tab_ref) {
                    snv_rows_format_tab(P, ch->name, cands + f.off, f.n, lim, tab_ref, ch->len, flush_lseq[k], snv_text);
                    continue;
                }
                std::vector<std::string> parts;
                snv_rows_format(P, ch->name, cands + f.off, f.n, lim, parts);
                for (auto &part : parts) snv_text += part;
            }
        });
        struct Joiner {
            std::thread &t;
            ~Joiner() { if (t.joinable()) t.join(); }
        } fmt_join{fmt};
        const double t_snv = ms_since(t_start);

        // per-base indel / insertion / breakpoint tests (row A10) on the device,
        // then the candidate lists, SV assembly and rows on the host (A13)
        double ms_sv = 0, t_sv_eval = 0, t_sv_ref = 0;
        std::string sv_text, ctx_text;
        size_t n_hits = 0;
        const SvHit *hits = nullptr;  // pinned, in base order (the SV scratch owns it)
        size_t nh = 0;
        // the rows' INV depth sums read caf_rd/caf_low on the copy stream, so
        // the row thread never waits behind the CNV kernels on `st` (the CNV
        // path only rewrites caf_mq)
        if (!C.h_cafsum) {
            HIPCHK(hipHostMalloc((void **)&C.h_cafsum, 64, hipHostMallocMapped));
            HIPCHK(hipHostGetDevicePointer((void **)&C.d_cafsum, C.h_cafsum, 0));
        }
        CafSum cs{C.st_copy, (const int32_t *)C.caf_rd.p, (const int32_t *)C.caf_low.p, ch->len, GROM_OK, C.h_cafsum,
                  C.d_cafsum};
        const char *href = nullptr;
        std::thread svt;
        Joiner sv_join{svt};
        {
            char serr[512] = {0};
            rc = sv_evaluate(C.sv, st, P, svin, *ch, a.eval_lo, a.eval_hi, C.d_mq, C.d_hez, &hits, &nh, &ms_sv, serr,
                             sizeof(serr));
            if (rc != GROM_OK) {
                set_err("%s", serr);
                return rc;
            }
            n_hits = nh;
            t_sv_eval = ms_since(t_start);
            if (nh > 0) {
                // the rows read reference bases (REF text, homopolymer runs):
                // the caller's host copy when there is one, else the pinned
                // copy made beside the pileup
                href = C.host_ref;
                if (!href) {
                    HIPCHK(hipEventSynchronize(C.ref_ev));
                    ref_copy_pending = false;
                    href = C.h_ref;
                }
                t_sv_ref = ms_since(t_start);
                // candidate lists, SV assembly and rows on a host thread while
                // the CNV path runs on the GPU
                svt = std::thread([&P, ch, href, &cs, hits, nh, &sv_text, &ctx_text] {
                    SvRowsInput ri{&P, ch->name, href, ch->len, &CafSum::call, &cs};
                    static const char *rec_prefix = getenv("GROM_SV_HITS_DUMP");  // test hook (sv.h)
                    if (!rec_prefix) {
                        sv_rows(ri, hits, nh, sv_text, ctx_text);
                        return;
                    }
                    struct Rec {
                        CafSum *cs;
                        std::vector<SvCafRec> q;
                        static double call(void *u, int64_t lo, int64_t hi) {
                            Rec &r = *(Rec *)u;
                            const double v = CafSum::call(r.cs, lo, hi);
                            r.q.push_back({lo, hi, v});
                            return v;
                        }
                    } rec{&cs, {}};
                    SvRowsInput rr{&P, ch->name, href, ch->len, &Rec::call, &rec};
                    sv_rows(rr, hits, nh, sv_text, ctx_text);
                    std::string path = std::string(rec_prefix) + "." + ch->name + ".svh";
                    if (sv_rows_record_write(path.c_str(), rr, hits, nh, rec.q, sv_text, ctx_text))
                        fprintf(stderr, "grom: writing %s failed\n", path.c_str());
                });
            }
        }
        const double t_sv = ms_since(t_start);
        if (ch->cnv && !want_dbg) {
            // the CNV phase: the arena's pileup/breakpoint buffers are dead
            // (sv_evaluate waited for the stream; the rows read pinned copies)
            if (!C.cnv) C.cnv = cnv_scratch_new();
            if (par && grom_arena_begin(par)) {
                set_err("phase arena: device memory allocation failed");
                return GROM_E_NOMEM;
            }
            cnv_scratch_phase(C.cnv, par);
        }
        if (reads_done) {
            // every kernel that reads the input has finished (sv_evaluate
            // waited for the stream) and so has the reference's host copy
            if (ref_copy_pending) {
                HIPCHK(hipEventSynchronize(C.ref_ev));
                ref_copy_pending = false;
            }
            reads_done(reads_done_arg);
        }

        // read-depth CNV path after the SV rows (GROM.c:16633-17300); the
        // reference runs it only when the FASTA name matched a BAM target
        CnvTiming ct{};
        std::string cnv_text;
        if (ch->cnv && !want_dbg) {
            if (!C.cnv) C.cnv = cnv_scratch_new();
            std::string crow, side;
            char cerr[512] = {0};
            rc = cnv_chrom(C.cnv, st, P, ch->seed, ch->name, cnv_ref, ch->len, (int32_t *)C.caf_mq.p,
                           (const int32_t *)C.caf_rd.p, (const int32_t *)C.caf_low.p, crow, &ct, cerr, sizeof(cerr),
                           P.gen1000_window > 0 ? &side : nullptr);
            if (rc != GROM_OK) {
                set_err("%s", cerr);
                return rc;
            }
            cnv_text.swap(crow);
            if (P.gen1000_window > 0) {
                Text sdt{&out->side, &out->side_len, &out->side_cap};
                if (!side.empty()) sdt.add(side.data(), side.size());
                out->side_written = 1;
            }
        }
        const double t_cnv = ms_since(t_start);
        if (svt.joinable()) svt.join();
        if (cs.rc != GROM_OK) {
            set_err("INV depth check: device copy failed");  // raised on the row thread
            return cs.rc;
        }
        fmt.join();
        const double t_rows = ms_since(t_start);
        // SNV rows, the breakpoint rows (GROM.c:15163-16580), then the CNV rows (16633)
        vt.add(snv_text.data(), snv_text.size());
        vt.add(sv_text.data(), sv_text.size());
        vt.add(cnv_text.data(), cnv_text.size());
        Text ctt{&out->ctx, &out->ctx_len, &out->ctx_cap};
        if (!ctx_text.empty()) ctt.add(ctx_text.data(), ctx_text.size());

        if (timing)
            fprintf(stderr,
                    "grom timing %s: kernels %.3f ms, candidates ordered+copied %.3f ms (%u candidates), "
                    "breakpoint tests %.3f ms (device %.3f ms, %zu hit bases; eval %.3f, ref copy %.3f, rows %.3f), "
                    "cnv %.3f ms (device %.3f ms, %lld/%lld DEL/DUP calls, %lld rows), SNV rows (overlapped) "
                    "joined after %.3f ms more, %lld tiles\n",
                    ch->name ? ch->name : "?", t_kernels, t_snv - t_kernels, ncand, t_sv - t_snv, ms_sv,
                    n_hits, t_sv_eval - t_snv, t_sv_ref > 0 ? t_sv_ref - t_sv_eval : 0.0,
                    t_sv - (t_sv_ref > 0 ? t_sv_ref : t_sv_eval), t_cnv - t_sv, ct.ms_device, (long long)ct.del_calls,
                    (long long)ct.dup_calls, (long long)ct.rows, t_rows - t_cnv, (long long)n_tiles);
        HIPCHK(hipEventRecord(C.e1, st));
        HIPCHK(hipEventSynchronize(C.e1));
        if (ref_copy_pending) HIPCHK(hipEventSynchronize(C.ref_ev));
        if (stats) {
            float ms = 0, msp = 0;
            (void)hipEventElapsedTime(&ms, C.e0, C.e1);
            (void)hipEventElapsedTime(&msp, C.ep0, C.ep1);
            uint32_t nev = 0;
            (void)hipMemcpy(&nev, d_nev, 4, hipMemcpyDeviceToHost);
            stats->ms_total = ms;
            stats->ms_pileup = msp;
            stats->ms_cnv = ct.ms_device;
            stats->cnv_rows = ct.rows;
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
    static const uint32_t zero_off[1] = {0};
    const uint32_t *coff = (n > 0 && h->cigar_off) ? h->cigar_off : zero_off;  // an empty batch may hold no array
    if ((rc = up(C.r_pos, h->pos, n, st)) || (rc = up(C.r_flag, h->flag, n, st)) ||
        (rc = up(C.r_mapq, h->mapq, n, st)) || (rc = up(C.r_mtid, h->mtid, n, st)) ||
        (rc = up(C.r_mpos, h->mpos, n, st)) || (rc = up(C.r_isize, h->isize, n, st)) ||
        (rc = up(C.r_lq, h->l_qseq, n, st)) || (rc = up(C.r_coff, coff, n + 1, st)) ||
        (rc = up(C.r_cig, h->cigar, h->n_cigar_ops, st)) || (rc = up(C.r_boff, h->base_off, n, st)) ||
        (rc = up(C.r_seq, h->seq, (h->n_bases + 1) / 2, st)) || (rc = up(C.r_qual, h->qual, h->n_bases, st)) ||
        (rc = up(C.r_nid, h->name_id, n, st)) || (rc = up(C.ref, ch->ref, ch->len, st)))
        return rc;
    const bool has_aux = h->n_aux > 0 && h->aux_idx && h->aux;
    if (has_aux && ((rc = up(C.r_aidx, h->aux_idx, n, st)) || (rc = up(C.r_aux, h->aux, h->n_aux, st)))) return rc;
    const bool has_drop = h->n_drop > 0 && h->drop_pos && h->drop_lq && h->drop_before;
    if (has_drop && ((rc = up(C.r_dpos, h->drop_pos, h->n_drop, st)) || (rc = up(C.r_dlq, h->drop_lq, h->n_drop, st)) ||
                     (rc = up(C.r_dbef, h->drop_before, h->n_drop, st))))
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
    d->n_aux = has_aux ? h->n_aux : 0;
    d->aux_idx = has_aux ? (const int32_t *)C.r_aidx.p : nullptr;
    d->aux = has_aux ? (const grom_aux *)C.r_aux.p : nullptr;
    d->n_drop = has_drop ? h->n_drop : 0;
    d->drop_pos = has_drop ? (const int32_t *)C.r_dpos.p : nullptr;
    d->drop_lq = has_drop ? (const int32_t *)C.r_dlq.p : nullptr;
    d->drop_before = has_drop ? (const int64_t *)C.r_dbef.p : nullptr;
    return GROM_OK;
}

}  // namespace

extern "C" {

int grom_abi_version(void) { return GROM_AMD_ABI_VERSION; }
int grom_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}
size_t grom_abi_struct_size(int which) {
    switch (which) {
    case 0: return sizeof(grom_params);
    case 1: return sizeof(grom_chrom);
    case 2: return sizeof(grom_reads);
    case 3: return sizeof(grom_out);
    case 4: return sizeof(grom_stats);
    case 5: return sizeof(grom_indel_rec);
    case 6: return sizeof(grom_aux);
    case 7: return sizeof(grom_sv_rec);
    default: return 0;
    }
}
const char *grom_last_error(void) { return g_err; }
void grom_set_last_error(const char *msg) { set_err("%s", msg ? msg : ""); }
int64_t grom_device_mem_free(int device) {
    size_t fr = 0, tot = 0;
    if (hipSetDevice(device) != hipSuccess || hipMemGetInfo(&fr, &tot) != hipSuccess) return -1;
    return (int64_t)fr;
}

int grom_ctx_init(int slot, int device, const grom_params *params, const double *hez, const double *mq) {
    if (slot < 0 || slot >= 64 || device < 0 || !params || !hez || !mq) {
        set_err("grom_ctx_init: bad argument");
        return GROM_E_ARG;
    }
    Ctx &C = g_ctx[slot];
    if (C.init) grom_dev_fini(slot);
    HIPCHK(hipSetDevice(device));
    C.device = device;
    C.prm = *params;
    HIPCHK(hipStreamCreateWithFlags(&C.st, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&C.st_copy, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&C.ref_ev, hipEventDisableTiming));
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

int grom_ctx_set_params(int slot, const grom_params *params) {
    if (slot < 0 || slot >= 64 || !params || !g_ctx[slot].init) {
        set_err("grom_ctx_set_params: bad argument");
        return GROM_E_ARG;
    }
    g_ctx[slot].prm = *params;
    return GROM_OK;
}

int grom_dev_init(int device, const grom_params *params, const double *hez, const double *mq) {
    return grom_ctx_init(device, device, params, hez, mq);
}

void grom_dev_fini(int device) {
    if (device < 0 || device >= 64 || !g_ctx[device].init) return;
    Ctx &C = g_ctx[device];
    (void)hipSetDevice(C.device);
    (void)hipStreamSynchronize(C.st);
    DevBuf *all[] = {&C.r_pos, &C.r_flag, &C.r_mapq, &C.r_mtid, &C.r_mpos, &C.r_isize, &C.r_lq, &C.r_coff,
                     &C.r_cig, &C.r_boff, &C.r_seq, &C.r_qual, &C.r_nid, &C.ref, &C.keep, &C.meta, &C.cands2,
                     &C.runb, &C.runc, &C.segs, &C.fpart, &C.tlo, &C.thi, &C.caf_mq, &C.caf_rd, &C.caf_low, &C.cands,
                     &C.misc, &C.dbg, &C.slots, &C.r_aidx, &C.r_aux, &C.r_dpos, &C.r_dlq, &C.r_dbef};
    for (DevBuf *b : all)
        if (b->p) {
            if (b->own) grom_dev_free(b->p, b->cap, GROM_DEVCAT_SCAN);
            b->p = nullptr;
            b->cap = 0;
        }
    if (C.h_cands) (void)hipHostFree(C.h_cands);
    if (C.h_cafsum) (void)hipHostFree(C.h_cafsum);
    if (C.st_copy) (void)hipStreamSynchronize(C.st_copy);
    if (C.h_ref) (void)hipHostFree(C.h_ref);
    if (C.ref_ev) (void)hipEventDestroy(C.ref_ev);
    if (C.st_copy) (void)hipStreamDestroy(C.st_copy);
    cnv_scratch_free(C.cnv);
    sv_scratch_free(C.sv);
    grom_arena_free(C.ar);
    (void)hipFree(C.d_mq);
    (void)hipFree(C.d_hez);
    (void)hipEventDestroy(C.e0);
    (void)hipEventDestroy(C.e1);
    (void)hipEventDestroy(C.ep0);
    (void)hipEventDestroy(C.ep1);
    (void)hipStreamDestroy(C.st);
    g_ctx[device] = Ctx();
}


int grom_scan_chrom(int device, const grom_chrom *chrom, const grom_reads *reads, grom_out *out, grom_stats *stats) {
    Ctx *C = ctx_of(device);
    if (!C) return GROM_E_NODEV;
    if (!chrom || !reads || !out || !chrom->ref) { set_err("grom_scan_chrom: null argument"); return GROM_E_ARG; }
    HIPCHK(hipSetDevice(C->device));
    grom_chrom dch;
    grom_reads dr;
    int rc = upload(*C, chrom, reads, &dch, &dr);
    if (rc) return rc;
    C->host_ref = chrom->ref;
    rc = scan_device(*C, &dch, &dr, out, stats, nullptr, nullptr, 0, nullptr);
    C->host_ref = nullptr;
    return rc;
}

int grom_scan_chrom_device(int device, const grom_chrom *chrom, const grom_reads *dev_reads, grom_out *out,
                           grom_stats *stats) {
    Ctx *C = ctx_of(device);
    if (!C) return GROM_E_NODEV;
    if (!chrom || !dev_reads || !out) { set_err("grom_scan_chrom_device: null argument"); return GROM_E_ARG; }
    if (((uintptr_t)dev_reads->qual | (uintptr_t)dev_reads->seq) & 15) {
        set_err("grom_scan_chrom_device: qual and seq must be 16-byte aligned");
        return GROM_E_ARG;
    }
    HIPCHK(hipSetDevice(C->device));
    return scan_device(*C, chrom, dev_reads, out, stats, nullptr, nullptr, 0, nullptr);
}

int grom_upload(int device, const grom_chrom *chrom, const grom_reads *reads, grom_chrom *dev_chrom,
                grom_reads *dev_reads) {
    Ctx *C = ctx_of(device);
    if (!C) return GROM_E_NODEV;
    if (!chrom || !reads || !dev_chrom || !dev_reads) { set_err("grom_upload: null argument"); return GROM_E_ARG; }
    HIPCHK(hipSetDevice(C->device));
    int rc = upload(*C, chrom, reads, dev_chrom, dev_reads);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(C->st));
    return GROM_OK;
}

struct grom_resident {
    int device;
    void *base;
    int64_t bytes;
};

grom_resident *grom_resident_new(int device, const grom_chrom *ch, const grom_reads *h, grom_chrom *dch,
                                 grom_reads *d) {
    if (!ch || !h || !dch || !d || !ch->ref || ch->len <= 0) {
        set_err("grom_resident_new: bad argument");
        return nullptr;
    }
    const int64_t n = h->n;
    const bool has_aux = h->n_aux > 0 && h->aux_idx && h->aux;
    const bool has_drop = h->n_drop > 0 && h->drop_pos && h->drop_lq && h->drop_before;
    static const uint32_t zero_off[1] = {0};
    struct Part { const void *src; size_t bytes; size_t off; };
    // every array 256-byte aligned; qual/seq padded past their end (16-byte reads)
    Part parts[] = {
        {h->pos, 4 * (size_t)n}, {h->flag, 2 * (size_t)n}, {h->mapq, (size_t)n}, {h->mtid, 4 * (size_t)n},
        {h->mpos, 4 * (size_t)n}, {h->isize, 4 * (size_t)n}, {h->l_qseq, 4 * (size_t)n},
        {n > 0 && h->cigar_off ? h->cigar_off : zero_off, 4 * (size_t)(n + 1)},
        {h->cigar, 4 * (size_t)h->n_cigar_ops}, {h->base_off, 8 * (size_t)n}, {h->seq, (size_t)(h->n_bases + 1) / 2},
        {h->qual, (size_t)h->n_bases}, {h->name_id, 4 * (size_t)n}, {ch->ref, (size_t)ch->len},
        {has_aux ? h->aux_idx : nullptr, has_aux ? 4 * (size_t)n : 0},
        {has_aux ? h->aux : nullptr, has_aux ? sizeof(grom_aux) * (size_t)h->n_aux : 0},
        {has_drop ? h->drop_pos : nullptr, has_drop ? 4 * (size_t)h->n_drop : 0},
        {has_drop ? h->drop_lq : nullptr, has_drop ? 4 * (size_t)h->n_drop : 0},
        {has_drop ? h->drop_before : nullptr, has_drop ? 8 * (size_t)h->n_drop : 0},
    };
    size_t off = 0;
    for (Part &q : parts) {
        q.off = off;
        off += (q.bytes + 64 + 255) & ~(size_t)255;
    }
    grom_resident *r = new grom_resident{device, nullptr, (int64_t)off};
    if (hipSetDevice(device) != hipSuccess || hipMalloc(&r->base, off) != hipSuccess) {
        set_err("grom_resident_new: hipMalloc(%zu) on device %d failed", off, device);
        delete r;
        return nullptr;
    }
    for (const Part &q : parts)
        if (q.bytes && hipMemcpy((char *)r->base + q.off, q.src, q.bytes, hipMemcpyHostToDevice) != hipSuccess) {
            set_err("grom_resident_new: copy to device failed");
            (void)hipFree(r->base);
            delete r;
            return nullptr;
        }
    auto at = [&](int k) { return (const void *)((const char *)r->base + parts[k].off); };
    *dch = *ch;
    dch->ref = (const char *)at(13);
    *d = *h;
    d->pos = (const int32_t *)at(0);
    d->flag = (const uint16_t *)at(1);
    d->mapq = (const uint8_t *)at(2);
    d->mtid = (const int32_t *)at(3);
    d->mpos = (const int32_t *)at(4);
    d->isize = (const int32_t *)at(5);
    d->l_qseq = (const int32_t *)at(6);
    d->cigar_off = (const uint32_t *)at(7);
    d->cigar = (const uint32_t *)at(8);
    d->base_off = (const int64_t *)at(9);
    d->seq = (const uint8_t *)at(10);
    d->qual = (const uint8_t *)at(11);
    d->name_id = (const uint32_t *)at(12);
    d->n_aux = has_aux ? h->n_aux : 0;
    d->aux_idx = has_aux ? (const int32_t *)at(14) : nullptr;
    d->aux = has_aux ? (const grom_aux *)at(15) : nullptr;
    d->n_drop = has_drop ? h->n_drop : 0;
    d->drop_pos = has_drop ? (const int32_t *)at(16) : nullptr;
    d->drop_lq = has_drop ? (const int32_t *)at(17) : nullptr;
    d->drop_before = has_drop ? (const int64_t *)at(18) : nullptr;
    return r;
}

int64_t grom_resident_bytes(const grom_resident *r) { return r ? r->bytes : 0; }

void grom_resident_free(grom_resident *r) {
    if (!r) return;
    (void)hipSetDevice(r->device);
    (void)hipFree(r->base);
    delete r;
}

// ---------------------------------------------------------------------------
// Streamed input (include/grom_amd.h, "streamed input"): a chromosome's reads
// arrive as pieces in pinned host memory; each piece is appended with async
// copies on the stage's own stream, so the copies of chromosome k+1 overlap
// the scan of chromosome k on the contexts' streams.
// ---------------------------------------------------------------------------
void *grom_pinned_alloc(size_t bytes) {
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 16, hipHostMallocPortable) != hipSuccess) {
        set_err("hipHostMalloc(%zu) failed", bytes);
        return nullptr;
    }
    return p;
}

void grom_pinned_free(void *p) {
    if (p) (void)hipHostFree(p);
}

#define GROM_STAGE_EVENTS 64

// the arrays of a staged chromosome, all in one device block
enum { SA_POS, SA_FLAG, SA_MAPQ, SA_MTID, SA_MPOS, SA_ISIZE, SA_LQ, SA_COFF, SA_BOFF, SA_NID, SA_AIDX, SA_CIG, SA_QUAL,
       SA_SEQ, SA_AUX, SA_DPOS, SA_DLQ, SA_DBEF, SA_REF, SA_N };

struct grom_stage {
    int device = -1;
    hipStream_t st = nullptr;
    // one device block; array a at off[a] with cap[a] bytes (slack: kernels
    // read whole 16-byte words past an array's end)
    char *blk = nullptr;
    size_t blk_cap = 0;
    size_t off[SA_N] = {}, cap[SA_N] = {};
    int64_t n = 0, n_cig = 0, n_bases = 0, n_aux = 0, n_drop = 0, ref_len = 0;
    int64_t front = 0;  // reads trimmed from the front of the views (grom_stage_trim)
    int32_t patch_idx = -1;
    grom_aux patch_aux{};
    hipEvent_t ev[GROM_STAGE_EVENTS] = {};
    hipEvent_t all_ev = nullptr;  // every copy issued so far (the scans wait on it)
    int64_t tickets = 0;  // appends issued (ticket t uses ev[t % GROM_STAGE_EVENTS])
    int64_t done_upto = 0; // every ticket below this is known complete
    int64_t bytes_h2d = 0;
    // scratch of the stage's own operations (put_aux, trim_drops): grows, is
    // kept (a hipMalloc/hipFree pair per chromosome would wait for the device)
    char *scratch = nullptr;
    size_t scratch_cap = 0;
    // called by grom_scan_chrom_staged once the scan no longer reads the
    // stage (grom_stage_on_consumed)
    void (*consumed)(void *, grom_stage *) = nullptr;
    void *consumed_arg = nullptr;
    char *a(int k) const { return blk + off[k]; }
};

int64_t grom_stage_held(const grom_stage *s) { return s ? (int64_t)(s->blk_cap + s->scratch_cap) : 0; }

int64_t grom_stage_drop(grom_stage *s) {
    if (!s || (!s->blk && !s->scratch)) return 0;
    (void)hipSetDevice(s->device);
    (void)hipStreamSynchronize(s->st);
    const int64_t freed = (int64_t)(s->blk_cap + s->scratch_cap);
    if (s->blk) grom_dev_free(s->blk, s->blk_cap, GROM_DEVCAT_STAGE);
    if (s->scratch) grom_dev_free(s->scratch, s->scratch_cap, GROM_DEVCAT_STAGE);
    s->blk = nullptr;
    s->blk_cap = 0;
    s->scratch = nullptr;
    s->scratch_cap = 0;
    memset(s->cap, 0, sizeof(s->cap));
    memset(s->off, 0, sizeof(s->off));
    s->n = s->n_cig = s->n_bases = s->n_aux = s->n_drop = s->ref_len = 0;
    s->front = 0;
    return freed;
}

void grom_stage_on_consumed(grom_stage *s, void (*fn)(void *, grom_stage *), void *arg) {
    if (!s) return;
    s->consumed = fn;
    s->consumed_arg = arg;
}

static char *stage_scratch(grom_stage *s, size_t bytes) {
    if (bytes <= s->scratch_cap) return s->scratch;
    if (s->scratch) {
        (void)hipStreamSynchronize(s->st);
        grom_dev_free(s->scratch, s->scratch_cap, GROM_DEVCAT_STAGE);
    }
    s->scratch = nullptr;
    s->scratch_cap = 0;
    const size_t want = bytes + bytes / 2 + 4096;
    if (grom_dev_malloc((void **)&s->scratch, want, GROM_DEVCAT_STAGE)) return nullptr;
    s->scratch_cap = want;
    return s->scratch;
}

// bytes each array holds now (kept when the block grows)
static void stage_used(const grom_stage *s, size_t u[SA_N]) {
    u[SA_POS] = 4 * s->n; u[SA_FLAG] = 2 * s->n; u[SA_MAPQ] = s->n; u[SA_MTID] = 4 * s->n; u[SA_MPOS] = 4 * s->n;
    u[SA_ISIZE] = 4 * s->n; u[SA_LQ] = 4 * s->n; u[SA_COFF] = 4 * (s->n + 1); u[SA_BOFF] = 8 * s->n;
    u[SA_NID] = 4 * s->n; u[SA_AIDX] = 4 * s->n; u[SA_CIG] = 4 * s->n_cig; u[SA_QUAL] = s->n_bases;
    u[SA_SEQ] = s->n_bases / 2; u[SA_AUX] = sizeof(grom_aux) * s->n_aux; u[SA_DPOS] = 4 * s->n_drop;
    u[SA_DLQ] = 4 * s->n_drop; u[SA_DBEF] = 8 * s->n_drop; u[SA_REF] = s->ref_len;
}

// make every array hold need[a] bytes (+64 slack), keeping keep[a] bytes of
// its contents: one new block when anything is short (copies on the stage
// stream), else nothing.  A short array gets need + need/grow: appends grow
// by a quarter (grow 4, amortised), exact or estimated sizes by 1/64.
static int stage_reserve(grom_stage *s, const size_t need[SA_N], const size_t keep[SA_N], size_t grow = 64) {
    bool ok = s->blk != nullptr;
    for (int k = 0; k < SA_N && ok; k++) ok = s->cap[k] >= need[k] + 64;
    if (ok) return GROM_OK;
    size_t cap[SA_N], off[SA_N], tot = 0;
    for (int k = 0; k < SA_N; k++) {
        cap[k] = s->cap[k] >= need[k] + 64 ? s->cap[k] : need[k] + need[k] / grow + 4096;
        off[k] = tot;
        tot += (cap[k] + 255) & ~(size_t)255;
    }
    static const bool log = getenv("GROM_STAGE_LOG") != nullptr;
    if (log) {  // which arrays outgrew the block
        fprintf(stderr, "grom: stage %p block %.3f -> %.3f GB:", (void *)s, s->blk_cap / 1e9, tot / 1e9);
        for (int k = 0; k < SA_N; k++)
            if (s->cap[k] < need[k] + 64) fprintf(stderr, " [%d] %zu<%zu", k, s->cap[k], need[k]);
        fputc('\n', stderr);
    }
    char *nb = nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    bool kept = false;
    for (int k = 0; k < SA_N; k++) kept |= keep[k] != 0;
    if (s->blk && !kept) {  // nothing to carry over: the old block goes first
        HIPCHK(hipStreamSynchronize(s->st));
        grom_dev_free(s->blk, s->blk_cap, GROM_DEVCAT_STAGE);
        s->blk = nullptr;
        s->blk_cap = 0;
        memset(s->cap, 0, sizeof(s->cap));
    }
    if (grom_dev_malloc((void **)&nb, tot, GROM_DEVCAT_STAGE)) {
        set_err("grom_stage: hipMalloc(%zu) failed", tot);
        return GROM_E_NOMEM;
    }
    if (s->blk) {
        for (int k = 0; k < SA_N; k++)
            if (keep[k]) HIPCHK(hipMemcpyAsync(nb + off[k], s->a(k), keep[k], hipMemcpyDeviceToDevice, s->st));
        HIPCHK(hipStreamSynchronize(s->st));
        grom_dev_free(s->blk, s->blk_cap, GROM_DEVCAT_STAGE);
    }
    grom_note_alloc_ns(std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count(),
                       tot);
    s->blk = nb;
    s->blk_cap = tot;
    memcpy(s->off, off, sizeof(off));
    memcpy(s->cap, cap, sizeof(cap));
    return GROM_OK;
}

grom_stage *grom_stage_new(int device) {
    if (hipSetDevice(device) != hipSuccess) {
        set_err("grom_stage_new: no device %d", device);
        return nullptr;
    }
    grom_stage *s = new grom_stage();
    s->device = device;
    if (hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking) != hipSuccess) {
        set_err("grom_stage_new: stream creation failed");
        delete s;
        return nullptr;
    }
    for (int k = 0; k <= GROM_STAGE_EVENTS; k++)
        if (hipEventCreateWithFlags(k < GROM_STAGE_EVENTS ? &s->ev[k] : &s->all_ev, hipEventDisableTiming) !=
            hipSuccess) {
            set_err("grom_stage_new: event creation failed");
            grom_stage_free(s);
            return nullptr;
        }
    return s;
}

void grom_stage_free(grom_stage *s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    if (s->st) (void)hipStreamSynchronize(s->st);
    if (s->blk) grom_dev_free(s->blk, s->blk_cap, GROM_DEVCAT_STAGE);
    if (s->scratch) grom_dev_free(s->scratch, s->scratch_cap, GROM_DEVCAT_STAGE);
    for (int k = 0; k < GROM_STAGE_EVENTS; k++)
        if (s->ev[k]) (void)hipEventDestroy(s->ev[k]);
    if (s->all_ev) (void)hipEventDestroy(s->all_ev);
    if (s->st) (void)hipStreamDestroy(s->st);
    delete s;
}

int grom_stage_begin(grom_stage *s, const grom_stage_sizes *est) {
    if (!s) { set_err("grom_stage_begin: null stage"); return GROM_E_ARG; }
    HIPCHK(hipSetDevice(s->device));
    HIPCHK(hipStreamSynchronize(s->st));  // the previous chromosome's copies are done
    s->n = s->n_cig = s->n_bases = s->n_aux = s->n_drop = s->ref_len = 0;
    s->front = 0;
    s->done_upto = s->tickets;
    s->bytes_h2d = 0;
    if (est) {
        const size_t n = (size_t)std::max<int64_t>(est->n, 1), nd = (size_t)std::max<int64_t>(est->n_drop, 1);
        const size_t nb = (size_t)std::max<int64_t>(est->n_bases, 16);
        size_t need[SA_N] = {4 * n, 2 * n, n, 4 * n, 4 * n, 4 * n, 4 * n, 4 * (n + 1), 8 * n, 4 * n, 4 * n,
                             4 * (size_t)std::max<int64_t>(est->n_cigar_ops, 1), nb, nb / 2,
                             sizeof(grom_aux) * (size_t)std::max<int64_t>(est->n_aux, 1), 4 * nd, 4 * nd, 8 * nd,
                             (size_t)std::max<int64_t>(est->ref_len, 16)};
        const size_t keep[SA_N] = {};
        const int rc = stage_reserve(s, need, keep);
        if (rc == GROM_OK && !stage_scratch(s, std::max(16 * nd, 8 * (size_t)std::max<int64_t>(est->n_aux, 1)))) {
            set_err("grom_stage_begin: no device scratch");
            return GROM_E_NOMEM;
        }
        return rc;
    }
    return GROM_OK;
}

int grom_stage_set_ref(grom_stage *s, const char *ref, int64_t len) {
    if (!s || (!ref && len > 0) || len < 0) { set_err("grom_stage_set_ref: bad argument"); return GROM_E_ARG; }
    HIPCHK(hipSetDevice(s->device));
    size_t need[SA_N], keep[SA_N];
    stage_used(s, need);
    stage_used(s, keep);
    need[SA_REF] = (size_t)std::max<int64_t>(len, 16);
    keep[SA_REF] = 0;
    int rc = stage_reserve(s, need, keep);
    if (rc) return rc;
    if (len > 0) HIPCHK(hipMemcpyAsync(s->a(SA_REF), ref, (size_t)len, hipMemcpyHostToDevice, s->st));
    s->ref_len = len;
    s->bytes_h2d += len;
    return GROM_OK;
}

static int stage_ticket_wait(grom_stage *s, int64_t t) {
    if (t < s->done_upto) return GROM_OK;
    HIPCHK(hipEventSynchronize(s->ev[t % GROM_STAGE_EVENTS]));
    s->done_upto = t + 1;
    return GROM_OK;
}

int64_t grom_stage_append(grom_stage *s, const grom_reads *p) {
    if (!s || !p || p->n < 0 || (p->n > 0 && (!p->pos || !p->cigar_off || !p->base_off))) {
        set_err("grom_stage_append: bad argument");
        return GROM_E_ARG;
    }
    if (p->n_bases & 1) { set_err("grom_stage_append: n_bases must be even"); return GROM_E_ARG; }
    HIPCHK(hipSetDevice(s->device));
    // the event of this ticket's slot must be free (the append GROM_STAGE_EVENTS back is done)
    if (s->tickets >= GROM_STAGE_EVENTS) {
        int rc = stage_ticket_wait(s, s->tickets - GROM_STAGE_EVENTS);
        if (rc) return rc;
    }
    const bool has_aux = p->n_aux > 0 && p->aux;
    const bool has_drop = p->n_drop > 0 && p->drop_pos && p->drop_lq && p->drop_before;
    grom_stage after = {};  // the counts after this piece (for the sizes only)
    after.n = s->n + p->n;
    after.n_cig = s->n_cig + p->n_cigar_ops;
    after.n_bases = s->n_bases + p->n_bases;
    after.n_aux = s->n_aux + (has_aux ? p->n_aux : 0);
    after.n_drop = s->n_drop + (has_drop ? p->n_drop : 0);
    after.ref_len = s->ref_len;
    size_t need[SA_N], keep[SA_N];
    stage_used(&after, need);
    stage_used(s, keep);
    int rc = stage_reserve(s, need, keep, 4);
    if (rc) return rc;
    int64_t bytes = 0;
    auto cp = [&](int arr, int64_t off_bytes, const void *src, int64_t nbytes) -> int {
        if (nbytes <= 0) return GROM_OK;
        HIPCHK(hipMemcpyAsync(s->a(arr) + off_bytes, src, (size_t)nbytes, hipMemcpyHostToDevice, s->st));
        bytes += nbytes;
        return GROM_OK;
    };
    const int64_t k = p->n;
    if (k > 0) {
        if ((rc = cp(SA_POS, 4 * s->n, p->pos, 4 * k)) || (rc = cp(SA_FLAG, 2 * s->n, p->flag, 2 * k)) ||
            (rc = cp(SA_MAPQ, s->n, p->mapq, k)) || (rc = cp(SA_MTID, 4 * s->n, p->mtid, 4 * k)) ||
            (rc = cp(SA_MPOS, 4 * s->n, p->mpos, 4 * k)) || (rc = cp(SA_ISIZE, 4 * s->n, p->isize, 4 * k)) ||
            (rc = cp(SA_LQ, 4 * s->n, p->l_qseq, 4 * k)) || (rc = cp(SA_COFF, 4 * s->n, p->cigar_off, 4 * (k + 1))) ||
            (rc = cp(SA_BOFF, 8 * s->n, p->base_off, 8 * k)) || (rc = cp(SA_NID, 4 * s->n, p->name_id, 4 * k)) ||
            (rc = cp(SA_CIG, 4 * s->n_cig, p->cigar, 4 * p->n_cigar_ops)) ||
            (rc = cp(SA_QUAL, s->n_bases, p->qual, p->n_bases)) ||
            (rc = cp(SA_SEQ, s->n_bases / 2, p->seq, p->n_bases / 2)))
            return rc;
        if (p->aux_idx) {
            if ((rc = cp(SA_AIDX, 4 * s->n, p->aux_idx, 4 * k))) return rc;
        } else {
            HIPCHK(hipMemsetAsync(s->a(SA_AIDX) + 4 * s->n, 0xff, 4 * (size_t)k, s->st));
        }
    }
    if (has_aux && (rc = cp(SA_AUX, sizeof(grom_aux) * s->n_aux, p->aux, sizeof(grom_aux) * p->n_aux))) return rc;
    if (has_drop && ((rc = cp(SA_DPOS, 4 * s->n_drop, p->drop_pos, 4 * p->n_drop)) ||
                     (rc = cp(SA_DLQ, 4 * s->n_drop, p->drop_lq, 4 * p->n_drop)) ||
                     (rc = cp(SA_DBEF, 8 * s->n_drop, p->drop_before, 8 * p->n_drop))))
        return rc;
    const int64_t t = s->tickets++;
    HIPCHK(hipEventRecord(s->ev[t % GROM_STAGE_EVENTS], s->st));
    s->n = after.n;
    s->n_cig = after.n_cig;
    s->n_bases = after.n_bases;
    s->n_aux = after.n_aux;
    s->n_drop = after.n_drop;
    s->bytes_h2d += bytes;
    return t;
}

int grom_stage_ticket_done(grom_stage *s, int64_t ticket) {
    if (!s || ticket < 0 || ticket >= s->tickets) return 1;
    if (ticket < s->done_upto) return 1;
    if (s->tickets - ticket > GROM_STAGE_EVENTS) return 1;  // its slot was reused after it completed
    if (hipSetDevice(s->device) != hipSuccess) return 0;
    hipError_t e = hipEventQuery(s->ev[ticket % GROM_STAGE_EVENTS]);
    return e == hipSuccess ? 1 : 0;
}

int grom_stage_ticket_wait(grom_stage *s, int64_t ticket) {
    if (!s || ticket < 0 || ticket >= s->tickets || s->tickets - ticket > GROM_STAGE_EVENTS) return GROM_OK;
    HIPCHK(hipSetDevice(s->device));
    return stage_ticket_wait(s, ticket);
}

int grom_stage_view(grom_stage *s, const grom_chrom *chrom, grom_chrom *dch, grom_reads *d) {
    if (!s || !chrom || !dch || !d) { set_err("grom_stage_view: null argument"); return GROM_E_ARG; }
    if (s->ref_len != chrom->len) {
        set_err("grom_stage_view: reference of %lld bases staged, chromosome has %lld", (long long)s->ref_len,
                (long long)chrom->len);
        return GROM_E_ARG;
    }
    HIPCHK(hipSetDevice(s->device));
    if (s->n == 0) {  // an empty chromosome still needs cigar_off[0] = 0
        size_t need[SA_N], keep[SA_N];
        stage_used(s, need);
        stage_used(s, keep);
        int rc = stage_reserve(s, need, keep);
        if (rc) return rc;
        HIPCHK(hipMemsetAsync(s->a(SA_COFF), 0, 4, s->st));
    }
    *dch = *chrom;
    dch->ref = (const char *)s->a(SA_REF);
    memset(d, 0, sizeof(*d));
    const int64_t f = s->front;
    d->n = s->n - f;
    d->n_cigar_ops = s->n_cig;
    d->n_bases = s->n_bases;
    d->pos = (const int32_t *)s->a(SA_POS) + f;
    d->flag = (const uint16_t *)s->a(SA_FLAG) + f;
    d->mapq = (const uint8_t *)s->a(SA_MAPQ) + f;
    d->mtid = (const int32_t *)s->a(SA_MTID) + f;
    d->mpos = (const int32_t *)s->a(SA_MPOS) + f;
    d->isize = (const int32_t *)s->a(SA_ISIZE) + f;
    d->l_qseq = (const int32_t *)s->a(SA_LQ) + f;
    d->cigar_off = (const uint32_t *)s->a(SA_COFF) + f;  // absolute offsets into cigar
    d->cigar = (const uint32_t *)s->a(SA_CIG);
    d->base_off = (const int64_t *)s->a(SA_BOFF) + f;    // absolute offsets into seq/qual
    d->seq = (const uint8_t *)s->a(SA_SEQ);
    d->qual = (const uint8_t *)s->a(SA_QUAL);
    d->name_id = (const uint32_t *)s->a(SA_NID) + f;
    d->n_aux = s->n_aux;
    d->aux_idx = s->n_aux > 0 ? (const int32_t *)s->a(SA_AIDX) + f : nullptr;
    d->aux = s->n_aux > 0 ? (const grom_aux *)s->a(SA_AUX) : nullptr;
    d->n_drop = s->n_drop;
    d->drop_pos = s->n_drop > 0 ? (const int32_t *)s->a(SA_DPOS) : nullptr;
    d->drop_lq = s->n_drop > 0 ? (const int32_t *)s->a(SA_DLQ) : nullptr;
    d->drop_before = s->n_drop > 0 ? (const int64_t *)s->a(SA_DBEF) : nullptr;
    return GROM_OK;
}

int64_t grom_stage_bytes(const grom_stage *s) { return s ? s->bytes_h2d : 0; }

int grom_stage_trim(grom_stage *s, int64_t n_front) {
    if (!s || n_front < 0 || n_front > s->n) { set_err("grom_stage_trim: bad argument"); return GROM_E_ARG; }
    s->front = n_front;
    return GROM_OK;
}

int grom_stage_patch_aux(grom_stage *s, int64_t read_index, const grom_aux *aux) {
    if (!s || !aux || read_index < 0 || read_index >= s->n || read_index > INT32_MAX) {
        set_err("grom_stage_patch_aux: bad argument");
        return GROM_E_ARG;
    }
    HIPCHK(hipSetDevice(s->device));
    size_t need[SA_N], keep[SA_N];
    stage_used(s, keep);
    stage_used(s, need);
    need[SA_AUX] += sizeof(grom_aux);
    int rc = stage_reserve(s, need, keep);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(s->st));  // the values below are copied from the stage itself
    s->patch_idx = (int32_t)s->n_aux;
    s->patch_aux = *aux;
    HIPCHK(hipMemcpyAsync(s->a(SA_AUX) + sizeof(grom_aux) * s->n_aux, &s->patch_aux, sizeof(grom_aux),
                          hipMemcpyHostToDevice, s->st));
    HIPCHK(hipMemcpyAsync(s->a(SA_AIDX) + 4 * read_index, &s->patch_idx, 4, hipMemcpyHostToDevice, s->st));
    HIPCHK(hipStreamSynchronize(s->st));
    s->n_aux++;
    return GROM_OK;
}

// ---- device-side fills (ddecode.hip: the BAM decoded on the GPU) ----
__global__ void k_stage_aux_idx(int32_t *aidx, const int64_t *kidx, int64_t n, int32_t first) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
        aidx[kidx[k]] = first + (int32_t)k;
}

__global__ void k_stage_trim_drops(int32_t *dpos, int32_t *dlq, int64_t *dbef, const int32_t *spos, const int32_t *slq,
                                   const int64_t *sbef, int64_t n, int64_t sk) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        dpos[k] = spos[k];
        dlq[k] = slq[k];
        dbef[k] = sbef[k] >= sk ? sbef[k] - sk : 0;
    }
}

static void stage_dev_view(grom_stage *s, grom_reads *d) {
    memset(d, 0, sizeof(*d));
    d->n = s->n;
    d->n_cigar_ops = s->n_cig;
    d->n_bases = s->n_bases;
    d->pos = (const int32_t *)s->a(SA_POS);
    d->flag = (const uint16_t *)s->a(SA_FLAG);
    d->mapq = (const uint8_t *)s->a(SA_MAPQ);
    d->mtid = (const int32_t *)s->a(SA_MTID);
    d->mpos = (const int32_t *)s->a(SA_MPOS);
    d->isize = (const int32_t *)s->a(SA_ISIZE);
    d->l_qseq = (const int32_t *)s->a(SA_LQ);
    d->cigar_off = (const uint32_t *)s->a(SA_COFF);
    d->cigar = (const uint32_t *)s->a(SA_CIG);
    d->base_off = (const int64_t *)s->a(SA_BOFF);
    d->seq = (const uint8_t *)s->a(SA_SEQ);
    d->qual = (const uint8_t *)s->a(SA_QUAL);
    d->name_id = (const uint32_t *)s->a(SA_NID);
    d->n_aux = s->n_aux;
    d->aux_idx = (const int32_t *)s->a(SA_AIDX);
    d->aux = (const grom_aux *)s->a(SA_AUX);
    d->n_drop = s->n_drop;
    d->drop_pos = (const int32_t *)s->a(SA_DPOS);
    d->drop_lq = (const int32_t *)s->a(SA_DLQ);
    d->drop_before = (const int64_t *)s->a(SA_DBEF);
}

int grom_stage_fill_begin(grom_stage *s, const grom_stage_sizes *sz, grom_reads *dev) {
    if (!s || !sz || !dev) { set_err("grom_stage_fill_begin: null argument"); return GROM_E_ARG; }
    int rc = grom_stage_begin(s, nullptr);
    if (rc) return rc;
    grom_stage want = {};
    want.n = sz->n;
    want.n_cig = sz->n_cigar_ops;
    want.n_bases = sz->n_bases;
    want.n_aux = sz->n_aux;
    want.n_drop = sz->n_drop;
    want.ref_len = std::max<int64_t>(sz->ref_len, 16);
    size_t need[SA_N], keep[SA_N] = {};
    stage_used(&want, need);
    need[SA_AUX] += sizeof(grom_aux);  // the -S patch
    if ((rc = stage_reserve(s, need, keep))) return rc;
    s->n = sz->n;
    s->n_cig = sz->n_cigar_ops;
    s->n_bases = sz->n_bases;
    s->n_aux = 0;
    s->n_drop = sz->n_drop;
    s->bytes_h2d = 0;
    stage_dev_view(s, dev);
    return GROM_OK;
}

// the piece-wise device decode (ddecode.hip): room for `need` in every array,
// keeping what the earlier pieces wrote (`have`); the stage's counts become
// `need` until grom_stage_fill_set gives the final ones
int grom_stage_fill_ensure(grom_stage *s, const grom_stage_sizes *need, const grom_stage_sizes *have, grom_reads *dev) {
    if (!s || !need || !have || !dev) { set_err("grom_stage_fill_ensure: null argument"); return GROM_E_ARG; }
    HIPCHK(hipSetDevice(s->device));
    grom_stage w = {}, h = {};
    w.n = need->n;
    w.n_cig = need->n_cigar_ops;
    w.n_bases = need->n_bases;
    w.n_aux = need->n_aux;
    w.n_drop = need->n_drop;
    w.ref_len = std::max<int64_t>(need->ref_len, 16);
    h.n = have->n;
    h.n_cig = have->n_cigar_ops;
    h.n_bases = have->n_bases;
    h.n_drop = have->n_drop;
    size_t nd[SA_N], kp[SA_N];
    stage_used(&w, nd);
    nd[SA_AUX] += sizeof(grom_aux);  // the -S patch
    stage_used(&h, kp);
    kp[SA_COFF] = h.n > 0 ? 4 * (size_t)h.n : 0;  // (the closing entry is written last)
    kp[SA_AUX] = 0;
    kp[SA_REF] = 0;
    int rc = stage_reserve(s, nd, kp, 32);
    if (rc) return rc;
    s->n = w.n;
    s->n_cig = w.n_cig;
    s->n_bases = w.n_bases;
    s->n_aux = 0;
    s->n_drop = w.n_drop;
    s->bytes_h2d = 0;
    stage_dev_view(s, dev);
    return GROM_OK;
}

int grom_stage_fill_set(grom_stage *s, const grom_stage_sizes *sz) {
    if (!s || !sz) { set_err("grom_stage_fill_set: null argument"); return GROM_E_ARG; }
    s->n = sz->n;
    s->n_cig = sz->n_cigar_ops;
    s->n_bases = sz->n_bases;
    s->n_aux = 0;
    s->n_drop = sz->n_drop;
    return GROM_OK;
}

int grom_stage_put_aux(grom_stage *s, const grom_aux *aux, const int64_t *kidx, int64_t n) {
    if (!s || n < 0 || (n > 0 && (!aux || !kidx))) { set_err("grom_stage_put_aux: bad argument"); return GROM_E_ARG; }
    if (n == 0) return GROM_OK;
    HIPCHK(hipSetDevice(s->device));
    size_t need[SA_N], keep[SA_N];
    stage_used(s, keep);
    stage_used(s, need);
    need[SA_AUX] = sizeof(grom_aux) * (size_t)(s->n_aux + n + 1);
    int rc = stage_reserve(s, need, keep);
    if (rc) return rc;
    int64_t *d_k = (int64_t *)stage_scratch(s, sizeof(int64_t) * (size_t)n);
    if (!d_k) { set_err("grom_stage_put_aux: no device scratch"); return GROM_E_NOMEM; }
    HIPCHK(hipMemcpyAsync(s->a(SA_AUX) + sizeof(grom_aux) * s->n_aux, aux, sizeof(grom_aux) * (size_t)n,
                          hipMemcpyHostToDevice, s->st));
    HIPCHK(hipMemcpyAsync(d_k, kidx, sizeof(int64_t) * (size_t)n, hipMemcpyHostToDevice, s->st));
    hipLaunchKernelGGL(k_stage_aux_idx, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256), 0, s->st,
                       (int32_t *)s->a(SA_AIDX), d_k, n, (int32_t)s->n_aux);
    HIPCHK(hipStreamSynchronize(s->st));
    s->n_aux += n;
    return GROM_OK;
}

int grom_stage_trim_drops(grom_stage *s, int64_t sd, int64_t sk) {
    if (!s || sd < 0 || sd > s->n_drop || sk < 0) { set_err("grom_stage_trim_drops: bad argument"); return GROM_E_ARG; }
    HIPCHK(hipSetDevice(s->device));
    const int64_t n = s->n_drop - sd;
    if (n > 0) {
        // through a scratch copy: the source and destination ranges overlap
        char *tmp = stage_scratch(s, 16 * (size_t)n);
        if (!tmp) { set_err("grom_stage_trim_drops: no device scratch"); return GROM_E_NOMEM; }
        int32_t *tp = (int32_t *)tmp, *tl = tp + n;
        int64_t *tb = (int64_t *)(tmp + 8 * (size_t)n);
        HIPCHK(hipMemcpyAsync(tp, (int32_t *)s->a(SA_DPOS) + sd, 4 * (size_t)n, hipMemcpyDeviceToDevice, s->st));
        HIPCHK(hipMemcpyAsync(tl, (int32_t *)s->a(SA_DLQ) + sd, 4 * (size_t)n, hipMemcpyDeviceToDevice, s->st));
        HIPCHK(hipMemcpyAsync(tb, (int64_t *)s->a(SA_DBEF) + sd, 8 * (size_t)n, hipMemcpyDeviceToDevice, s->st));
        hipLaunchKernelGGL(k_stage_trim_drops, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256), 0,
                           s->st, (int32_t *)s->a(SA_DPOS), (int32_t *)s->a(SA_DLQ), (int64_t *)s->a(SA_DBEF), tp, tl,
                           tb, n, sk);
        HIPCHK(hipStreamSynchronize(s->st));
    }
    s->n_drop = n;
    return GROM_OK;
}

int grom_copy_d2h(void *dst, const void *src, size_t n, int device) {
    if (hipSetDevice(device) != hipSuccess) return -1;
    return hipMemcpy(dst, src, n, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}

int grom_stage_dev_reads(grom_stage *s, grom_reads *dev) {
    if (!s || !dev) { set_err("grom_stage_dev_reads: null argument"); return GROM_E_ARG; }
    stage_dev_view(s, dev);
    return GROM_OK;
}

int grom_scan_chrom_staged(int slot, grom_stage *s, const grom_chrom *chrom, grom_out *out, grom_stats *stats) {
    Ctx *C = ctx_of(slot);
    if (!C) return GROM_E_NODEV;
    if (!s || !chrom || !out || !chrom->ref) { set_err("grom_scan_chrom_staged: null argument"); return GROM_E_ARG; }
    if (s->device != C->device) {
        set_err("grom_scan_chrom_staged: stage on device %d, context %d on device %d", s->device, slot, C->device);
        return GROM_E_ARG;
    }
    HIPCHK(hipSetDevice(C->device));
    grom_chrom dch;
    grom_reads dr;
    int rc = grom_stage_view(s, chrom, &dch, &dr);
    if (rc) return rc;
    // the scan's stream waits for every copy of the stage (device-side order)
    HIPCHK(hipEventRecord(s->all_ev, s->st));
    HIPCHK(hipStreamWaitEvent(C->st, s->all_ev, 0));
    C->host_ref = chrom->ref;
    struct Done {
        grom_stage *s;
        static void call(void *u) {
            grom_stage *s = ((Done *)u)->s;
            s->consumed(s->consumed_arg, s);
        }
    } done{s};
    rc = scan_device(*C, &dch, &dr, out, stats, nullptr, nullptr, 0, nullptr, s->consumed ? &Done::call : nullptr, &done);
    C->host_ref = nullptr;
    return rc;
}

int grom_debug_counts_staged(int slot, grom_stage *s, const grom_chrom *chrom, int32_t *first_pos, int32_t *counts,
                             int64_t counts_cap, int32_t *caf3) {
    Ctx *C = ctx_of(slot);
    if (!C) return GROM_E_NODEV;
    if (!s || !chrom || !chrom->ref) { set_err("grom_debug_counts_staged: null argument"); return GROM_E_ARG; }
    HIPCHK(hipSetDevice(C->device));
    grom_chrom dch;
    grom_reads dr;
    int rc = grom_stage_view(s, chrom, &dch, &dr);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(s->st));
    grom_out tmp{};
    C->host_ref = chrom->ref;
    rc = scan_device(*C, &dch, &dr, &tmp, nullptr, first_pos, counts, counts_cap, caf3);
    C->host_ref = nullptr;
    grom_out_free(&tmp);
    return rc;
}

int grom_debug_counts(int device, const grom_chrom *chrom, const grom_reads *reads, int32_t *first_pos,
                      int32_t *counts, int64_t counts_cap, int32_t *caf3) {
    Ctx *C = ctx_of(device);
    if (!C) return GROM_E_NODEV;
    HIPCHK(hipSetDevice(C->device));
    grom_chrom dch;
    grom_reads dr;
    int rc = upload(*C, chrom, reads, &dch, &dr);
    if (rc) return rc;
    grom_out tmp{};
    rc = scan_device(*C, &dch, &dr, &tmp, nullptr, first_pos, counts, counts_cap, caf3);
    grom_out_free(&tmp);
    return rc;
}

int64_t grom_debug_indels(int device, grom_indel_rec *out, int64_t cap) {
    Ctx *C = ctx_of(device);
    if (!C) return GROM_E_NODEV;
    if (!C->sv) return 0;
    const int64_t n = sv_indel_count(C->sv);
    const int64_t m = std::min<int64_t>(n, std::max<int64_t>(cap, 0));
    if (m > 0 && out) {
        HIPCHK(hipSetDevice(C->device));
        HIPCHK(hipMemcpy(out, sv_indel_records(C->sv), sizeof(grom_indel_rec) * (size_t)m, hipMemcpyDeviceToHost));
    }
    return n;
}

int64_t grom_debug_sv(int device, grom_sv_rec *out, int64_t cap) {
    Ctx *C = ctx_of(device);
    if (!C) return GROM_E_NODEV;
    if (!C->sv) return 0;
    const int64_t n = sv_debug_count(C->sv);
    const int64_t m = std::min<int64_t>(n, std::max<int64_t>(cap, 0));
    if (m > 0 && out) {
        HIPCHK(hipSetDevice(C->device));
        HIPCHK(hipMemcpy(out, sv_debug_records(C->sv), sizeof(grom_sv_rec) * (size_t)m, hipMemcpyDeviceToHost));
    }
    return n;
}

}  // extern "C"
