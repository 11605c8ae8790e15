// indel.hip -- CIGAR indel evidence (GROM.c:7187-7423) on
// MI355X.
//
// The reference folds every I/D op of every ingested read into per-base ring
// state as it reads the stream: the first length seen at a base becomes the
// primary (count, length) pair, equal lengths add to it, a different length
// goes to one of the base's 50 "other" slots, and a slot that overtakes the
// primary swaps with it.  That fold is order-dependent, so the GPU form keeps
// the stream order explicitly instead of replaying the ring:
//
//   k_indel_count  one lane per read: how many events its CIGAR emits inside
//                  the evaluated range (I: 1, D: 2 -- first and last base)
//   exclusive scan event slots in (read, op) order
//   k_indel_emit   one lane per read: position keys + compact event records
//   radix sort     stable on the 32-bit position, so events of one base stay
//                  in stream order (the order the ring sees them)
//   run-length     one run per base
//   k_indel_fold   one lane per base folds its events sequentially and writes
//                  one grom_indel_rec
//
// Indels are sparse (≈1e-4 per base per haplotype), so the pass moves a few MB
// per 100 Mb chromosome: it is launch- and latency-bound, never HBM-bound.
// Only indel-typed "other" slots exist here; the discordant-pair and
// split-read evidence types that share those slots in the reference (rows
// A8/A9) are not built yet.

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdio>
#include <cstring>

#include "indel.h"

namespace {

constexpr int OTHER_LEN = 50;  // g_other_len, GROM.c:837
constexpr int ISEQ_LEN = 50;   // g_indel_i_seq_len, GROM.c:904
constexpr int MAX_CIGAR = 1000;  // the reference copies at most 1000 ops, GROM.c:6740-6750
enum : uint8_t { OT_EMPTY = 0, OT_I = 11, OT_DF = 12, OT_DR = 13 };  // GROM.c:668-681

__constant__ char c_nt16_ind[16] = {'=', 'A', 'C', 'M', 'G', 'R', 'S', 'V', 'T', 'W', 'Y', 'H', 'K', 'D', 'B', 'N'};

struct IndelEvent {
    int64_t seq_nib;  // nibble offset of the inserted bases (I only)
    int32_t len;      // op length
    int32_t lq_left;  // read bases left from seq_nib (I only)
    uint8_t type;     // OT_I / OT_DF / OT_DR
    uint8_t add;      // 6 or 0 (cdp_add, GROM.c:5829-5836)
    uint8_t pad[6];
};

struct ReadView {
    const int32_t *pos;
    const uint8_t *mapq;
    const uint8_t *keep;
    const uint32_t *cig_off;
    const uint32_t *cigar;
    const int64_t *base_off;
    const int32_t *lqseq;
};

// walk one read's CIGAR as the reference does (GROM.c:7187-7420) and hand
// every in-range event to f(position, type, len, seq_base_index)
template <class F>
__device__ __forceinline__ void walk_indels(const ReadView &R, int64_t i, int32_t lo, int32_t hi, F &&f) {
    if (R.keep && R.keep[i] == 0) return;
    const uint32_t cb = R.cig_off[i];
    uint32_t ce = R.cig_off[i + 1];
    if (ce - cb > (uint32_t)MAX_CIGAR) ce = cb + MAX_CIGAR;
    int64_t tp = R.pos[i];
    int32_t sb = 0;
    for (uint32_t k = cb; k < ce; k++) {
        const uint32_t cw = R.cigar[k];
        const int op = cw & 15;
        const int32_t len = (int32_t)(cw >> 4);
        if (op == 4) {  // S
            sb += len;
        } else if (op == 0 || op == 3 || op == 7 || op == 8) {  // M N = X
            tp += len;
            if (op != 3) sb += len;
        } else if (op == 1) {  // I
            if (tp >= lo && tp <= hi) f((int32_t)tp, OT_I, len, sb);
            sb += len;
        } else if (op == 2) {  // D
            if (tp >= lo && tp <= hi) f((int32_t)tp, OT_DF, len, 0);
            const int64_t te = tp + len - 1;
            if (te >= lo && te <= hi) f((int32_t)te, OT_DR, len, 0);
            tp += len;
        }
    }
}

__global__ void k_indel_count(int64_t n, ReadView R, int32_t lo, int32_t hi, uint32_t *__restrict__ cnt) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t c = 0;
        walk_indels(R, i, lo, hi, [&](int32_t, uint8_t, int32_t, int32_t) { c++; });
        cnt[i] = c;
    }
}

__global__ void k_indel_emit(int64_t n, ReadView R, int32_t lo, int32_t hi, int32_t min_mapq,
                             const uint32_t *__restrict__ off, uint32_t *__restrict__ keys,
                             uint32_t *__restrict__ vals, IndelEvent *__restrict__ ev) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t o = off[i];
        const uint8_t add = (int32_t)R.mapq[i] >= min_mapq ? 6 : 0;
        const int64_t bo = R.base_off[i];
        const int32_t lq = R.lqseq[i];
        walk_indels(R, i, lo, hi, [&](int32_t p, uint8_t type, int32_t len, int32_t sb) {
            IndelEvent e;
            e.seq_nib = bo + sb;
            e.len = len;
            e.lq_left = lq - sb;
            e.type = type;
            e.add = add;
            ev[o] = e;
            keys[o] = (uint32_t)p;
            vals[o] = o;
            o++;
        });
    }
}

// One lane per base: the reference's fold (GROM.c:7209-7283 insertion,
// 7289-7352 forward end, 7356-7420 reverse end) over the base's events in
// stream order.  The 50 "other" slots live in scratch; bases with any event
// are rare, so this kernel is small.
__global__ void k_indel_fold(uint32_t n_runs, const uint32_t *__restrict__ run_pos,
                             const uint32_t *__restrict__ run_len, const uint32_t *__restrict__ run_off,
                             const uint32_t *__restrict__ order, const IndelEvent *__restrict__ ev,
                             const uint8_t *__restrict__ seq, grom_indel_rec *__restrict__ out) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_runs) return;
    grom_indel_rec rec;
    memset(&rec, 0, sizeof(rec));
    rec.pos = (int32_t)run_pos[r];
    uint8_t ot_type[OTHER_LEN];
    int32_t ot_cnt[OTHER_LEN];
    int32_t ot_len[OTHER_LEN];  // the reference keeps a double; every indel length is an exact integer
    for (int o = 0; o < OTHER_LEN; o++) { ot_type[o] = OT_EMPTY; ot_cnt[o] = 0; ot_len[o] = 0; }
    const uint32_t b = run_off[r], e = b + run_len[r];
    for (uint32_t j = b; j < e; j++) {
        const IndelEvent E = ev[order[j]];
        const int32_t add = E.add;
        int32_t *cnt, *dist;
        if (E.type == OT_I) { cnt = &rec.ins; dist = &rec.ins_len; }
        else if (E.type == OT_DF) { cnt = &rec.del_f; dist = &rec.del_f_len; rec.del_f_rd += 1; }
        else { cnt = &rec.del_r; dist = &rec.del_r_len; rec.del_r_rd += 1; }
        if (*cnt == 0) {
            *cnt = add;
            *dist = E.len;
            if (E.type == OT_I && E.len <= ISEQ_LEN) {
                for (int q = 0; q < E.len; q++) {
                    const int64_t nb = E.seq_nib + q;
                    const uint8_t byte = seq[nb >> 1];
                    rec.ins_seq[q] = q < E.lq_left ? c_nt16_ind[(nb & 1) ? (byte & 15) : (byte >> 4)] : 0;
                }
            }
        } else if ((uint32_t)E.len == (uint32_t)*dist) {
            *cnt += add;
        } else {
            bool found = false;
            for (int o = 0; o < OTHER_LEN; o++) {
                if (ot_type[o] == E.type) {
                    if (E.len == ot_len[o]) {
                        found = true;
                        ot_cnt[o] += add;
                        if (ot_cnt[o] > *cnt) {  // the slot overtakes the primary: swap
                            const int32_t tc = ot_cnt[o], tl = ot_len[o];
                            ot_cnt[o] = *cnt;
                            ot_len[o] = *dist;
                            *cnt = tc;
                            *dist = tl;
                        }
                        break;
                    }
                } else if (ot_type[o] == OT_EMPTY) {
                    found = true;
                    ot_cnt[o] = add;
                    ot_type[o] = E.type;
                    ot_len[o] = E.len;
                    break;
                }
            }
            if (!found) {
                for (int o = 0; o < OTHER_LEN; o++) {
                    if (ot_cnt[o] <= add) {
                        ot_cnt[o] = add;
                        ot_type[o] = E.type;
                        ot_len[o] = E.len;
                        break;
                    }
                }
            }
        }
    }
    rec.other_len = OTHER_LEN;  // GROM.c:11415-11425: index of the first empty slot
    for (int o = 0; o < OTHER_LEN; o++)
        if (ot_type[o] == OT_EMPTY) { rec.other_len = o; break; }
    out[r] = rec;
}

struct Buf {
    void *p = nullptr;
    size_t cap = 0;
};

}  // namespace

struct IndelScratch {
    Buf cnt, off, keys, vals, keys2, vals2, ev, run_pos, run_len, run_off, n_runs, tmp, rec;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int64_t n_rec = 0;
};

static int ibuf(Buf &b, size_t bytes, char *err, size_t errlen) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return GROM_OK;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    const size_t want = bytes + bytes / 8 + 64;
    if (hipMalloc(&b.p, want) != hipSuccess) {
        snprintf(err, errlen, "indel pass: hipMalloc(%zu) failed", want);
        return GROM_E_NOMEM;
    }
    b.cap = want;
    return GROM_OK;
}

IndelScratch *indel_scratch_new() { return new IndelScratch(); }

void indel_scratch_free(IndelScratch *s) {
    if (!s) return;
    Buf *all[] = {&s->cnt, &s->off, &s->keys, &s->vals, &s->keys2, &s->vals2, &s->ev,
                  &s->run_pos, &s->run_len, &s->run_off, &s->n_runs, &s->tmp, &s->rec};
    for (Buf *b : all)
        if (b->p) (void)hipFree(b->p);
    if (s->e0) (void)hipEventDestroy(s->e0);
    if (s->e1) (void)hipEventDestroy(s->e1);
    delete s;
}

const grom_indel_rec *indel_records(const IndelScratch *S) { return (const grom_indel_rec *)S->rec.p; }
int64_t indel_count(const IndelScratch *S) { return S->n_rec; }

#define ICHK(x)                                                                      \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            snprintf(err, errlen, "indel pass: %s: %s", #x, hipGetErrorString(e_)); \
            return GROM_E_HIP;                                                       \
        }                                                                            \
    } while (0)

int indel_chrom(IndelScratch *S, hipStream_t st, int64_t n, const int32_t *pos, const uint8_t *mapq,
                const uint8_t *keep, const uint32_t *cig_off, const uint32_t *cigar, const int64_t *base_off,
                const int32_t *lqseq, const uint8_t *seq, int32_t min_mapq, int32_t lo, int32_t hi,
                int64_t *n_out, double *ms_device, char *err, size_t errlen) {
    int rc;
    S->n_rec = 0;
    *n_out = 0;
    if (ms_device) *ms_device = 0;
    if (n <= 0 || hi < lo) return GROM_OK;
    if (n >= (int64_t)UINT32_MAX) {
        snprintf(err, errlen, "indel pass: %lld reads exceed the 32-bit event index", (long long)n);
        return GROM_E_ARG;
    }
    if (!S->e0) {
        ICHK(hipEventCreate(&S->e0));
        ICHK(hipEventCreate(&S->e1));
    }
    ICHK(hipEventRecord(S->e0, st));
    const ReadView R{pos, mapq, keep, cig_off, cigar, base_off, lqseq};
    const int g = (int)std::min<int64_t>((n + 255) / 256, 8192);
    if ((rc = ibuf(S->cnt, sizeof(uint32_t) * (n + 1), err, errlen)) ||
        (rc = ibuf(S->off, sizeof(uint32_t) * (n + 1), err, errlen)))
        return rc;
    uint32_t *cnt = (uint32_t *)S->cnt.p, *off = (uint32_t *)S->off.p;
    ICHK(hipMemsetAsync(cnt + n, 0, sizeof(uint32_t), st));
    hipLaunchKernelGGL(k_indel_count, dim3(g), dim3(256), 0, st, n, R, lo, hi, cnt);
    ICHK(hipGetLastError());
    // exclusive scan over n+1 entries: off[n] is the event total
    size_t tmp_bytes = 0;
    ICHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, cnt, off, (int)(n + 1), st));
    if ((rc = ibuf(S->tmp, tmp_bytes, err, errlen))) return rc;
    ICHK(hipcub::DeviceScan::ExclusiveSum(S->tmp.p, tmp_bytes, cnt, off, (int)(n + 1), st));
    uint32_t n_ev = 0;
    ICHK(hipMemcpyAsync(&n_ev, off + n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    ICHK(hipStreamSynchronize(st));
    if (n_ev == 0) return GROM_OK;
    if ((rc = ibuf(S->keys, sizeof(uint32_t) * n_ev, err, errlen)) ||
        (rc = ibuf(S->vals, sizeof(uint32_t) * n_ev, err, errlen)) ||
        (rc = ibuf(S->keys2, sizeof(uint32_t) * n_ev, err, errlen)) ||
        (rc = ibuf(S->vals2, sizeof(uint32_t) * n_ev, err, errlen)) ||
        (rc = ibuf(S->ev, sizeof(IndelEvent) * n_ev, err, errlen)) ||
        (rc = ibuf(S->run_pos, sizeof(uint32_t) * n_ev, err, errlen)) ||
        (rc = ibuf(S->run_len, sizeof(uint32_t) * n_ev, err, errlen)) ||
        (rc = ibuf(S->run_off, sizeof(uint32_t) * n_ev, err, errlen)) ||
        (rc = ibuf(S->n_runs, sizeof(uint32_t) * 2, err, errlen)))
        return rc;
    uint32_t *keys = (uint32_t *)S->keys.p, *vals = (uint32_t *)S->vals.p;
    uint32_t *keys2 = (uint32_t *)S->keys2.p, *vals2 = (uint32_t *)S->vals2.p;
    hipLaunchKernelGGL(k_indel_emit, dim3(g), dim3(256), 0, st, n, R, lo, hi, min_mapq, off, keys, vals,
                       (IndelEvent *)S->ev.p);
    ICHK(hipGetLastError());
    // stable LSD radix sort on the position: equal positions keep stream order
    size_t t_sort = 0, t_rle = 0, t_scan = 0;
    ICHK(hipcub::DeviceRadixSort::SortPairs(nullptr, t_sort, keys, keys2, vals, vals2, (int)n_ev, 0, 32, st));
    ICHK(hipcub::DeviceRunLengthEncode::Encode(nullptr, t_rle, keys2, (uint32_t *)S->run_pos.p,
                                               (uint32_t *)S->run_len.p, (uint32_t *)S->n_runs.p, (int)n_ev, st));
    ICHK(hipcub::DeviceScan::ExclusiveSum(nullptr, t_scan, (uint32_t *)S->run_len.p, (uint32_t *)S->run_off.p,
                                          (int)n_ev, st));
    if ((rc = ibuf(S->tmp, std::max(t_sort, std::max(t_rle, t_scan)), err, errlen))) return rc;
    ICHK(hipcub::DeviceRadixSort::SortPairs(S->tmp.p, t_sort, keys, keys2, vals, vals2, (int)n_ev, 0, 32, st));
    ICHK(hipcub::DeviceRunLengthEncode::Encode(S->tmp.p, t_rle, keys2, (uint32_t *)S->run_pos.p,
                                               (uint32_t *)S->run_len.p, (uint32_t *)S->n_runs.p, (int)n_ev, st));
    uint32_t n_runs = 0;
    ICHK(hipMemcpyAsync(&n_runs, S->n_runs.p, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    ICHK(hipStreamSynchronize(st));
    if (n_runs == 0 || n_runs > n_ev) {
        snprintf(err, errlen, "indel pass: %u position runs for %u events", n_runs, n_ev);
        return GROM_E_HIP;
    }
    ICHK(hipcub::DeviceScan::ExclusiveSum(S->tmp.p, t_scan, (uint32_t *)S->run_len.p, (uint32_t *)S->run_off.p,
                                          (int)n_runs, st));
    if ((rc = ibuf(S->rec, sizeof(grom_indel_rec) * n_runs, err, errlen))) return rc;
    hipLaunchKernelGGL(k_indel_fold, dim3((n_runs + 63) / 64), dim3(64), 0, st, n_runs,
                       (const uint32_t *)S->run_pos.p, (const uint32_t *)S->run_len.p,
                       (const uint32_t *)S->run_off.p, (const uint32_t *)vals2, (const IndelEvent *)S->ev.p, seq,
                       (grom_indel_rec *)S->rec.p);
    ICHK(hipGetLastError());
    ICHK(hipEventRecord(S->e1, st));
    ICHK(hipEventSynchronize(S->e1));
    float ms = 0;
    ICHK(hipEventElapsedTime(&ms, S->e0, S->e1));
    if (ms_device) *ms_device = ms;
    S->n_rec = n_runs;
    *n_out = n_runs;
    return GROM_OK;
}
