// k_scan_scatter.h -- the pileup tile kernel in scatter form (included by
// scan.hip after k_scan_tile.h, whose LaneCounts / pile_emit it shares).
//
// A workgroup owns TG consecutive reference positions.  Its waves take the
// tile's reads round-robin; a read's fields are wave-uniform, and the lanes
// take 64 of its aligned bases at a time, so each base is loaded once,
// coalesced, and no lane idles on a read that does not cover it.
//
// What a read adds to the per-position counters is split three ways, so that
// the common base costs one LDS atomic:
//   - intervals, as +v/-v at the two ends of difference arrays (prefix-summed
//     once per tile): the caf_* read depth of each M/=/X block
//     (GROM.c:6605-6671), the physical read depth [pos, E) (GROM.c:7173-7181),
//     and -- for a read with MAPQ >= -q -- what each tallied base would add if
//     it matched the reference with base quality >= -b: the base count and
//     forward count, the MAPQ sum, and the position-in-read sum, which is
//     linear in the position: sum(x - e) = n*x - sum(e) on the forward strand,
//     sum(lsm + e - x) on the reverse (e = position of read offset 0);
//   - per base, only the base-quality sum of such matching bases (ds_add_u32);
//   - every other base of such a read (low base quality, a mismatch, a
//     reference base outside ACGT) is an exception event: the fold removes the
//     interval's assumed contribution and applies the base's real tally,
//     including the order-dependent read-name de-duplication of mismatches
//     (GROM.c:6805-6824).  Bases of reads with MAPQ < -q add to three
//     low-quality counters, or are events when they mismatch.  Soft-clip
//     evidence (GROM.c:7105-7169) is an event too.
// After the reads, the events are bucketed by position (counting sort), each
// lane sorts its bucket by read index -- the reference's ring order -- and
// folds it; pile_emit writes the outputs.  Every sum is an int32 counter in
// the reference and is kept modulo 2^32 here, so the identities are exact.
// A tile whose events exceed the LDS budget writes nothing and is listed for
// the gather kernel (k_scan_tile_list).

#define SEVCAP GROM_EVENT_CAP
#define SNW (TG / 64)

// event word w: position in tile (bits 0-10) | type << 11 | code << 13 |
// fwd << 16 | base quality << 17 | assumed << 25 | matches reference << 26;
// z: offset in read (EV_X, EV_LQ) or clip mask; evx: mapq | lsm << 8
#define EV_X 0     // a base of a MAPQ >= -q read that is not a plain match
#define EV_LQ 1    // a mismatching ACGT base of a MAPQ < -q read
#define EV_CLIP 2  // soft-clip evidence: z = category mask | MAPQ >= -q << 6

// difference arrays
enum { D_CMQ, D_CRD, D_CLOW, D_RD, D_NF, D_NR, D_MQ, D_SF, D_SR, NDIF };
#define NSCAN (NDIF + 1)

struct __align__(16) ScatLds {
    int32_t dif[NDIF][TG + 1];
    uint32_t bqh[TG];                     // base-quality sum of plain matches
    uint32_t lcnt[TG], bql[TG], mql[TG];  // MAPQ < -q reads' matches: count, base quality, mapq
    uint4 ev[SEVCAP];                     // x: read index, y: name id, z, w: see above
    uint32_t evx[SEVCAP];
    uint32_t evn[TG];                     // events per position, then bucket cursors
    uint16_t sidx[SEVCAP];                // event indices bucketed by position
    uint8_t rinfo[TG];                    // reference base: 4-bit code (16: none) | ACGT index << 5
    uint32_t nev;
    int32_t scan[SNW][NSCAN];
    TileTail tail;
};

__device__ __forceinline__ int32_t tile_index(int64_t p, int32_t t0) {
    const int64_t d = p - t0;
    return (int32_t)(d < 0 ? 0 : (d > TG ? TG : d));
}

__device__ __forceinline__ void scat_event(ScatLds &L, uint32_t evcap, uint32_t r, uint32_t nid, uint32_t z,
                                           uint32_t w, uint32_t x) {
    const uint32_t k = atomicAdd(&L.nev, 1u);
    if (k < evcap) {
        L.ev[k] = make_uint4(r, nid, z, w);
        L.evx[k] = x;
        atomicAdd(&L.evn[w & 2047u], 1u);
    }
}

// the uniform fields of one read that the tally needs
struct ReadU {
    int64_t bo;
    int32_t p0, lq, r;
    uint32_t nid, mq;
    bool fwd, hq_read;
};

// one base: read offset qi lands on tile position i; q, s4 the base (s4 = 15,
// q = 0 past the read's sequence), ri the reference info, lsm the length
// with hard clips at this block (GROM.c:6769-7059; tally_base in
// k_scan_tile.h is the same tally in register form)
__device__ __forceinline__ void tally_one(ScatLds &L, const grom_scan_args &a, uint32_t evcap, const ReadU &u, int i,
                                          int32_t qi, int32_t lsm, uint32_t q, uint32_t s4, uint32_t ri) {
    const uint32_t rcode = ri >> 5;
    const bool mv = rcode < 4, match = s4 == (ri & 31u);
    const uint32_t code = (uint32_t)acgt_code((int)s4);
    const uint32_t w = (uint32_t)i | (code << 13) | ((u.fwd ? 1u : 0u) << 16) | (q << 17) | ((mv ? 1u : 0u) << 25) |
                       ((match ? 1u : 0u) << 26);
    if (u.hq_read) {
        if (mv && match && (int)q >= a.min_base_qual)
            atomicAdd(&L.bqh[i], q);
        else if (mv || !match)
            scat_event(L, evcap, (uint32_t)u.r, u.nid, (uint32_t)qi, w | (EV_X << 11), u.mq | ((uint32_t)lsm << 8));
    } else if (match) {
        if (mv) {
            atomicAdd(&L.lcnt[i], 1u);
            atomicAdd(&L.bql[i], q);
            atomicAdd(&L.mql[i], u.mq);
        }
    } else if (code < 4) {
        scat_event(L, evcap, (uint32_t)u.r, u.nid, (uint32_t)qi, w | (EV_LQ << 11), u.mq);
    }
}

// interval ends, one per lane: lanes 0-3 a caf block [cs, ce) (if caf_ok),
// 4-5 the physical depth [rs, re) (if rd_ok), 6-11 the assumed tally of the
// bases on [ps, pe) with read offset 0 at position e (if tal_ok)
__device__ __forceinline__ void interval_ends(ScatLds &L, const ReadU &u, const grom_scan_args &a, int32_t t0,
                                              bool caf_ok, int64_t cs, int64_t ce, bool rd_ok, int64_t rs, int64_t re,
                                              bool tal_ok, int64_t ps, int64_t pe, int64_t e, int32_t lsm) {
    const int lane = threadIdx.x & 63;
    const bool end = lane & 1;
    int k = 0;
    int64_t at = 0;
    int32_t v = 0;
    bool on = false;
    if (lane < 4) {
        on = caf_ok;
        k = (lane < 2) ? D_CMQ : (((int)u.mq >= a.rd_min_mapq) ? D_CRD : D_CLOW);
        v = (lane < 2) ? (int32_t)u.mq : 1;
        at = end ? ce : cs;
    } else if (lane < 6) {
        on = rd_ok;
        k = D_RD;
        v = 1;
        at = end ? re : rs;
    } else if (lane < 12) {
        on = tal_ok && u.hq_read;
        const int f = (lane - 6) >> 1;  // 0 count, 1 mapq, 2 position sum
        k = (f == 0) ? (u.fwd ? D_NF : D_NR) : (f == 1) ? D_MQ : (u.fwd ? D_SF : D_SR);
        v = (f == 0) ? 1 : (f == 1) ? (int32_t)u.mq : (int32_t)(uint32_t)(u.fwd ? (e - t0) : (lsm + e - t0));
        at = end ? pe : ps;
    }
    if (on) atomicAdd(&L.dif[k][tile_index(at, t0)], end ? -v : v);
}

// lanes take read offsets [o_lo, o_hi) of one aligned block starting at
// position xb, read offset qb; all bounds are wave-uniform
__device__ __forceinline__ void scat_block(ScatLds &L, const grom_scan_args &a, const ReadArrays &R, uint32_t evcap,
                                           const ReadU &u, int32_t t0, int64_t xb, int32_t qb, int32_t o_lo,
                                           int32_t o_hi, int32_t lsm) {
    const int lane = threadIdx.x & 63;
    for (int32_t ob = o_lo; ob < o_hi; ob += 64) {
        const int32_t o = ob + lane;
        if (o < o_hi) {
            const int32_t qi = qb + o;
            uint32_t q = 0, s4 = 15;
            if (qi < u.lq) {
                const int64_t b = u.bo + qi;
                q = R.qual[b];
                const uint32_t sb = R.seq[b >> 1];
                s4 = (b & 1) ? (sb & 15u) : (sb >> 4);
            }
            const int i = (int)(xb + o - t0);
            tally_one(L, a, evcap, u, i, qi, lsm, q, s4, L.rinfo[i]);
        }
    }
}

// a read with any other CIGAR: the walk of GROM.c:6605-7181 restated as in
// the gather kernel, wave-uniform, with the lanes taking each aligned block
__device__ __forceinline__ void scat_general(ScatLds &L, const grom_scan_args &a, const ReadArrays &R,
                                             const ReadMeta *__restrict__ meta, uint32_t evcap, int32_t r, int32_t t0,
                                             int32_t lo_x, int32_t hi_x) {
    const int lane = threadIdx.x & 63;
    const int32_t clen = (int32_t)a.chr_len;
    const ReadMeta m = meta[r];
    ReadU u;
    u.r = r;
    u.p0 = (int32_t)m.a.x;
    u.lq = (int32_t)m.a.z;
    u.nid = m.a.w;
    u.mq = m.b.z & 255u;
    u.bo = ((int64_t)m.c.x << 32) | m.b.w;
    const uint32_t cb = m.b.x, ncig = m.b.y & 0xffffu, fl = m.b.y >> 16;
    u.fwd = !(fl & 0x10);
    u.hq_read = (int)u.mq >= a.min_mapq;
    const int32_t p0 = u.p0, lq = u.lq;
    const bool pos_ok = p0 >= 0 && p0 < clen;
    const uint32_t ce = cb + ncig;
    int32_t snv_base = 0, srb = 0, lseq_mod = lq, eai = 0;
    int64_t caf_pos = p0;
    int first_op = -1, first_len = 0, last_op = -1, last_len = 0;
    const uint32_t ncap = (ce - cb > 1000u) ? cb + 1000u : ce;  // GROM.c:6743
    for (uint32_t k = cb; k < ce; k++) {
        const uint32_t cg = R.cigar[k];
        const int op = cg & 15;
        const int32_t len = (int32_t)(cg >> 4);
        const bool in_cap = k < ncap;
        if (op == 0 || op == 7 || op == 8) {
            const bool caf_ok = caf_pos >= 0 && caf_pos + len < clen;
            bool tal_ok = false;
            int64_t xb = 0, lo = 0, hi = 0;
            int32_t loop_end = 0;
            if (in_cap && pos_ok) {
                xb = (int64_t)p0 + srb;
                loop_end = (xb + len >= clen) ? (clen - p0) : len;
                lo = max((int64_t)0, (int64_t)lo_x - xb);
                hi = min((int64_t)loop_end, (int64_t)hi_x + 1 - xb);
                tal_ok = lo < hi;
            }
            interval_ends(L, u, a, t0, caf_ok, caf_pos, caf_pos + len, false, 0, 0, tal_ok, xb + lo, xb + hi,
                          xb - snv_base, lseq_mod);
            if (tal_ok) scat_block(L, a, R, evcap, u, t0, xb, snv_base, (int32_t)lo, (int32_t)hi, lseq_mod);
            caf_pos += len;
            if (!in_cap) continue;
            if (pos_ok) {
                snv_base += loop_end;
                srb += loop_end;
            }
        } else if (op == 2) {
            caf_pos += len;
            if (!in_cap) continue;
            srb += len;
            eai -= len;
        } else if (in_cap) {
            if (op == 4) snv_base += len;
            else if (op == 5) lseq_mod += len;
            else if (op == 1) { snv_base += len; eai += len; }
            else if (op == 3) srb += len;
        } else {
            continue;
        }
        if (first_op < 0) { first_op = op; first_len = len; }
        last_op = op;
        last_len = len;
    }
    // clip lengths and the aligned end E, GROM.c:7067-7100
    const int start_adj = (first_op == 4 || first_op == 5) ? first_len : 0;
    const int end_adj = (last_op == 4 || last_op == 5) ? last_len : 0;
    const int64_t E = (int64_t)p0 - start_adj + lseq_mod - end_adj - eai;
    interval_ends(L, u, a, t0, false, 0, 0, E > p0, p0, E, false, 0, 0, 0, 0);
    // soft-clip evidence at pos-1 and E, GROM.c:7105-7169
    const bool at_l = start_adj >= a.sc_min && (int64_t)p0 - 1 >= lo_x && (int64_t)p0 - 1 <= hi_x;
    const bool at_r = end_adj >= a.sc_min && E >= lo_x && E <= hi_x;
    if ((at_l || at_r) && lane < 2) {
        const bool paired = fl & 0x1, munmap = fl & 0x8, rev = fl & 0x10;
        const bool same_chr = (int32_t)m.c.y == a.chr_tid;
        const int32_t mp = (int32_t)m.c.z, tl = (int32_t)m.c.w;
        uint32_t mask = 0;
        int32_t at = -1;
        if (lane == 0 && at_l) {
            if (!paired || (!rev && (munmap || (!munmap && same_chr && mp > p0)))) mask |= 1u;
            if (paired && !munmap && !same_chr && rev) mask |= 4u;
            if (paired && !munmap && same_chr && rev && abs(tl) <= a.insert_max && mp < p0) mask |= 16u;
            at = p0 - 1;
        }
        if (lane == 1 && at_r) {
            if (!paired || (rev && (munmap || (!munmap && same_chr && mp < p0)))) mask |= 2u;
            if (paired && !munmap && !same_chr && !rev) mask |= 8u;
            if (paired && !munmap && same_chr && !rev && abs(tl) <= a.insert_max && mp > p0) mask |= 32u;
            at = (int32_t)E;
        }
        if (mask)
            scat_event(L, evcap, (uint32_t)r, u.nid, mask | ((u.hq_read ? 1u : 0u) << 6),
                       (uint32_t)(at - t0) | (EV_CLIP << 11), u.mq);
    }
}

// ---- single-op reads, with the next read's bases loaded ahead ----
struct FastRead {
    ReadU u;
    int32_t len, o_lo, o_hi;
};
#define NCH 3  // 64-base chunks loaded ahead (reads up to 192 bases)
struct FastLoads {
    uint32_t q[NCH], s[NCH], ri[NCH];
};

__device__ __forceinline__ FastRead fast_view(const grom_scan_args &a, int32_t rb, int j, int32_t lo_x, int32_t hi_x,
                                              uint32_t vp0, uint32_t vlq, uint32_t vnid, uint32_t vnf, uint32_t vmk,
                                              uint32_t vbl, uint32_t vbh, uint32_t vcw) {
    FastRead f;
    f.u.r = rb + j * SNW;
    f.u.p0 = (int32_t)lane_get(vp0, j);
    f.u.lq = (int32_t)lane_get(vlq, j);
    f.u.nid = lane_get(vnid, j);
    const uint32_t fl = lane_get(vnf, j) >> 16;
    f.u.mq = lane_get(vmk, j) & 255u;
    f.u.bo = ((int64_t)lane_get(vbh, j) << 32) | lane_get(vbl, j);
    f.len = (int32_t)(lane_get(vcw, j) >> 4);
    f.u.fwd = !(fl & 0x10);
    f.u.hq_read = (int)f.u.mq >= a.min_mapq;
    const int32_t clen = (int32_t)a.chr_len;
    const bool pos_ok = f.u.p0 >= 0 && f.u.p0 < clen;
    f.o_lo = max(0, lo_x - f.u.p0);
    f.o_hi = pos_ok ? min(min(f.len, clen - f.u.p0), hi_x + 1 - f.u.p0) : 0;
    return f;
}

__device__ __forceinline__ void fast_issue(const ScatLds &L, const ReadArrays &R, const FastRead &f, int32_t t0,
                                           FastLoads &ld) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        ld.q[c] = 0;
        ld.s[c] = 0;
        ld.ri[c] = 0;
        if (f.o_lo + c * 64 < f.o_hi) {  // wave-uniform
            const int32_t o = f.o_lo + c * 64 + lane;
            const bool v = o < f.o_hi && o < f.u.lq;
            const int64_t b = f.u.bo + o;
            if (v) {
                ld.q[c] = R.qual[b];
                ld.s[c] = R.seq[b >> 1];
            }
            if (o < f.o_hi) ld.ri[c] = L.rinfo[f.u.p0 + o - t0];
        }
    }
}

__device__ __forceinline__ void fast_tally(ScatLds &L, const grom_scan_args &a, const ReadArrays &R, uint32_t evcap,
                                           const FastRead &f, const FastLoads &ld, int32_t t0) {
    const int lane = threadIdx.x & 63;
    const int32_t clen = (int32_t)a.chr_len;
    const int64_t p0 = f.u.p0;
    // the caf block is kept only if it ends before the chromosome end
    // (GROM.c:6625); physical depth [pos, pos + l_qseq)
    interval_ends(L, f.u, a, t0, f.u.p0 >= 0 && f.len < clen - f.u.p0, p0, p0 + f.len, true, p0, p0 + f.u.lq,
                  f.o_lo < f.o_hi, p0 + f.o_lo, p0 + f.o_hi, p0, f.u.lq);
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        const int32_t o = f.o_lo + c * 64 + lane;
        if (o < f.o_hi) {
            const int64_t b = f.u.bo + o;
            const uint32_t s4 = (o < f.u.lq) ? ((b & 1) ? (ld.s[c] & 15u) : (ld.s[c] >> 4)) : 15u;
            tally_one(L, a, evcap, f.u, (int)(p0 + o - t0), o, f.u.lq, ld.q[c], s4, ld.ri[c]);
        }
    }
    if (f.o_lo + NCH * 64 < f.o_hi)  // longer reads: the rest without lookahead
        scat_block(L, a, R, evcap, f.u, t0, p0, 0, f.o_lo + NCH * 64, f.o_hi, f.u.lq);
}

// inclusive scan of NSCAN int32 over the workgroup (lane = position); the
// last one is returned exclusive
__device__ __forceinline__ void scat_scan(ScatLds &L, int32_t (&v)[NSCAN]) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int32_t el = v[NSCAN - 1];
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
#pragma unroll
        for (int k = 0; k < NSCAN; k++) {
            const int32_t t = __shfl_up(v[k], d, 64);
            if (lane >= d) v[k] += t;
        }
    }
    if (lane == 63) {
#pragma unroll
        for (int k = 0; k < NSCAN; k++) L.scan[wave][k] = v[k];
    }
    __syncthreads();
    for (int w = 0; w < wave; w++) {
#pragma unroll
        for (int k = 0; k < NSCAN; k++) v[k] += L.scan[w][k];
    }
    v[NSCAN - 1] -= el;
}

#ifndef GROM_SCAT_WAVES_PER_EU
#define GROM_SCAT_WAVES_PER_EU 4
#endif

__global__ __launch_bounds__(TG) __attribute__((amdgpu_waves_per_eu(GROM_SCAT_WAVES_PER_EU))) void k_scan_scatter(
    grom_scan_args a, const char *__restrict__ ref, ReadArrays R, const ReadMeta *__restrict__ meta,
    const int32_t *__restrict__ tile_lo, const int32_t *__restrict__ tile_hi, PileOut O,
    const double *__restrict__ mq_tab, const double *__restrict__ hez_tab, int64_t n_tiles, uint32_t evcap,
    uint32_t *__restrict__ ovf_list, uint32_t *__restrict__ n_ovf) {
    __shared__ ScatLds L;
    const int64_t per_xcd = (n_tiles + 7) / 8;
    const int64_t tile = (int64_t)(blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
    if (tile >= n_tiles) return;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int32_t clen = (int32_t)a.chr_len;
    const int32_t t0 = (int32_t)(tile * TG);
    const int32_t x = t0 + tid;
    const int32_t r0 = tile_lo[tile], r1 = tile_hi[tile];

    const char rb = (x < clen) ? upcase(ref[x]) : 'N';
    int rb4 = 16;
    for (int k = 0; k < 16; k++) rb4 = (c_nt16[k] == rb) ? k : rb4;
    const int rcode = (rb4 < 16) ? acgt_code(rb4) : 4;
    L.rinfo[tid] = (uint8_t)(rb4 | (rcode << 5));
#pragma unroll
    for (int k = 0; k < NDIF; k++) L.dif[k][tid] = 0;
    L.bqh[tid] = 0;
    L.lcnt[tid] = 0;
    L.bql[tid] = 0;
    L.mql[tid] = 0;
    L.evn[tid] = 0;
    if (tid == 0) L.nev = 0;
    __syncthreads();

    // evaluated positions of this tile (GROM.c:11086, 5842)
    const int32_t lo_x = max(t0, a.eval_lo), hi_x = min(t0 + TG - 1, a.eval_hi);
    const int32_t t1 = t0 + TG;

#ifndef GROM_SCAT_PROF
#define GROM_SCAT_PROF 0  // profiling variants only: 1 skips the reads, 2 their tally
#endif
    for (int32_t rb0 = r0 + wave; rb0 < r1 && GROM_SCAT_PROF != 1; rb0 += 64 * SNW) {
        // ---- lane j holds read rb0 + j*SNW: its record and first CIGAR word ----
        const int32_t rj = rb0 + lane * SNW;
        uint32_t vp0 = 0, vlq = 0, vnid = 0, vnf = 0, vmk = 0, vbl = 0, vbh = 0, vcw = 0;
        bool rel = false, fast = false;
        if (rj < r1) {
            const ReadMeta m = meta[rj];
            vp0 = m.a.x; vlq = m.a.z; vnid = m.a.w; vnf = m.b.y; vmk = m.b.z; vbl = m.b.w; vbh = m.c.x;
            const uint32_t ncig = m.b.y & 0xffffu;
            vcw = ncig ? R.cigar[m.b.x] : 0u;
            // kept by -M (GROM.c:6590) and touching [t0, t1) at all
            rel = ((m.b.z >> 8) & 255u) != 0 && (int32_t)m.a.x - 1 <= t1 - 1 && (int32_t)m.a.y > t0;
            const uint32_t op = vcw & 15u;
            fast = rel && ncig == 1 && (op == 0 || op == 7 || op == 8);
        }
        uint64_t fm = __ballot(fast && GROM_SCAT_PROF != 2);
        uint64_t gm = __ballot(rel && !fast && GROM_SCAT_PROF != 2);
        // one M/=/X op (the common case), software-pipelined: the next read's
        // bases are in flight while this one is tallied
        if (fm) {
            FastRead cur = fast_view(a, rb0, __builtin_ctzll(fm), lo_x, hi_x, vp0, vlq, vnid, vnf, vmk, vbl, vbh, vcw);
            fm &= fm - 1;
            FastLoads lc;
            fast_issue(L, R, cur, t0, lc);
            for (;;) {
                const bool more = fm != 0;
                FastRead nxt = cur;
                FastLoads ln = lc;
                if (more) {
                    nxt = fast_view(a, rb0, __builtin_ctzll(fm), lo_x, hi_x, vp0, vlq, vnid, vnf, vmk, vbl, vbh, vcw);
                    fm &= fm - 1;
                    fast_issue(L, R, nxt, t0, ln);
                }
                fast_tally(L, a, R, evcap, cur, lc, t0);
                if (!more) break;
                cur = nxt;
                lc = ln;
            }
        }
        while (gm) {
            const int32_t r = rb0 + __builtin_ctzll(gm) * SNW;
            gm &= gm - 1;
            scat_general(L, a, R, meta, evcap, r, t0, lo_x, hi_x);
        }
    }
    __syncthreads();

    // ---- a tile over the event budget goes to the gather kernel ----
    const uint32_t nev = L.nev;
    if (nev > evcap) {
        if (tid == 0) {
            const uint32_t k = atomicAdd(n_ovf, 1u);
            ovf_list[k] = (uint32_t)tile;
        }
        return;  // nev is the same for the whole workgroup
    }

    // ---- interval prefix sums; event buckets by position ----
    int32_t v[NSCAN];
#pragma unroll
    for (int k = 0; k < NDIF; k++) v[k] = L.dif[k][tid];
    v[NDIF] = (int32_t)L.evn[tid];
    const int32_t ecnt = v[NDIF];
    scat_scan(L, v);
    const int32_t ebeg = v[NDIF];
    L.evn[tid] = (uint32_t)ebeg;
    __syncthreads();
    for (uint32_t k = tid; k < nev; k += TG) {
        const uint32_t s = atomicAdd(&L.evn[L.ev[k].w & 2047u], 1u);
        L.sidx[s] = (uint16_t)k;
    }
    __syncthreads();
    // this position's events in read order (insertion sort; buckets are small)
    for (int32_t i = ebeg + 1; i < ebeg + ecnt; i++) {
        const uint16_t e = L.sidx[i];
        const uint32_t key = L.ev[e].x;
        int32_t j = i - 1;
        while (j >= ebeg && L.ev[L.sidx[j]].x > key) {
            L.sidx[j + 1] = L.sidx[j];
            j--;
        }
        L.sidx[j + 1] = e;
    }

    // ---- fold: the intervals' plain matches, then the events in order ----
    const bool mv = rcode < 4;
    const uint32_t xr = (uint32_t)(x - t0);
    // plain matches of MAPQ >= -q reads (kept only where the reference is ACGT)
    int32_t m_cnt = mv ? (int32_t)((uint32_t)v[D_NF] + (uint32_t)v[D_NR]) : 0;
    int32_t m_fs = mv ? v[D_NF] : 0;
    int32_t m_pir = mv ? (int32_t)((uint32_t)v[D_NF] * xr - (uint32_t)v[D_SF] + (uint32_t)v[D_SR] -
                                   (uint32_t)v[D_NR] * xr)
                       : 0;
    LaneCounts c = {};
    c.mq_hi = mv ? v[D_MQ] : 0;
    c.bq_hi = (int32_t)L.bqh[tid];
    int32_t m_low = (int32_t)L.lcnt[tid];
    c.bq_lo = (int32_t)L.bql[tid];
    c.mq_lo = (int32_t)L.mql[tid];
    int32_t sch[6] = {0, 0, 0, 0, 0, 0}, scn[6] = {0, 0, 0, 0, 0, 0};
    uint32_t slot[GROM_MAX_NAME_SLOTS];
#pragma unroll
    for (int k = 0; k < GROM_MAX_NAME_SLOTS; k++) slot[k] = 0;
    for (int32_t i = ebeg; i < ebeg + ecnt; i++) {
        const uint32_t e = L.sidx[i];
        const uint4 ev = L.ev[e];
        const uint32_t ex = L.evx[e];
        const uint32_t type = (ev.w >> 11) & 3u, code = (ev.w >> 13) & 7u;
        const bool efwd = (ev.w >> 16) & 1u, assumed = (ev.w >> 25) & 1u, ematch = (ev.w >> 26) & 1u;
        const int32_t q = (int32_t)((ev.w >> 17) & 255u), emq = (int32_t)(ex & 255u);
        const int32_t qi = (int32_t)ev.z;
        if (type == EV_X) {
            if (assumed) {  // the interval counted this base as a plain match
                m_cnt -= 1;
                m_fs -= efwd ? 1 : 0;
                m_pir -= efwd ? qi : (int32_t)(ex >> 8) - qi;
                c.mq_hi -= emq;
            }
            if (q >= a.min_base_qual) {
                // a high-quality mismatch: read-name slots (GROM.c:6805-6824)
                bool done = false, found = false;
#pragma unroll
                for (int s = 0; s < GROM_MAX_NAME_SLOTS; s++) {
                    const bool active = !done && s < a.min_snv;
                    const bool empty = active && slot[s] == 0;
                    const bool hit = active && !empty && slot[s] == ev.y;
                    slot[s] = (empty && ev.y != 0) ? ev.y : slot[s];
                    found = found || hit;
                    done = done || empty || hit;
                }
                const bool count = code < 4 && !found;
                const int32_t ch = count ? 1 : 0;
                GROM_ADD4(c, snv, code, ch);
                GROM_ADD4(c, fs, code, efwd ? ch : 0);
                GROM_ADD4(c, pir, code, count ? qi : 0);  // both strands add the offset (GROM.c:6896)
                c.bq_hi += count ? q : 0;
                c.mq_hi += count ? emq : 0;
            } else if (ematch ? mv : code < 4) {  // low base quality
                if (ematch) m_low += 1;
                else GROM_ADD4(c, low, code, 1);
                c.bq_lo += q;
                c.mq_lo += emq;
            }
        } else if (type == EV_LQ) {
            GROM_ADD4(c, low, code, 1);
            c.bq_lo += q;
            c.mq_lo += emq;
        } else {
            const int32_t h = (ev.z >> 6) & 1;
#pragma unroll
            for (int k = 0; k < 6; k++) {
                const bool b = (ev.z >> k) & 1u;
                sch[k] += b ? h : 0;
                scn[k] += b ? 1 : 0;
            }
        }
    }
    GROM_ADD4(c, snv, rcode, m_cnt);
    GROM_ADD4(c, fs, rcode, m_fs);
    GROM_ADD4(c, pir, rcode, m_pir);
    GROM_ADD4(c, low, rcode, m_low);

    const bool evals = x >= a.eval_lo && x <= a.eval_hi;
    pile_emit(a, ref, O, mq_tab, hez_tab, L.tail, tile, x, rb, evals, c, v[D_RD], v[D_CMQ], v[D_CRD], v[D_CLOW], sch,
              scn);
}

#undef GROM_ADD4
