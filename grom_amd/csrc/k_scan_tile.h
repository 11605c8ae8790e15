// k_scan_tile.h -- the per-chromosome scan's tile kernel (included by scan.hip).
//
// One workgroup owns GROM_TILE consecutive reference positions and one thread
// owns one position.  The reads that can touch the tile (sorted by position,
// GROM's file order) are staged in LDS in chunks -- metadata, CIGAR words and
// the contiguous run of their qualities and packed bases, copied with wide
// coalesced loads -- and every wave then walks them in order while each lane
// folds the read's contribution to *its* position into registers.  That
// per-position, in-read-order fold is exactly the order in which the
// reference's ring accumulates a base (GROM.c:6406-7185), so the
// order-dependent read-name de-duplication of mismatching bases
// (GROM.c:6805-6824) needs no sorting and no atomics, and every counter stays in
// a register until the base is evaluated in place (GROM.c:11096-11199).
//
// Tiles are mapped so that consecutive tiles run on one XCD (blocks are dealt
// round-robin over the 8 XCDs): a read straddling two tiles is then fetched
// from HBM once and served to the second tile from that XCD's L2.

#define TG GROM_TILE
#define RCHUNK 192
#define CIGCAP 1024
#define QBYTES 16384  // staged qualities per chunk (bytes)

struct __align__(16) ScanLds {
    int64_t boff[RCHUNK];
    int32_t pos[RCHUNK], lq[RCHUNK], ext[RCHUNK], mtid[RCHUNK], mpos[RCHUNK], isize[RCHUNK];
    uint32_t coff[RCHUNK], cend[RCHUNK], nid[RCHUNK];
    uint16_t flag[RCHUNK];
    uint8_t mapq[RCHUNK], keep[RCHUNK];
    uint32_t cig[CIGCAP];
    uint32_t qual[QBYTES / 4 + 2];
    uint32_t seq[QBYTES / 8 + 2];
    char ref[TG];
    unsigned long long red[TG / 64][2];
    int32_t m2;  // reads of the chunk that fit the staging budgets
};

// per-lane counters of one position (cdp_one_base_*)
struct LaneCounts {
    int32_t snv0, snv1, snv2, snv3, fs0, fs1, fs2, fs3, low0, low1, low2, low3, pir0, pir1, pir2, pir3;
    int32_t bq_hi, mq_hi, bq_lo, mq_lo;
};

#define GROM_ADD4(cnt, f, code, v)                    \
    do {                                              \
        cnt.f##0 += ((code) == 0) ? (v) : 0;          \
        cnt.f##1 += ((code) == 1) ? (v) : 0;          \
        cnt.f##2 += ((code) == 2) ? (v) : 0;          \
        cnt.f##3 += ((code) == 3) ? (v) : 0;          \
    } while (0)

// one aligned base of a read at this lane's position: the SNV tally body of
// GROM.c:6800-6992 (high-quality branch with read-name slots) and
// GROM.c:6995-7040 (low-quality branch)
__device__ __forceinline__ void tally_base(LaneCounts &c, uint32_t (&slot)[GROM_MAX_NAME_SLOTS], int min_snv,
                                           bool hq, int q, int s4, char rb, bool fwd, int qi, int lseq_mod, int mq,
                                           uint32_t nid) {
    const char sb = c_nt16[s4];
    const int code = c_nt16_acgt[s4];
    // branch-free updates: every counter is touched with a 0/1 increment, so
    // the counters stay in registers (no select of addresses)
    bool count = hq && code < 4;
    int32_t pv = fwd ? qi : lseq_mod - qi;
    {
        if (hq && rb != sb) {
            // first empty slot takes the name (names >= 50 chars are never
            // stored); a slot holding the name marks the base as seen.  Written
            // with selects so the slots stay in registers.
            bool done = false, found = false;
#pragma unroll
            for (int s = 0; s < GROM_MAX_NAME_SLOTS; s++) {
                const bool active = !done && s < min_snv;
                const bool empty = active && slot[s] == 0;
                const bool match = active && !empty && slot[s] == nid;
                slot[s] = (empty && nid != 0) ? nid : slot[s];
                found = found || match;
                done = done || empty || match;
            }
            count = count && !found;
            pv = qi;  // mismatches add the offset on both strands (GROM.c:6896)
        }
    }
    const bool low = !hq && code < 4;
    const int32_t ch = count ? 1 : 0, cl = low ? 1 : 0;
    GROM_ADD4(c, snv, code, ch);
    GROM_ADD4(c, fs, code, fwd ? ch : 0);
    GROM_ADD4(c, pir, code, count ? pv : 0);
    GROM_ADD4(c, low, code, cl);
    c.bq_hi += count ? q : 0;
    c.mq_hi += count ? mq : 0;
    c.bq_lo += low ? q : 0;
    c.mq_lo += low ? mq : 0;
}

// a CIGAR word of the current chunk: from LDS when the chunk was staged,
// else (a read too large to stage) from global memory
__device__ __forceinline__ uint32_t cigar_word(const ScanLds &L, const ReadArrays &R, bool staged, uint32_t k,
                                               uint32_t cf) {
    uint32_t w;
    if (staged) w = L.cig[k - cf];
    else w = R.cigar[k];
    return w;
}

// quality and 4-bit base of global base offset `nib` (BAM nibble order)
__device__ __forceinline__ void load_base(const ScanLds &L, const ReadArrays &R, bool staged, int64_t qb0,
                                          int64_t sb0, int64_t nib, int &q, int &s4) {
    uint32_t qv, sv;
    if (staged) {
        const int64_t qo = nib - qb0, so = (nib >> 1) - sb0;
        qv = (L.qual[qo >> 2] >> ((qo & 3) * 8)) & 255u;
        sv = (L.seq[so >> 2] >> ((so & 3) * 8)) & 255u;
    } else {
        qv = R.qual[nib];
        sv = R.seq[nib >> 1];
    }
    q = (int)qv;
    s4 = (int)((sv >> ((~nib & 1) << 2)) & 15u);
}

__global__ __launch_bounds__(TG) void k_scan_tile(grom_scan_args a, const char *__restrict__ ref, ReadArrays R,
                                                  const int32_t *__restrict__ tile_lo,
                                                  const int32_t *__restrict__ tile_hi, PileOut O,
                                                  const double *__restrict__ mq_tab,
                                                  const double *__restrict__ hez_tab, int64_t n_tiles) {
    __shared__ ScanLds L;
    // XCD-contiguous tile order (speed only; any mapping is correct)
    const int64_t per_xcd = (n_tiles + 7) / 8;
    const int64_t tile = (int64_t)(blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
    if (tile >= n_tiles) return;  // whole workgroup leaves together
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t t0 = tile * TG;
    const int64_t x = t0 + tid;         // this lane's reference position
    const int64_t x0 = t0 + wave * 64;  // first position of this wave
    const int32_t r0 = tile_lo[tile], r1 = tile_hi[tile];
    L.ref[tid] = (x < a.chr_len) ? upcase(ref[x]) : 'N';
    const char rb = L.ref[tid];
    const bool evals = x >= a.eval_lo && x <= a.eval_hi;  // GROM.c:11086, 5842

    LaneCounts c = {};
    int32_t rd = 0, caf_mq = 0, caf_rd = 0, caf_low = 0;
    int32_t sc[15];
#pragma unroll
    for (int k = 0; k < 15; k++) sc[k] = 0;
    uint32_t slot[GROM_MAX_NAME_SLOTS];
#pragma unroll
    for (int k = 0; k < GROM_MAX_NAME_SLOTS; k++) slot[k] = 0;

    int32_t c0 = r0;
    while (c0 < r1) {
        const int32_t m = min(RCHUNK, r1 - c0);
        __syncthreads();  // previous chunk fully consumed
        if (tid == 0) L.m2 = 0;
        __syncthreads();
        // ---- stage metadata ----
        bool fits = false;
        if (tid < m) {
            const int32_t r = c0 + tid;
            const uint32_t cb = R.cig_off[r], ce = R.cig_off[r + 1];
            const int32_t p = R.pos[r], lq = R.lqseq[r];
            const int64_t bo = R.base_off[r];
            L.pos[tid] = p;
            L.lq[tid] = lq;
            L.coff[tid] = cb;
            L.cend[tid] = ce;
            L.boff[tid] = bo;
            L.nid[tid] = R.name_id[r];
            L.flag[tid] = R.flag[r];
            L.mapq[tid] = R.mapq[r];
            L.keep[tid] = R.keep ? R.keep[r] : 1;
            L.mtid[tid] = R.mtid[r];
            L.mpos[tid] = R.mpos[r];
            L.isize[tid] = R.isize[r];
            // furthest position the read can touch (tally extent, or the
            // clip / depth end E = pos - start_adj + lseq - end_adj - (I - D))
            int32_t s = 0, e = lq;
            for (uint32_t k = cb; k < ce; k++) {
                const uint32_t cw = R.cigar[k];
                const int op = cw & 15;
                const int32_t len = (int32_t)(cw >> 4);
                if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) s += len;
                if (op == 2 || op == 5) e += len;
            }
            L.ext[tid] = p + max(s, e) + 1;
            // reads are contiguous in cigar[] and in qual/seq, so these budgets
            // hold for a prefix of the chunk
            fits = (bo + lq - R.base_off[c0]) <= (int64_t)QBYTES - 16 && ce - R.cig_off[c0] <= CIGCAP;
        }
        if (fits) atomicMax(&L.m2, tid + 1);
        __syncthreads();
        int32_t m2 = min(L.m2, m);
        const bool staged = m2 > 0;
        if (!staged) m2 = 1;  // one oversized read: served from global memory
        const int64_t b0 = L.boff[0];
        const uint32_t cf = L.coff[0], cl = L.cend[m2 - 1];
        // ---- stage CIGAR words, qualities and packed bases ----
        const int64_t qw0 = b0 >> 2, sw0 = (b0 >> 1) >> 2;  // first qual / seq word
        if (staged) {
            const int64_t bend = L.boff[m2 - 1] + L.lq[m2 - 1];
            const int64_t qw1 = min((bend + 3) >> 2, qw0 + (int64_t)(QBYTES / 4 + 2));
            const int64_t sw1 = min((((bend + 1) >> 1) + 3) >> 2, sw0 + (int64_t)(QBYTES / 8 + 2));
            const uint32_t nc = min(cl - cf, (uint32_t)CIGCAP);  // guards only; the budget check implies them
            for (uint32_t k = tid; k < nc; k += TG) L.cig[k] = R.cigar[cf + k];
            const uint32_t *gq = (const uint32_t *)R.qual;
            for (int64_t w = qw0 + tid; w < qw1; w += TG) L.qual[w - qw0] = gq[w];
            const uint32_t *gs = (const uint32_t *)R.seq;
            for (int64_t w = sw0 + tid; w < sw1; w += TG) L.seq[w - sw0] = gs[w];
        }
        __syncthreads();
        const int64_t qb0 = qw0 << 2, sb0 = sw0 << 2;  // global byte offsets of L.qual[0] / L.seq[0]

        for (int i = 0; i < m2; i++) {
            const int32_t p0 = L.pos[i];
            // wave-uniform overlap test with [x0, x0+64): contributions span
            // [pos-1 (left clip), ext)
            if (p0 - 1 > x0 + 63 || L.ext[i] < x0) continue;
            if (L.keep[i] == 0) continue;  // -M duplicate (GROM.c:6590)
            const uint16_t fl = L.flag[i];
            const int mq = L.mapq[i];
            const int lq = L.lq[i];
            const int64_t bo = L.boff[i];
            const uint32_t nid = L.nid[i];
            const uint32_t cb = L.coff[i], ce = L.cend[i];
            const bool fwd = !(fl & 0x10);
            const bool hq_read = mq >= a.min_mapq;
            const bool pos_ok = p0 >= 0 && p0 < a.chr_len;
            const uint32_t cw0 = (ce > cb) ? cigar_word(L, R, staged, cb, cf) : 0u;
            const int op0 = cw0 & 15;
            if (ce - cb == 1 && (op0 == 0 || op0 == 7 || op0 == 8)) {
                // ---- fast path: a single M/=/X op ----
                const int len = (int)(cw0 >> 4);
                if (p0 >= 0 && (int64_t)p0 + len < a.chr_len && x >= p0 && x < (int64_t)p0 + len) {
                    caf_mq += mq;
                    if (mq >= a.rd_min_mapq) caf_rd += 1;
                    else caf_low += 1;
                }
                if (pos_ok && evals) {
                    const int loop_end = ((int64_t)p0 + len >= a.chr_len) ? (int)(a.chr_len - p0) : len;
                    if (x >= p0 && x < (int64_t)p0 + loop_end) {
                        const int qi = (int)(x - p0);
                        int q = 0, s4 = 15;
                        if (qi < lq) load_base(L, R, staged, qb0, sb0, bo + qi, q, s4);
                        tally_base(c, slot, a.min_snv, hq_read && q >= a.min_base_qual, q, s4, rb, fwd, qi, lq, mq,
                                   nid);
                    }
                }
                if (x >= p0 && x < (int64_t)p0 + lq) rd += 1;  // E = pos + l_qseq
                continue;
            }
            // ---- general CIGAR walk ----
            int snv_base = 0, srb = 0, lseq_mod = lq, eai = 0;
            int64_t caf_pos = p0;
            int first_op = -1, first_len = 0, last_op = -1, last_len = 0;
            const uint32_t ncap = (ce - cb > 1000u) ? cb + 1000u : ce;  // GROM.c:6743
            for (uint32_t k = cb; k < ce; k++) {
                const uint32_t cg = cigar_word(L, R, staged, k, cf);
                const int op = cg & 15;
                const int len = (int)(cg >> 4);
                const bool in_cap = k < ncap;
                if (op == 0 || op == 7 || op == 8) {
                    // whole-chromosome read depth, GROM.c:6605-6671 (all ops)
                    if (caf_pos >= 0 && caf_pos + len < a.chr_len && x >= caf_pos && x < caf_pos + len) {
                        caf_mq += mq;
                        if (mq >= a.rd_min_mapq) caf_rd += 1;
                        else caf_low += 1;
                    }
                    caf_pos += len;
                    if (!in_cap) continue;
                    if (pos_ok) {
                        // SNV tally, GROM.c:6769-7059
                        const int64_t xb = (int64_t)p0 + srb;
                        const int loop_end = (xb + len >= a.chr_len) ? (int)(a.chr_len - p0) : len;
                        if (evals && x >= xb && x < xb + loop_end) {
                            const int qi = snv_base + (int)(x - xb);
                            int q = 0, s4 = 15;
                            if (qi < lq) load_base(L, R, staged, qb0, sb0, bo + qi, q, s4);
                            tally_base(c, slot, a.min_snv, hq_read && q >= a.min_base_qual, q, s4, rb, fwd, qi,
                                       lseq_mod, mq, nid);
                        }
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
            if (x >= p0 && x < E) rd += 1;  // physical read depth, GROM.c:7173-7181
            // soft-clip evidence, GROM.c:7105-7169
            const bool at_l = start_adj >= a.sc_min && x == (int64_t)p0 - 1;
            const bool at_r = end_adj >= a.sc_min && x == E;
            if (evals && (at_l || at_r)) {
                const bool paired = fl & 0x1, munmap = fl & 0x8, rev = fl & 0x10;
                const bool same_chr = L.mtid[i] == a.chr_tid;
                const int32_t mp = L.mpos[i], tl = L.isize[i];
                const int add = hq_read ? 6 : 0;  // cdp_add, GROM.c:5829-5836
                if (at_l) {
                    if (!paired || (!rev && (munmap || (!munmap && same_chr && mp > p0)))) {
                        sc[0] += add; sc[2] += 1; sc[4] += 1;
                    }
                    if (paired && !munmap && !same_chr && rev) {
                        sc[5] += add; sc[7] += 1; sc[9] += 1;
                    }
                    if (paired && !munmap && same_chr && rev && abs(tl) <= a.insert_max && mp < p0) {
                        sc[10] += add; sc[12] += 1; sc[14] += 1;
                    }
                }
                if (at_r) {
                    if (!paired || (rev && (munmap || (!munmap && same_chr && mp < p0)))) {
                        sc[1] += add; sc[3] += 1; sc[4] += 1;
                    }
                    if (paired && !munmap && !same_chr && !rev) {
                        sc[6] += add; sc[8] += 1; sc[9] += 1;
                    }
                    if (paired && !munmap && same_chr && !rev && abs(tl) <= a.insert_max && mp > p0) {
                        sc[11] += add; sc[13] += 1; sc[14] += 1;
                    }
                }
            }
        }
        c0 += m2;
    }

    // ---- outputs of this position ----
    unsigned long long fsum = 0, fcnt = 0;
    if (x < a.chr_len) {
        O.caf_mq[x] = caf_mq;
        O.caf_rd[x] = caf_rd;
        O.caf_low[x] = caf_low;
        if (x < a.flush_end && rb != 'N') {  // SNV flush depth sums, GROM.c:15066-15073
            fsum = (unsigned long long)((int64_t)caf_rd + caf_low);
            fcnt = 1;
        }
    }
    if (evals) {
        const int32_t total = c.snv0 + c.snv1 + c.snv2 + c.snv3;
        const int32_t rc_all = total + c.low0 + c.low1 + c.low2 + c.low3;
        const int32_t bq_all = c.bq_hi + c.bq_lo, mq_all = c.mq_hi + c.mq_lo;
        if (O.dbg) {
            int32_t *d = O.dbg + (size_t)(x - a.eval_lo) * GC_COUNT;
            d[GC_POS] = (int32_t)x;
            d[GC_SNV + 0] = c.snv0; d[GC_SNV + 1] = c.snv1; d[GC_SNV + 2] = c.snv2; d[GC_SNV + 3] = c.snv3;
            d[GC_SNV_LOWMQ + 0] = c.low0; d[GC_SNV_LOWMQ + 1] = c.low1;
            d[GC_SNV_LOWMQ + 2] = c.low2; d[GC_SNV_LOWMQ + 3] = c.low3;
            d[GC_PIR + 0] = c.pir0; d[GC_PIR + 1] = c.pir1; d[GC_PIR + 2] = c.pir2; d[GC_PIR + 3] = c.pir3;
            d[GC_FS + 0] = c.fs0; d[GC_FS + 1] = c.fs1; d[GC_FS + 2] = c.fs2; d[GC_FS + 3] = c.fs3;
            d[GC_BQ] = c.bq_hi;
            d[GC_BQ_ALL] = bq_all;
            d[GC_MQ] = c.mq_hi;
            d[GC_MQ_ALL] = mq_all;
            d[GC_BQ_RC] = total;
            d[GC_MQ_RC] = total;
            d[GC_RC_ALL] = rc_all;
            d[GC_RD] = rd;
#pragma unroll
            for (int k = 0; k < 15; k++) d[GC_SC_LEFT + k] = sc[k];
        }
        // SNV test, GROM.c:11096-11199
        if (rd + sc[14] > 0 && rb != 'N') {
            const int32_t snv[4] = {c.snv0, c.snv1, c.snv2, c.snv3};
            int best = -1;
            float best_ratio = 0.f;
            const bool bq_ok = (double)bq_all / (double)rc_all >= a.min_ave_bq;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const float ratio = (float)snv[k] / (float)total;
                if (rb != c_acgt[k] && (double)ratio >= a.min_snv_ratio && snv[k] >= a.min_snv && bq_ok) {
                    if (best < 0 || ratio > best_ratio) {
                        best = k;
                        best_ratio = ratio;
                    }
                }
            }
            if (best >= 0) {
                const uint32_t ci = atomicAdd(O.n_cands, 1u);
                if (ci < O.cand_cap) {  // else the host sees n_cands > cap and re-runs with room
                    grom_snv_cand cd;
                    cd.pos = (int32_t)x;
                    cd.base = best;
                    cd.ratio = best_ratio;
                    cd.ref_base = (int32_t)(unsigned char)ref[x];
                    const int32_t sk = best == 0 ? c.snv0 : best == 1 ? c.snv1 : best == 2 ? c.snv2 : c.snv3;
                    const size_t ti = (total > GROM_MAX_TRIALS)
                                          ? (size_t)GROM_MAX_TRIALS * (GROM_MAX_TRIALS + 1) + sk * GROM_MAX_TRIALS / total
                                          : (size_t)total * (GROM_MAX_TRIALS + 1) + sk;
                    cd.binom = mq_tab[ti];
                    cd.hez = hez_tab[ti];
                    cd.snv[0] = c.snv0; cd.snv[1] = c.snv1; cd.snv[2] = c.snv2; cd.snv[3] = c.snv3;
                    cd.lowmq[0] = c.low0; cd.lowmq[1] = c.low1; cd.lowmq[2] = c.low2; cd.lowmq[3] = c.low3;
                    cd.pir[0] = c.pir0; cd.pir[1] = c.pir1; cd.pir[2] = c.pir2; cd.pir[3] = c.pir3;
                    cd.fs[0] = c.fs0; cd.fs[1] = c.fs1; cd.fs[2] = c.fs2; cd.fs[3] = c.fs3;
                    cd.bq = c.bq_hi;
                    cd.bq_all = bq_all;
                    cd.mq = c.mq_hi;
                    cd.mq_all = mq_all;
                    cd.bq_rc = total;
                    cd.mq_rc = total;
                    cd.rc_all = rc_all;
                    cd.pad1 = 0;
                    O.cands[ci] = cd;
                }
            }
        }
    }
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
        unsigned long long s = 0, cc = 0;
        for (int w = 0; w < TG / 64; w++) {
            s += L.red[w][0];
            cc += L.red[w][1];
        }
        if (cc) {
            atomicAdd(&O.flush_acc[0], s);
            atomicAdd(&O.flush_acc[1], cc);
        }
    }
}

#undef GROM_ADD4
