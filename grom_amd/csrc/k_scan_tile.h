// k_scan_tile.h -- the per-chromosome scan's tile kernel (included by scan.hip).
//
// One workgroup owns GROM_TILE consecutive reference positions and one thread
// owns one position.  The reads that can touch the tile (sorted by position,
// GROM's file order) are staged in LDS in chunks; every wave then walks them
// in order and each lane folds the read's contribution to *its* position into
// registers.  That per-position, in-read-order fold is exactly the order in
// which the reference's ring accumulates a base (GROM.c:6406-7185), so the
// order-dependent read-name de-duplication of mismatching bases
// (GROM.c:6805-6824) needs no sorting and no atomics, and every counter sits
// in a register until the base is evaluated (GROM.c:11096-11199) in place.
//
// HBM traffic per launch: each read's metadata and CIGAR once per tile it
// overlaps, each base's quality and packed sequence byte once (consecutive
// lanes read consecutive bytes of a read), the reference tile, and the three
// whole-chromosome read-depth arrays written once.

#define TG GROM_TILE
#define RCHUNK 256
#define CIGCAP 2048

struct __align__(16) ScanLds {
    int64_t boff[RCHUNK];
    int32_t pos[RCHUNK], lq[RCHUNK], ext[RCHUNK], mtid[RCHUNK], mpos[RCHUNK], isize[RCHUNK];
    uint32_t coff[RCHUNK], cend[RCHUNK], nid[RCHUNK];
    uint16_t flag[RCHUNK];
    uint8_t mapq[RCHUNK], keep[RCHUNK];
    uint32_t cig[CIGCAP];
    char ref[TG];
    unsigned long long red[TG / 64][2];
    uint32_t cig_first;
    int32_t cig_staged;
};

// add one counted base to the per-lane counters (code in 0..3)
#define GROM_ADD4(arr, code, v)          \
    do {                                 \
        arr##0 += ((code) == 0) ? (v) : 0; \
        arr##1 += ((code) == 1) ? (v) : 0; \
        arr##2 += ((code) == 2) ? (v) : 0; \
        arr##3 += ((code) == 3) ? (v) : 0; \
    } while (0)

__global__ __launch_bounds__(TG) void k_scan_tile(grom_scan_args a, const char *__restrict__ ref, ReadArrays R,
                                                  const int32_t *__restrict__ tile_lo,
                                                  const int32_t *__restrict__ tile_hi, PileOut O,
                                                  const double *__restrict__ mq_tab,
                                                  const double *__restrict__ hez_tab) {
    __shared__ ScanLds L;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t t0 = (int64_t)blockIdx.x * TG;
    const int64_t x = t0 + tid;            // this lane's reference position
    const int64_t x0 = t0 + wave * 64;     // first position of this wave
    const int32_t r0 = tile_lo[blockIdx.x], r1 = tile_hi[blockIdx.x];
    L.ref[tid] = (x < a.chr_len) ? upcase(ref[x]) : 'N';
    const bool evals = x >= a.eval_lo && x <= a.eval_hi;  // GROM.c:11086, 5842

    // per-position counters (cdp_one_base_*), in registers
    int32_t snv0 = 0, snv1 = 0, snv2 = 0, snv3 = 0, fs0 = 0, fs1 = 0, fs2 = 0, fs3 = 0;
    int32_t low0 = 0, low1 = 0, low2 = 0, low3 = 0, pir0 = 0, pir1 = 0, pir2 = 0, pir3 = 0;
    int32_t bq_hi = 0, mq_hi = 0, bq_lo = 0, mq_lo = 0, rd = 0, caf_mq = 0, caf_rd = 0, caf_low = 0;
    int32_t sc[15];
#pragma unroll
    for (int k = 0; k < 15; k++) sc[k] = 0;
    uint32_t slot[GROM_MAX_NAME_SLOTS];
#pragma unroll
    for (int k = 0; k < GROM_MAX_NAME_SLOTS; k++) slot[k] = 0;

    for (int32_t c0 = r0; c0 < r1; c0 += RCHUNK) {
        const int32_t m = min(RCHUNK, r1 - c0);
        __syncthreads();  // previous chunk fully consumed
        for (int i = tid; i < m; i += TG) {
            const int32_t r = c0 + i;
            const uint32_t cb = R.cig_off[r], ce = R.cig_off[r + 1];
            L.pos[i] = R.pos[r];
            L.lq[i] = R.lqseq[r];
            L.coff[i] = cb;
            L.cend[i] = ce;
            L.boff[i] = R.base_off[r];
            L.nid[i] = R.name_id[r];
            L.flag[i] = R.flag[r];
            L.mapq[i] = R.mapq[r];
            L.keep[i] = R.keep ? R.keep[r] : 1;
            L.mtid[i] = R.mtid[r];
            L.mpos[i] = R.mpos[r];
            L.isize[i] = R.isize[r];
            // furthest position the read can touch (tally extent, or the
            // clip / depth end E = pos - start_adj + lseq - end_adj - (I - D))
            int32_t s = 0, e = L.lq[i];
            for (uint32_t k = cb; k < ce; k++) {
                const uint32_t c = R.cigar[k];
                const int op = c & 15;
                const int32_t len = (int32_t)(c >> 4);
                if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) s += len;
                if (op == 2 || op == 5) e += len;
            }
            L.ext[i] = L.pos[i] + max(s, e) + 1;
        }
        if (tid == 0) {
            const uint32_t cf = R.cig_off[c0], cl = R.cig_off[c0 + m];
            L.cig_first = cf;
            L.cig_staged = (cl - cf) <= CIGCAP;
        }
        __syncthreads();
        const uint32_t cf = L.cig_first;
        const bool staged = L.cig_staged;
        if (staged)
            for (uint32_t k = tid; k < R.cig_off[c0 + m] - cf; k += TG) L.cig[k] = R.cigar[cf + k];
        __syncthreads();

        for (int i = 0; i < m; i++) {
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
            int snv_base = 0, srb = 0, lseq_mod = lq, eai = 0;
            int64_t caf_pos = p0;
            int first_op = -1, first_len = 0, last_op = -1, last_len = 0;
            const uint32_t ncap = (ce - cb > 1000u) ? cb + 1000u : ce;  // GROM.c:6743
            for (uint32_t k = cb; k < ce; k++) {
                const uint32_t cg = staged ? L.cig[k - cf] : R.cigar[k];
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
                            if (qi < lq) {
                                const int64_t nib = bo + qi;
                                q = R.qual[nib];
                                s4 = (R.seq[nib >> 1] >> ((~nib & 1) << 2)) & 15;
                            }
                            const char sb = c_nt16[s4];
                            const int code = c_nt16_acgt[s4];
                            const char rb = L.ref[tid];
                            if (hq_read && q >= a.min_base_qual) {
                                bool count = code < 4;
                                int32_t pv = fwd ? qi : lseq_mod - qi;
                                if (rb != sb) {
                                    // read-name slots of the position, GROM.c:6805-6824
                                    bool done = false, found = false;
#pragma unroll
                                    for (int s = 0; s < GROM_MAX_NAME_SLOTS; s++) {
                                        if (!done && s < a.min_snv) {
                                            if (slot[s] == 0) {
                                                if (nid != 0) slot[s] = nid;
                                                done = true;
                                            } else if (slot[s] == nid) {
                                                found = done = true;
                                            }
                                        }
                                    }
                                    count = count && !found;
                                    pv = qi;  // mismatches add the offset on both strands (GROM.c:6896)
                                }
                                if (count) {
                                    GROM_ADD4(snv, code, 1);
                                    GROM_ADD4(fs, code, fwd ? 1 : 0);
                                    GROM_ADD4(pir, code, pv);
                                    bq_hi += q;
                                    mq_hi += mq;
                                }
                            } else if (code < 4) {
                                GROM_ADD4(low, code, 1);
                                bq_lo += q;
                                mq_lo += mq;
                            }
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
            if (evals && ((start_adj >= a.sc_min && x == (int64_t)p0 - 1) || (end_adj >= a.sc_min && x == E))) {
                const bool paired = fl & 0x1, munmap = fl & 0x8, rev = fl & 0x10;
                const bool same_chr = L.mtid[i] == a.chr_tid;
                const int32_t mp = L.mpos[i], tl = L.isize[i];
                const int add = hq_read ? 6 : 0;  // cdp_add, GROM.c:5829-5836
                if (start_adj >= a.sc_min && x == (int64_t)p0 - 1) {
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
                if (end_adj >= a.sc_min && x == E) {
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
    }

    // ---- outputs of this position ----
    unsigned long long fsum = 0, fcnt = 0;
    const char rb = L.ref[tid];
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
        const int32_t total = snv0 + snv1 + snv2 + snv3;
        const int32_t rc_all = total + low0 + low1 + low2 + low3;
        const int32_t bq_all = bq_hi + bq_lo, mq_all = mq_hi + mq_lo;
        if (O.dbg) {
            int32_t *d = O.dbg + (size_t)(x - a.eval_lo) * GC_COUNT;
            d[GC_POS] = (int32_t)x;
            d[GC_SNV + 0] = snv0; d[GC_SNV + 1] = snv1; d[GC_SNV + 2] = snv2; d[GC_SNV + 3] = snv3;
            d[GC_SNV_LOWMQ + 0] = low0; d[GC_SNV_LOWMQ + 1] = low1; d[GC_SNV_LOWMQ + 2] = low2; d[GC_SNV_LOWMQ + 3] = low3;
            d[GC_PIR + 0] = pir0; d[GC_PIR + 1] = pir1; d[GC_PIR + 2] = pir2; d[GC_PIR + 3] = pir3;
            d[GC_FS + 0] = fs0; d[GC_FS + 1] = fs1; d[GC_FS + 2] = fs2; d[GC_FS + 3] = fs3;
            d[GC_BQ] = bq_hi;
            d[GC_BQ_ALL] = bq_all;
            d[GC_MQ] = mq_hi;
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
            const int32_t snv[4] = {snv0, snv1, snv2, snv3};
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
                    grom_snv_cand c;
                    c.pos = (int32_t)x;
                    c.base = best;
                    c.ratio = best_ratio;
                    c.ref_base = (int32_t)(unsigned char)ref[x];
                    const int32_t sk = snv[best];
                    const size_t ti = (total > GROM_MAX_TRIALS)
                                          ? (size_t)GROM_MAX_TRIALS * (GROM_MAX_TRIALS + 1) + sk * GROM_MAX_TRIALS / total
                                          : (size_t)total * (GROM_MAX_TRIALS + 1) + sk;
                    c.binom = mq_tab[ti];
                    c.hez = hez_tab[ti];
                    c.snv[0] = snv0; c.snv[1] = snv1; c.snv[2] = snv2; c.snv[3] = snv3;
                    c.lowmq[0] = low0; c.lowmq[1] = low1; c.lowmq[2] = low2; c.lowmq[3] = low3;
                    c.pir[0] = pir0; c.pir[1] = pir1; c.pir[2] = pir2; c.pir[3] = pir3;
                    c.fs[0] = fs0; c.fs[1] = fs1; c.fs[2] = fs2; c.fs[3] = fs3;
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
        unsigned long long s = 0, c = 0;
        for (int w = 0; w < TG / 64; w++) {
            s += L.red[w][0];
            c += L.red[w][1];
        }
        if (c) {
            atomicAdd(&O.flush_acc[0], s);
            atomicAdd(&O.flush_acc[1], c);
        }
    }
}

#undef GROM_ADD4
