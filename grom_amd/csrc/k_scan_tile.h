// k_scan_tile.h -- the per-chromosome scan's tile kernel (included by scan.hip).
//
// One workgroup owns GROM_TILE consecutive reference positions and one thread
// owns one position.  The reads that can touch the tile (sorted by position,
// GROM's file order) are staged in LDS in chunks -- their packed metadata
// records (k_prep), CIGAR words, and the contiguous run of their qualities and
// packed bases, all copied with 16-byte loads issued together.  Each wave then
// takes the chunk 64 reads at a time: lane j holds read j's record in
// registers, a ballot picks the reads that touch the wave's 64 positions, and
// the wave walks those in order with the record broadcast by v_readlane (no
// LDS round trip per read) while each lane folds the read's contribution to
// *its* position into registers.  That per-position, in-read-order fold is
// exactly the order in which the reference's ring accumulates a base
// (GROM.c:6406-7185), so the order-dependent read-name de-duplication of
// mismatching bases (GROM.c:6805-6824) needs no sorting and no atomics, and
// every counter stays in a register until the base is evaluated in place
// (GROM.c:11096-11199).  Reads whose CIGAR is one M/=/X op (the common case)
// take a fast path without the CIGAR walk.
//
// Positions are int32 (BAM positions are; scan_device rejects longer
// chromosomes).  Tiles are mapped so that consecutive tiles run on one XCD
// (blocks are dealt round-robin over the 8 XCDs): a read straddling two tiles
// is then fetched from HBM once and served to the second tile from that XCD's
// L2.

#define TG GROM_TILE
#define RCHUNK 128
#define CIGCAP 1024
#define QBYTES 12288                 // staged qualities per chunk (bytes)
#define QV (QBYTES / 16 + 2)          // uint4 slots for qualities
#define SV (QBYTES / 32 + 2)          // uint4 slots for packed bases
#define QLOADS ((QV + TG - 1) / TG)   // 16-byte loads per thread
#define SLOADS ((SV + TG - 1) / TG)

// Packed per-read record written by k_prep (3 x 16 bytes):
//   a: pos, ext (one past the furthest position the read can touch), l_qseq, name id
//   b: cigar offset, n_cigar | flag << 16, mapq | keep << 8, base offset (low 32)
//   c: base offset (high 32), mate tid, mate pos, isize
struct ReadMeta {
    uint4 a, b, c;
};

// Bits of ReadMeta.b.z above mapq | keep << 8.  k_prep sets MK_FAST (one
// M/=/X op of l_qseq bases inside the chromosome, kept), MK_REV (reverse
// strand) and MK_HQ (mapq >= -m, the reference's high-quality read test);
// the staging step sets DIFFED on the MK_FAST reads it staged: their caf and
// depth intervals went to the difference arrays, and the fold takes them on
// the fast path, which only tallies each one's base at the lane.
#define DIFFED (1u << 16)
#define MK_REV (1u << 17)
#define MK_HQ (1u << 18)
#define MK_FAST (1u << 19)

// k_prep: one record per read, and the tile halo (max ext - pos)
__global__ void k_prep(int64_t n, ReadArrays R, ReadMeta *__restrict__ meta, int32_t *__restrict__ halo,
                       int64_t clen, int32_t min_mapq) {
    int32_t best = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t cb = R.cig_off[i], ce = R.cig_off[i + 1];
        const int32_t p = R.pos[i], lq = R.lqseq[i];
        // tally extent (M/D/N/=/X) or the clip / depth end
        // E = pos - start_adj + lseq - end_adj - (I - D), whichever is larger
        int32_t s = 0, e = lq;
        for (uint32_t k = cb; k < ce; k++) {
            const uint32_t cw = R.cigar[k];
            const int op = cw & 15;
            const int32_t len = (int32_t)(cw >> 4);
            if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) s += len;
            if (op == 2 || op == 5) e += len;
        }
        const int32_t span = max(s, e) + 1;
        best = max(best, span);
        const int64_t bo = R.base_off[i];
        const uint32_t keep = R.keep ? R.keep[i] : 1u;
        const uint32_t mq = R.mapq[i], fl = R.flag[i];
        // the fast path's candidates: one M/=/X op of l_qseq bases inside the
        // chromosome, kept (the staging step makes them DIFFED)
        const uint32_t op0 = ce - cb == 1 ? (R.cigar[cb] & 15u) : 15u;
        const bool fast = ce - cb == 1 && (op0 == 0 || op0 == 7 || op0 == 8) && keep && s == lq && p >= 0 &&
                          (int64_t)s < clen - p;
        ReadMeta m;
        m.a = make_uint4((uint32_t)p, (uint32_t)(p + span), (uint32_t)lq, R.name_id[i]);
        m.b = make_uint4(cb, (ce - cb) | (fl << 16),
                         mq | (keep << 8) | (fast ? MK_FAST : 0u) | ((fl & 0x10u) ? MK_REV : 0u) |
                             ((int32_t)mq >= min_mapq ? MK_HQ : 0u),  // signed, as tally_base (-q may be < 0)
                         (uint32_t)(bo & 0xffffffffu));
        m.c = make_uint4((uint32_t)((uint64_t)bo >> 32), (uint32_t)R.mtid[i], (uint32_t)R.mpos[i],
                         (uint32_t)R.isize[i]);
        meta[i] = m;
    }
    for (int o = 32; o > 0; o >>= 1) best = max(best, __shfl_xor(best, o, 64));
    if ((threadIdx.x & 63) == 0) atomicMax(halo, best);
}

// per-tile reductions of the output step (pile_emit)
struct TileTail {
    unsigned long long red[TG / 64][2];
    uint32_t wcnt[TG / 64];  // candidates per wave
    uint32_t cbase;          // the tile's first candidate slot
};

// the chunk's records in LDS at a stride of 13 words: a lane per record reads
// and writes them, and the plain 12-word stride put every 8th lane of a
// 32-lane half on the same bank (4-way conflicts; 13 is odd: none)
#define META_W 13

struct __align__(16) ScanLds {
    uint32_t meta[RCHUNK * META_W];
    uint4 qual[QV + 1];  // + a slot the clamped loads past the window are stored to
    uint4 seq[SV + 1];
    uint32_t cig[CIGCAP];
    char ref[TG];
    TileTail tail;
    int32_t m2;  // reads of the chunk that fit the staging budgets
    // interval sums of the single-op reads (DIFFED below): the caf MAPQ sum
    // and, packed, the caf counts (MAPQ >= -q in the low half, the rest in
    // the high half; their sum is also the read's physical depth), as
    // difference arrays over the tile, prefix-summed once at the end
    int32_t dmq[TG + 1];
    uint32_t dcnt[TG + 1];
};

// tiles with more reads than this keep the per-lane interval updates (the
// packed 16-bit caf counts could overflow)
#define DIFF_MAX_READS 30000

__device__ __forceinline__ ReadMeta meta_ld(const ScanLds &L, int i) {
    const uint32_t *p = L.meta + META_W * i;
    ReadMeta r;
    r.a = make_uint4(p[0], p[1], p[2], p[3]);
    r.b = make_uint4(p[4], p[5], p[6], p[7]);
    r.c = make_uint4(p[8], p[9], p[10], p[11]);
    return r;
}

__device__ __forceinline__ void meta_st(ScanLds &L, int i, const ReadMeta &r) {
    uint32_t *p = L.meta + META_W * i;
    p[0] = r.a.x; p[1] = r.a.y; p[2] = r.a.z; p[3] = r.a.w;
    p[4] = r.b.x; p[5] = r.b.y; p[6] = r.b.z; p[7] = r.b.w;
    p[8] = r.c.x; p[9] = r.c.y; p[10] = r.c.z; p[11] = r.c.w;
}

// per-lane counters of one position (cdp_one_base_*)
struct LaneCounts {
    int32_t snv0, snv1, snv2, snv3, fs0, fs1, fs2, fs3, low0, low1, low2, low3, pir0, pir1, pir2, pir3;
    int32_t bq_hi, mq_hi, bq_lo, mq_lo;
};

#define GROM_ADD4(cnt, f, code, v)           \
    do {                                     \
        cnt.f##0 += ((code) == 0) ? (v) : 0; \
        cnt.f##1 += ((code) == 1) ? (v) : 0; \
        cnt.f##2 += ((code) == 2) ? (v) : 0; \
        cnt.f##3 += ((code) == 3) ? (v) : 0; \
    } while (0)

// The same counters with the per-code counts (snv, fs, low) kept as 16-bit
// pairs: fewer registers for the tile kernel.  Each count is bounded by the
// position's depth, hence by the tile's read count; tiles with more than
// PACK_MAX_READS reads go to the unpacked kernel (k_scan_tile_mem).
#define PACK_MAX_READS 65535
struct PackedCounts {
    uint32_t snv01, snv23, fs01, fs23, low01, low23;
    int32_t pir0, pir1, pir2, pir3;
    int32_t bq_hi, mq_hi, bq_lo, mq_lo;
};

// per-code adds of one base (or of the matched-base totals): code 0..3, or 4
// (not ACGT: nothing)
__device__ __forceinline__ void add_codes(LaneCounts &c, int code, int32_t snv, int32_t fs, int32_t pir, int32_t low) {
    GROM_ADD4(c, snv, code, snv);
    GROM_ADD4(c, fs, code, fs);
    GROM_ADD4(c, pir, code, pir);
    GROM_ADD4(c, low, code, low);
}
__device__ __forceinline__ void add_codes(PackedCounts &c, int code, int32_t snv, int32_t fs, int32_t pir, int32_t low) {
    const uint32_t sh = (code & 1) ? 16u : 0u;
    const bool lo2 = code < 2, hi2 = code >= 2 && code < 4;
    c.snv01 += lo2 ? ((uint32_t)snv << sh) : 0u;
    c.snv23 += hi2 ? ((uint32_t)snv << sh) : 0u;
    c.fs01 += lo2 ? ((uint32_t)fs << sh) : 0u;
    c.fs23 += hi2 ? ((uint32_t)fs << sh) : 0u;
    c.low01 += lo2 ? ((uint32_t)low << sh) : 0u;
    c.low23 += hi2 ? ((uint32_t)low << sh) : 0u;
    c.pir0 += (code == 0) ? pir : 0;
    c.pir1 += (code == 1) ? pir : 0;
    c.pir2 += (code == 2) ? pir : 0;
    c.pir3 += (code == 3) ? pir : 0;
}
__device__ __forceinline__ LaneCounts unpack(const LaneCounts &c) { return c; }
__device__ __forceinline__ LaneCounts unpack(const PackedCounts &c) {
    LaneCounts u;
    u.snv0 = (int32_t)(c.snv01 & 0xffffu); u.snv1 = (int32_t)(c.snv01 >> 16);
    u.snv2 = (int32_t)(c.snv23 & 0xffffu); u.snv3 = (int32_t)(c.snv23 >> 16);
    u.fs0 = (int32_t)(c.fs01 & 0xffffu); u.fs1 = (int32_t)(c.fs01 >> 16);
    u.fs2 = (int32_t)(c.fs23 & 0xffffu); u.fs3 = (int32_t)(c.fs23 >> 16);
    u.low0 = (int32_t)(c.low01 & 0xffffu); u.low1 = (int32_t)(c.low01 >> 16);
    u.low2 = (int32_t)(c.low23 & 0xffffu); u.low3 = (int32_t)(c.low23 >> 16);
    u.pir0 = c.pir0; u.pir1 = c.pir1; u.pir2 = c.pir2; u.pir3 = c.pir3;
    u.bq_hi = c.bq_hi; u.mq_hi = c.mq_hi; u.bq_lo = c.bq_lo; u.mq_lo = c.mq_lo;
    return u;
}

// soft-clip evidence per category (plain, ctx, indel) x side (L, R): reads
// with mapq >= -q (h) and all reads (n); packed as h | n << 16 under the same
// bound as PackedCounts
template <bool PK>
struct ClipCounts {
    int32_t h[6], n[6];
    __device__ __forceinline__ void add(int k, int hv) { h[k] += hv; n[k] += 1; }
    __device__ __forceinline__ int32_t hi(int k) const { return h[k]; }
    __device__ __forceinline__ int32_t all(int k) const { return n[k]; }
};
template <>
struct ClipCounts<true> {
    uint32_t v[6];
    __device__ __forceinline__ void add(int k, int hv) { v[k] += (uint32_t)hv + 65536u; }
    __device__ __forceinline__ int32_t hi(int k) const { return (int32_t)(v[k] & 0xffffu); }
    __device__ __forceinline__ int32_t all(int k) const { return (int32_t)(v[k] >> 16); }
};

// bases matching the reference base of the lane (the common case), counted
// without selecting a counter by base code; folded into LaneCounts at the end
struct MatchCounts {
    int32_t cnt, fs, pir, low;
};

// 4-bit BAM code -> index into "ACGT" (A=1, C=2, G=4, T=8), 4 for anything else
__device__ __forceinline__ int acgt_code(int s4) {
    return (s4 != 0 && (s4 & (s4 - 1)) == 0) ? __builtin_ctz((unsigned)s4) : 4;
}

// The read-name slots of one position (GROM.c:6805-6824): the first empty
// slot takes the name (names >= 50 chars are never stored, id 0); a slot
// holding the name marks the base as seen.  Slots fill from 0 and are never
// emptied while the position is open, so "first empty" is the fill count.
//
// RegSlots: NS slots in registers (-n <= NS), written with selects so they
// stay in registers; the kernel is built for NS = 4, 8, 16, 32.
template <int NS>
struct RegSlots {
    uint32_t s[NS];
    __device__ __forceinline__ void reset() {
#pragma unroll
        for (int k = 0; k < NS; k++) s[k] = 0;
    }
    __device__ __forceinline__ bool probe(uint32_t nid, int min_snv, bool on = true) {
        bool done = !on, found = false;
#pragma unroll
        for (int k = 0; k < NS; k++) {
            const bool active = !done && k < min_snv;
            const bool empty = active && s[k] == 0;
            const bool match = active && !empty && s[k] == nid;
            s[k] = (empty && nid != 0) ? nid : s[k];
            found = found || match;
            done = done || empty || match;
        }
        return found;
    }
};

// MemSlots: any -n.  The slots live in global scratch, [slot][lane] per
// workgroup (one column per position, stride GROM_TILE, so a wave's probes
// are coalesced); the fill count is a register.  Only mismatching bases with
// a high-quality read probe the slots (<1% of visits), so the L2 round trips
// are off the common path.
struct MemSlots {
    uint32_t *col;
    int nf;
    __device__ __forceinline__ void reset() { nf = 0; }
    __device__ __forceinline__ bool probe(uint32_t nid, int min_snv, bool on = true) {
        if (!on) return false;
        const int lim = min(nf, min_snv);
        for (int k = 0; k < lim; k++)
            if (col[(size_t)k * TG] == nid) return true;  // stored ids are never 0
        if (nf < min_snv && nid != 0) {
            col[(size_t)nf * TG] = nid;
            nf++;
        }
        return false;
    }
};

// one aligned base of a read at this lane's position: the SNV tally body of
// GROM.c:6800-6992 (high-quality branch with read-name slots) and
// GROM.c:6995-7040 (low-quality branch).  rb4 is the 4-bit code whose
// character (bam_nt16_rev_table) equals the reference base, or 16 if none, so
// `s4 == rb4` is the reference's `ref != read base` test negated; mv says the
// reference base is one of ACGT.
template <class SLOTS, class CNT>
__device__ __forceinline__ void tally_base(CNT &c, MatchCounts &m, SLOTS &slot,
                                           int min_snv, bool hq, bool mv, int q, int s4, int rb4, bool fwd, int qi,
                                           int lseq_mod, int mq, uint32_t nid) {
    if (s4 == rb4) {
        const bool h = hq && mv, l = !hq && mv;
        m.cnt += h ? 1 : 0;
        m.fs += (h && fwd) ? 1 : 0;
        m.pir += h ? (fwd ? qi : lseq_mod - qi) : 0;
        m.low += l ? 1 : 0;
        c.bq_hi += h ? q : 0;
        c.mq_hi += h ? mq : 0;
        c.bq_lo += l ? q : 0;
        c.mq_lo += l ? mq : 0;
        return;
    }
    const int code = acgt_code(s4);
    bool count = hq && code < 4;
    if (hq) count = count && !slot.probe(nid, min_snv);
    const bool low = !hq && code < 4;
    const int32_t ch = count ? 1 : 0, cl = low ? 1 : 0;
    // mismatches add the offset on both strands (GROM.c:6896)
    add_codes(c, code, ch, fwd ? ch : 0, count ? qi : 0, cl);
    c.bq_hi += count ? q : 0;
    c.mq_hi += count ? mq : 0;
    c.bq_lo += low ? q : 0;
    c.mq_lo += low ? mq : 0;
}

// a mismatching base of the fast path (the second half of tally_base),
// predicated by `on` instead of branched on, so a wave with any mismatching
// lane runs it once for all lanes
template <class SLOTS, class CNT>
__device__ __forceinline__ void tally_mismatch(CNT &c, SLOTS &slot, bool on, int min_snv, bool hq, int q, int s4,
                                               bool fwd, int qi, int mq, uint32_t nid) {
    const int code = acgt_code(s4);
    const bool probe_on = on && hq;
    const bool found = slot.probe(nid, min_snv, probe_on);
    const bool count = probe_on && code < 4 && !found;
    const bool low = on && !hq && code < 4;
    const int32_t ch = count ? 1 : 0, cl = low ? 1 : 0;
    add_codes(c, code, ch, fwd ? ch : 0, count ? qi : 0, cl);  // GROM.c:6896
    c.bq_hi += count ? q : 0;
    c.mq_hi += count ? mq : 0;
    c.bq_lo += low ? q : 0;
    c.mq_lo += low ? mq : 0;
}

// lane i's value of v, as a wave-uniform (scalar) value
__device__ __forceinline__ uint32_t lane_get(uint32_t v, int i) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, i);
}

// lane j's registers: read g + j of the chunk
struct GroupRegs {
    uint32_t p0, lq, nid, cb, nf, mk, bo, cw0;
};

// the scalar view of read g + i
struct ReadView {
    int32_t p0, lq, bo;  // bo: base offset relative to the staged window
    uint32_t cw0, ncig, fl, mq, mkf, nid, cb;
    int i;
};

__device__ __forceinline__ ReadView view_of(const GroupRegs &G, int i) {
    ReadView v;
    v.i = i;
    v.p0 = (int32_t)lane_get(G.p0, i);
    v.lq = (int32_t)lane_get(G.lq, i);
    v.bo = (int32_t)lane_get(G.bo, i);
    v.cw0 = lane_get(G.cw0, i);
    const uint32_t nf = lane_get(G.nf, i);
    v.ncig = nf & 0xffffu;
    v.fl = nf >> 16;
    v.mkf = lane_get(G.mk, i);
    v.mq = v.mkf & 255u;
    v.nid = lane_get(G.nid, i);
    v.cb = lane_get(G.cb, i);
    return v;
}

__device__ __forceinline__ bool fast_read(const ReadView &v) {
    const uint32_t op = v.cw0 & 15u;
    return v.ncig == 1 && (op == 0 || op == 7 || op == 8);
}

// Byte b of a staged LDS array, read as its whole dword and shifted: lanes
// of a wave look up consecutive bytes of one read (consecutive positions),
// and whole-dword reads of one address broadcast, where byte reads of
// neighbouring bytes of a dword are told apart by address (GROM_LDS_BYTE=1:
// the byte reads, for A/B)
__device__ __forceinline__ uint32_t lds_byte(const uint32_t *w, int32_t b) {
#if defined(GROM_LDS_BYTE) && GROM_LDS_BYTE
    return reinterpret_cast<const uint8_t *>(w)[b];
#else
    return (w[b >> 2] >> ((b & 3) << 3)) & 0xffu;
#endif
}

// quality byte and 4-bit base (BAM nibble order) of staged base `rel`
// (relative to the window start, which is a multiple of 16)
__device__ __forceinline__ void staged_base(const uint32_t *lq, const uint32_t *ls, int32_t soff, int32_t rel,
                                            uint32_t &q, uint32_t &sbyte) {
    q = lds_byte(lq, rel);
    sbyte = lds_byte(ls, soff + (rel >> 1));
}

// The outputs of position x (one lane per position; every lane of the
// workgroup calls this, it has barriers): caf arrays, flush depth sums, the
// debug counters, the SNV test (GROM.c:11096-11199) and the tile's candidate
// run.
__device__ __forceinline__ void pile_emit(const grom_scan_args &a, const char *__restrict__ ref, const PileOut &O,
                                          const double *__restrict__ mq_tab, const double *__restrict__ hez_tab,
                                          TileTail &T_, int64_t tile, int32_t x, char rb, bool evals,
                                          const LaneCounts &c, int32_t rd, int32_t caf_mq, int32_t caf_rd,
                                          int32_t caf_low, const int32_t (&sch)[6], const int32_t (&scn)[6]) {
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int32_t clen = (int32_t)a.chr_len;
    // soft-clip counters in the reference's order (GC_SC_LEFT..GC_INDEL_SC+4)
    int32_t sc[15];
    sc[0] = 6 * sch[0]; sc[1] = 6 * sch[1]; sc[2] = scn[0]; sc[3] = scn[1]; sc[4] = scn[0] + scn[1];
    sc[5] = 6 * sch[2]; sc[6] = 6 * sch[3]; sc[7] = scn[2]; sc[8] = scn[3]; sc[9] = scn[2] + scn[3];
    sc[10] = 6 * sch[4]; sc[11] = 6 * sch[5]; sc[12] = scn[4]; sc[13] = scn[5]; sc[14] = scn[4] + scn[5];

    // ---- outputs of this position ----
    unsigned long long fsum = 0, fcnt = 0;
    if (x < clen) {
        O.caf_mq[x] = caf_mq;
        O.caf_rd[x] = caf_rd;
        O.caf_low[x] = caf_low;
        if (x < a.flush_end && rb != 'N') {  // SNV flush depth sums, GROM.c:15066-15073
            fsum = (unsigned long long)((int64_t)caf_rd + caf_low);
            fcnt = 1;
        }
    }
    int best = -1;  // candidate base of this position, if any
    float best_ratio = 0.f;
    if (evals) {
        const int32_t total = c.snv0 + c.snv1 + c.snv2 + c.snv3;
        const int32_t rc_all = total + c.low0 + c.low1 + c.low2 + c.low3;
        const int32_t bq_all = c.bq_hi + c.bq_lo, mq_all = c.mq_hi + c.mq_lo;
        if (O.dbg) {
            int32_t *d = O.dbg + (size_t)(x - a.eval_lo) * GC_COUNT;
            d[GC_POS] = x;
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
            d[GC_RD] = rd + (O.rd_add ? O.rd_add[x] : 0);  // + the breakpoint ranges (row A9)
#pragma unroll
            for (int k = 0; k < 15; k++) d[GC_SC_LEFT + k] = sc[k];
        }
        // SNV test, GROM.c:11096-11199
        // (the divisions only where some non-reference base reaches -n: the
        // tests are pure, so skipping them elsewhere changes no result)
        const int32_t snv[4] = {c.snv0, c.snv1, c.snv2, c.snv3};
        bool any = false;
#pragma unroll
        for (int k = 0; k < 4; k++) any = any || (rb != c_acgt[k] && snv[k] >= a.min_snv);
        if (any && rd + sc[14] > 0 && rb != 'N') {
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
        }
    }
    // ---- breakpoint-test context (row A10, sv.hip): positions the SV fold
    // marked, and every position with soft-clip evidence (whose absence then
    // means zero counters) ----
    if (O.sv_ctx) {
        const bool want = evals && (((O.sv_bits[x >> 5] >> (x & 31)) & 1u) || sc[0] || sc[1] || sc[2] || sc[3]);
        const uint64_t wm = __ballot(want);
        if (wm) {
            uint32_t wb = 0;
            if (lane == 0) wb = atomicAdd(O.n_sv_ctx, (uint32_t)__popcll(wm));
            wb = __shfl(wb, 0, 64);
            if (want) {
                const uint32_t k = wb + (uint32_t)__popcll(wm & ((1ull << lane) - 1));
                if (k < O.sv_ctx_cap) {
                    grom_sv_ctx r;
                    r.pos = x;
                    r.rd = rd;
                    r.sc_rd = sc[4];
                    r.indel_sc_rd = sc[14];
                    r.sc_left = sc[0];
                    r.sc_right = sc[1];
                    r.sc_left_rd = sc[2];
                    r.sc_right_rd = sc[3];
                    r.indel_sc_left = sc[10];
                    r.indel_sc_right = sc[11];
                    r.snv_all = c.snv0 + c.snv1 + c.snv2 + c.snv3 + c.low0 + c.low1 + c.low2 + c.low3;
                    r.pad = 0;
                    O.sv_ctx[k] = r;
                }
            }
        }
    }
    // ---- block totals: flush depth sums and the tile's candidate run ----
    // Candidates of a tile are written contiguously in position order at a
    // base taken with one atomic per tile; k_run_* put the runs in tile order.
    const uint64_t cmask = __ballot(best >= 0);
    for (int o = 32; o > 0; o >>= 1) {
        fsum += __shfl_xor(fsum, o, 64);
        fcnt += __shfl_xor(fcnt, o, 64);
    }
    if (lane == 0) {
        T_.red[wave][0] = fsum;
        T_.red[wave][1] = fcnt;
        T_.wcnt[wave] = (uint32_t)__popcll(cmask);
    }
    __syncthreads();
    if (tid == 0) {
        unsigned long long s = 0, cc = 0;
        uint32_t nc = 0;
        for (int w = 0; w < TG / 64; w++) {
            s += T_.red[w][0];
            cc += T_.red[w][1];
            nc += T_.wcnt[w];
        }
        // per-tile flush sums, reduced by k_flush_reduce (one global atomic
        // per tile on a single address serialises the whole grid)
        O.flush_part[2 * tile] = s;
        O.flush_part[2 * tile + 1] = cc;
        const uint32_t base = nc ? atomicAdd(O.n_cands, nc) : 0u;
        T_.cbase = base;
        O.run_base[tile] = base;
        O.run_cnt[tile] = nc;
    }
    __syncthreads();
    if (best >= 0) {
        uint32_t ci = T_.cbase + (uint32_t)__popcll(cmask & ((1ull << lane) - 1));
        for (int w = 0; w < wave; w++) ci += T_.wcnt[w];
        if (ci < O.cand_cap) {  // else the host sees n_cands > cap and re-runs with room
            const int32_t total = c.snv0 + c.snv1 + c.snv2 + c.snv3;
            grom_snv_cand cd;
            cd.pos = x;
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
            cd.bq_all = c.bq_hi + c.bq_lo;
            cd.mq = c.mq_hi;
            cd.mq_all = c.mq_hi + c.mq_lo;
            cd.bq_rc = total;
            cd.mq_rc = total;
            cd.rc_all = total + c.low0 + c.low1 + c.low2 + c.low3;
            cd.pad1 = 0;
            O.cands[ci] = cd;
        }
    }
}


// DIFFED reads looked up per step of the fast path (their LDS reads in flight together)
#ifndef GROM_FAST_READS
#define GROM_FAST_READS 2
#endif
#define FR GROM_FAST_READS

// occupancy target: 5 waves per SIMD (a 96-register budget) measured faster
// than the unconstrained 4 despite a few spills; GROM_WAVES_PER_EU overrides
#ifndef GROM_WAVES_PER_EU
#define GROM_WAVES_PER_EU 5
#endif
#define GROM_OCCUPANCY __attribute__((amdgpu_waves_per_eu(GROM_WAVES_PER_EU)))

// SLOTS: the read-name slots of the lane's position (RegSlots<NS> with
// NS >= -n: fewer slots, fewer VGPRs; MemSlots for any -n).  PK: packed
// 16-bit counters (tiles of at most PACK_MAX_READS reads).
template <bool PK, class SLOTS>
__device__ __forceinline__ void scan_tile_gather(ScanLds &L, SLOTS &slot, int64_t tile, const grom_scan_args &a,
                                                 const char *__restrict__ ref, const ReadArrays &R,
                                                 const ReadMeta *__restrict__ meta, const int32_t *__restrict__ tile_lo,
                                                 const int32_t *__restrict__ tile_hi, const PileOut &O,
                                                 const double *__restrict__ mq_tab, const double *__restrict__ hez_tab) {
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int32_t clen = (int32_t)a.chr_len;
    const int32_t t0 = (int32_t)(tile * TG);
    const int32_t x = t0 + tid;         // this lane's reference position
    const int32_t x0 = t0 + wave * 64;  // first position of this wave
#ifdef GROM_PROF_NOREADS  // timing probe only: the tile's fixed work
    const int32_t r0 = tile_lo[tile], r1 = r0;
#else
    const int32_t r0 = tile_lo[tile], r1 = tile_hi[tile];
#endif
    L.ref[tid] = (x < clen) ? upcase(ref[x]) : 'N';
    const char rb = L.ref[tid];
    int rb4 = 16;  // the 4-bit code printed as rb (GROM compares characters)
    for (int k = 0; k < 16; k++) rb4 = (c_nt16[k] == rb) ? k : rb4;
    const int rcode = (rb4 < 16) ? acgt_code(rb4) : 4;
    const bool mv = rcode < 4;
    const bool evals = x >= a.eval_lo && x <= a.eval_hi;  // GROM.c:11086, 5842
    // the fast path's lane position: outside the evaluated range no read's
    // offset (x - pos, unsigned) falls inside it, so no base is tallied
    const int32_t xe = evals ? x : (int32_t)(INT32_MIN / 2);
    const uint32_t *lq32 = reinterpret_cast<const uint32_t *>(L.qual);
    const uint32_t *ls32 = reinterpret_cast<const uint32_t *>(L.seq);

    typename std::conditional<PK, PackedCounts, LaneCounts>::type c = {};
    MatchCounts mc = {0, 0, 0, 0};
    int32_t rd = 0, caf_mq = 0, caf_rd = 0, caf_low = 0;
    // soft-clip evidence per category (plain, ctx, indel) x side (L, R):
    // reads with mapq >= -q (each adds 6, GROM.c:5829-5836) and all reads
    ClipCounts<PK> sc = {};
    slot.reset();

    const uint4 *gq4 = reinterpret_cast<const uint4 *>(R.qual);
    const uint4 *gs4 = reinterpret_cast<const uint4 *>(R.seq);

    const bool use_diff = r1 - r0 <= DIFF_MAX_READS;  // workgroup-uniform
    L.dmq[tid] = 0;
    L.dcnt[tid] = 0;
    if (tid == 0) { L.dmq[TG] = 0; L.dcnt[TG] = 0; }

    int32_t c0 = r0;
    while (c0 < r1) {
        const int32_t m = min(RCHUNK, r1 - c0);
        __syncthreads();  // previous chunk fully consumed
        if (tid == 0) L.m2 = 0;
        __syncthreads();
        // ---- stage the packed records; find the prefix within the budgets ----
        if (tid < m) {
            const ReadMeta rm = meta[c0 + tid];
            meta_st(L, tid, rm);
            const ReadMeta f = meta[c0];
            const int64_t bo = ((int64_t)rm.c.x << 32) | rm.b.w, b0 = ((int64_t)f.c.x << 32) | f.b.w;
            const uint32_t ce = rm.b.x + (rm.b.y & 0xffffu);
            // reads are contiguous in cigar[] and in qual/seq, so this holds
            // for a prefix of the chunk
            if (bo + (int32_t)rm.a.z - b0 <= (int64_t)QBYTES - 64 && ce - f.b.x <= CIGCAP) atomicMax(&L.m2, tid + 1);
        }
        __syncthreads();
        int32_t m2 = min(L.m2, m);
        const bool staged = m2 > 0;
        if (!staged) m2 = 1;  // one oversized read: served from global memory
        const ReadMeta first = meta_ld(L, 0), last = meta_ld(L, m2 - 1);
        const int64_t b0 = ((int64_t)first.c.x << 32) | first.b.w;
        const int64_t bend = (((int64_t)last.c.x << 32) | last.b.w) + (int32_t)last.a.z;
        const uint32_t cf = first.b.x, cl = last.b.x + (last.b.y & 0xffffu);
        // ---- stage CIGAR words, qualities and packed bases ----
        const int64_t qv0 = b0 >> 4, sv0 = b0 >> 5;  // first 16-byte slot of each
        if (staged) {
            const int64_t qv1 = min((bend + 15) >> 4, qv0 + (int64_t)QV);
            const int64_t sv1 = min((((bend + 1) >> 1) + 15) >> 4, sv0 + (int64_t)SV);
            uint4 vq[QLOADS], vs[SLOADS];
            // clamped indices: every load is unconditional and all are in
            // flight before the first LDS store
#pragma unroll
            for (int k = 0; k < QLOADS; k++) vq[k] = gq4[min(qv0 + tid + k * TG, qv1 - 1)];
#pragma unroll
            for (int k = 0; k < SLOADS; k++) vs[k] = gs4[min(sv0 + tid + k * TG, sv1 - 1)];
            const uint32_t nc = min(cl - cf, (uint32_t)CIGCAP);
            for (uint32_t k = tid; k < nc; k += TG) L.cig[k] = R.cigar[cf + k];
#pragma unroll
            for (int k = 0; k < QLOADS; k++) {
                const int64_t w = qv0 + tid + k * TG;
                L.qual[w < qv1 ? (int)(w - qv0) : QV] = vq[k];  // unconditional: the loads stay in flight together
            }
#pragma unroll
            for (int k = 0; k < SLOADS; k++) {
                const int64_t w = sv0 + tid + k * TG;
                L.seq[w < sv1 ? (int)(w - sv0) : SV] = vs[k];
            }
        }
        // single-op staged reads: their caf and physical-depth intervals go
        // to the tile's difference arrays (one lane per read), so the fold
        // below skips those per-lane updates (GROM.c:6605-6671, 7173-7181)
        // Reads that start before the tile all add at index 0 and those that
        // end past it all subtract at TG, which the scan never reads: one
        // wave-summed add at 0 instead of up to a chunk of same-address
        // atomics (most of the kernel's LDS bank-conflict cycles), and no
        // update at TG.
        if (use_diff && staged) {
            int32_t mq0 = 0;
            uint32_t inc0 = 0;
            if (tid < m2) {
                const uint32_t bz = L.meta[META_W * tid + 6];
                const int32_t p0 = (int32_t)L.meta[META_W * tid], len = (int32_t)L.meta[META_W * tid + 2];
                const uint32_t mq = bz & 255u;
                if (bz & MK_FAST) {
                    const int32_t lo = max(p0, t0) - t0, hi = min(p0 + len, t0 + TG) - t0;
                    if (lo < hi) {
                        const uint32_t inc = ((int32_t)mq >= a.rd_min_mapq) ? 1u : 65536u;  // signed, as the oracle
                        if (lo > 0) {
                            atomicAdd(&L.dmq[lo], (int32_t)mq);
                            atomicAdd(&L.dcnt[lo], inc);
                        } else {
                            mq0 = (int32_t)mq;
                            inc0 = inc;
                        }
                        if (hi < TG) {
                            atomicSub(&L.dmq[hi], (int32_t)mq);
                            atomicSub(&L.dcnt[hi], inc);
                        }
                    }
                    L.meta[META_W * tid + 6] = bz | DIFFED;  // read by the fold, written only here
                }
            }
            if (__ballot(mq0 != 0 || inc0 != 0)) {  // (wave-uniform)
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    mq0 += __shfl_xor(mq0, o, 64);
                    inc0 += (uint32_t)__shfl_xor((int)inc0, o, 64);
                }
                if (lane == 0) {
                    atomicAdd(&L.dmq[0], mq0);
                    atomicAdd(&L.dcnt[0], inc0);
                }
            }
        }
        __syncthreads();
        // window: base qb0 + rel has its quality at L.qual byte rel and its
        // packed base at L.seq byte soff + (rel >> 1) (qb0 is a multiple of 16)
        const int64_t qb0 = qv0 << 4;
        const int32_t soff = (int32_t)((qb0 >> 1) - (sv0 << 4));

        for (int g = 0; g < m2; g += 64) {
            // ---- lane j holds read g + j of the chunk ----
            const int j = g + lane;
            GroupRegs G = {0, 0, 0, 0, 0, 0, 0, 0};
            bool rel = false;
            if (j < m2) {
                const ReadMeta rm = meta_ld(L, j);
                G.p0 = rm.a.x;
                G.lq = rm.a.z;
                G.nid = rm.a.w;
                G.cb = rm.b.x;
                G.nf = rm.b.y;
                G.mk = rm.b.z;
                G.bo = (uint32_t)((((int64_t)rm.c.x << 32) | rm.b.w) - qb0);
                // DIFFED reads sit in the staged window (offset and length
                // below QBYTES): both travel in one word to the fast path
                if (rm.b.z & DIFFED) G.bo |= rm.a.z << 16;
                G.cw0 = (staged && (rm.b.y & 0xffffu) != 0) ? L.cig[rm.b.x - cf] : 0u;
                // touches [x0, x0+64)?  contributions span [pos-1 (left clip), ext)
                rel = ((rm.b.z >> 8) & 255u) != 0 &&  // -M duplicate (GROM.c:6590)
                      (int32_t)rm.a.x - 1 <= x0 + 63 && (int32_t)rm.a.y > x0;
            }
            uint64_t mask = __ballot(rel);
            if (!mask) continue;
            const uint64_t dmask = __ballot(j < m2 && (G.mk & DIFFED));
            while (mask) {
                // ---- fast path: the next one or two reads in order are
                // DIFFED (one aligned block of l_qseq bases): each lane only
                // looks up the read's base at its position.  Both pairs of
                // LDS reads are issued before either base is tallied; the
                // order-free matched-base sums are added first, then the
                // mismatching bases in read order (the read-name slots are
                // order-dependent, GROM.c:6805-6824) ----
                const uint64_t b0 = mask & (0ull - mask);
                if (b0 & dmask) {
                    // the run of up to FR consecutive DIFFED reads at the front
                    // of the mask (wave-uniform); empty slots tally nothing
                    int32_t fp[FR], fl[FR], fb[FR], fi[FR];
                    uint32_t fm[FR];
                    uint64_t mm = mask;
                    bool run = true;
#pragma unroll
                    for (int k = 0; k < FR; k++) {
                        const uint64_t b = mm & (0ull - mm);
                        run = run && (b & dmask) != 0;
                        mm = run ? (mm ^ b) : mm;
                        const int i = run ? __builtin_ctzll(b) : __builtin_ctzll(b0);
                        fp[k] = (int32_t)lane_get(G.p0, i);
                        const uint32_t bl = lane_get(G.bo, i);
                        fl[k] = run ? (int32_t)(bl >> 16) : 0;
                        fb[k] = (int32_t)(bl & 0xffffu);
                        fi[k] = i;
                        fm[k] = lane_get(G.mk, i);
                    }
                    mask = mm;
#ifdef GROM_PROF_NOFAST  // timing probe only: the fast reads are skipped
                    continue;
#endif
                    uint32_t fq[FR], fs4[FR], fdx[FR];
                    bool fhit[FR];
#pragma unroll
                    for (int k = 0; k < FR; k++) {
                        fdx[k] = (uint32_t)(xe - fp[k]);
                        fhit[k] = fdx[k] < (uint32_t)fl[k];
                        const int32_t r = fhit[k] ? fb[k] + (int32_t)fdx[k] : 0;
                        fq[k] = lds_byte(lq32, r);
                        fs4[k] = lds_byte(ls32, soff + (r >> 1)) >> ((((uint32_t)r & 1u) ^ 1u) << 2);
                    }
#pragma unroll
                    for (int k = 0; k < FR; k++) {
                        const int s4 = (int)(fs4[k] & 15u), q = (int)fq[k], mq = (int)(fm[k] & 255u);
                        const bool fwd = !(fm[k] & MK_REV);
                        const bool hq = (fm[k] & MK_HQ) && q >= a.min_base_qual;
                        const bool mt = fhit[k] && s4 == rb4 && mv;
                        const bool h = mt && hq, l = mt && !hq;
                        mc.cnt += h ? 1 : 0;
                        mc.fs += (h && fwd) ? 1 : 0;
                        mc.pir += h ? (fwd ? (int32_t)fdx[k] : fl[k] - (int32_t)fdx[k]) : 0;
                        mc.low += l ? 1 : 0;
                        c.bq_hi += h ? q : 0;
                        c.mq_hi += h ? mq : 0;
                        c.bq_lo += l ? q : 0;
                        c.mq_lo += l ? mq : 0;
                    }
                    bool anymm = false;
#pragma unroll
                    for (int k = 0; k < FR; k++) anymm = anymm || (fhit[k] && (int)(fs4[k] & 15u) != rb4);
                    if (__ballot(anymm)) {  // wave-uniform: predicated for every lane
#pragma unroll
                        for (int k = 0; k < FR; k++) {
                            const int s4 = (int)(fs4[k] & 15u), q = (int)fq[k], mq = (int)(fm[k] & 255u);
                            tally_mismatch(c, slot, fhit[k] && s4 != rb4, a.min_snv,
                                           (fm[k] & MK_HQ) && q >= a.min_base_qual, q, s4, !(fm[k] & MK_REV),
                                           (int)fdx[k], mq, lane_get(G.nid, fi[k]));
                        }
                    }
                    continue;
                }
#ifdef GROM_PROF_NOGENERAL  // timing probe only: skip the reads off the fast path
                mask &= mask - 1;
                continue;
#endif
                const ReadView u = view_of(G, __builtin_ctzll(mask));
                mask &= mask - 1;
                const int32_t p0 = u.p0;
                const int mq = (int)u.mq;
                const bool fwd = !(u.fl & 0x10);
                const bool hq_read = mq >= a.min_mapq;
                const bool pos_ok = p0 >= 0 && p0 < clen;
                const bool fastr = staged && fast_read(u);  // wave-uniform
                // the read's base at this lane's position, if the SNV tally
                // takes one: read offset and the hard-clip-extended length
                int32_t hit_qi = -1, hit_lsm = u.lq;
                if (fastr) {
                    // ---- fast path: a single M/=/X op ----
                    const int32_t len = (int32_t)(u.cw0 >> 4);
                    const uint32_t dx = (uint32_t)(x - p0);
                    if (!(u.mkf & DIFFED)) {  // wave-uniform
                        if (p0 >= 0 && len < clen - p0 && dx < (uint32_t)len) {
                            caf_mq += mq;
                            caf_rd += (mq >= a.rd_min_mapq) ? 1 : 0;
                            caf_low += (mq >= a.rd_min_mapq) ? 0 : 1;
                        }
                        rd += (dx < (uint32_t)u.lq) ? 1 : 0;  // E = pos + l_qseq
                    }
                    if (pos_ok && evals && dx < (uint32_t)min(len, clen - p0)) hit_qi = (int32_t)dx;
                } else {
                    // ---- general CIGAR walk (rare: int64 arithmetic) ----
                    const uint32_t cb = u.cb, ce = u.cb + u.ncig;
                    int snv_base = 0, srb = 0, lseq_mod = u.lq, eai = 0;
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
                            if (caf_pos >= 0 && caf_pos + len < clen && x >= caf_pos && x < caf_pos + len) {
                                caf_mq += mq;
                                if (mq >= a.rd_min_mapq) caf_rd += 1;
                                else caf_low += 1;
                            }
                            caf_pos += len;
                            if (!in_cap) continue;
                            if (pos_ok) {
                                // SNV tally, GROM.c:6769-7059: blocks advance
                                // monotonically, so at most one covers x
                                const int64_t xb = (int64_t)p0 + srb;
                                const int loop_end = (xb + len >= clen) ? (int)(clen - p0) : len;
                                if (evals && x >= xb && x < xb + loop_end) {
                                    hit_qi = snv_base + (int)(x - xb);
                                    hit_lsm = lseq_mod;
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
                    const bool at_l = start_adj >= a.sc_min && x == p0 - 1;
                    const bool at_r = end_adj >= a.sc_min && x == E;
                    if (evals && (at_l || at_r)) {
                        const uint32_t *mw = L.meta + META_W * (g + u.i) + 8;
                        const uint4 mate = make_uint4(mw[0], mw[1], mw[2], mw[3]);
                        const uint32_t fl = u.fl;
                        const bool paired = fl & 0x1, munmap = fl & 0x8, rev = fl & 0x10;
                        const bool same_chr = (int32_t)mate.y == a.chr_tid;
                        const int32_t mp = (int32_t)mate.z, tl = (int32_t)mate.w;
                        const int h = hq_read ? 1 : 0;
                        // category: plain (mate unmapped / proper orientation),
                        // ctx (mate on another chromosome), indel (close mate)
                        if (at_l) {
                            if (!paired || (!rev && (munmap || (!munmap && same_chr && mp > p0)))) {
                                sc.add(0, h);
                            }
                            if (paired && !munmap && !same_chr && rev) sc.add(2, h);
                            if (paired && !munmap && same_chr && rev && abs(tl) <= a.insert_max && mp < p0) {
                                sc.add(4, h);
                            }
                        }
                        if (at_r) {
                            if (!paired || (rev && (munmap || (!munmap && same_chr && mp < p0)))) {
                                sc.add(1, h);
                            }
                            if (paired && !munmap && !same_chr && !rev) sc.add(3, h);
                            if (paired && !munmap && same_chr && !rev && abs(tl) <= a.insert_max && mp > p0) {
                                sc.add(5, h);
                            }
                        }
                    }
                }
                // ---- SNV tally of the base at this lane (one per read) ----
                if (hit_qi >= 0) {
                    int q = 0, s4 = 15;
                    if (hit_qi < u.lq) {
                        uint32_t qb, sbv;
                        int odd = (u.bo + hit_qi) & 1;
                        {
                            if (staged) {
                                staged_base(lq32, ls32, soff, u.bo + hit_qi, qb, sbv);
                            } else {
                                const int64_t nib = qb0 + u.bo + (int64_t)hit_qi;
                                qb = R.qual[nib];
                                sbv = R.seq[nib >> 1];
                                odd = (int)(nib & 1);
                            }
                        }
                        q = (int)qb;
                        s4 = (int)((sbv >> ((odd ^ 1) << 2)) & 15u);
                    }
                    tally_base(c, mc, slot, a.min_snv, hq_read && q >= a.min_base_qual, mv, q, s4, rb4, fwd, hit_qi,
                               hit_lsm, mq, u.nid);
                }
            }
        }
        c0 += m2;
    }

    // the difference arrays: an inclusive scan over the tile (wave scans,
    // then the earlier waves' totals)
    if (use_diff) {
        __syncthreads();
        int32_t vm = L.dmq[tid];
        uint32_t vc = L.dcnt[tid];
        for (int d = 1; d < 64; d <<= 1) {
            const int32_t tm = __shfl_up(vm, d, 64);
            const uint32_t tc = __shfl_up(vc, d, 64);
            if (lane >= d) { vm += tm; vc += tc; }
        }
        __syncthreads();  // every lane has read its entry
        if (lane == 63) { L.dmq[wave] = vm; L.dcnt[wave] = vc; }
        __syncthreads();
        for (int w = 0; w < wave; w++) { vm += L.dmq[w]; vc += L.dcnt[w]; }
        caf_mq += vm;
        caf_rd += (int32_t)(vc & 0xffffu);
        caf_low += (int32_t)(vc >> 16);
        rd += (int32_t)(vc & 0xffffu) + (int32_t)(vc >> 16);
    }

    // matched bases go to the reference base's counters
    add_codes(c, rcode, mc.cnt, mc.fs, mc.pir, mc.low);
    int32_t sch[6], scn[6];
#pragma unroll
    for (int k = 0; k < 6; k++) { sch[k] = sc.hi(k); scn[k] = sc.all(k); }

    pile_emit(a, ref, O, mq_tab, hez_tab, L.tail, tile, x, rb, evals, unpack(c), rd, caf_mq, caf_rd, caf_low, sch, scn);
}

// every tile of the chromosome (GROM_PILEUP=gather)
template <int NS>
__global__ __launch_bounds__(TG) GROM_OCCUPANCY void k_scan_tile(grom_scan_args a, const char *__restrict__ ref, ReadArrays R,
                                                  const ReadMeta *__restrict__ meta,
                                                  const int32_t *__restrict__ tile_lo,
                                                  const int32_t *__restrict__ tile_hi, PileOut O,
                                                  const double *__restrict__ mq_tab,
                                                  const double *__restrict__ hez_tab, int64_t n_tiles,
                                                  uint32_t *__restrict__ heavy, int32_t pack_max) {
    __shared__ ScanLds L;
    // XCD-contiguous tile order (speed only; any mapping is correct)
    const int64_t per_xcd = (n_tiles + 7) / 8;
    const int64_t tile = (int64_t)(blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
    if (tile >= n_tiles) return;  // whole workgroup leaves together
    if (tile_hi[tile] - tile_lo[tile] > pack_max) {  // k_scan_tile_mem takes it (pack_max <= PACK_MAX_READS)
        if (threadIdx.x == 0) atomicOr(heavy, 1u);
        return;
    }
    RegSlots<NS> slot;
    scan_tile_gather<true>(L, slot, tile, a, ref, R, meta, tile_lo, tile_hi, O, mq_tab, hez_tab);
}

// -n above the register builds: a fixed grid of workgroups, each walking
// tiles blockIdx.x, blockIdx.x + gridDim.x, ... with its own slot columns in
// `slots` ([gridDim.x][min_snv][GROM_TILE] uint32, sized by the host), with
// 32-bit counters.  heavy_only: only the tiles k_scan_tile leaves (more than
// PACK_MAX_READS reads).
__global__ __launch_bounds__(TG) void k_scan_tile_mem(grom_scan_args a, const char *__restrict__ ref, ReadArrays R,
                                                     const ReadMeta *__restrict__ meta,
                                                     const int32_t *__restrict__ tile_lo,
                                                     const int32_t *__restrict__ tile_hi, PileOut O,
                                                     const double *__restrict__ mq_tab,
                                                     const double *__restrict__ hez_tab, int64_t n_tiles,
                                                     uint32_t *__restrict__ slots, int heavy_only,
                                                     const uint32_t *__restrict__ heavy, int32_t pack_max) {
    __shared__ ScanLds L;
    if (heavy_only && *heavy == 0) return;  // k_scan_tile left no tile (the usual case)
    MemSlots slot;
    slot.col = slots + (size_t)blockIdx.x * a.min_snv * TG + threadIdx.x;
    for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        if (heavy_only && tile_hi[tile] - tile_lo[tile] <= pack_max) continue;  // workgroup-uniform
        __syncthreads();  // the previous tile's LDS is no longer read
        scan_tile_gather<false>(L, slot, tile, a, ref, R, meta, tile_lo, tile_hi, O, mq_tab, hez_tab);
    }
}

// ---- candidate runs in tile order: exclusive scan of run_cnt, then gather ----
#define RUN_ITEMS 8
#define RUN_SEG (256 * RUN_ITEMS)

// exclusive scan of v over a 256-thread block; *total = block sum
__device__ __forceinline__ uint32_t block_scan_excl(uint32_t v, uint32_t *wsum, uint32_t *total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t inc = v;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(inc, d, 64);
        if (lane >= d) inc += t;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (int w = 0; w < 4; w++) {
        off += (w < wave) ? wsum[w] : 0u;
        tot += wsum[w];
    }
    __syncthreads();
    *total = tot;
    return off + inc - v;
}

// per RUN_SEG-tile segment: the number of candidates
__global__ __launch_bounds__(256) void k_run_sums(int64_t n_tiles, const uint32_t *__restrict__ cnt,
                                                  uint32_t *__restrict__ seg_sum) {
    __shared__ uint32_t wsum[4];
    const int64_t t0 = (int64_t)blockIdx.x * RUN_SEG + threadIdx.x * RUN_ITEMS;
    uint32_t s = 0;
    for (int k = 0; k < RUN_ITEMS; k++) s += (t0 + k < n_tiles) ? cnt[t0 + k] : 0u;
    uint32_t tot;
    (void)block_scan_excl(s, wsum, &tot);
    if (threadIdx.x == 0) seg_sum[blockIdx.x] = tot;
}

// exclusive scan of the segment sums (one block)
__global__ __launch_bounds__(256) void k_run_scan(int64_t n_seg, uint32_t *__restrict__ seg_sum) {
    __shared__ uint32_t wsum[4];
    uint32_t carry = 0;
    for (int64_t b = 0; b < n_seg; b += 256) {
        const int64_t i = b + threadIdx.x;
        const uint32_t v = (i < n_seg) ? seg_sum[i] : 0u;
        uint32_t tot;
        const uint32_t ex = block_scan_excl(v, wsum, &tot);
        if (i < n_seg) seg_sum[i] = carry + ex;
        carry += tot;
    }
}

// copy each tile's run to its place in position order
__global__ __launch_bounds__(256) void k_run_gather(int64_t n_tiles, const uint32_t *__restrict__ base,
                                                    const uint32_t *__restrict__ cnt,
                                                    const uint32_t *__restrict__ seg_off,
                                                    const grom_snv_cand *__restrict__ src,
                                                    grom_snv_cand *__restrict__ dst) {
    __shared__ uint32_t wsum[4];
    const int64_t t0 = (int64_t)blockIdx.x * RUN_SEG + threadIdx.x * RUN_ITEMS;
    uint32_t s = 0;
    for (int k = 0; k < RUN_ITEMS; k++) s += (t0 + k < n_tiles) ? cnt[t0 + k] : 0u;
    uint32_t tot;
    uint32_t o = seg_off[blockIdx.x] + block_scan_excl(s, wsum, &tot);
    for (int k = 0; k < RUN_ITEMS; k++) {
        if (t0 + k >= n_tiles) break;
        const uint32_t n = cnt[t0 + k], b = base[t0 + k];
        for (uint32_t j = 0; j < n; j++) dst[o + j] = src[b + j];
        o += n;
    }
}

