// inflate.h -- DEFLATE (RFC 1951) decoder for one BGZF block per lane.
//
// The reference reads its BAM through htslib's BGZF layer on the host
// (my_samread, GROM.c:981-992; bgzf_read inflates each <= 64 KiB block with
// zlib).  Here every BGZF block of a chromosome's compressed run is inflated on
// the GPU, one block per lane: a BAM's blocks are independent DEFLATE streams
// with their own Huffman trees, so a chromosome's 10^4-10^5 blocks fill the
// chip without any cross-lane work.
//
// The decoder is a flat state machine that takes one bounded STEP per loop
// trip -- a block header, or one symbol plus at most 16 bytes of a match --
// so the 64 lanes of a wave, each in its own block, stay in step: no lane
// waits for another's long match or for the end of another's DEFLATE block
// (a nested per-block/per-match loop makes the whole wave wait for its
// slowest lane at every level).  A match step is four 16-byte loads and four
// 16-byte stores (unaligned dwordx4; one wait for the loads per 64 bytes):
// the bytes past the match's end that the stores also write are garbage
// that this lane overwrites later, since a block's output is produced front
// to back; near the end of the block's output the step falls back to single
// bytes.  A match whose distance is below 64 copies its first distance bytes,
// then doubles the distance (the output is periodic with the distance, so any
// multiple of it is a valid source): 1, 2, 4, ..., 64, 64, ... bytes per step
// for a run of one byte.
//
// Per lane, the Huffman tables are canonical: for each code length l the
// left-justified end of its code range (lim[l]) and the offset from a code to
// its symbol's index in the sorted-symbol array (base[l]) sit in registers;
// the length of the code at the stream's front is the number of lim[l] at or
// below the next 15 bits (bit-reversed), found by one unrolled compare chain,
// and only the sorted symbols live in LDS, one byte each (plus a bit per
// literal/length entry for symbols >= 256), interleaved across the lanes a
// dword at a time so any per-lane index is bank-conflict free.  A dynamic
// header's run-length-coded code lengths are decoded twice -- once to count
// the lengths, once to place the symbols -- so they need no storage.  376
// bytes of LDS per lane: 6 waves of 64 blocks per CU.
//
// The same code is compiled for the host (LANES = 1, plain arrays) as the
// library's test twin (grom_inflate_selftest), checked against zlib on the CPU.
#pragma once
#include <stdint.h>

#if defined(__HIP_DEVICE_COMPILE__)
#define GI_KEEP(x) asm volatile("" : "+v"(x))
#else
#define GI_KEEP(x) (void)0
#endif
#if defined(__HIPCC__)
#define GI_FN __host__ __device__ __forceinline__
#define GI_UNROLL _Pragma("unroll")
#else
#define GI_FN static inline
#define GI_UNROLL _Pragma("GCC unroll 16")
#endif

// sorted-symbol tables per lane, in dwords of 4 one-byte cells: literal/length
// (288 cells), its >= 256 bitmap (288 bits), distance (32), code-length (19)
#define GI_T_LIT 0
#define GI_T_LITHI 72
#define GI_T_DIST 81
// GI_CLREG (a variant, off): the code-length code's 19 sorted symbols in
// four registers of the header state (5 bits each) instead of 5 LDS rows, so
// that 89 dwords per lane let 7 waves of 64 blocks share a CU's LDS instead
// of 6: measured slower (38.5 against 36.7 ms on the 140 k-block probe,
// profiles/r05ar)
#ifndef GI_CLREG
#define GI_CLREG 0
#endif
#if GI_CLREG
#define GI_LANE_DWORDS 89
#else
#define GI_T_CL 89
#define GI_LANE_DWORDS 94
#endif
#define GI_LANE_BYTES (GI_LANE_DWORDS * 4)

// per-trip statistics hooks (tools/inflate_trips.cpp); nothing by default
#ifndef GI_TRIP
#define GI_TRIP(mode) (void)0
#define GI_BYTES(kind, n) (void)0
#endif

// bytes a match step copies: four 16-byte loads, then four stores
#define GI_COPY 64u

enum { GI_OK = 0, GI_E_HEADER = 1, GI_E_TREE = 2, GI_E_CODE = 3, GI_E_DIST = 4, GI_E_OVERRUN = 5, GI_E_INPUT = 6,
       GI_E_SIZE = 7 };
enum { GI_M_HDR = 0, GI_M_SYM = 1, GI_M_COPY = 2, GI_M_STORED = 3, GI_M_DONE = 4, GI_M_P1 = 5, GI_M_P2 = 6 };

GI_FN uint32_t gi_rev15(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_bitreverse32(x) >> 17;
#else
    uint32_t r = 0;
    for (int i = 0; i < 15; i++) r |= ((x >> i) & 1u) << (14 - i);
    return r;
#endif
}

// LSB-first bit reader over the block's DEFLATE data.  A BGZF block's data is
// followed by its 8-byte trailer (CRC32, ISIZE) and then the next block or the
// buffer's padding (>= 64 bytes), so reading a little past the data is safe;
// the caller checks that no more than the data was consumed.
//
// Aligned 32-bit words with the next word loaded one refill ahead.  GI_QUAD=1
// (a variant, off): 16-byte loads with the next quad loaded a whole quad
// ahead, so a refill waits for a load issued about four refills earlier;
// measured 20% slower on the 140 k-block probe (46.5 against 38.6 ms,
// profiles/r05ao/probe.jsonl).  It reads at most 40 bytes past the consumed
// bits.
#ifndef GI_QUAD
#define GI_QUAD 0
#endif
struct GiBits {
#if GI_QUAD
    const uint32_t *wp;  // the next quad to load
    uint32_t q0, q1, q2, q3;  // the current quad's words not yet merged, q0 next
    uint32_t n0, n1, n2, n3;  // the next quad (loaded)
    int kq;                   // words left in the current quad (1..4)
#else
    const uint32_t *wp;  // the word after `nxt`
    uint32_t nxt;        // the next word to merge (already loaded)
#endif
    uint64_t buf;
    int cnt;             // valid bits in buf
    int sh0;             // bits of the first word before the data
    int64_t merged;      // words merged into buf so far
};

GI_FN uint32_t gi_ldw(const uint32_t *p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return *p;
#else
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
#endif
}

#if GI_QUAD
GI_FN void gi_ldq(const uint32_t *p, uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef uint32_t gi_q4 __attribute__((ext_vector_type(4), aligned(4)));
    const gi_q4 v = *(const gi_q4 *)p;  // one dwordx4 load
    a = v.x;
    b = v.y;
    c = v.z;
    d = v.w;
#else
    uint32_t v[4];
    __builtin_memcpy(v, p, 16);
    a = v[0];
    b = v[1];
    c = v[2];
    d = v[3];
#endif
}
#endif

// the reader at word `k` of `base` (4-byte aligned), bit r of that word
GI_FN void gi_start(GiBits &b, const uint32_t *base, int k, int r) {
#if GI_QUAD
    gi_ldq(base + k, b.q0, b.q1, b.q2, b.q3);
    gi_ldq(base + k + 4, b.n0, b.n1, b.n2, b.n3);
    b.wp = base + k + 8;
    b.buf = (uint64_t)(b.q0 >> r);
    b.q0 = b.q1;
    b.q1 = b.q2;
    b.q2 = b.q3;
    b.kq = 3;
#else
    const uint32_t w0 = gi_ldw(base + k);
    b.nxt = gi_ldw(base + k + 1);
    b.wp = base + k + 2;
    b.buf = (uint64_t)(w0 >> r);
#endif
    b.cnt = 32 - r;
    b.merged = k + 1;
}

GI_FN void gi_open(GiBits &b, const uint8_t *in) {
    // (pointer arithmetic on `in`, not an integer round trip: the compiler
    // keeps the global address space, so the loads are global_load, not flat
    // loads that an LDS wait would also wait for)
    const int mis = (int)((uintptr_t)in & 3);
    b.sh0 = mis * 8;
    gi_start(b, (const uint32_t *)(in - mis), 0, b.sh0);
}

// at least 32 bits in the buffer
GI_FN void gi_refill(GiBits &b) {
    if (b.cnt < 32) {
#if GI_QUAD
        b.buf |= (uint64_t)b.q0 << b.cnt;
        b.q0 = b.q1;
        b.q1 = b.q2;
        b.q2 = b.q3;
        if (--b.kq == 0) {
            b.q0 = b.n0;
            b.q1 = b.n1;
            b.q2 = b.n2;
            b.q3 = b.n3;
            gi_ldq(b.wp, b.n0, b.n1, b.n2, b.n3);
            b.wp += 4;
            b.kq = 4;
        }
#else
        b.buf |= (uint64_t)b.nxt << b.cnt;
        b.nxt = gi_ldw(b.wp);
        b.wp++;
#endif
        b.cnt += 32;
        b.merged++;
    }
}

GI_FN uint32_t gi_bits(GiBits &b, int n) {  // n <= 32, after a refill that covers them
    const uint32_t v = (uint32_t)(b.buf & ((n >= 32) ? 0xffffffffull : ((1ull << n) - 1)));
    b.buf >>= n;
    b.cnt -= n;
    return v;
}

// cell r of the table at dword t0 in the lane's column
template <int LANES>
GI_FN uint8_t *gi_cell(uint32_t *tab, int t0, int r, int lane) {
    return (uint8_t *)(tab + (t0 + (r >> 2)) * LANES + lane) + (r & 3);
}

// A canonical Huffman code with code lengths 1..N, one register per length:
// e[l] = lim[l] << 16 | (uint16)base[l], where lim[l] is the left-justified
// (15-bit) end of the codes of length <= l and a length-l code c is the
// symbol at sorted index base[l] + c.  With the bit-reversed next 15 bits
// `rev`, key = rev << 16 | 0xffff is >= e[l] exactly when rev >= lim[l], so
// one unsigned compare per length finds the code length.
template <int N>
struct GiHuffT {
    uint32_t e[N + 1];
};
typedef GiHuffT<15> GiHuff;   // literal/length and distance codes
typedef GiHuffT<7> GiHuffCL;  // the code-length code

// Kraft check and the code's entries from its length counts, the 16-bit field
// at bit `sh` of cnt[l] (l = 1..N), which then becomes the first sorted index
// of the length-l symbols.  GI_E_TREE for an over-subscribed set (DEFLATE
// permits an incomplete one: a code outside the tree fails at decode time).
template <int N>
GI_FN int gi_code(GiHuffT<N> &h, uint32_t *cnt, int sh) {
    int32_t left = 1;
    uint32_t code = 0, off = 0;
GI_UNROLL
    for (int l = 1; l <= N; l++) {
        const uint32_t c = (cnt[l] >> sh) & 0xffffu;
        left = (left << 1) - (int32_t)c;
        if (left < 0) return GI_E_TREE;
        cnt[l] = (cnt[l] & ~(0xffffu << sh)) | (off << sh);
        h.e[l] = (((code + c) << (15 - l)) << 16) | ((off - code) & 0xffffu);
        code = (code + c) << 1;
        off += c;
    }
    h.e[0] = 0;
    return GI_OK;
}

// symbol i of code length L (1..N) into its sorted cell (stable in symbol
// order); the 16-bit fields at bit `sh` of off[] are the next free indices
template <int LANES, int N, bool HI>
GI_FN void gi_place(uint32_t *tab, int t0, int lane, uint32_t *off, int sh, uint32_t L, int i) {
    uint32_t o = 0;
GI_UNROLL
    for (int l = 1; l <= N; l++) {
        o = (L == (uint32_t)l) ? off[l] : o;
        off[l] += (L == (uint32_t)l) ? (1u << sh) : 0u;
    }
    o = (o >> sh) & 0xffffu;
    *gi_cell<LANES>(tab, t0, (int)o, lane) = (uint8_t)i;
    if (HI && i >= 256) tab[(GI_T_LITHI + (int)(o >> 5)) * LANES + lane] |= 1u << (o & 31);
}

template <int LANES, bool HI>
GI_FN void gi_clear_hi(uint32_t *tab, int lane) {
    if (HI) {
GI_UNROLL
        for (int w = 0; w < 9; w++) tab[(GI_T_LITHI + w) * LANES + lane] = 0;
    }
}

// Build from n code lengths (len[i] for symbol i, read through `get`)
template <int LANES, int N, bool HI, class Get>
GI_FN int gi_build(GiHuffT<N> &h, uint32_t *tab, int lane, int t0, int n, Get get) {
    uint32_t cnt[N + 1];
GI_UNROLL
    for (int l = 0; l <= N; l++) cnt[l] = 0;
    for (int i = 0; i < n; i++) {
        const uint32_t L = get(i);
GI_UNROLL
        for (int l = 1; l <= N; l++) cnt[l] += (L == (uint32_t)l) ? 1u : 0u;
    }
    const int rc = gi_code<N>(h, cnt, 0);
    if (rc) return rc;
    gi_clear_hi<LANES, HI>(tab, lane);
    for (int i = 0; i < n; i++) {
        const uint32_t L = get(i);
        if (L) gi_place<LANES, N, HI>(tab, t0, lane, cnt, 0, L, i);
    }
    return GI_OK;
}

// the symbol at the front of the stream and its code length L (nothing
// consumed); -1 for a code outside the tree
template <int N>
GI_FN int gi_index(const GiBits &b, const GiHuffT<N> &h, int &L) {
    const uint32_t rev = gi_rev15((uint32_t)b.buf);
    const uint32_t key = rev << 16 | 0xffffu;
    L = 1;
    uint32_t bs = h.e[1];
GI_UNROLL
    for (int l = 1; l < N; l++) {
        const bool ge = key >= h.e[l];
        L += ge ? 1 : 0;
        bs = ge ? h.e[l + 1] : bs;
        // keep the chain of selects (the compiler would otherwise fold it into
        // e[L], a dynamic index that moves the table to scratch memory)
        GI_KEEP(bs);
    }
    if (key >= h.e[N]) return -1;
    return (int)(int16_t)(uint16_t)bs + (int)(rev >> (15 - L));
}

template <int LANES, int N, bool HI>
GI_FN int gi_lookup(const GiBits &b, const GiHuffT<N> &h, const uint32_t *tab, int lane, int t0, int &L) {
    const int idx = gi_index<N>(b, h, L);
    if (idx < 0) return -1;
    int s = *gi_cell<LANES>((uint32_t *)tab, t0, idx, lane);
    if (HI) s |= (int)((tab[(GI_T_LITHI + (idx >> 5)) * LANES + lane] >> (idx & 31)) & 1u) << 8;
    return s;
}

// decode one symbol; -1 for a code outside the tree
template <int LANES, int N, bool HI>
GI_FN int gi_decode(GiBits &b, const GiHuffT<N> &h, const uint32_t *tab, int lane, int t0) {
    int L;
    const int s = gi_lookup<LANES, N, HI>(b, h, tab, lane, t0, L);
    if (s < 0) return -1;
    b.buf >>= L;
    b.cnt -= L;
    return s;
}

// the RFC 1951 length / distance bases, computed (no tables)
GI_FN void gi_len_code(int s, int &base, int &extra) {  // s = 257..285
    if (s < 265) { base = s - 254; extra = 0; }
    else if (s < 285) { extra = (s - 261) >> 2; base = 3 + ((4 + ((s - 265) & 3)) << extra); }
    else { base = 258; extra = 0; }
}
GI_FN void gi_dist_code(int d, int &base, int &extra) {  // d = 0..29
    if (d < 4) { base = d + 1; extra = 0; }
    else { extra = (d >> 1) - 1; base = ((2 + (d & 1)) << extra) + 1; }
}

// one repeat item of the code-length code: its value and repeat count, or -1
GI_FN int gi_cl_item(GiBits &b, int s, int prev, int &val) {
    if (s < 16) { val = s; return 1; }
    if (s == 16) { val = prev; return prev < 0 ? -1 : 3 + (int)gi_bits(b, 2); }
    val = 0;
    return s == 17 ? 3 + (int)gi_bits(b, 3) : 11 + (int)gi_bits(b, 7);
}

// The fixed codes (RFC 1951 3.2.6) straight into the tables: literal/length
// code lengths 8 (0-143), 9 (144-255), 7 (256-279), 8 (280-287), so the
// sorted order is 256-279, 0-143, 280-287, 144-255; distances all 5 bits.
template <int LANES>
GI_FN int gi_fixed(GiHuff &lit, GiHuff &dist, uint32_t *tab, int lane) {
GI_UNROLL
    for (int w = 0; w < 72; w++) {
        uint32_t v = 0;
        for (int k = 0; k < 4; k++) {
            const int i = 4 * w + k;
            const int sym = i < 24 ? 256 + i : i < 168 ? i - 24 : i < 176 ? 280 + (i - 168) : 144 + (i - 176);
            v |= (uint32_t)(sym & 0xff) << (8 * k);
        }
        tab[(GI_T_LIT + w) * LANES + lane] = v;
    }
GI_UNROLL
    for (int w = 0; w < 9; w++) tab[(GI_T_LITHI + w) * LANES + lane] = w == 0 ? 0x00ffffffu : (w == 5 ? 0x0000ff00u : 0u);
GI_UNROLL
    for (int w = 0; w < 8; w++)
        tab[(GI_T_DIST + w) * LANES + lane] = (uint32_t)(4 * w) | (uint32_t)(4 * w + 1) << 8 | (uint32_t)(4 * w + 2) << 16 |
                                              (uint32_t)(4 * w + 3) << 24;
    uint32_t cn[16];
GI_UNROLL
    for (int l = 0; l < 16; l++) cn[l] = (l == 7 ? 24u : l == 8 ? 152u : l == 9 ? 112u : 0u) | (l == 5 ? 30u << 16 : 0u);
    int rc = gi_code<15>(lit, cn, 0);
    if (!rc) rc = gi_code<15>(dist, cn, 16);
    return rc;
}

// A dynamic block's header in progress.  Its code lengths are read one
// run-length item per step, twice: pass 1 counts the literal/length (low 16
// bits of cn[l]) and distance (high 16 bits) code lengths; the counts are
// checked and become each length's first sorted index; pass 2 reads the same
// items again (from bit `at`) and places the symbols, leaving each length's
// end index, from which the codes are formed.  A lane in a header thus takes
// a few hundred short steps beside its wave's symbol steps, instead of holding
// the whole wave for the header's length.  cn[] is the literal/length code's
// register array (lit.e), which a header does not otherwise need.
// GI_P2ONE (the default): pass 2 places one symbol per step (a variant
// with 0: a whole repeat item, up to 6 placements, per step)
#ifndef GI_P2ONE
#define GI_P2ONE 1
#endif
struct GiHdr {
    GiHuffCL clh;
#if GI_CLREG
    uint32_t clt[4];  // the code-length code's sorted symbols, 5 bits each, 6 per word
#endif
    int at;  // bit offset of the code lengths in the block's data
    int n, ntot, nlit, prev, eob;
    int rl;  // pass 2 (GI_P2ONE): symbols of the current repeat item still to place
};

// the bit reader positioned at bit `pos` of the data starting at `in`
GI_FN void gi_seek(GiBits &b, const uint8_t *in, int pos) {
    const int mis = (int)((uintptr_t)in & 3);
    const int abs = mis * 8 + pos;
    b.sh0 = mis * 8;
    gi_start(b, (const uint32_t *)(in - mis), abs >> 5, abs & 31);
}

// bits consumed so far
GI_FN int64_t gi_used(const GiBits &b) { return b.merged * 32 - b.sh0 - b.cnt; }

#if GI_CLREG
// the code-length code from its 19 3-bit lengths (cl, symbol i at bit 3i)
GI_FN int gi_build_cl(GiHdr &H, uint64_t cl) {
    uint32_t cnt[8];
GI_UNROLL
    for (int l = 0; l < 8; l++) cnt[l] = 0;
GI_UNROLL
    for (int i = 0; i < 19; i++) {
        const uint32_t L = (uint32_t)(cl >> (3 * i)) & 7u;
GI_UNROLL
        for (int l = 1; l <= 7; l++) cnt[l] += (L == (uint32_t)l) ? 1u : 0u;
    }
    const int rc = gi_code<7>(H.clh, cnt, 0);
    if (rc) return rc;
    H.clt[0] = H.clt[1] = H.clt[2] = H.clt[3] = 0;
GI_UNROLL
    for (int i = 0; i < 19; i++) {
        const uint32_t L = (uint32_t)(cl >> (3 * i)) & 7u;
        if (!L) continue;
        uint32_t o = 0;
GI_UNROLL
        for (int l = 1; l <= 7; l++) {
            o = (L == (uint32_t)l) ? cnt[l] : o;
            cnt[l] += (L == (uint32_t)l) ? 1u : 0u;
        }
        const uint32_t r = o / 6u, v = (uint32_t)i << (5u * (o - 6u * r));
        H.clt[0] |= r == 0 ? v : 0u;
        H.clt[1] |= r == 1 ? v : 0u;
        H.clt[2] |= r == 2 ? v : 0u;
        H.clt[3] |= r == 3 ? v : 0u;
    }
    return GI_OK;
}

// decode one code-length symbol; -1 for a code outside the tree
GI_FN int gi_decode_cl(GiBits &b, const GiHdr &H) {
    int L;
    const int idx = gi_index<7>(b, H.clh, L);
    if (idx < 0) return -1;
    b.buf >>= L;
    b.cnt -= L;
    const uint32_t r = (uint32_t)idx / 6u;
    // (selects kept apart: folded, they become a dynamic index into H,
    // which moves the header state to scratch memory)
    uint32_t w = H.clt[0];
    w = r == 1 ? H.clt[1] : w;
    GI_KEEP(w);
    w = r == 2 ? H.clt[2] : w;
    GI_KEEP(w);
    w = r == 3 ? H.clt[3] : w;
    return (int)((w >> (5u * ((uint32_t)idx - 6u * r))) & 31u);
}
#define GI_CL_DECODE(b, H) gi_decode_cl(b, H)
#else
#define GI_CL_DECODE(b, H) gi_decode<LANES, 7, false>(b, (H).clh, tab, lane, GI_T_CL)
#endif

// the 3-bit block header and, for a dynamic block, its counts and the
// code-length code (after a refill): the next mode or -GI_E_*
template <int LANES>
GI_FN int gi_header(GiBits &b, GiHuff &lit, GiHuff &dist, GiHdr &H, uint32_t *tab, int lane, uint32_t &bfinal,
                    uint32_t &rem) {
    const uint32_t hdr = gi_bits(b, 3);
    bfinal = hdr & 1;
    const uint32_t btype = hdr >> 1;
    if (btype == 0) {  // stored: to the byte boundary, LEN, NLEN, bytes
        gi_bits(b, b.cnt & 7);
        gi_refill(b);
        const uint32_t len = gi_bits(b, 16);
        gi_refill(b);
        const uint32_t nlen = gi_bits(b, 16);
        if ((len ^ 0xffffu) != nlen) return -GI_E_HEADER;
        rem = len;
        return len ? GI_M_STORED : (bfinal ? GI_M_DONE : GI_M_HDR);
    }
    if (btype == 1) {  // fixed codes
        const int rc = gi_fixed<LANES>(lit, dist, tab, lane);
        return rc ? -rc : GI_M_SYM;
    }
    if (btype != 2) return -GI_E_HEADER;
    H.nlit = (int)gi_bits(b, 5) + 257;
    const int ndist = (int)gi_bits(b, 5) + 1;
    const int ncl = (int)gi_bits(b, 4) + 4;
    if (H.nlit > 286 || ndist > 30) return -GI_E_HEADER;
    // code-length code lengths, 3 bits each in the order
    // 16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1,15 (5 bits per entry in two
    // words), packed 3 bits per symbol
    const uint64_t ord_lo = 16ull | 17ull << 5 | 18ull << 10 | 0ull << 15 | 8ull << 20 | 7ull << 25 | 9ull << 30 |
                            6ull << 35 | 10ull << 40 | 5ull << 45 | 11ull << 50 | 4ull << 55;
    const uint64_t ord_hi = 12ull | 3ull << 5 | 13ull << 10 | 2ull << 15 | 14ull << 20 | 1ull << 25 | 15ull << 30;
    uint64_t cl = 0;
    for (int k = 0; k < ncl; k++) {
        gi_refill(b);
        const uint32_t v = gi_bits(b, 3);
        const int s = (int)((k < 12 ? ord_lo >> (5 * k) : ord_hi >> (5 * (k - 12))) & 31u);
        cl |= (uint64_t)v << (3 * s);
    }
#if GI_CLREG
    const int rc = gi_build_cl(H, cl);
#else
    const int rc = gi_build<LANES, 7, false>(H.clh, tab, lane, GI_T_CL, 19,
                                             [cl](int i) -> uint32_t { return (uint32_t)(cl >> (3 * i)) & 7u; });
#endif
    if (rc) return -rc;
    H.ntot = H.nlit + ndist;
    H.at = (int)gi_used(b);
GI_UNROLL
    for (int l = 0; l < 16; l++) lit.e[l] = 0;
    H.n = 0;
    H.prev = -1;
    H.eob = 0;
    return GI_M_P1;
}

// Kraft check of the 16-bit counts at bit `sh` of cnt[1..15] (an
// over-subscribed set is GI_E_TREE; DEFLATE permits an incomplete one)
GI_FN int gi_kraft(const uint32_t *cnt, int sh) {
    int32_t left = 1;
GI_UNROLL
    for (int l = 1; l <= 15; l++) {
        left = (left << 1) - (int32_t)((cnt[l] >> sh) & 0xffffu);
        if (left < 0) return GI_E_TREE;
    }
    return GI_OK;
}

// one run-length item of the code lengths (after a refill): pass 1 or 2
template <int LANES, bool PASS2>
GI_FN int gi_cl_step(GiBits &b, const uint8_t *in, GiHuff &lit, GiHuff &dist, GiHdr &H, uint32_t *tab, int lane) {
    uint32_t *cn = lit.e;
#if GI_P2ONE
    if (PASS2) {
        // one symbol placed per step: a repeat item's symbols over several
        // steps, so no step holds its wave for a whole item
        if (H.rl == 0) {
            const int s = GI_CL_DECODE(b, H);
            if (s < 0) return -GI_E_TREE;
            int val;
            const int rep = gi_cl_item(b, s, H.prev, val);
            if (rep < 0 || H.n + rep > H.ntot) return -GI_E_TREE;
            H.prev = val;
            if (val) H.rl = rep;
            else H.n += rep;
        }
        if (H.rl > 0) {
            const int i = H.n;
            if (i < H.nlit) gi_place<LANES, 15, true>(tab, GI_T_LIT, lane, cn, 0, (uint32_t)H.prev, i);
            else gi_place<LANES, 15, false>(tab, GI_T_DIST, lane, cn, 16, (uint32_t)H.prev, i - H.nlit);
            H.n++;
            H.rl--;
        }
        if (H.n < H.ntot) return GI_M_P2;
        for (int l = 15; l >= 1; l--) cn[l] -= cn[l - 1];
        int rc = gi_code<15>(dist, cn, 16);
        if (!rc) rc = gi_code<15>(lit, cn, 0);
        return rc ? -rc : GI_M_SYM;
    }
#endif
    const int s = GI_CL_DECODE(b, H);
    if (s < 0) return -GI_E_TREE;
    int val;
    const int rep = gi_cl_item(b, s, H.prev, val);
    if (rep < 0 || H.n + rep > H.ntot) return -GI_E_TREE;
    if (!PASS2) {
        int rl = H.nlit - H.n;
        rl = rl < 0 ? 0 : (rl > rep ? rep : rl);
        const uint32_t add = (uint32_t)rl | (uint32_t)(rep - rl) << 16;
GI_UNROLL
        for (int l = 1; l < 16; l++) cn[l] += (val == l) ? add : 0u;
        if (val && H.n <= 256 && 256 < H.n + rep) H.eob = 1;
    } else if (val) {
        for (int k = 0; k < rep; k++) {
            const int i = H.n + k;
            if (i < H.nlit) gi_place<LANES, 15, true>(tab, GI_T_LIT, lane, cn, 0, (uint32_t)val, i);
            else gi_place<LANES, 15, false>(tab, GI_T_DIST, lane, cn, 16, (uint32_t)val, i - H.nlit);
        }
    }
    H.n += rep;
    H.prev = val;
    if (H.n < H.ntot) return PASS2 ? GI_M_P2 : GI_M_P1;
    if (PASS2) {
        // cn[l] = each length's end index: the counts again, then both codes
        // (the distance code first: the literal code is formed in place)
        for (int l = 15; l >= 1; l--) cn[l] -= cn[l - 1];
        int rc = gi_code<15>(dist, cn, 16);
        if (!rc) rc = gi_code<15>(lit, cn, 0);
        return rc ? -rc : GI_M_SYM;
    }
    // pass 1 done: the counts checked and turned into first sorted indices,
    // then the items again from their start
    if (!H.eob) return -GI_E_TREE;  // no end-of-block code (zlib refuses it too)
    if (gi_kraft(cn, 0) || gi_kraft(cn, 16)) return -GI_E_TREE;
    uint32_t off = 0;
GI_UNROLL
    for (int l = 1; l <= 15; l++) {
        const uint32_t c = cn[l];
        cn[l] = off;
        off += c;  // both 16-bit fields at once: neither exceeds 286
    }
    cn[0] = 0;
    gi_clear_hi<LANES, true>(tab, lane);
    gi_seek(b, in, H.at);
    H.n = 0;
    H.prev = -1;
    H.rl = 0;
    return GI_M_P2;
}

// Literals (and stored bytes) gather in a 64-bit register and go out as one
// 8-byte store per 8 bytes (round 4 stored them one byte per step: ~6x the
// output in write traffic).  Before a match the pending bytes are stored, 8
// bytes wide when the block's output has room (the bytes past the pending
// ones are garbage this lane overwrites later, as a match step's are), so a
// match always reads final bytes.
GI_FN void gi_put8(uint8_t *q, uint64_t v) {
    __builtin_memcpy(q, &v, 8);
}

GI_FN void gi_flush(uint8_t *out, uint32_t o, uint32_t out_len, uint64_t &pend, uint32_t &pn) {
    if (!pn) return;
    uint8_t *q = out + (o - pn);
    if (o - pn + 8 <= out_len) {
        gi_put8(q, pend);
    } else {
        for (uint32_t j = 0; j < pn; j++) q[j] = (uint8_t)(pend >> (8 * j));
    }
    pend = 0;
    pn = 0;
}

// one literal or stored byte into the pending register
GI_FN void gi_lit(uint8_t *out, uint32_t &o, uint64_t &pend, uint32_t &pn, uint32_t s) {
    pend |= (uint64_t)s << (8 * pn);
    pn++;
    o++;
    if (pn == 8) {
        gi_put8(out + (o - 8), pend);
        pend = 0;
        pn = 0;
    }
}

// A match step's stores wait for its loads (an L2 round trip).  GI_DEFER
// (the default): the step issues its loads and leaves the stores to the next
// trip, which stores them after its own refill and symbol decode (LDS work)
// and before its first output access -- a literal group's store, a flush, or
// the next match step's loads (whose source may be the pending bytes) -- so
// the round trip overlaps the next symbol's decode.  Stores keep their
// program order: the pending chunk's store (and its garbage tail past m)
// always precedes every later store.  36.7 against 38.6 ms on the 140 k-block
// probe (profiles/r05ao/probe.jsonl).
#ifndef GI_DEFER
#define GI_DEFER 1
#endif
// GI_DEFER2: a match's later chunk whose source lies wholly before the
// pending chunk loads before the pending chunk's stores (a variant)
#ifndef GI_DEFER2
#define GI_DEFER2 0
#endif
// GI_LIT2: a literal step also takes a second literal when the bit buffer
// holds its code (a variant)
#ifndef GI_LIT2
#define GI_LIT2 0
#endif

// Inflate one block's raw DEFLATE data (in[0..in_len)) into out[0..out_len).
// `tab` is the LDS (device) or local (host) table storage of GI_LANE_DWORDS
// rows x LANES columns.  Bytes outside out[0..out_len) are never written.
template <int LANES>
GI_FN int gi_inflate(const uint8_t *in, uint32_t in_len, uint8_t *out, uint32_t out_len, uint32_t *tab, int lane) {
    typedef uint32_t gi_u32x4 __attribute__((vector_size(16)));
    GiBits b;
    gi_open(b, in);
    GiHuff lit = {}, dist = {};
    GiHdr H = {};
    uint32_t o = 0, bfinal = 0;
    uint32_t rem = 0;  // bytes left of the match or stored block
    uint32_t D = 0;    // the match's current source distance (a multiple of its distance)
    uint64_t pend = 0; // literals not yet stored: the output bytes [o - pn, o)
    uint32_t pn = 0;
    gi_u32x4 v0 = {}, v1 = {}, v2 = {}, v3 = {};
    uint32_t cq = 0, cm = 0;  // GI_DEFER: a loaded match chunk of cm bytes (0: none) for out + cq
    // the pending chunk's stores (16-byte pieces that cover its cm bytes)
    auto commit = [&]() {
        if (cm) {
            uint8_t *q = out + cq;
            __builtin_memcpy(q, &v0, 16);
            if (cm > 16) __builtin_memcpy(q + 16, &v1, 16);
            if (cm > 32) __builtin_memcpy(q + 32, &v2, 16);
            if (cm > 48) __builtin_memcpy(q + 48, &v3, 16);
            cm = 0;
        }
    };
    int mode = GI_M_HDR, rc = GI_OK;
    while (mode != GI_M_DONE) {
        GI_TRIP(mode);
        gi_refill(b);
        if (mode == GI_M_HDR) {
            const int m = gi_header<LANES>(b, lit, dist, H, tab, lane, bfinal, rem);
            if (m < 0) {
                rc = -m;
                break;
            }
            if (m == GI_M_STORED && o + rem > out_len) {
                rc = GI_E_OVERRUN;
                break;
            }
            mode = m;
        } else if (mode == GI_M_P1 || mode == GI_M_P2) {
            const int m = mode == GI_M_P1 ? gi_cl_step<LANES, false>(b, in, lit, dist, H, tab, lane)
                                          : gi_cl_step<LANES, true>(b, in, lit, dist, H, tab, lane);
            if (m < 0) {
                rc = -m;
                break;
            }
            mode = m;
        } else if (mode == GI_M_SYM) {
            const int s = gi_decode<LANES, 15, true>(b, lit, tab, lane, GI_T_LIT);
            if (s < 0 || s > 285) {
                rc = GI_E_CODE;
                break;
            }
            if (s < 256) {
                if (o >= out_len) {
                    rc = GI_E_OVERRUN;
                    break;
                }
                if (pn == 7) commit();  // (this literal completes a group: its store follows the chunk's)
                gi_lit(out, o, pend, pn, (uint32_t)s);
                GI_BYTES(0, 1);
#if GI_LIT2
                // a second literal in the same step when the buffer holds its code
                if (b.cnt >= 15 && o < out_len) {
                    int L2;
                    const int s2 = gi_lookup<LANES, 15, true>(b, lit, tab, lane, GI_T_LIT, L2);
                    if (s2 >= 0 && s2 < 256) {
                        b.buf >>= L2;
                        b.cnt -= L2;
                        if (pn == 7) commit();
                        gi_lit(out, o, pend, pn, (uint32_t)s2);
                        GI_BYTES(0, 1);
                    }
                }
#endif
            } else if (s == 256) {
                mode = bfinal ? GI_M_DONE : GI_M_HDR;
            } else {
                int lb, le;
                gi_len_code(s, lb, le);
                const uint32_t len = (uint32_t)lb + gi_bits(b, le);
                gi_refill(b);
                const int d = gi_decode<LANES, 15, false>(b, dist, tab, lane, GI_T_DIST);
                if (d < 0 || d > 29) {
                    rc = GI_E_DIST;
                    break;
                }
                int db, de;
                gi_dist_code(d, db, de);
                const uint32_t dd = (uint32_t)db + gi_bits(b, de);
                if (dd > o) {
                    rc = GI_E_DIST;
                    break;
                }
                if (o + len > out_len) {
                    rc = GI_E_OVERRUN;
                    break;
                }
                rem = len;
                D = dd;
                mode = GI_M_COPY;
                commit();
                gi_flush(out, o, out_len, pend, pn);  // the match reads final bytes
            }
        }
        // (a match starts copying in the step that decoded it)
        if (mode == GI_M_COPY) {
            uint32_t m = rem < GI_COPY ? rem : GI_COPY;
            m = m < D ? m : D;
            uint8_t *q = out + o;
            // 16-byte pieces that cover m bytes (sources all final: o - D + m <= o)
            const uint32_t span = (m + 15u) & ~15u;
#if GI_DEFER2
            if (cm && D >= m + cm && o + span <= out_len) {
                // the source lies before the pending chunk (which ends at o):
                // this chunk's loads go out before the pending chunk's stores
                gi_u32x4 w0 = {}, w1 = {}, w2 = {}, w3 = {};
                __builtin_memcpy(&w0, q - D, 16);
                if (m > 16) __builtin_memcpy(&w1, q - D + 16, 16);
                if (m > 32) __builtin_memcpy(&w2, q - D + 32, 16);
                if (m > 48) __builtin_memcpy(&w3, q - D + 48, 16);
                commit();
                v0 = w0;
                v1 = w1;
                v2 = w2;
                v3 = w3;
                cq = o;
                cm = m;
            } else
#endif
            if (o + span <= out_len) {
                commit();  // (its bytes may be this step's source)
                __builtin_memcpy(&v0, q - D, 16);
                if (m > 16) __builtin_memcpy(&v1, q - D + 16, 16);
                if (m > 32) __builtin_memcpy(&v2, q - D + 32, 16);
                if (m > 48) __builtin_memcpy(&v3, q - D + 48, 16);
                cq = o;
                cm = m;
#if !GI_DEFER
                commit();
#endif
            } else {
                commit();
                for (uint32_t j = 0; j < m; j++) q[j] = q[(int64_t)j - D];
            }
            o += m;
            rem -= m;
            GI_BYTES(1, m);
            if (m == D && D < GI_COPY) D <<= 1;
            if (!rem) mode = GI_M_SYM;
        } else if (mode == GI_M_STORED) {
            // byte-aligned: up to 4 bytes from the bit buffer per step
            commit();
            gi_refill(b);
            const uint32_t m = rem < 4u ? rem : 4u;
            for (uint32_t j = 0; j < m; j++) gi_lit(out, o, pend, pn, gi_bits(b, 8));
            GI_BYTES(2, m);
            rem -= m;
            if (!rem) mode = bfinal ? GI_M_DONE : GI_M_HDR;
        }
    }
    if (rc) return rc;
    commit();
    gi_flush(out, o, out_len, pend, pn);
    // consumed bits: every merged word minus the first word's lead and the buffer
    const int64_t used_bits = gi_used(b);
    if (used_bits > 8 * (int64_t)in_len) return GI_E_INPUT;
    if (o != out_len) return GI_E_SIZE;
    return GI_OK;
}

// ---------------------------------------------------------------------------
// Two-phase inflate (round 6).  gi_inflate above copies every match from the
// block's own output in global memory inside the decode loop: the match's
// loads are an L2 round trip on the lane's chain (its stores before them
// must land first: one in-order memory counter), and a wave carries the
// union of the header, symbol and copy paths every trip.  Split:
//   phase 1 (gi_tokens, one block per lane, LDS code tables): the Huffman
//     decode alone.  Literals go to their final places in the block's output
//     (8-byte groups, as gi_inflate's); each match becomes a 32-bit token in
//     the block's token area; no output byte is read back.
//   phase 2 (gi_lz, one block per lane, no LDS, few registers: a full chip
//     of waves): the tokens replayed -- each match copied from the output
//     before it, 16-byte pieces, the match's last piece cut to its bytes so
//     the literals already in place after it are never touched.
// Token: bits 0-7 the literals before it (lc), bit 31 set: literals only
// (the block's last token, or a run of 255), else bits 8-15 the match length
// - 3 and bits 16-30 its distance - 1.  A block with more than `tokcap`
// tokens is GI_E_TOKCAP: the caller inflates it with gi_inflate instead.
// ---------------------------------------------------------------------------
enum { GI_E_TOKCAP = 9 };
#define GI_TOK_LITONLY 0x80000000u

template <int LANES>
GI_FN int gi_tokens(const uint8_t *in, uint32_t in_len, uint8_t *out, uint32_t out_len, uint32_t *tok, uint32_t tokcap,
                    uint32_t *ntok, uint32_t *tab, int lane) {
    typedef uint32_t gi_u32x4 __attribute__((vector_size(16)));
    GiBits b;
    gi_open(b, in);
    GiHuff lit_h = {}, dist_h = {};
    GiHdr H = {};
    uint32_t o = 0, bfinal = 0, rem = 0;
    uint64_t pend = 0;   // literals not yet stored: the output bytes [o - pn, o)
    uint32_t pn = 0;
    uint32_t lc = 0;     // literals since the last token
    uint32_t nt = 0;     // tokens so far
    gi_u32x4 tv = {};    // the current group of four tokens, oldest in [0] once full
    int mode = GI_M_HDR, rc = GI_OK;
    // one token into the group; a full group leaves as one 16-byte store
    auto emit = [&](uint32_t t) -> bool {
        if (nt >= tokcap) return false;
        tv = (gi_u32x4){tv[1], tv[2], tv[3], t};
        nt++;
        if ((nt & 3u) == 0) __builtin_memcpy(tok + (nt - 4), &tv, 16);
        return true;
    };
    auto put_lit = [&](uint32_t s) -> bool {
        gi_lit(out, o, pend, pn, s);
        if (++lc == 255) {
            lc = 0;
            return emit(GI_TOK_LITONLY | 255u);
        }
        return true;
    };
    while (mode != GI_M_DONE) {
        GI_TRIP(mode);
        gi_refill(b);
        if (mode == GI_M_HDR) {
            const int m = gi_header<LANES>(b, lit_h, dist_h, H, tab, lane, bfinal, rem);
            if (m < 0) {
                rc = -m;
                break;
            }
            if (m == GI_M_STORED && o + rem > out_len) {
                rc = GI_E_OVERRUN;
                break;
            }
            mode = m;
        } else if (mode == GI_M_P1 || mode == GI_M_P2) {
            const int m = mode == GI_M_P1 ? gi_cl_step<LANES, false>(b, in, lit_h, dist_h, H, tab, lane)
                                          : gi_cl_step<LANES, true>(b, in, lit_h, dist_h, H, tab, lane);
            if (m < 0) {
                rc = -m;
                break;
            }
            mode = m;
        } else if (mode == GI_M_SYM) {
            const int s = gi_decode<LANES, 15, true>(b, lit_h, tab, lane, GI_T_LIT);
            if (s < 0 || s > 285) {
                rc = GI_E_CODE;
                break;
            }
            if (s < 256) {
                if (o >= out_len) {
                    rc = GI_E_OVERRUN;
                    break;
                }
                if (!put_lit((uint32_t)s)) {
                    rc = GI_E_TOKCAP;
                    break;
                }
                GI_BYTES(0, 1);
            } else if (s == 256) {
                mode = bfinal ? GI_M_DONE : GI_M_HDR;
            } else {
                int lb, le;
                gi_len_code(s, lb, le);
                const uint32_t len = (uint32_t)lb + gi_bits(b, le);
                gi_refill(b);
                const int d = gi_decode<LANES, 15, false>(b, dist_h, tab, lane, GI_T_DIST);
                if (d < 0 || d > 29) {
                    rc = GI_E_DIST;
                    break;
                }
                int db, de;
                gi_dist_code(d, db, de);
                const uint32_t dd = (uint32_t)db + gi_bits(b, de);
                if (dd > o) {
                    rc = GI_E_DIST;
                    break;
                }
                if (o + len > out_len) {
                    rc = GI_E_OVERRUN;
                    break;
                }
                if (!emit(lc | (len - 3u) << 8 | (dd - 1u) << 16)) {
                    rc = GI_E_TOKCAP;
                    break;
                }
                lc = 0;
                // the pending literals out (their garbage tail lands in this
                // match's bytes, which phase 2 writes)
                gi_flush(out, o, out_len, pend, pn);
                o += len;
                GI_BYTES(1, len);
            }
        } else if (mode == GI_M_STORED) {
            // byte-aligned: up to 4 bytes from the bit buffer per step
            const uint32_t m = rem < 4u ? rem : 4u;
            bool ok = true;
            for (uint32_t j = 0; j < m; j++) ok = put_lit(gi_bits(b, 8)) && ok;
            if (!ok) {
                rc = GI_E_TOKCAP;
                break;
            }
            GI_BYTES(2, m);
            rem -= m;
            if (!rem) mode = bfinal ? GI_M_DONE : GI_M_HDR;
        }
    }
    if (rc) return rc;
    if (lc && !emit(GI_TOK_LITONLY | lc)) return GI_E_TOKCAP;
    gi_flush(out, o, out_len, pend, pn);
    // the last group, shifted down to its start
    const uint32_t tail = nt & 3u;
    if (tail) {
        for (uint32_t k = tail; k < 4; k++) tv = (gi_u32x4){tv[1], tv[2], tv[3], 0u};
        __builtin_memcpy(tok + (nt - tail), &tv, 16);
    }
    *ntok = nt;
    const int64_t used_bits = gi_used(b);
    if (used_bits > 8 * (int64_t)in_len) return GI_E_INPUT;
    if (o != out_len) return GI_E_SIZE;
    return GI_OK;
}

// the first n (< 16) bytes of a 16-byte piece, exactly: 8, 4, 2, 1-byte stores
GI_FN void gi_put_part(uint8_t *q, const uint32_t *w, uint32_t n) {
    uint32_t k = 0;  // words done
    if (n & 8) {
        const uint64_t v = (uint64_t)w[0] | (uint64_t)w[1] << 32;
        __builtin_memcpy(q, &v, 8);
        k = 2;
    }
    uint32_t x = w[k], y = w[k + 1];
    // (select, not a dynamic index: the piece stays in registers)
    if (n & 4) {
        __builtin_memcpy(q + (n & 8), &x, 4);
        x = y;
    }
    const uint32_t at = n & 12u;
    if (n & 2) {
        const uint16_t h = (uint16_t)x;
        __builtin_memcpy(q + at, &h, 2);
        x >>= 16;
    }
    if (n & 1) q[at + (n & 2)] = (uint8_t)x;
}

// One match: out[o, o + rem) from D bytes back (all of it before o final).
// A step copies up to 64 bytes (at most the current source distance D,
// doubled after each step that copies D bytes: the output is periodic with
// the distance) in 16-byte pieces; the pieces are cut at the match's end, so
// whatever follows the match (literals already in place) is never touched.
GI_FN void gi_match(uint8_t *out, uint32_t o, uint32_t rem, uint32_t D) {
    typedef uint32_t gi_u32x4 __attribute__((vector_size(16)));
    while (rem) {
        uint32_t m = rem < GI_COPY ? rem : GI_COPY;
        m = m < D ? m : D;
        uint8_t *q = out + o;
        const uint8_t *src = q - D;
        gi_u32x4 v0 = {}, v1 = {}, v2 = {}, v3 = {};
        __builtin_memcpy(&v0, src, 16);
        if (m > 16) __builtin_memcpy(&v1, src + 16, 16);
        if (m > 32) __builtin_memcpy(&v2, src + 32, 16);
        if (m > 48) __builtin_memcpy(&v3, src + 48, 16);
        // (bytes past m but inside the match are garbage the next step overwrites)
        const uint32_t span = (m + 15u) & ~15u;
        const uint32_t lim = rem < span ? rem : span;
        const uint32_t full = lim >> 4, part = lim & 15u;
        if (full > 0) __builtin_memcpy(q, &v0, 16);
        if (full > 1) __builtin_memcpy(q + 16, &v1, 16);
        if (full > 2) __builtin_memcpy(q + 32, &v2, 16);
        if (full > 3) __builtin_memcpy(q + 48, &v3, 16);
        if (part) {
            const gi_u32x4 lp = full == 0 ? v0 : full == 1 ? v1 : full == 2 ? v2 : v3;
            uint32_t w[4] = {lp[0], lp[1], lp[2], lp[3]};
            gi_put_part(q + 16 * full, w, part);
        }
        o += m;
        rem -= m;
        if (m == D && D < GI_COPY) D <<= 1;
    }
}

// Phase 2 for one block on one lane (the host twin's; the device's takes a
// wave per block, ddecode.hip k_lz77): the tokens tok[0..n) over
// out[0..out_len), whose literal bytes are already in place, in order.
// Tokens come four per load.
GI_FN int gi_lz(const uint32_t *tok, uint32_t n, uint8_t *out, uint32_t out_len) {
    typedef uint32_t gi_u32x4 __attribute__((vector_size(16)));
    uint32_t o = 0;
    gi_u32x4 g = {};
    for (uint32_t k = 0; k < n; k++) {
        if ((k & 3u) == 0) __builtin_memcpy(&g, tok + k, 16);
        const uint32_t t = g[0];
        g = (gi_u32x4){g[1], g[2], g[3], 0u};
        o += t & 255u;
        if (o > out_len) return GI_E_OVERRUN;
        if (t & GI_TOK_LITONLY) continue;
        const uint32_t len = ((t >> 8) & 255u) + 3u, d = ((t >> 16) & 0x7fffu) + 1u;
        if (d > o) return GI_E_DIST;
        if (o + len > out_len) return GI_E_OVERRUN;
        gi_match(out, o, len, d);
        o += len;
    }
    return o == out_len ? GI_OK : GI_E_SIZE;
}
