// inflate.h -- DEFLATE (RFC 1951) decoder for one BGZF block per lane.
//
// The reference reads its BAM through htslib's BGZF layer on the host
// (my_samread, GROM.c:981-992; bgzf_read inflates each <= 64 KiB block with
// zlib).  Here every BGZF block of a chromosome's compressed run is inflated on
// the GPU, one block per lane: a BAM's blocks are independent DEFLATE streams
// with their own Huffman trees, so a chromosome's 10^4-10^5 blocks fill the
// chip without any cross-lane work.
//
// Per lane, the Huffman tables are canonical: for each code length l the
// left-justified end of its code range (lim[l]) and the offset from a code to
// its symbol's index in the sorted-symbol array (base[l]) sit in registers;
// the length of the code at the stream's front is the number of lim[l] at or
// below the next 15 bits (bit-reversed), found by one unrolled compare chain,
// and only the sorted symbols live in LDS (element-major across the lanes, so
// any per-lane index is bank-conflict free).  No table of 2^n entries per
// block: the 64 blocks of a wave need 43 KiB of LDS in all.
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

// sorted-symbol rows per lane: literal/length (288), distance (32), code-length (19)
#define GI_ROW_LIT 0
#define GI_ROW_DIST 288
#define GI_ROW_CL 320
#define GI_ROWS 339
// 4-bit code-length cells of a dynamic block's 286 + 30 symbols, after the rows
#define GI_NIB_ROWS 160
// storage per lane (bytes): the symbol rows (uint16) and the length cells
#define GI_LANE_BYTES (GI_ROWS * 2 + GI_NIB_ROWS)

enum { GI_OK = 0, GI_E_HEADER = 1, GI_E_TREE = 2, GI_E_CODE = 3, GI_E_DIST = 4, GI_E_OVERRUN = 5, GI_E_INPUT = 6,
       GI_E_SIZE = 7 };

GI_FN uint32_t gi_rev15(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_bitreverse32(x) >> 17;
#else
    uint32_t r = 0;
    for (int i = 0; i < 15; i++) r |= ((x >> i) & 1u) << (14 - i);
    return r;
#endif
}

// LSB-first bit reader over the block's DEFLATE data, fed by aligned 32-bit
// words with the next word loaded one refill ahead (the load's latency hides
// behind the symbols decoded meanwhile).  A BGZF block's data is followed by
// its 8-byte trailer (CRC32, ISIZE) and then the next block or the buffer's
// padding, so reading up to 15 bytes past the data is safe; the caller checks
// that no more than the data was consumed.
struct GiBits {
    const uint32_t *wp;  // the word after `nxt`
    uint32_t nxt;        // the next word to merge (already loaded)
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

GI_FN void gi_open(GiBits &b, const uint8_t *in) {
    // (pointer arithmetic on `in`, not an integer round trip: the compiler
    // keeps the global address space, so the loads are global_load, not flat
    // loads that an LDS wait would also wait for)
    const int mis = (int)((uintptr_t)in & 3);
    b.wp = (const uint32_t *)(in - mis);
    b.sh0 = mis * 8;
    const uint32_t w0 = gi_ldw(b.wp);
    b.nxt = gi_ldw(b.wp + 1);
    b.wp += 2;
    b.buf = (uint64_t)(w0 >> b.sh0);
    b.cnt = 32 - b.sh0;
    b.merged = 1;
}

// at least 32 bits in the buffer
GI_FN void gi_refill(GiBits &b) {
    if (b.cnt < 32) {
        b.buf |= (uint64_t)b.nxt << b.cnt;
        b.cnt += 32;
        b.nxt = gi_ldw(b.wp);
        b.wp++;
        b.merged++;
    }
}

GI_FN uint32_t gi_bits(GiBits &b, int n) {  // n <= 32, after a refill that covers them
    const uint32_t v = (uint32_t)(b.buf & ((n >= 32) ? 0xffffffffull : ((1ull << n) - 1)));
    b.buf >>= n;
    b.cnt -= n;
    return v;
}

// a canonical Huffman code: code lengths 1..15
struct GiHuff {
    uint32_t lim[16];  // lim[l]: left-justified (15-bit) end of the codes of length <= l
    int32_t base[16];  // symbol index of a length-l code c: base[l] + c
};

// Build from n code lengths (len[i] for symbol i, read through `get`): the
// sorted symbols go to rows row0.. of the lane's column.  Returns GI_OK, or
// GI_E_TREE for an over-subscribed set.  allow_incomplete: DEFLATE permits an
// incomplete distance tree (a single code) -- any code outside the tree fails
// at decode time.
template <int LANES, class Get>
GI_FN int gi_build(GiHuff &h, uint16_t *sym, int lane, int row0, int n, Get get) {
    uint32_t cnt[16];
GI_UNROLL
    for (int l = 0; l < 16; l++) cnt[l] = 0;
    for (int i = 0; i < n; i++) {
        const uint32_t L = get(i);
GI_UNROLL
        for (int l = 1; l < 16; l++) cnt[l] += (L == (uint32_t)l) ? 1u : 0u;
    }
    // Kraft check, first codes, offsets
    int32_t left = 1;
    uint32_t code = 0, off = 0, off_l[16];
GI_UNROLL
    for (int l = 1; l < 16; l++) {
        left = (left << 1) - (int32_t)cnt[l];
        if (left < 0) return GI_E_TREE;
        off_l[l] = off;
        h.base[l] = (int32_t)off - (int32_t)code;
        code += cnt[l];
        h.lim[l] = code << (15 - l);
        off += cnt[l];
        code <<= 1;
    }
    h.base[0] = 0;
    h.lim[0] = 0;
    // place the symbols in code order (stable in symbol order)
    for (int i = 0; i < n; i++) {
        const uint32_t L = get(i);
        uint32_t o = 0;
GI_UNROLL
        for (int l = 1; l < 16; l++) {
            o = (L == (uint32_t)l) ? off_l[l] : o;
            off_l[l] += (L == (uint32_t)l) ? 1u : 0u;
        }
        if (L) sym[(row0 + (int)o) * LANES + lane] = (uint16_t)i;
    }
    return GI_OK;
}

// decode one symbol; -1 for a code outside the tree
template <int LANES>
GI_FN int gi_decode(GiBits &b, const GiHuff &h, const uint16_t *sym, int lane, int row0) {
    const uint32_t rev = gi_rev15((uint32_t)b.buf);
    int L = 1;
    int32_t bs = h.base[1];
GI_UNROLL
    for (int l = 1; l < 15; l++) {
        const bool ge = rev >= h.lim[l];
        L += ge ? 1 : 0;
        bs = ge ? h.base[l + 1] : bs;
        // keep the chain of selects (the compiler would otherwise fold it into
        // base[L], a dynamic index that moves the tables to scratch memory)
        GI_KEEP(bs);
    }
    if (rev >= h.lim[15]) return -1;
    const int idx = bs + (int)(rev >> (15 - L));
    b.buf >>= L;
    b.cnt -= L;
    return sym[(row0 + idx) * LANES + lane];
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

// Inflate one block's raw DEFLATE data (in[0..in_len)) into out[0..out_len).
// `sym` is the LDS (device) or local (host) sorted-symbol storage of GI_ROWS
// rows x LANES columns.  Every output byte is written exactly once.
template <int LANES>
GI_FN int gi_inflate(const uint8_t *in, uint32_t in_len, uint8_t *out, uint32_t out_len, uint16_t *sym, int lane) {
    GiBits b;
    gi_open(b, in);
    uint32_t o = 0;
    GiHuff lit, dist;
    for (;;) {
        gi_refill(b);
        const uint32_t hdr = gi_bits(b, 3);
        const uint32_t bfinal = hdr & 1, btype = hdr >> 1;
        if (btype == 0) {  // stored: to the byte boundary, LEN, NLEN, bytes
            gi_bits(b, b.cnt & 7);
            gi_refill(b);
            const uint32_t len = gi_bits(b, 16);
            gi_refill(b);
            const uint32_t nlen = gi_bits(b, 16);
            if ((len ^ 0xffffu) != nlen) return GI_E_HEADER;
            if (o + len > out_len) return GI_E_OVERRUN;
            for (uint32_t k = 0; k < len; k++) {
                if (b.cnt < 8) gi_refill(b);
                out[o++] = (uint8_t)gi_bits(b, 8);
            }
        } else if (btype == 1 || btype == 2) {
            int nlit = 288, ndist = 30;
            if (btype == 1) {  // fixed codes
                int rc = gi_build<LANES>(lit, sym, lane, GI_ROW_LIT, 288, [](int i) -> uint32_t {
                    return i < 144 ? 8u : (i < 256 ? 9u : (i < 280 ? 7u : 8u));
                });
                if (rc) return rc;
                rc = gi_build<LANES>(dist, sym, lane, GI_ROW_DIST, 30, [](int) -> uint32_t { return 5u; });
                if (rc) return rc;
            } else {  // dynamic codes
                gi_refill(b);
                nlit = (int)gi_bits(b, 5) + 257;
                ndist = (int)gi_bits(b, 5) + 1;
                const int ncl = (int)gi_bits(b, 4) + 4;
                if (nlit > 286 || ndist > 30) return GI_E_HEADER;
                // code-length code lengths, 3 bits each in the order
                // 16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1,15 (5 bits per
                // entry in two words), packed 3 bits per symbol
                const uint64_t ord_lo = 16ull | 17ull << 5 | 18ull << 10 | 0ull << 15 | 8ull << 20 | 7ull << 25 |
                                        9ull << 30 | 6ull << 35 | 10ull << 40 | 5ull << 45 | 11ull << 50 | 4ull << 55;
                const uint64_t ord_hi = 12ull | 3ull << 5 | 13ull << 10 | 2ull << 15 | 14ull << 20 | 1ull << 25 |
                                        15ull << 30;
                uint64_t cl = 0;
                for (int k = 0; k < ncl; k++) {
                    gi_refill(b);
                    const uint32_t v = gi_bits(b, 3);
                    const int s = (int)((k < 12 ? ord_lo >> (5 * k) : ord_hi >> (5 * (k - 12))) & 31u);
                    cl |= (uint64_t)v << (3 * s);
                }
                GiHuff clh;
                int rc = gi_build<LANES>(clh, sym, lane, GI_ROW_CL, 19,
                                         [cl](int i) -> uint32_t { return (uint32_t)(cl >> (3 * i)) & 7u; });
                if (rc) return rc;
                // the literal/length and distance code lengths, run-length
                // coded: into 4-bit cells after the symbol rows (GI_NIB_ROWS
                // rows of two lengths per lane), then both trees from them
                uint8_t *nib = (uint8_t *)(sym + GI_ROWS * LANES);
                const int ntot = nlit + ndist;
                int n = 0, prev = -1;
                while (n < ntot) {
                    gi_refill(b);
                    const int s = gi_decode<LANES>(b, clh, sym, lane, GI_ROW_CL);
                    if (s < 0) return GI_E_TREE;
                    int rep = 1, val = s;
                    if (s == 16) {
                        if (prev < 0) return GI_E_TREE;
                        rep = 3 + (int)gi_bits(b, 2);
                        val = prev;
                    } else if (s == 17) {
                        rep = 3 + (int)gi_bits(b, 3);
                        val = 0;
                    } else if (s == 18) {
                        rep = 11 + (int)gi_bits(b, 7);
                        val = 0;
                    }
                    if (n + rep > ntot) return GI_E_TREE;
                    for (int k = 0; k < rep; k++, n++) {
                        uint8_t *c = nib + (n >> 1) * LANES + lane;
                        *c = (n & 1) ? (uint8_t)(*c | (val << 4)) : (uint8_t)val;
                    }
                    prev = val;
                }
                rc = gi_build<LANES>(lit, sym, lane, GI_ROW_LIT, nlit, [nib, lane](int i) -> uint32_t {
                    return (uint32_t)(nib[(i >> 1) * LANES + lane] >> (4 * (i & 1))) & 15u;
                });
                if (rc) return rc;
                rc = gi_build<LANES>(dist, sym, lane, GI_ROW_DIST, ndist, [nib, lane, nlit](int i) -> uint32_t {
                    const int k = i + nlit;
                    return (uint32_t)(nib[(k >> 1) * LANES + lane] >> (4 * (k & 1))) & 15u;
                });
                if (rc) return rc;
            }
            // the block's symbols
            for (;;) {
                gi_refill(b);
                const int s = gi_decode<LANES>(b, lit, sym, lane, GI_ROW_LIT);
                if (s < 0) return GI_E_CODE;
                if (s < 256) {
                    if (o >= out_len) return GI_E_OVERRUN;
                    out[o++] = (uint8_t)s;
                    continue;
                }
                if (s == 256) break;
                if (s > 285) return GI_E_CODE;
                int lb, le;
                gi_len_code(s, lb, le);
                const uint32_t len = (uint32_t)lb + gi_bits(b, le);
                gi_refill(b);
                const int d = gi_decode<LANES>(b, dist, sym, lane, GI_ROW_DIST);
                if (d < 0 || d > 29) return GI_E_DIST;
                int db, de;
                gi_dist_code(d, db, de);
                const uint32_t dd = (uint32_t)db + gi_bits(b, de);
                if (dd > o) return GI_E_DIST;
                if (o + len > out_len) return GI_E_OVERRUN;
                uint8_t *q = out + o;
                if (dd < len && dd <= 8) {  // a short repeating pattern: loaded once, stored from registers
                    uint64_t pat = 0;
                    GI_UNROLL
                    for (uint32_t k = 0; k < 8; k++)
                        if (k < dd) pat |= (uint64_t)q[(int64_t)k - dd] << (8 * k);
                    uint32_t r = 0;
                    for (uint32_t k = 0; k < len; k++) {
                        q[k] = (uint8_t)(pat >> (8 * r));
                        r = (r + 1 == dd) ? 0 : r + 1;
                    }
                } else {  // chunks of up to 16 bytes whose sources are final: all loads, then the stores
                    for (uint32_t k = 0; k < len;) {
                        uint32_t m = len - k;
                        m = m < 16u ? m : 16u;
                        m = m < dd ? m : dd;
                        uint8_t t[16];
                        GI_UNROLL
                        for (uint32_t j = 0; j < 16; j++) t[j] = j < m ? q[(int64_t)(k + j) - dd] : 0;
                        GI_UNROLL
                        for (uint32_t j = 0; j < 16; j++)
                            if (j < m) q[k + j] = t[j];
                        k += m;
                    }
                }
                o += len;
            }
        } else {
            return GI_E_HEADER;
        }
        if (bfinal) break;
    }
    // consumed bits: every merged word minus the first word's lead and the buffer
    const int64_t used_bits = b.merged * 32 - b.sh0 - b.cnt;
    if (used_bits > 8 * (int64_t)in_len) return GI_E_INPUT;
    if (o != out_len) return GI_E_SIZE;
    return GI_OK;
}
