// inflate_host.cpp -- the host twin of the device BGZF inflater (inflate.h):
// the same decoder compiled for the CPU with one lane, and a self-test that
// checks it against zlib on every block of a BAM (tests/test_host.py).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <vector>

#include "../../include/grom_amd.h"
#include "inflate.h"

extern "C" int grom_inflate_block_host(const uint8_t *in, uint32_t in_len, uint8_t *out, uint32_t out_len) {
    thread_local uint32_t tab[GI_LANE_DWORDS];
    return gi_inflate<1>(in, in_len, out, out_len, tab, 0);
}

// the two-phase decoder (gi_tokens, then the tokens replayed): the same bytes
// as gi_inflate, or GI_E_TOKCAP for a block with more than tokcap tokens
extern "C" int grom_inflate_block_host2(const uint8_t *in, uint32_t in_len, uint8_t *out, uint32_t out_len,
                                        uint32_t tokcap) {
    thread_local uint32_t tab[GI_LANE_DWORDS];
    thread_local std::vector<uint32_t> tok;
    tok.assign(((size_t)tokcap + 3) & ~(size_t)3, 0);
    uint32_t nt = 0;
    const int rc = gi_tokens<1>(in, in_len, out, out_len, tok.data(), tokcap & ~3u, &nt, tab, 0);
    return rc ? rc : gi_lz(tok.data(), nt, out, out_len);
}

static uint16_t rd16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static uint32_t rd32(const uint8_t *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }

// Every BGZF block of `bam_path` (at most max_blocks; <= 0: all) inflated by
// the twin and by zlib: the number of blocks whose output or status differ,
// or a negative value if the file is not BGZF.  *n_blocks gets the blocks
// checked, *bytes their inflated size.
extern "C" int64_t grom_inflate_selftest(const char *bam_path, int64_t max_blocks, int64_t *n_blocks, int64_t *bytes) {
    FILE *f = fopen(bam_path, "rb");
    if (!f) return -1;
    fseek(f, 0, SEEK_END);
    const long size = ftell(f);
    fseek(f, 0, SEEK_SET);
    std::vector<uint8_t> file((size_t)size + 64);
    if (fread(file.data(), 1, (size_t)size, f) != (size_t)size) {
        fclose(f);
        return -1;
    }
    fclose(f);
    std::vector<uint8_t> a(65536 + 64), b(65536 + 64);
    int64_t bad = 0, nb = 0, nbytes = 0;
    long off = 0;
    while (off + 18 <= size && (max_blocks <= 0 || nb < max_blocks)) {
        const uint8_t *h = file.data() + off;
        if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || !(h[3] & 4)) return -2;
        const int xlen = rd16(h + 10);
        int bsize = -1;
        for (int o = 0; o + 4 <= xlen;) {
            const int sl = rd16(h + 12 + o + 2);
            if (h[12 + o] == 'B' && h[12 + o + 1] == 'C' && sl == 2) bsize = rd16(h + 12 + o + 4);
            o += 4 + sl;
        }
        if (bsize < 0 || off + bsize + 1 > size) return -3;
        const long blen = bsize + 1;
        const uint32_t isize = rd32(h + blen - 4);
        const uint8_t *data = h + 12 + xlen;
        const uint32_t dlen = (uint32_t)(blen - 12 - xlen - 8);
        if (isize > 65536) return -4;
        // zlib
        z_stream zs;
        memset(&zs, 0, sizeof(zs));
        int zrc = inflateInit2(&zs, -15);
        zs.next_in = (Bytef *)data;
        zs.avail_in = dlen;
        zs.next_out = a.data();
        zs.avail_out = (uInt)a.size();
        if (zrc == Z_OK) zrc = inflate(&zs, Z_FINISH);
        const bool zok = zrc == Z_STREAM_END && zs.total_out == isize;
        inflateEnd(&zs);
        // the twin
        memset(b.data(), 0xa5, b.size());
        const int rc = grom_inflate_block_host(data, dlen, b.data(), isize);
        bool same = zok ? (rc == GI_OK && memcmp(a.data(), b.data(), isize) == 0) : (rc != GI_OK);
        // the two-phase decoder: the same bytes, or a refusal (a block over
        // the token cap) that the one-phase decoder then covers
        memset(b.data(), 0x5a, b.size());
        const int rc2 = grom_inflate_block_host2(data, dlen, b.data(), isize, 65536);
        same = same && (zok ? (rc2 == GI_OK && memcmp(a.data(), b.data(), isize) == 0) : (rc2 != GI_OK));
        if (!same) {
            if (bad < 5) fprintf(stderr, "inflate selftest: block at %ld (isize %u): zlib %d, twin %d\n", off, isize, zrc, rc);
            bad++;
        }
        nbytes += isize;
        nb++;
        off += blen;
    }
    if (n_blocks) *n_blocks = nb;
    if (bytes) *bytes = nbytes;
    return bad;
}
