// tools/match_dist.cpp -- analysis only: the LZ77 match distances of every BGZF block
// of a BAM (the host twin's token pass, inflate.h gi_tokens), weighted by match
// length.  g++ -O2 -std=c++17 -o /tmp/match_dist tools/match_dist.cpp; /tmp/match_dist g.bam
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "../include/grom_amd.h"
#include "../grom_amd/csrc/inflate.h"
static uint16_t rd16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static uint32_t rd32(const uint8_t *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }
int main(int argc, char **argv) {
    FILE *f = fopen(argv[1], "rb"); fseek(f, 0, SEEK_END); long size = ftell(f); fseek(f, 0, SEEK_SET);
    std::vector<uint8_t> file(size + 64); if (fread(file.data(), 1, size, f) != (size_t)size) return 1;
    static uint32_t tab[GI_LANE_DWORDS];
    std::vector<uint32_t> tok(70000); std::vector<uint8_t> out(65536 + 64);
    double lit = 0, mat = 0; double hist[17] = {0}; double nmatch = 0; double nm_h[17] = {0};
    long off = 0; int nb = 0;
    while (off + 18 <= size) {
        const uint8_t *h = file.data() + off; int xlen = rd16(h + 10); int bsize = -1;
        for (int o = 0; o + 4 <= xlen;) { int sl = rd16(h + 12 + o + 2); if (h[12+o]=='B' && h[13+o]=='C' && sl==2) bsize = rd16(h+12+o+4); o += 4 + sl; }
        long blen = bsize + 1; uint32_t isize = rd32(h + blen - 4);
        uint32_t nt = 0;
        int rc = gi_tokens<1>(h + 12 + xlen, (uint32_t)(blen - 20 - xlen), out.data(), isize, tok.data(), 65536, &nt, tab, 0);
        if (rc) { fprintf(stderr, "rc %d\n", rc); return 1; }
        for (uint32_t i = 0; i < nt; i++) {
            uint32_t t = tok[i]; lit += t & 255;
            if (t & 0x80000000u) continue;
            uint32_t len = ((t >> 8) & 255) + 3, dist = ((t >> 16) & 0x7fff) + 1;
            int b = 0; while ((1u << b) < dist) b++;
            hist[b] += len; mat += len; nmatch++; nm_h[b]++;
        }
        off += blen; nb++;
    }
    printf("blocks %d literal bytes %.0f match bytes %.0f (%.1f%%) matches %.0f\n", nb, lit, mat, 100*mat/(lit+mat), nmatch);
    double c = 0;
    for (int b = 0; b < 17; b++) { c += hist[b]; printf("dist <= %6u: match bytes %5.1f%% cum %5.1f%%  matches %5.1f%%\n", 1u << b, 100*hist[b]/mat, 100*c/mat, 100*nm_h[b]/nmatch); }
}
