// tools/inflate_trips.cpp -- where the device inflater's loop trips go: the
// host twin of inflate.h (one lane) over every BGZF block of a BAM, counting
// trips per mode and output bytes per kind (literal, match, stored), and the
// trips of the slowest block per 64 (a wave's length is its slowest lane's).
//   g++ -O2 -I grom_amd/csrc tools/inflate_trips.cpp -o /tmp/inflate_trips && /tmp/inflate_trips x.bam
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
static long long g_trips[8], g_bytes[3], g_cur;
#define GI_TRIP(mode) (g_trips[(mode)]++, g_cur++)
#define GI_BYTES(kind, n) (g_bytes[(kind)] += (n))
#include "inflate.h"

int main(int argc, char **argv) {
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 1;
    std::vector<uint8_t> file;
    {
        fseek(f, 0, SEEK_END);
        long n = ftell(f);
        fseek(f, 0, SEEK_SET);
        file.resize(n + 64);
        if (fread(file.data(), 1, n, f) != (size_t)n) return 1;
        file.resize(n);
    }
    std::vector<uint8_t> out(65536 + 64);
    uint32_t tab[GI_LANE_DWORDS];
    size_t off = 0;
    long long nb = 0, tot = 0, wave_max = 0, wave_sum = 0, lane_sum = 0;
    std::vector<long long> per;
    while (off + 18 <= file.size()) {
        const uint8_t *h = file.data() + off;
        const int xlen = h[10] | h[11] << 8;
        const int bsize = h[16] | h[17] << 8;
        const long blen = bsize + 1;
        const uint32_t isize = *(const uint32_t *)(h + blen - 4);
        g_cur = 0;
        if (gi_inflate<1>(h + 12 + xlen, (uint32_t)(blen - 12 - xlen - 8), out.data(), isize, tab, 0)) return 2;
        per.push_back(g_cur);
        tot += isize;
        nb++;
        off += blen;
    }
    for (size_t i = 0; i < per.size(); i += 64) {
        long long m = 0;
        for (size_t j = i; j < per.size() && j < i + 64; j++) { m = per[j] > m ? per[j] : m; lane_sum += per[j]; }
        wave_sum += m * (long long)std::min<size_t>(64, per.size() - i);
    }
    long long trips = 0;
    for (int k = 0; k < 8; k++) trips += g_trips[k];
    printf("blocks %lld, output %lld bytes (%.1f per block), trips %lld (%.1f per block, %.3f per byte)\n", nb, tot,
           (double)tot / nb, trips, (double)trips / nb, (double)trips / tot);
    const char *names[] = {"header", "symbol", "copy", "stored", "done", "cl pass 1", "cl pass 2"};
    for (int k = 0; k < 7; k++) printf("  trips in %-10s %12lld (%.1f%%)\n", names[k], g_trips[k], 100.0 * g_trips[k] / trips);
    printf("bytes: literal %lld (%.1f%%), match %lld (%.1f%%), stored %lld\n", g_bytes[0], 100.0 * g_bytes[0] / tot,
           g_bytes[1], 100.0 * g_bytes[1] / tot, g_bytes[2]);
    printf("lane-trips: sum %lld, as waves of 64 (slowest lane) %lld: %.1f%% lanes idle\n", lane_sum, wave_sum,
           100.0 * (1.0 - (double)lane_sum / wave_sum));
    return 0;
}
