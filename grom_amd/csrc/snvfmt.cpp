// snvfmt.cpp -- VCF text of the SNV rows without printf on the hot path.
//
// The reference prints each row with one fprintf (GROM.c:11203-11274,
// 15063-15107); at ~1e5 rows per 100 Mb that call dominates the host side of
// the scan.  Here integers are written directly, "%.2f" is computed exactly
// from the double's binary value (glibc rounds the exact value half to even,
// and so does fmt_2f), and the two "%e" fields -- table p-values and float
// ratios, which take few distinct values -- are formatted once per distinct
// bit pattern by snprintf itself and reused.  Output is byte-identical to the
// fprintf form (tests/test_host.py::test_fmt_2f_matches_printf and every VCF
// parity test).
#include "snvfmt.h"

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>
#include <unordered_map>

int fmt_2f(char *out, double v) {
    if (!std::isfinite(v) || std::fabs(v) >= 1e15) return snprintf(out, 400, "%.2f", v);
    char *p = out;
    if (std::signbit(v)) {
        *p++ = '-';
        v = -v;
    }
    uint64_t ip = 0;  // round(v * 100), half to even on the exact value
    if (v != 0) {
        int e;
        const double fr = std::frexp(v, &e);                // v = fr * 2^e, fr in [0.5, 1)
        const uint64_t m = (uint64_t)std::ldexp(fr, 53);    // exact 53-bit mantissa
        const int sh = 53 - e;                              // v = m * 2^-sh, sh > 0 for v < 2^52
        const unsigned __int128 x = (unsigned __int128)m * 100u;  // < 2^60
        if (sh < 127) {
            ip = (uint64_t)(x >> sh);
            const unsigned __int128 one = 1;
            const unsigned __int128 rem = x & ((one << sh) - 1), half = one << (sh - 1);
            if (rem > half || (rem == half && (ip & 1))) ip++;
        }  // else x < 2^60 < half: rounds to 0
    }
    char tmp[24];
    int n = 0;
    uint64_t whole = ip / 100;
    do {
        tmp[n++] = (char)('0' + whole % 10);
        whole /= 10;
    } while (whole);
    while (n) *p++ = tmp[--n];
    *p++ = '.';
    *p++ = (char)('0' + (ip % 100) / 10);
    *p++ = (char)('0' + ip % 10);
    *p = 0;
    return (int)(p - out);
}

namespace {

inline char *put_i32(char *p, int32_t v) {
    uint32_t u = (uint32_t)v;
    if (v < 0) {
        *p++ = '-';
        u = 0u - u;
    }
    char tmp[12];
    int n = 0;
    do {
        tmp[n++] = (char)('0' + u % 10);
        u /= 10;
    } while (u);
    while (n) *p++ = tmp[--n];
    return p;
}

inline char *put_str(char *p, const char *s, size_t n) {
    memcpy(p, s, n);
    return p + n;
}

// "%e" of a double, memoised per bit pattern
struct ECache {
    std::unordered_map<uint64_t, std::string> m;
    char *put(char *p, double v) {
        uint64_t key;
        memcpy(&key, &v, 8);
        auto it = m.find(key);
        if (it == m.end()) {
            char b[64];
            const int w = snprintf(b, sizeof(b), "%e", v);
            it = m.emplace(key, std::string(b, (size_t)w)).first;
        }
        return put_str(p, it->second.data(), it->second.size());
    }
};

void rows_range(const grom_params &P, const char *name, const grom_snv_cand *c, size_t lo, size_t hi, double lim,
                std::string &out) {
    static const char dna[4] = {'A', 'C', 'G', 'T'};
    static const char fmt_col[] = "\t.\t.\t.\tGT:PR:AF:A:C:G:T:AL:CL:GL:TL:BQ:MQ:PIR:FS\t";
    const size_t name_len = strlen(name);
    ECache ec;
    std::string line;
    line.resize(name_len + 4 * 400 + 512 + 2 * (size_t)P.ploidy);  // fmt_2f may write up to 400 bytes
    out.reserve(out.size() + (hi - lo) * 120);
    for (size_t i = lo; i < hi; i++) {
        const grom_snv_cand &s = c[i];
        const double ratio = (double)s.ratio;
        if (!(s.rc_all <= lim || ratio >= P.high_cov_min_snv_ratio)) continue;
        int cn = (int)round(ratio * P.ploidy);
        if (cn == 0) cn = 1;
        const int b = s.base;
        char *p0 = &line[0], *p = p0;
        p = put_str(p, name, name_len);
        *p++ = '\t';
        p = put_i32(p, s.pos + 1);
        *p++ = '\t';
        *p++ = '\t';
        *p++ = (char)s.ref_base;
        *p++ = '\t';
        *p++ = dna[b];
        p = put_str(p, fmt_col, sizeof(fmt_col) - 1);
        for (int k = 0; k < P.ploidy; k++) {
            *p++ = (k < cn) ? '1' : '0';
            if (k < P.ploidy - 1) *p++ = '/';
        }
        *p++ = ':';
        p = ec.put(p, s.binom);
        *p++ = ':';
        p = ec.put(p, ratio);
        for (int k = 0; k < 4; k++) {
            *p++ = ':';
            p = put_i32(p, s.snv[k]);
        }
        for (int k = 0; k < 4; k++) {
            *p++ = ':';
            p = put_i32(p, s.lowmq[k]);
        }
        *p++ = ':';
        p += fmt_2f(p, (double)s.bq_all / (double)s.rc_all);
        *p++ = ':';
        p += fmt_2f(p, (double)s.mq_all / (double)s.rc_all);
        *p++ = ':';
        p += fmt_2f(p, (double)s.pir[b] / (double)s.snv[b]);
        *p++ = ':';
        p += fmt_2f(p, (double)s.fs[b] / (double)s.snv[b]);
        *p++ = '\n';
        out.append(p0, (size_t)(p - p0));
    }
}

}  // namespace

void snv_rows_format(const grom_params &P, const char *chr_name, const grom_snv_cand *c, size_t n, double lim,
                     std::vector<std::string> &parts) {
    unsigned nt = std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
    if (n < 16384) nt = 1;
    parts.assign(nt, std::string());
    if (nt == 1) {
        rows_range(P, chr_name, c, 0, n, lim, parts[0]);
        return;
    }
    std::vector<std::thread> th;
    th.reserve(nt);
    for (unsigned t = 0; t < nt; t++)
        th.emplace_back(rows_range, std::cref(P), chr_name, c, n * t / nt, n * (t + 1) / nt, lim, std::ref(parts[t]));
    for (auto &t : th) t.join();
}

extern "C" int64_t grom_fmt_selftest(int64_t n, uint64_t seed) {
    // test hook: fmt_2f against printf on ratios of integers (the values the
    // rows print) plus edge cases; returns the number of mismatches
    static const double edge[] = {0.0, -0.0, 0.005, 0.015, 0.125, 0.375, 2.675, 1.005, 99.995, 1e14 + 0.125,
                                  0.0 / 1.0, 1.0 / 0.0, -1.0 / 0.0, 123456.785, 5e-324, 0.994999999999999,
                                  0.995, 29.5 / 3.0};
    int64_t bad = 0;
    char a[400], b[400];
    auto check = [&](double v) {
        fmt_2f(a, v);
        snprintf(b, sizeof(b), "%.2f", v);
        if (strcmp(a, b) != 0) bad++;
    };
    for (double v : edge) check(v);
    check(std::nan(""));
    volatile double z = 0.0;
    check(z / z);
    uint64_t s = seed ? seed : 0x9e3779b97f4a7c15ull;
    for (int64_t i = 0; i < n; i++) {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        const int64_t num = (int64_t)(s % 200000), den = (int64_t)((s >> 32) % 5000) + 1;
        check((double)num / (double)den);
        check((double)(num % 1000) / 8.0);  // exact binary ties
    }
    return bad;
}

void snv_rows_format_tab(const grom_params &P, const char *chr_name, const grom_snv_cand *c, size_t n, double lim,
                         const char *ref, int64_t len, int32_t lseq, std::string &out) {
    static const char dna[4] = {'A', 'C', 'G', 'T'};
    char b[512];
    for (size_t i = 0; i < n; i++) {
        const grom_snv_cand &s = c[i];
        const double ratio = (double)s.ratio;
        if (!(s.rc_all <= lim || ratio >= P.high_cov_min_snv_ratio)) continue;
        const int k = s.base;
        // the two depth lists of this row are never written by the reference
        // (GROM.c:3771-3778, malloc'ed and printed only): fresh pages read 0
        int w = snprintf(b, sizeof b, "SNV\t%s\t%d\t%c\t%e\t%d\t%d", chr_name, s.pos, dna[k], ratio, 0, 0);
        out.append(b, (size_t)w);
        for (int j = 0; j < 4; j++) out.append(b, (size_t)snprintf(b, sizeof b, "\t%d", s.snv[j]));
        for (int j = 0; j < 4; j++) out.append(b, (size_t)snprintf(b, sizeof b, "\t%d", s.lowmq[j]));
        w = snprintf(b, sizeof b, "\t%d\t%d\t%d\t%d\t%d\t%d\t%d", s.bq, s.bq_all, s.mq, s.mq_all, s.bq_rc, s.mq_rc, s.rc_all);
        out.append(b, (size_t)w);
        const double pir = (double)s.pir[k] / (double)s.snv[k], fs = (double)s.fs[k] / (double)s.snv[k];
        const bool inner = s.pos > 0 && s.pos < len - 1;
        w = snprintf(b, sizeof b, "\t%.2f\t%.2f\t%c%c%c\t", pir, fs, inner ? ref[s.pos - 1] : '.', inner ? ref[s.pos] : '.',
                     inner ? ref[s.pos + 1] : '.');
        out.append(b, (size_t)w);
        for (int32_t j = 0; j < lseq; j++) {
            const int64_t x = (int64_t)s.pos - lseq + 1 + j;
            out.push_back(x < 0 ? 'N' : ref[x]);
        }
        for (int32_t j = 0; j < lseq - 1; j++) {
            const int64_t x = (int64_t)s.pos + lseq - 1 - j;
            out.push_back(x >= len - 1 ? 'N' : ref[x]);
        }
        out.append(b, (size_t)snprintf(b, sizeof b, "\t%e\t%e\n", s.binom, s.hez));
    }
}
