/*
 * synth.c -- deterministic synthetic genome + paired-end read generator.
 * See synth.h for the model.  Everything is driven by xoshiro256** streams
 * seeded from (cfg->seed, chromosome index, purpose), so a given config
 * always yields byte-identical FASTA/BAM files.
 */
#include "synth.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---------------- RNG ---------------- */
typedef struct { uint64_t s[4]; } xrng;

static uint64_t splitmix(uint64_t *x) {
    uint64_t z = (*x += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
static void xseed(xrng *r, uint64_t seed, uint64_t a, uint64_t b) {
    uint64_t x = seed ^ (a * 0x9E3779B97F4A7C15ULL) ^ (b * 0xD1B54A32D192ED03ULL);
    for (int i = 0; i < 4; i++) r->s[i] = splitmix(&x);
}
static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
static inline uint64_t xnext(xrng *r) {
    uint64_t *s = r->s;
    uint64_t res = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return res;
}
static inline double xunif(xrng *r) { return (xnext(r) >> 11) * (1.0 / 9007199254740992.0); }
static inline long xint(xrng *r, long n) { return (long)(xunif(r) * (double)n); }
static double xnorm(xrng *r) {
    double u1 = xunif(r), u2 = xunif(r);
    if (u1 < 1e-300) u1 = 1e-300;
    return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}
static double xexp(xrng *r, double mean) {
    double u = xunif(r);
    if (u < 1e-300) u = 1e-300;
    return -log(u) * mean;
}

static const char ACGT[4] = {'A', 'C', 'G', 'T'};

void synth_default_cfg(synth_cfg *c) {
    memset(c, 0, sizeof(*c));
    c->n_chr = 1;
    c->chr_len[0] = 1000000;
    strcpy(c->chr_name[0], "chr1");
    c->coverage = 30.0;
    for (int i = 0; i < SYNTH_MAX_CHR; i++) c->chr_cov[i] = -1.0;
    c->read_len = 150;
    c->insert_mean = 500.0;
    c->insert_sd = 50.0;
    c->snv_rate = 1e-3;
    c->indel_rate = 1e-4;
    c->max_indel = 20;
    c->err_rate = 0.002;
    c->lowq_frac = 0.02;
    c->hi_q = 30;
    c->lo_q = 10;
    c->lowmapq_frac = 0.03;
    c->softclip_frac = 0.01;
    c->munmap_frac = 0.002;
    c->dup_frac = 0.0;
    c->telomere_n = 10000;
    c->lower_frac = 0.1;
    c->gc_lo = 0.35;
    c->gc_hi = 0.55;
    c->repeat_rate = 2e-5;
    c->fasta_line = 60;
    c->cnv_rate = 0.0;
    c->multi_indel = 0.0;
    c->cnv_min = 10000;
    c->cnv_max = 300000;
    c->sv_per_mb = 0.0;
    c->sv_evidence = 0.5;
    c->ploidy = 2;
    c->seed = 2;
}

/* record i of a FASTA: its letters (case kept), NUL-terminated */
static char *fasta_record(const char *path, int want, long *len_out) {
    FILE *f = fopen(path, "r");
    if (!f) return NULL;
    char line[1 << 16];
    int rec = -1;
    long n = 0, cap = 1 << 20;
    char *s = NULL;
    while (fgets(line, sizeof(line), f)) {
        if (line[0] == '>') {
            if (rec == want) break;
            rec++;
            if (rec == want) s = (char *)malloc((size_t)cap);
            continue;
        }
        if (rec != want) continue;
        for (const char *q = line; *q; q++) {
            if (!((*q >= 'A' && *q <= 'Z') || (*q >= 'a' && *q <= 'z'))) continue;
            if (n + 1 >= cap) { cap *= 2; s = (char *)realloc(s, (size_t)cap); }
            s[n++] = *q;
        }
    }
    fclose(f);
    if (s) s[n] = 0;
    if (len_out) *len_out = n;
    return s;
}

int synth_cfg_from_fasta(synth_cfg *c, const char *path) {
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    char line[1 << 16];
    c->n_chr = 0;
    while (fgets(line, sizeof(line), f)) {
        if (line[0] == '>') {
            if (c->n_chr == SYNTH_MAX_CHR) break;
            int k = 0;
            while (line[1 + k] && line[1 + k] > ' ' && k < 47) { c->chr_name[c->n_chr][k] = line[1 + k]; k++; }
            c->chr_name[c->n_chr][k] = 0;
            c->chr_len[c->n_chr++] = 0;
            continue;
        }
        if (c->n_chr == 0) continue;
        for (const char *q = line; *q; q++)
            if ((*q >= 'A' && *q <= 'Z') || (*q >= 'a' && *q <= 'z')) c->chr_len[c->n_chr - 1]++;
    }
    fclose(f);
    c->ref_fasta = path;
    return c->n_chr > 0 ? 0 : -1;
}

char *synth_reference(const synth_cfg *c, int ci) {
    if (c->ref_fasta) return fasta_record(c->ref_fasta, ci, NULL);
    long n = c->chr_len[ci];
    char *s = (char *)malloc((size_t)n + 1);
    xrng r;
    xseed(&r, c->seed, (uint64_t)ci + 1, 1);
    double gc = 0.41;
    if (c->ref_period > 0) { /* one pattern, repeated */
        const long P = c->ref_period < n ? c->ref_period : n;
        for (long i = 0; i < P; i++) {
            double u = xunif(&r);
            if (u < gc) s[i] = (u < gc * 0.5) ? 'G' : 'C';
            else s[i] = (u < gc + (1.0 - gc) * 0.5) ? 'A' : 'T';
        }
        for (long i = P; i < n; i++) s[i] = s[i - P];
    } else {
        for (long i = 0; i < n; i++) {
            if (i % 100000 == 0) gc = c->gc_lo + (c->gc_hi - c->gc_lo) * xunif(&r);
            double u = xunif(&r);
            if (u < gc) s[i] = (u < gc * 0.5) ? 'G' : 'C';
            else s[i] = (u < gc + (1.0 - gc) * 0.5) ? 'A' : 'T';
        }
    }
    /* dinucleotide repeat runs */
    if (c->repeat_rate > 0) {
        long i = (long)xexp(&r, 1.0 / c->repeat_rate);
        while (i < n) {
            int len = 20 + (int)xint(&r, 60);
            char a = ACGT[xint(&r, 4)], b = ACGT[xint(&r, 4)];
            for (int k = 0; k < len && i + k < n; k++) s[i + k] = (k & 1) ? b : a;
            i += len + (long)xexp(&r, 1.0 / c->repeat_rate);
        }
    }
    /* soft-masked blocks */
    if (c->lower_frac > 0) {
        long i = (long)xexp(&r, 5000.0 / c->lower_frac);
        while (i < n) {
            long len = 200 + xint(&r, 4800);
            for (long k = 0; k < len && i + k < n; k++) s[i + k] = (char)(s[i + k] + 32);
            i += len + (long)xexp(&r, 5000.0 / c->lower_frac);
        }
    }
    long tn = c->telomere_n;
    if (tn * 3 > n) tn = n / 3;
    for (long i = 0; i < tn; i++) { s[i] = 'N'; s[n - 1 - i] = 'N'; }
    s[n] = 0;
    return s;
}

/* ---------------- donor haplotypes ---------------- */
typedef struct {
    char *seq;     /* donor bases (upper case) */
    int32_t *map;  /* donor index -> reference index, -1 for inserted base */
    int32_t *inv;  /* reference index -> first donor index with map >= it */
    long len;
} haplo;

static int synth_ploidy(const synth_cfg *c) {
    return c->ploidy >= 1 && c->ploidy <= SYNTH_MAX_PLOIDY ? c->ploidy : 2;
}

/* Donor haplotypes of chromosome ci: `ploidy` copies (synth_cfg.ploidy, 2 by
 * default).  A diploid variant is on haplotype 0, 1 or both (gt 0/1/2); with
 * another ploidy it is on a random non-empty subset (carrier mask), so allele
 * fractions take every value k/ploidy.  The diploid random stream is the one
 * the generator has always drawn. */
static void build_haplos(const synth_cfg *c, int ci, const char *ref, haplo *h) {
    long n = c->chr_len[ci];
    const int P = synth_ploidy(c);
    xrng r;
    xseed(&r, c->seed, (uint64_t)ci + 1, 2);
    for (int k = 0; k < P; k++) {
        long cap = n + n / 50 + 1024;
        h[k].seq = (char *)malloc(cap);
        h[k].map = (int32_t *)malloc(cap * sizeof(int32_t));
        h[k].len = 0;
    }
    double vrate = c->snv_rate + c->indel_rate;
    long next_var = vrate > 0 ? (long)xexp(&r, 1.0 / vrate) : n + 1;
    long i = 0;
    while (i < n) {
        char rb = ref[i];
        char ub = (rb >= 'a' && rb <= 'z') ? (char)(rb - 32) : rb;
        if (i == next_var && ub != 'N' && i > 0 && i + c->max_indel + 2 < n) {
            unsigned carriers;
            if (P == 2) {
                int gt = (int)xint(&r, 3); /* 0: hap0 only, 1: hap1 only, 2: both */
                carriers = gt == 2 ? 3u : (1u << gt);
            } else {
                do { carriers = (unsigned)xint(&r, 1L << P); } while (carriers == 0);
            }
            double u = xunif(&r) * vrate;
            int consumed = 1;
            if (u < c->snv_rate) {
                char alt;
                do { alt = ACGT[xint(&r, 4)]; } while (alt == ub);
                for (int k = 0; k < P; k++) {
                    int has = (carriers >> k) & 1;
                    h[k].seq[h[k].len] = has ? alt : ub;
                    h[k].map[h[k].len++] = (int32_t)i;
                }
            } else {
                int len = 1 + (int)xint(&r, c->max_indel);
                int ins = xunif(&r) < 0.5;
                /* multi-allelic: the carriers after the first carry a second length */
                int lens[SYNTH_MAX_PLOIDY];
                for (int k = 0; k < P; k++) lens[k] = len;
                if (c->multi_indel > 0 && xunif(&r) < c->multi_indel) {
                    carriers = (1u << P) - 1;
                    int len2 = 1 + (int)xint(&r, c->max_indel);
                    for (int k = 1; k < P; k++) lens[k] = len2;
                }
                if (ins) {
                    for (int k = 0; k < P; k++) {
                        int has = (carriers >> k) & 1;
                        h[k].seq[h[k].len] = ub;
                        h[k].map[h[k].len++] = (int32_t)i;
                        if (has)
                            for (int q = 0; q < lens[k]; q++) {
                                h[k].seq[h[k].len] = ACGT[xint(&r, 4)];
                                h[k].map[h[k].len++] = -1;
                            }
                    }
                } else {
                    /* deletion of ref[i+1 .. i+lens[k]] on the haplotypes that carry it */
                    int span = 0;
                    for (int k = 0; k < P; k++) span = lens[k] > span ? lens[k] : span;
                    for (int k = 0; k < P; k++) {
                        int has = (carriers >> k) & 1;
                        h[k].seq[h[k].len] = ub;
                        h[k].map[h[k].len++] = (int32_t)i;
                        for (int q = has ? lens[k] + 1 : 1; q <= span; q++) {
                            char b = ref[i + q];
                            h[k].seq[h[k].len] = (b >= 'a' && b <= 'z') ? (char)(b - 32) : b;
                            h[k].map[h[k].len++] = (int32_t)(i + q);
                        }
                    }
                    consumed = 1 + span;
                }
            }
            i += consumed;
            next_var = i + 2 * c->max_indel + (long)xexp(&r, 1.0 / vrate);
            continue;
        }
        if (i == next_var) next_var++;
        for (int k = 0; k < P; k++) {
            h[k].seq[h[k].len] = ub;
            h[k].map[h[k].len++] = (int32_t)i;
        }
        i++;
    }
    for (int k = 0; k < P; k++) {
        h[k].inv = (int32_t *)malloc((size_t)(n + 1) * sizeof(int32_t));
        long ri = 0;
        for (long d = 0; d < h[k].len; d++) {
            int32_t m = h[k].map[d];
            if (m < 0) continue;
            while (ri <= m) h[k].inv[ri++] = (int32_t)d;
        }
        while (ri <= n) h[k].inv[ri++] = (int32_t)h[k].len;
    }
}

static void free_haplos(haplo *h, int P) {
    for (int k = 0; k < P; k++) { free(h[k].seq); free(h[k].map); free(h[k].inv); }
}

/* ---------------- record heap (sorted emission) ---------------- */
typedef struct { int32_t pos; uint64_t order; bam_rec rec; } hent;
typedef struct { hent *a; long n, cap; } rheap;

static int hless(const hent *x, const hent *y) {
    return x->pos < y->pos || (x->pos == y->pos && x->order < y->order);
}
static void hpush(rheap *h, hent e) {
    if (h->n == h->cap) {
        h->cap = h->cap ? h->cap * 2 : 4096;
        h->a = (hent *)realloc(h->a, h->cap * sizeof(hent));
    }
    long i = h->n++;
    h->a[i] = e;
    while (i > 0) {
        long p = (i - 1) / 2;
        if (!hless(&h->a[i], &h->a[p])) break;
        hent t = h->a[i]; h->a[i] = h->a[p]; h->a[p] = t;
        i = p;
    }
}
static hent hpop(rheap *h) {
    hent top = h->a[0];
    h->a[0] = h->a[--h->n];
    long i = 0;
    for (;;) {
        long l = 2 * i + 1, r = l + 1, m = i;
        if (l < h->n && hless(&h->a[l], &h->a[m])) m = l;
        if (r < h->n && hless(&h->a[r], &h->a[m])) m = r;
        if (m == i) break;
        hent t = h->a[i]; h->a[i] = h->a[m]; h->a[m] = t;
        i = m;
    }
    return top;
}

/* ---------------- read construction ---------------- */
typedef struct {
    int32_t pos;        /* leftmost mapped reference base */
    int32_t ref_end;    /* one past last mapped reference base */
    int n_cigar;
    uint32_t cigar[512];
    char seq[1024];
    uint8_t qual[1024];
    int len;
} aln;

static void push_op(aln *a, int op, int len) {
    if (len <= 0) return;
    if (a->n_cigar > 0 && (int)(a->cigar[a->n_cigar - 1] & 0xf) == op) {
        a->cigar[a->n_cigar - 1] += (uint32_t)len << 4;
        return;
    }
    a->cigar[a->n_cigar++] = ((uint32_t)len << 4) | (uint32_t)op;
}

/* align donor[d0, d0+L) of haplotype h; clip_left/right bases become random
 * soft-clipped sequence.  Returns 0 if no base maps. */
static int make_aln(const haplo *h, long d0, int L, int clip_left, int clip_right, xrng *r, aln *a) {
    a->n_cigar = 0;
    a->len = L;
    int first = -1, last = -1;
    for (int k = 0; k < L; k++) {
        int32_t m = (k < clip_left || k >= L - clip_right) ? -1 : h->map[d0 + k];
        a->seq[k] = (k < clip_left || k >= L - clip_right) ? ACGT[xint(r, 4)] : h->seq[d0 + k];
        if (m >= 0) { if (first < 0) first = k; last = k; }
    }
    if (first < 0) return 0;
    push_op(a, GC_SOFT_CLIP, first);
    int32_t prev = -1;
    for (int k = first; k <= last; k++) {
        int32_t m = (k < clip_left || k >= L - clip_right) ? -1 : h->map[d0 + k];
        if (m < 0) { push_op(a, GC_INS, 1); continue; }
        if (prev >= 0 && m > prev + 1) push_op(a, GC_DEL, m - prev - 1);
        push_op(a, GC_MATCH, 1);
        prev = m;
    }
    push_op(a, GC_SOFT_CLIP, L - 1 - last);
    a->pos = h->map[d0 + first];
    a->ref_end = prev + 1;
    return 1;
}

static void fill_rec(bam_rec *b, const char *name, int tid, const aln *a, int with_cigar, int flag,
                     int mapq, int mtid, int mpos, int isize, int pos_override) {
    int lq = (int)strlen(name) + 1;
    int nc = with_cigar ? a->n_cigar : 0;
    int L = a->len;
    b->data_len = lq + 4 * nc + (L + 1) / 2 + L;
    b->m_data = b->data_len;
    b->data = (uint8_t *)malloc(b->data_len);
    memcpy(b->data, name, lq);
    if (nc) memcpy(b->data + lq, a->cigar, 4 * nc);
    uint8_t *s = b->data + lq + 4 * nc;
    memset(s, 0, (L + 1) / 2);
    for (int k = 0; k < L; k++) {
        int code;
        switch (a->seq[k]) {
        case 'A': code = 1; break;
        case 'C': code = 2; break;
        case 'G': code = 4; break;
        case 'T': code = 8; break;
        default: code = 15;
        }
        s[k >> 1] |= (uint8_t)(code << ((~k & 1) << 2));
    }
    memcpy(s + (L + 1) / 2, a->qual, L);
    b->tid = tid;
    b->pos = with_cigar ? a->pos : pos_override;
    b->l_qname = (uint8_t)lq;
    b->mapq = (uint8_t)mapq;
    b->n_cigar = (uint16_t)nc;
    b->flag = (uint16_t)flag;
    b->l_qseq = L;
    b->mtid = mtid;
    b->mpos = mpos;
    b->isize = isize;
    int end = with_cigar ? a->ref_end : pos_override + 1;
    b->bin = (uint16_t)bam_reg2bin(b->pos, end > b->pos ? end : b->pos + 1);
}

static void add_errors(aln *a, const synth_cfg *c, xrng *r) {
    for (int k = 0; k < a->len; k++) {
        if (xunif(r) < c->err_rate) {
            char o = a->seq[k], n;
            do { n = ACGT[xint(r, 4)]; } while (n == o);
            a->seq[k] = n;
        }
        a->qual[k] = (uint8_t)(xunif(r) < c->lowq_frac ? c->lo_q : c->hi_q);
    }
}

static int draw_mapq(const synth_cfg *c, xrng *r) {
    return xunif(r) < c->lowmapq_frac ? (int)xint(r, 20) : 60;
}

/* Copy-number regions of chromosome ci: fragment start rate is multiplied
 * by the region's depth factor (0 = homozygous loss, 0.5, 1.5, 2).  Regions
 * are sorted and disjoint; drawn from their own stream so that a genome with
 * no regions reads exactly as before. */
typedef struct { long start, end; double f; } cnv_reg;
static int synth_cnv_regions(const synth_cfg *c, int ci, cnv_reg **out) {
    long n = c->chr_len[ci];
    int k = (int)(c->cnv_rate * (double)n + 0.5);
    *out = NULL;
    if (k <= 0 || c->cnv_max <= 0) return 0;
    static const double fs[4] = {0.0, 0.5, 1.5, 2.0};
    cnv_reg *r = (cnv_reg *)malloc(sizeof(cnv_reg) * k);
    xrng g;
    xseed(&g, c->seed, (uint64_t)ci + 1, 7);
    long span = n / k;
    int m = 0;
    for (int i = 0; i < k; i++) {
        long lo = (long)i * span + c->telomere_n, hi = (long)(i + 1) * span - c->telomere_n;
        long len = c->cnv_min + xint(&g, c->cnv_max - c->cnv_min + 1);
        if (hi - lo <= len + 2) continue;
        long s = lo + xint(&g, hi - lo - len);
        r[m].start = s;
        r[m].end = s + len;
        r[m].f = fs[xint(&g, 4)];
        m++;
    }
    *out = r;
    return m;
}

/* ---------------- breakpoint SVs (alignment-level model) ----------------
 * Each SV is simulated as the alignments an aligner would report around its
 * breakpoints, on top of the normal reference-like coverage: discordant
 * pairs (orientation and insert size of the rearranged donor), split reads
 * with SA:Z tags, soft-clipped reads and unmapped mates.  Read sequence is
 * the reference at the mapped bases (no mismatches), quality hi_q.  Events
 * are drawn genome-wide from their own stream, so both sides of a
 * translocation are generated consistently by the two chromosomes' passes. */
enum { SV_DEL, SV_DUP, SV_INV, SV_INS, SV_CTX, SV_NTYPES };
typedef struct { int type, chr, chr2; long s, e, y; uint64_t id; } sv_event;

static int synth_sv_events(const synth_cfg *c, sv_event **out) {
    *out = NULL;
    if (c->sv_per_mb <= 0) return 0;
    int cap = 64, n = 0;
    sv_event *ev = (sv_event *)malloc(sizeof(sv_event) * cap);
    for (int ci = 0; ci < c->n_chr; ci++) {
        long len = c->chr_len[ci];
        int k = (int)(c->sv_per_mb * (double)len / 1e6 + 0.5);
        if (k <= 0) continue;
        xrng g;
        xseed(&g, c->seed, (uint64_t)ci + 1, 11);
        long span = len / k;
        for (int i = 0; i < k; i++) {
            long lo = (long)i * span + c->telomere_n + 4000, hi = (long)(i + 1) * span - c->telomere_n - 4000;
            int type = (int)xint(&g, SV_NTYPES);
            if (type == SV_CTX && c->n_chr < 2) type = SV_DEL;
            long L;
            switch (type) {
            case SV_DEL: L = xunif(&g) < 0.5 ? 40 + xint(&g, 120) : 300 + xint(&g, 3000); break;
            case SV_DUP: L = 200 + xint(&g, 3000); break;
            case SV_INV: L = 600 + xint(&g, 4000); break;
            case SV_INS: L = 150 + xint(&g, 300); break; /* inserted length (novel sequence) */
            default: L = 1;
            }
            if (hi - lo <= L + 2) { /* dense SVs: a slot narrower than two telomere margins */
                lo = (long)i * span + 1500;
                hi = (long)(i + 1) * span - 1500;
                if (lo < c->telomere_n + 4000) lo = c->telomere_n + 4000;
                if (hi > len - c->telomere_n - 4000) hi = len - c->telomere_n - 4000;
            }
            if (hi - lo <= L + 2) continue;
            long st = lo + xint(&g, hi - lo - (type == SV_INS || type == SV_CTX ? 1 : L));
            if (n == cap) { cap *= 2; ev = (sv_event *)realloc(ev, sizeof(sv_event) * cap); }
            sv_event *e = &ev[n++];
            e->type = type;
            e->chr = ci;
            e->s = st;
            e->e = (type == SV_INS || type == SV_CTX) ? st : st + L;
            e->chr2 = -1;
            e->y = L; /* INS: inserted length */
            if (type == SV_CTX) {
                e->chr2 = (ci + 1) % c->n_chr;
                long l2 = c->chr_len[e->chr2];
                e->y = c->telomere_n + 4000 + xint(&g, l2 - 2 * (c->telomere_n + 4000));
            }
            e->id = ((uint64_t)ci << 32) | (uint64_t)i;
        }
    }
    *out = ev;
    return n;
}

typedef struct {
    const synth_cfg *c;
    int ci;
    const char *ref;
    long len;
    rheap *heap;
    uint64_t *order;
    long n;
} sv_out;

/* one alignment: ops (op,len) pairs; SEQ is the reference under M ops */
static void sv_emit(sv_out *o, const char *name, long pos, const int *ops, int n_ops, int flag, int mapq, int mtid,
                    long mpos, long isize, const char *sa) {
    const synth_cfg *c = o->c;
    int L = c->read_len;
    if (pos < 0 || pos + L >= o->len) return;
    aln a;
    a.n_cigar = 0;
    a.len = L;
    long rp = pos;
    int q = 0;
    for (int k = 0; k < n_ops; k++) {
        int op = ops[2 * k], ln = ops[2 * k + 1];
        push_op(&a, op, ln);
        for (int j = 0; j < ln && q < L; j++) {
            char b;
            if (op == GC_MATCH) b = o->ref[rp++];
            else b = o->ref[(pos + L + 7 * q) % o->len]; /* clipped bases: some other sequence */
            if (b >= 'a' && b <= 'z') b = (char)(b - 32);
            a.seq[q] = b;
            a.qual[q] = (uint8_t)c->hi_q;
            q++;
        }
    }
    a.pos = (int32_t)pos;
    a.ref_end = (int32_t)rp;
    hent e;
    memset(&e, 0, sizeof(e));
    fill_rec(&e.rec, name, o->ci, &a, 1, flag, mapq, mtid, (int)mpos, (int)isize, 0);
    if (sa) {
        /* append SA:Z:<sa> (GROM parses it when the record's aux is 1..99 bytes) */
        int sl = (int)strlen(sa) + 1;
        e.rec.data = (uint8_t *)realloc(e.rec.data, e.rec.data_len + 3 + sl);
        uint8_t *p = e.rec.data + e.rec.data_len;
        p[0] = 'S'; p[1] = 'A'; p[2] = 'Z';
        memcpy(p + 3, sa, sl);
        e.rec.data_len += 3 + sl;
        e.rec.m_data = e.rec.data_len;
    }
    e.pos = e.rec.pos;
    e.order = (*o->order)++;
    hpush(o->heap, e);
    o->n++;
}

/* a read-pair: (pos1, flag1) on this chromosome, its mate at mpos; isize
 * from the reference span (positive for the leftmost read) */
static long sv_isize(long p1, long p2, int L, int first) {
    long lo = p1 < p2 ? p1 : p2, hi = (p1 > p2 ? p1 : p2) + L;
    long v = hi - lo;
    return first ? v : -v;
}

static int sv_mapq(const synth_cfg *c, xrng *r) { return xunif(r) < c->lowmapq_frac ? (int)xint(r, 20) : 60; }

static void sv_pair(sv_out *o, xrng *r, const char *name, long p1, int rev1, long p2, int rev2) {
    int L = o->c->read_len;
    int f1 = GF_PAIRED | GF_READ1 | (rev1 ? GF_REVERSE : 0) | (rev2 ? GF_MREVERSE : 0);
    int f2 = GF_PAIRED | GF_READ2 | (rev2 ? GF_REVERSE : 0) | (rev1 ? GF_MREVERSE : 0);
    int m = GC_MATCH;
    int ops[2] = {m, L};
    int q1 = sv_mapq(o->c, r), q2 = sv_mapq(o->c, r);
    sv_emit(o, name, p1, ops, 1, f1, q1, o->ci, p2, sv_isize(p1, p2, L, p1 <= p2), NULL);
    sv_emit(o, name, p2, ops, 1, f2, q2, o->ci, p1, sv_isize(p1, p2, L, p2 < p1), NULL);
}

/* a split read: k bases at ref a (then clipped), the other L-k at ref b
 * (after a clip); the longer part is the primary alignment, the other one
 * its SA:Z entry; `rev` strand for both parts (sa_rev flips the SA strand). */
static void sv_split(sv_out *o, xrng *r, const char *name, long a, long b, int k, int rev, int sa_rev, long mpos,
                     int mrev, int flag_mate_unmapped) {
    int L = o->c->read_len;
    char sa[96];
    int ops[4];
    long pos;
    const char *cn = o->c->chr_name[o->ci];
    if (k >= L - k) {
        pos = a;
        ops[0] = GC_MATCH; ops[1] = k; ops[2] = GC_SOFT_CLIP; ops[3] = L - k;
        snprintf(sa, sizeof(sa), "%s,%ld,%c,%dS%dM,60,0;", cn, b + 1, (rev ^ sa_rev) ? '-' : '+', k, L - k);
    } else {
        pos = b;
        ops[0] = GC_SOFT_CLIP; ops[1] = k; ops[2] = GC_MATCH; ops[3] = L - k;
        snprintf(sa, sizeof(sa), "%s,%ld,%c,%dM%dS,60,0;", cn, a + 1, (rev ^ sa_rev) ? '-' : '+', k, L - k);
    }
    int flag = GF_PAIRED | GF_READ1 | (rev ? GF_REVERSE : 0);
    if (flag_mate_unmapped) flag |= GF_MUNMAP;
    else if (mrev) flag |= GF_MREVERSE;
    long isz = flag_mate_unmapped ? 0 : sv_isize(pos, mpos, L, pos <= mpos);
    sv_emit(o, name, pos, ops, 2, flag, sv_mapq(o->c, r), o->ci, flag_mate_unmapped ? pos : mpos, isz, sa);
    if (!flag_mate_unmapped) {
        int m_ops[2] = {GC_MATCH, L};
        int mf = GF_PAIRED | GF_READ2 | (mrev ? GF_REVERSE : 0) | (rev ? GF_MREVERSE : 0);
        sv_emit(o, name, mpos, m_ops, 1, mf, sv_mapq(o->c, r), o->ci, pos, sv_isize(pos, mpos, L, mpos < pos), NULL);
    }
}

/* every record chromosome ci contributes to the SV events */
static long synth_sv_records(const synth_cfg *c, int ci, const char *ref, rheap *heap, uint64_t *order) {
    sv_event *ev;
    int n_ev = synth_sv_events(c, &ev);
    sv_out o = {c, ci, ref, c->chr_len[ci], heap, order, 0};
    const int L = c->read_len;
    const double cov = c->chr_cov[ci] >= 0 ? c->chr_cov[ci] : c->coverage;
    const int ins = (int)c->insert_mean;
    /* spanning fragments over one breakpoint: depth x insert / (2 L), scaled */
    int npair = (int)(cov * (double)(ins - L) / (2.0 * L) * c->sv_evidence + 0.5);
    int nsplit = (int)(cov * 0.5 * c->sv_evidence + 0.5);
    if (npair < 1) npair = 1;
    char name[64];
    for (int k = 0; k < n_ev; k++) {
        const sv_event *e = &ev[k];
        if (e->chr != ci && e->chr2 != ci) continue;
        xrng r;
        xseed(&r, c->seed, e->id + 1000003ULL, 13);
        const long s = e->s, en = e->e;
        int f = 0;
#define NAME() snprintf(name, sizeof(name), "SV%02d:%06d:%04d", e->chr, k, f++)
        switch (e->type) {
        case SV_DEL:
            for (int j = 0; j < npair; j++) {
                int fi = (int)lround(c->insert_mean + c->insert_sd * xnorm(&r));
                long a = s - L - xint(&r, fi > 2 * L ? fi - 2 * L : 1);
                long b = en + (fi - (s - a)) - L;
                if (b < en) b = en;
                NAME();
                sv_pair(&o, &r, name, a, 0, b, 1);
            }
            for (int j = 0; j < nsplit; j++) {
                int kk = 30 + (int)xint(&r, L - 60);
                int fi = (int)lround(c->insert_mean + c->insert_sd * xnorm(&r));
                NAME();
                if (j & 1) {
                    /* F read over the junction, its R mate downstream in the donor */
                    long mp = en + (fi - kk) - L;
                    sv_split(&o, &r, name, s - kk, en, kk, 0, 0, mp, 1, 0);
                } else {
                    /* R read over the junction, its F mate upstream */
                    long mp = s - kk - (fi - L);
                    sv_split(&o, &r, name, s - kk, en, kk, 1, 0, mp, 0, 0);
                }
            }
            break;
        case SV_DUP:
            for (int j = 0; j < npair; j++) {
                int fi = (int)lround(c->insert_mean + c->insert_sd * xnorm(&r));
                long a = en - L - xint(&r, fi > 2 * L ? fi - 2 * L : 1);
                long b = s + (fi - (en - a)) - L;
                if (b < s) b = s;
                NAME();
                sv_pair(&o, &r, name, a, 0, b, 1); /* F at the dup end, R mate near its start */
            }
            for (int j = 0; j < nsplit; j++) {
                int kk = 30 + (int)xint(&r, L - 60);
                int fi = (int)lround(c->insert_mean + c->insert_sd * xnorm(&r));
                NAME();
                if (j & 1) {
                    /* F read: k bases before the dup end, then its start; R mate downstream of the start */
                    long mp = s + (fi - kk) - L;
                    sv_split(&o, &r, name, en - kk, s, kk, 0, 0, mp, 1, 0);
                } else {
                    /* R read over the junction, its F mate upstream (before the dup end) */
                    long mp = en - kk - (fi - L);
                    sv_split(&o, &r, name, en - kk, s, kk, 1, 0, mp, 0, 0);
                }
            }
            break;
        case SV_INV:
            for (int j = 0; j < npair; j++) {
                int fi = (int)lround(c->insert_mean + c->insert_sd * xnorm(&r));
                /* junction at s: F outside, the mate reads the inverted segment forward */
                long a = s - L - xint(&r, fi > 2 * L ? fi - 2 * L : 1);
                long t = fi - L - (s - a);
                if (t < 0) t = 0;
                NAME();
                sv_pair(&o, &r, name, a, 0, en - t - L, 0);
                /* junction at e: both reverse */
                fi = (int)lround(c->insert_mean + c->insert_sd * xnorm(&r));
                long u = (en - s) - L - xint(&r, fi > 2 * L ? fi - 2 * L : 1);
                if (u < 0) u = 0;
                long p1 = en - u - L, p2 = s + u + fi - L;
                if (p2 < en) p2 = en;
                NAME();
                sv_pair(&o, &r, name, p1, 1, p2, 1);
            }
            for (int j = 0; j < nsplit; j++) {
                int kk = 30 + (int)xint(&r, L - 60);
                int fi = (int)lround(c->insert_mean + c->insert_sd * xnorm(&r));
                NAME();
                /* the inverted part aligns on the other strand */
                sv_split(&o, &r, name, s - kk, en - (L - kk), kk, 0, 1, s - kk + fi - L, 1, 0);
            }
            break;
        case SV_INS: {
            const long I = e->y;
            for (int j = 0; j < npair; j++) {
                int fi = (int)lround(c->insert_mean + c->insert_sd * xnorm(&r));
                long a = s - L - xint(&r, 40);
                long b = s + (fi - I - (s - a)) - L + L / 2;
                if (b < s + 1) b = s + 1;
                NAME();
                if (j % 3 == 2) {
                    /* the mate lies inside the insertion: unmapped */
                    int ops[2] = {GC_MATCH, L};
                    sv_emit(&o, name, a, ops, 1, GF_PAIRED | GF_READ1 | GF_MUNMAP, sv_mapq(c, &r), ci, a, 0, NULL);
                } else {
                    sv_pair(&o, &r, name, a, 0, b, 1);
                }
                /* reads clipped at the insertion point */
                int kk = 10 + (int)xint(&r, 60);
                int ops1[4] = {GC_MATCH, L - kk, GC_SOFT_CLIP, kk};
                NAME();
                sv_emit(&o, name, s + 1 - (L - kk), ops1, 2, 0, sv_mapq(c, &r), -1, -1, 0, NULL);
                int ops2[4] = {GC_SOFT_CLIP, kk, GC_MATCH, L - kk};
                NAME();
                sv_emit(&o, name, s + 1, ops2, 2, GF_REVERSE, sv_mapq(c, &r), -1, -1, 0, NULL);
            }
            break;
        }
        case SV_CTX: {
            /* fragments joining (chr, s) to (chr2, y); both sides from the same stream */
            for (int j = 0; j < npair; j++) {
                int fi = (int)lround(c->insert_mean + c->insert_sd * xnorm(&r));
                long a = s - L - xint(&r, fi > 2 * L ? fi - 2 * L : 1);
                long t = fi - (s - a) - L;
                if (t < 0) t = 0;
                int orient = (int)xint(&r, 2); /* partner read reverse (0) or forward (1) */
                long b = orient == 0 ? e->y + t : e->y - t - L;
                int q1 = sv_mapq(c, &r), q2 = sv_mapq(c, &r);
                snprintf(name, sizeof(name), "SX%02d:%06d:%04d", e->chr, k, f++);
                int ops[2] = {GC_MATCH, L};
                int rev2 = orient == 0;
                if (ci == e->chr) {
                    int fl = GF_PAIRED | GF_READ1 | (rev2 ? GF_MREVERSE : 0);
                    sv_emit(&o, name, a, ops, 1, fl, q1, e->chr2, b, 0, NULL);
                }
                if (ci == e->chr2) {
                    int fl = GF_PAIRED | GF_READ2 | (rev2 ? GF_REVERSE : 0);
                    sv_emit(&o, name, b, ops, 1, fl, q2, e->chr, a, 0, NULL);
                }
            }
            break;
        }
        }
#undef NAME
    }
    free(ev);
    return o.n;
}

long synth_reads(const synth_cfg *c, int ci, const char *ref, synth_emit_fn emit, void *ctx) {
    long n = c->chr_len[ci];
    int L = c->read_len;
    haplo h[SYNTH_MAX_PLOIDY];
    const int ploidy = synth_ploidy(c);
    build_haplos(c, ci, ref, h);
    /* prefix count of N bases so fragments never touch an N block */
    int32_t *ncount = (int32_t *)malloc((size_t)(n + 1) * sizeof(int32_t));
    ncount[0] = 0;
    for (long i = 0; i < n; i++) ncount[i + 1] = ncount[i] + (ref[i] == 'N' || ref[i] == 'n');

    xrng r;
    xseed(&r, c->seed, (uint64_t)ci + 1, 3);
    double cov = c->chr_cov[ci] >= 0 ? c->chr_cov[ci] : c->coverage;
    double n_frag = cov * (double)n / (2.0 * L);
    if (n_frag <= 0) n_frag = 0;
    double gap = n_frag > 0 ? (double)n / n_frag : (double)n;
    rheap heap = {0};
    long emitted = 0;
    uint64_t order = 0;
    double start_f = n_frag > 0 ? xexp(&r, gap) : (double)n;
    uint64_t frag_id = 0;
    cnv_reg *creg;
    int n_creg = synth_cnv_regions(c, ci, &creg), ic = 0;
    /* the SV evidence records wait in the heap until their position comes up */
    synth_sv_records(c, ci, ref, &heap, &order);
    aln a1, a2;
    char name[64];
    while (start_f < (double)n) {
        long start = (long)start_f;
        double f = 1.0;
        while (ic < n_creg && creg[ic].end <= start) ic++;
        if (ic < n_creg && creg[ic].start <= start) f = creg[ic].f;
        if (f == 0.0) {
            start_f = (double)creg[ic].end + xexp(&r, gap);
            continue;
        }
        start_f += (f == 1.0) ? xexp(&r, gap) : xexp(&r, gap / f);
        int hk = (int)xint(&r, ploidy);
        const haplo *hp = &h[hk];
        int ins = (int)lround(c->insert_mean + c->insert_sd * xnorm(&r));
        if (ins < L) ins = L;
        /* fragment start in reference coordinates, mapped onto the donor */
        long d0 = hp->inv[start];
        if (d0 + ins >= hp->len) continue;
        int32_t rs = hp->map[d0], re = hp->map[d0 + ins - 1];
        if (rs < 0 || re < 0 || re <= rs) continue;
        if (ncount[re + 1] - ncount[rs] != 0) continue;
        int ndup = (xunif(&r) < c->dup_frac) ? 2 : 1;
        frag_id++;
        /* flush everything that now sorts before this fragment */
        while (heap.n > 0 && heap.a[0].pos < start && !(c->max_emit > 0 && emitted >= c->max_emit)) {
            hent e = hpop(&heap);
            emit(ctx, &e.rec);
            free(e.rec.data);
            emitted++;
        }
        if (c->max_emit > 0 && emitted >= c->max_emit) break;
        for (int dup = 0; dup < ndup; dup++) {
            int cl1 = 0, cr2 = 0;
            if (xunif(&r) < c->softclip_frac) cl1 = 5 + (int)xint(&r, 26);
            if (xunif(&r) < c->softclip_frac) cr2 = 5 + (int)xint(&r, 26);
            if (!make_aln(hp, d0, L, cl1, 0, &r, &a1)) continue;
            if (!make_aln(hp, d0 + ins - L, L, 0, cr2, &r, &a2)) continue;
            add_errors(&a1, c, &r);
            add_errors(&a2, c, &r);
            int mq1 = draw_mapq(c, &r), mq2 = draw_mapq(c, &r);
            int left_is_r1 = xunif(&r) < 0.5;
            int munmap = xunif(&r) < c->munmap_frac;
            if (dup == 0) snprintf(name, sizeof(name), "SYN%02d:%010llu", ci, (unsigned long long)frag_id);
            else snprintf(name, sizeof(name), "SYN%02d:%010llu:d", ci, (unsigned long long)frag_id);
            int tlen = a2.ref_end - a1.pos;
            int f1 = GF_PAIRED | (left_is_r1 ? GF_READ1 : GF_READ2);
            int f2 = GF_PAIRED | GF_REVERSE | (left_is_r1 ? GF_READ2 : GF_READ1);
            hent e1, e2;
            memset(&e1, 0, sizeof(e1));
            memset(&e2, 0, sizeof(e2));
            if (munmap) {
                f1 |= GF_MUNMAP;
                f2 |= GF_UNMAP;
                f2 &= ~GF_REVERSE;
                fill_rec(&e1.rec, name, ci, &a1, 1, f1, mq1, ci, a1.pos, 0, 0);
                fill_rec(&e2.rec, name, ci, &a2, 0, f2, 0, ci, a1.pos, 0, a1.pos);
            } else {
                f1 |= GF_PROPER | GF_MREVERSE;
                f2 |= GF_PROPER;
                fill_rec(&e1.rec, name, ci, &a1, 1, f1, mq1, ci, a2.pos, tlen, 0);
                fill_rec(&e2.rec, name, ci, &a2, 1, f2, mq2, ci, a1.pos, -tlen, 0);
            }
            e1.pos = e1.rec.pos; e1.order = order++;
            e2.pos = e2.rec.pos; e2.order = order++;
            hpush(&heap, e1);
            hpush(&heap, e2);
        }
    }
    while (heap.n > 0) {
        hent e = hpop(&heap);
        if (!(c->max_emit > 0 && emitted >= c->max_emit)) {
            emit(ctx, &e.rec);
            emitted++;
        }
        free(e.rec.data);
    }
    free(heap.a);
    free(creg);
    free(ncount);
    free_haplos(h, ploidy);
    return emitted;
}

/* ---------------- the files: FASTA, BAM and its index ----------------
 * Chromosomes are generated on parallel threads; each fills 0xff00-byte BGZF
 * payloads (records kept inside one block when they fit, as htslib does) and
 * queues them for a pool of compressor threads.  The index is accumulated
 * while the records are written, with offsets as (block number << 16 | offset
 * in the block), and mapped to file offsets once the compressed block sizes
 * are known. */
#include <pthread.h>
#include <unistd.h>

typedef struct {
    unsigned char *raw, *comp;
    int len, clen;
} sblock;

typedef struct {
    sblock **blk;
    int n_blk, cap_blk;
    unsigned char *cur;
    int cur_len;
    bai_racc *acc;
    char *ref;
    int done;
    struct swriter *w;
} schrom;

typedef struct swriter {
    const synth_cfg *c;
    schrom *ch;
    pthread_mutex_t mu;
    pthread_cond_t cv;
    sblock **q;       /* blocks waiting for compression */
    int q_head, q_tail, q_cap;
    int next_chr, gens_left, err;
    int order[SYNTH_MAX_CHR];
} swriter;

static void q_push(swriter *w, sblock *b) {
    pthread_mutex_lock(&w->mu);
    if (w->q_tail - w->q_head == w->q_cap) {
        int nc = w->q_cap ? 2 * w->q_cap : 1024;
        sblock **nq = (sblock **)malloc(sizeof(sblock *) * (size_t)nc);
        for (int i = 0; i < w->q_tail - w->q_head; i++) nq[i] = w->q[(w->q_head + i) % (w->q_cap ? w->q_cap : 1)];
        free(w->q);
        w->q = nq;
        w->q_tail -= w->q_head;
        w->q_head = 0;
        w->q_cap = nc;
    }
    w->q[w->q_tail % w->q_cap] = b;
    w->q_tail++;
    pthread_cond_signal(&w->cv);
    pthread_mutex_unlock(&w->mu);
}

/* BGZF compression level: 6 (zlib's and samtools' default) unless
 * GROM_SYNTH_LEVEL says otherwise (the bench's large BAMs) */
static int synth_level(void) {
    const char *e = getenv("GROM_SYNTH_LEVEL");
    const int l = e ? atoi(e) : 6;
    return l < 1 ? 1 : (l > 9 ? 9 : l);
}

static int compress_one(sblock *b) {
    unsigned char out[65536 + 64];
    const int n = bgzf_block_compress(b->raw, b->len, out, synth_level());
    if (n < 0) return -1;
    b->comp = (unsigned char *)malloc((size_t)n);
    if (!b->comp) return -1;
    memcpy(b->comp, out, (size_t)n);
    b->clen = n;
    free(b->raw);
    b->raw = NULL;
    return 0;
}

static int compress_one(sblock *b);

/* a generator that gets ahead of the compressors compresses queued blocks
 * itself until at most SYNTH_QUEUE_MAX wait (the raw blocks of a 30x genome
 * would otherwise pile up: 190 GB); which thread compresses a block does not
 * change its bytes */
#define SYNTH_QUEUE_MAX 2048

static void q_help(swriter *w) {
    for (;;) {
        pthread_mutex_lock(&w->mu);
        if (w->q_tail - w->q_head <= SYNTH_QUEUE_MAX) {
            pthread_mutex_unlock(&w->mu);
            return;
        }
        sblock *b = w->q[w->q_head % w->q_cap];
        w->q_head++;
        pthread_mutex_unlock(&w->mu);
        if (compress_one(b)) w->err = 1;
    }
}

static void sc_flush(schrom *c) {
    if (c->cur_len == 0) return;
    sblock *b = (sblock *)calloc(1, sizeof(sblock));
    b->raw = c->cur;
    b->len = c->cur_len;
    if (c->n_blk == c->cap_blk) {
        c->cap_blk = c->cap_blk ? 2 * c->cap_blk : 1024;
        c->blk = (sblock **)realloc(c->blk, sizeof(sblock *) * (size_t)c->cap_blk);
    }
    c->blk[c->n_blk++] = b;
    c->cur = (unsigned char *)malloc(BGZF_PAYLOAD);
    c->cur_len = 0;
    q_push(c->w, b);
    q_help(c->w);
}

static void sc_write(schrom *c, const void *src, int n) {
    const unsigned char *p = (const unsigned char *)src;
    while (n > 0) {
        int take = BGZF_PAYLOAD - c->cur_len;
        if (take > n) take = n;
        memcpy(c->cur + c->cur_len, p, (size_t)take);
        c->cur_len += take;
        p += take;
        n -= take;
        if (c->cur_len >= BGZF_PAYLOAD) sc_flush(c);
    }
}

static void le32(unsigned char *p, uint32_t v) { p[0] = v & 0xff; p[1] = (v >> 8) & 0xff; p[2] = (v >> 16) & 0xff; p[3] = v >> 24; }
static void le16(unsigned char *p, uint16_t v) { p[0] = v & 0xff; p[1] = v >> 8; }

static void emit_par(void *ctx, const bam_rec *b) {
    schrom *c = (schrom *)ctx;
    unsigned char h[36];
    le32(h, (uint32_t)(32 + b->data_len));
    le32(h + 4, (uint32_t)b->tid);
    le32(h + 8, (uint32_t)b->pos);
    h[12] = b->l_qname;
    h[13] = b->mapq;
    le16(h + 14, b->bin);
    le16(h + 16, b->n_cigar);
    le16(h + 18, b->flag);
    le32(h + 20, (uint32_t)b->l_qseq);
    le32(h + 24, (uint32_t)b->mtid);
    le32(h + 28, (uint32_t)b->mpos);
    le32(h + 32, (uint32_t)b->isize);
    if (c->cur_len + 36 + b->data_len > BGZF_PAYLOAD && c->cur_len > 0) sc_flush(c);
    const uint64_t vb = ((uint64_t)c->n_blk << 16) | (uint64_t)c->cur_len;
    sc_write(c, h, 36);
    sc_write(c, b->data, b->data_len);
    const uint64_t ve = ((uint64_t)c->n_blk << 16) | (uint64_t)c->cur_len;
    bai_racc_push(c->acc, b->pos < 0 ? 0 : b->pos, bam_end_pos(b), vb, ve, (b->flag & 4) != 0);
}

static void *gen_main(void *arg) {
    swriter *w = (swriter *)arg;
    for (;;) {
        pthread_mutex_lock(&w->mu);
        const int k = w->next_chr < w->c->n_chr ? w->order[w->next_chr++] : -1;
        pthread_mutex_unlock(&w->mu);
        if (k < 0) break;
        schrom *c = &w->ch[k];
        c->w = w;
        c->acc = bai_racc_new();
        c->cur = (unsigned char *)malloc(BGZF_PAYLOAD);
        c->ref = synth_reference(w->c, k);
        synth_reads(w->c, k, c->ref, emit_par, c);
        sc_flush(c);
        free(c->cur);
        c->cur = NULL;
        bai_racc_flush(c->acc);
    }
    pthread_mutex_lock(&w->mu);
    w->gens_left--;
    pthread_cond_broadcast(&w->cv);
    pthread_mutex_unlock(&w->mu);
    /* then help compress */
    for (;;) {
        pthread_mutex_lock(&w->mu);
        while (w->q_head == w->q_tail && w->gens_left > 0) pthread_cond_wait(&w->cv, &w->mu);
        if (w->q_head == w->q_tail) {
            pthread_mutex_unlock(&w->mu);
            break;
        }
        sblock *b = w->q[w->q_head % w->q_cap];
        w->q_head++;
        pthread_mutex_unlock(&w->mu);
        if (compress_one(b)) w->err = 1;
    }
    return NULL;
}

typedef struct {
    const schrom *ch;
    int64_t *base; /* file offset of each chromosome's first block */
    int64_t **coff; /* per chromosome: file offset of block b (n_blk + 1 entries) */
} voff_map;

static uint64_t map_voff(void *ctx, int ref, uint64_t v) {
    const voff_map *m = (const voff_map *)ctx;
    const int64_t b = (int64_t)(v >> 16);
    /* the end of a block is written as the start of the next one, as
     * bgzf_tell (and htslib) report it */
    if (b < m->ch[ref].n_blk && (int)(v & 0xffff) == m->ch[ref].blk[b]->len) return (uint64_t)m->coff[ref][b + 1] << 16;
    return ((uint64_t)m->coff[ref][b] << 16) | (v & 0xffff);
}

int synth_write_files(const synth_cfg *c, const char *fasta_path, const char *bam_path) {
    {  /* a new FASTA under an old name: drop its <fasta>.info cache, which the
        * CLI (like GROM.c:22308) would otherwise trust */
        char info[4096];
        snprintf(info, sizeof(info), "%s.info", fasta_path);
        remove(info);
    }
    swriter w;
    memset(&w, 0, sizeof(w));
    w.c = c;
    w.ch = (schrom *)calloc((size_t)c->n_chr, sizeof(schrom));
    pthread_mutex_init(&w.mu, NULL);
    pthread_cond_init(&w.cv, NULL);
    for (int i = 0; i < c->n_chr; i++) w.order[i] = i;
    for (int a = 1; a < c->n_chr; a++) /* longest first */
        for (int b = a; b > 0 && c->chr_len[w.order[b]] > c->chr_len[w.order[b - 1]]; b--) {
            int t = w.order[b]; w.order[b] = w.order[b - 1]; w.order[b - 1] = t;
        }
    long ncpu = sysconf(_SC_NPROCESSORS_ONLN);
    int n_thr = getenv("GROM_SYNTH_THREADS") ? atoi(getenv("GROM_SYNTH_THREADS")) : (int)(ncpu < 16 ? ncpu : 16);
    if (n_thr < 1) n_thr = 1;
    w.gens_left = n_thr;
    pthread_t thr[64];
    if (n_thr > 64) n_thr = 64;
    for (int t = 0; t < n_thr; t++) pthread_create(&thr[t], NULL, gen_main, &w);
    for (int t = 0; t < n_thr; t++) pthread_join(thr[t], NULL);
    int rc = w.err ? -1 : 0;

    FILE *fa = fopen(fasta_path, "w");
    if (!fa) rc = -1;
    if (fa && c->ref_fasta) { /* the given FASTA, byte for byte */
        FILE *in = fopen(c->ref_fasta, "rb");
        char buf[1 << 16];
        size_t k;
        if (!in) rc = -1;
        while (in && (k = fread(buf, 1, sizeof(buf), in)) > 0) fwrite(buf, 1, k, fa);
        if (in) fclose(in);
    }
    for (int i = 0; i < c->n_chr && fa && !c->ref_fasta; i++) {
        fprintf(fa, ">%s synthetic\n", c->chr_name[i]);
        for (long k = 0; k < c->chr_len[i]; k += c->fasta_line) {
            long m = c->chr_len[i] - k;
            if (m > c->fasta_line) m = c->fasta_line;
            fwrite(w.ch[i].ref + k, 1, m, fa);
            fputc('\n', fa);
        }
    }
    if (fa && fclose(fa) != 0) rc = -1;

    /* header blocks, then each chromosome's blocks in order, then EOF */
    bam_hdr h;
    memset(&h, 0, sizeof(h));
    char text[64 * 96 + 64];
    int tl = snprintf(text, sizeof(text), "@HD\tVN:1.4\tSO:coordinate\n");
    for (int i = 0; i < c->n_chr; i++)
        tl += snprintf(text + tl, sizeof(text) - tl, "@SQ\tSN:%s\tLN:%ld\n", c->chr_name[i], c->chr_len[i]);
    h.text = text;
    h.l_text = tl;
    h.n_ref = c->n_chr;
    h.ref_name = (char **)calloc(c->n_chr, sizeof(char *));
    h.ref_len = (int32_t *)calloc(c->n_chr, sizeof(int32_t));
    for (int i = 0; i < c->n_chr; i++) {
        h.ref_name[i] = (char *)c->chr_name[i];
        h.ref_len[i] = (int32_t)c->chr_len[i];
    }
    voff_map vm;
    vm.ch = w.ch;
    vm.base = (int64_t *)calloc((size_t)c->n_chr + 1, sizeof(int64_t));
    vm.coff = (int64_t **)calloc((size_t)c->n_chr, sizeof(int64_t *));
    bgzf_writer bw;
    if (rc == 0 && bgzf_open_write(&bw, bam_path, synth_level()) != 0) rc = -1;
    if (rc == 0) {
        rc = bam_write_header(&bw, &h);
        if (rc == 0 && bgzf_flush_block(&bw) != 0) rc = -1;
        int64_t off = ftell(bw.fp);
        for (int i = 0; i < c->n_chr && rc == 0; i++) {
            schrom *s = &w.ch[i];
            vm.coff[i] = (int64_t *)malloc(sizeof(int64_t) * ((size_t)s->n_blk + 1));
            for (int b = 0; b < s->n_blk; b++) {
                vm.coff[i][b] = off;
                if (fwrite(s->blk[b]->comp, 1, (size_t)s->blk[b]->clen, bw.fp) != (size_t)s->blk[b]->clen) rc = -1;
                off += s->blk[b]->clen;
            }
            vm.coff[i][s->n_blk] = off;
        }
        if (bgzf_close_write(&bw) != 0) rc = -1;
    }
    if (rc == 0) {
        char path[4096];
        snprintf(path, sizeof(path), "%s.bai", bam_path);
        bai_racc **R = (bai_racc **)calloc((size_t)c->n_chr, sizeof(bai_racc *));
        for (int i = 0; i < c->n_chr; i++) R[i] = w.ch[i].acc;
        rc = bai_write_racc(path, R, c->n_chr, 0, map_voff, &vm);  /* a real index, as samtools index writes */
        free(R);
    }
    for (int i = 0; i < c->n_chr; i++) {
        schrom *s = &w.ch[i];
        for (int b = 0; b < s->n_blk; b++) {
            free(s->blk[b]->raw);
            free(s->blk[b]->comp);
            free(s->blk[b]);
        }
        free(s->blk);
        free(s->ref);
        bai_racc_free(s->acc);
        free(vm.coff[i]);
    }
    free(vm.coff);
    free(vm.base);
    free(w.ch);
    free(w.q);
    free(h.ref_name);
    free(h.ref_len);
    pthread_mutex_destroy(&w.mu);
    pthread_cond_destroy(&w.cv);
    return rc;
}
