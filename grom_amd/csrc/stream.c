/*
 * stream.c -- host front end (see stream.h).
 */
#include "stream.h"

#include <ctype.h>
#include <math.h>
#include <pthread.h>
#include <unistd.h>
#include <stdlib.h>
#include <string.h>

/* ---------------- FASTA ---------------- */

static int fasta_grow(grom_fasta *f, int want, int *cap) {
    if (want <= *cap) return 0;
    int c = *cap ? *cap : 64;
    while (c < want) c *= 2;
    void *a = realloc(f->names, sizeof(*f->names) * c), *b = realloc(f->name_len, sizeof(int) * c),
         *d = realloc(f->file_pos, sizeof(long) * c), *e = realloc(f->len, sizeof(long) * c);
    if (a) f->names = a;
    if (b) f->name_len = b;
    if (d) f->file_pos = d;
    if (e) f->len = e;
    if (!a || !b || !d || !e) return -1;
    *cap = c;
    return 0;
}

/* load_genome_info (GROM.c:1047-1081): "<n> <mappable>" then per chromosome
 * "<i> <name_len> <file_pos> <len> <name>"; a line that does not parse or is
 * out of order drops the whole table (n = 0) but, as in the reference, keeps
 * the mappable length already read from the first line. */
static void fasta_load_info(grom_fasta *f, const char *path, int *cap) {
    char name[4096];
    snprintf(name, sizeof(name), "%s.info", path);
    FILE *fp = fopen(name, "r");
    if (!fp) return;
    int n = 0;
    long mappable = 0;
    if (fscanf(fp, "%d %ld\n", &n, &mappable) == 2) {
        f->mappable = mappable;
        if (n < 0 || n > GROM_MAX_CHR_NAMES || fasta_grow(f, n, cap) != 0) n = 0;
        for (int i = 0; i < n; i++) {
            int idx = -1, nl = 0;
            long pos = 0, len = 0;
            char nm[GROM_MAX_CHR_NAME_LEN];
            if (fscanf(fp, "%d %d %ld %ld %49s\n", &idx, &nl, &pos, &len, nm) != 5 || idx != i) {
                n = 0;
                break;
            }
            memset(f->names[i], 0, GROM_MAX_CHR_NAME_LEN);
            memcpy(f->names[i], nm, strlen(nm));
            f->name_len[i] = nl;
            f->file_pos[i] = pos;
            f->len[i] = len;
        }
        f->n = n;
    }
    fclose(fp);
}

/* save_genome_info (GROM.c:1028-1045) */
static void fasta_save_info(const grom_fasta *f, const char *path) {
    char name[4096];
    snprintf(name, sizeof(name), "%s.info", path);
    FILE *fp = fopen(name, "w");
    if (!fp) return;
    fprintf(fp, "%d %ld\n", f->n, f->mappable);
    for (int i = 0; i < f->n; i++) fprintf(fp, "%d %d %ld %ld %s\n", i, f->name_len[i], f->file_pos[i], f->len[i], f->names[i]);
    fclose(fp);
}

int grom_fasta_open_cached(grom_fasta *f, const char *path) {
    memset(f, 0, sizeof(*f));
    f->fh = fopen(path, "r");
    if (!f->fh) return -1;
    int cap = 0;
    fasta_load_info(f, path, &cap);
    if (f->n > 0) return 0;
    /* GROM.c:22308-22311: no usable cache -> index the FASTA and save it
     * (find_genome_length adds to a mappable length a failed load kept) */
    const long kept = f->mappable;
    fclose(f->fh);
    free(f->names);
    free(f->name_len);
    free(f->file_pos);
    free(f->len);
    if (grom_fasta_open(f, path) != 0) return -1;
    f->mappable += kept;
    fasta_save_info(f, path);
    return 0;
}

int grom_fasta_open(grom_fasta *f, const char *path) {
    memset(f, 0, sizeof(*f));
    f->fh = fopen(path, "r");
    if (!f->fh) return -1;
    int cap = 64;
    f->names = malloc(sizeof(*f->names) * cap);
    f->name_len = malloc(sizeof(int) * cap);
    f->file_pos = malloc(sizeof(long) * cap);
    f->len = malloc(sizeof(long) * cap);
    /* find_genome_length, GROM.c:1321-1428: lines read with fgets(1000);
     * a header's name runs to its first non-graph character. */
    char line[1000];
    long cur_len = 0;
    while (fgets(line, sizeof(line), f->fh)) {
        if (line[0] != '>') {
            for (const char *c = line; *c; c++)
                if (isalpha((unsigned char)*c)) {
                    if (*c != 'N' && *c != 'n') f->mappable++;
                    cur_len++;
                }
            continue;
        }
        long here = ftell(f->fh);
        int L = (int)strlen(line), name_end = L;
        for (int w = L - 1; w > 0; w--)
            if (!isgraph((unsigned char)line[w])) name_end = w;
        if (f->n > 0) f->len[f->n - 1] = cur_len;
        cur_len = 0;
        if (f->n >= GROM_MAX_CHR_NAMES) { f->n++; continue; }
        if (f->n == cap) {
            cap *= 2;
            f->names = realloc(f->names, sizeof(*f->names) * cap);
            f->name_len = realloc(f->name_len, sizeof(int) * cap);
            f->file_pos = realloc(f->file_pos, sizeof(long) * cap);
            f->len = realloc(f->len, sizeof(long) * cap);
        }
        if (name_end >= GROM_MAX_CHR_NAME_LEN) name_end = GROM_MAX_CHR_NAME_LEN;
        memset(f->names[f->n], 0, GROM_MAX_CHR_NAME_LEN);
        for (int a = 1; a < name_end; a++) f->names[f->n][a - 1] = (char)tolower((unsigned char)line[a]);
        f->name_len[f->n] = name_end - 1;
        f->file_pos[f->n] = here;
        f->len[f->n] = 0;
        f->n++;
    }
    if (f->n > 0 && f->n <= GROM_MAX_CHR_NAMES) f->len[f->n - 1] = cur_len;
    if (f->n > GROM_MAX_CHR_NAMES) f->n = GROM_MAX_CHR_NAMES;
    return 0;
}

void grom_fasta_close(grom_fasta *f) {
    if (f->fh) fclose(f->fh);
    free(f->names);
    free(f->name_len);
    free(f->file_pos);
    free(f->len);
    memset(f, 0, sizeof(*f));
}

long grom_fasta_load(grom_fasta *f, int i, char *buf, long cap) {
    /* find_disc_svs' loader, GROM.c:21009-21045: per line keep everything up
     * to the last letter; that cut is only re-measured when the line length
     * changes. */
    char line[1000];
    long len = 0;
    fseek(f->fh, f->file_pos[i], SEEK_SET);
    while (fgets(line, sizeof(line), f->fh) && line[0] != '>') {
        int L = (int)strlen(line);
        if (len == 0 || L != f->loader_line_len) {
            f->loader_line_len = L;
            int w = L - 1;
            while (!isalpha((unsigned char)line[w]) && w > 0) w--;
            f->loader_alpha_len = w + 1;
        }
        if (buf && len + f->loader_alpha_len <= cap) memcpy(buf + len, line, f->loader_alpha_len);
        len += f->loader_alpha_len;
    }
    return len;
}

/* grom_fasta_load's result without the shared stream: the chromosome's bytes
 * by pread into a private buffer and fgets(line, 1000)'s chunks found with
 * memchr (a chunk ends after its newline or at 999 bytes), so chromosomes
 * load on several threads at once.  -2 when the chromosome holds a NUL byte
 * (strlen would cut the chunk; the caller takes grom_fasta_load). */
long grom_fasta_load_at(const grom_fasta *f, int i, char *buf, long cap) {
    enum { BLK = 1 << 22 };
    char *b = malloc((size_t)BLK + 1024);
    if (!b) return -1;
    const int fd = fileno(f->fh);
    off_t off = (off_t)f->file_pos[i];
    size_t have = 0, p = 0;
    int eof = 0, prev_l = -1, alpha = 0;
    long len = 0;
    for (;;) {
        if (have - p < 1000 && !eof) {
            memmove(b, b + p, have - p);
            have -= p;
            p = 0;
            const ssize_t k = pread(fd, b + have, BLK, off);
            if (k < 0) { free(b); return -1; }
            if (k == 0) eof = 1;
            if (k > 0 && memchr(b + have, 0, (size_t)k)) { free(b); return -2; }
            have += (size_t)k;
            off += k;
            continue;
        }
        if (p >= have) break; /* fgets at end of file */
        const size_t avail = have - p, lim = avail < 999 ? avail : 999;
        const char *line = b + p;
        const char *nl = memchr(line, '\n', lim);
        const int L = (int)(nl ? (size_t)(nl - line) + 1 : lim);
        if (line[0] == '>') break;
        if (len == 0 || L != prev_l) {
            prev_l = L;
            int w = L - 1;
            while (!isalpha((unsigned char)line[w]) && w > 0) w--;
            alpha = w + 1;
        }
        if (buf && len + alpha <= cap) memcpy(buf + len, line, (size_t)alpha);
        len += alpha;
        p += (size_t)L;
    }
    free(b);
    return len;
}

typedef struct {
    const grom_fasta *f;
    const int *idx;
    long *out;
    int n, next, bad;
    pthread_mutex_t mu;
} fasta_len_job;

static void *fasta_len_main(void *arg) {
    fasta_len_job *j = (fasta_len_job *)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        const int k = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (k >= j->n) break;
        const long L = grom_fasta_load_at(j->f, j->idx[k], NULL, 0);
        if (L < 0) {
            pthread_mutex_lock(&j->mu);
            j->bad = 1;
            pthread_mutex_unlock(&j->mu);
        }
        j->out[k] = L;
    }
    return NULL;
}

int grom_fasta_lengths(const grom_fasta *f, const int *idx, int n, long *out, int threads) {
    if (n <= 0) return 0;
    if (threads > n) threads = n;
    if (threads < 1) threads = 1;
    if (threads > 64) threads = 64;
    fasta_len_job j;
    memset(&j, 0, sizeof(j));
    j.f = f;
    j.idx = idx;
    j.out = out;
    j.n = n;
    pthread_mutex_init(&j.mu, NULL);
    pthread_t th[64];
    int started = 0;
    for (int t = 1; t < threads; t++) {
        if (pthread_create(&th[started], NULL, fasta_len_main, &j) != 0) break;
        started++;
    }
    fasta_len_main(&j);
    for (int t = 0; t < started; t++) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&j.mu);
    return j.bad ? -1 : 0;
}

int grom_target_name_lc(const char *target, char *out, int cap) {
    int L = (int)strlen(target);
    if (L > cap - 1) L = cap - 1;
    for (int i = 0; i < L; i++) out[i] = (char)tolower((unsigned char)target[i]);
    out[L] = 0;
    for (int i = L - 1; i > 0; i--)
        if (!isgraph((unsigned char)out[i])) L = i;
    return L;
}

static int name_rule(const char *bam, int bl, const char *fa, int fl) {
    char t[GROM_MAX_CHR_NAME_LEN + 8];
    if (bl == fl && strncmp(bam, fa, fl) == 0) return 1;
    if (bl - 3 == fl && strncmp(bam, "chr", 3) == 0) {
        snprintf(t, sizeof(t), "chr%.*s", fl, fa);
        return strncmp(bam, t, bl) == 0;
    }
    if (bl + 3 == fl && strncmp(fa, "chr", 3) == 0) {
        snprintf(t, sizeof(t), "chr%.*s", bl, bam);
        return strncmp(fa, t, fl) == 0;
    }
    return 0;
}

int grom_match_target(const grom_fasta *f, const char *target) {
    char lc[GROM_MAX_CHR_NAMES];
    int bl = grom_target_name_lc(target, lc, (int)sizeof(lc));
    for (int i = 0; i < f->n; i++)
        if (name_rule(lc, bl, f->names[i], f->name_len[i])) return i;
    return -1;
}

/* ---------------- insert-size pre-pass ---------------- */

double grom_prob2(double num_sd) {
    double x = num_sd / sqrt(2), t = 1.0 / (1.0 + 0.3275911 * x);
    double e = 1.0 - (0.254829592 * t + -0.284496736 * pow(t, 2) + 1.421413741 * pow(t, 3) +
                      -1.453152027 * pow(t, 4) + 1.061405429 * pow(t, 5)) *
                         exp(-pow(x, 2));
    return (1.0 - e) / 2.0;
}

static int icmp_slow(const void *a, const void *b) {
    const int x = *(const int *)a, y = *(const int *)b;
    return (x > y) - (x < y);
}

/* ascending sort of ints in O(n): LSD radix, 3 passes of 11 bits over the
 * value with its sign bit flipped (the order qsort with an int comparator
 * gives, GROM.c:1276-1310, is the plain numeric order: the result is the
 * same array) */
void grom_sort_ints(int *a, int64_t n) {
    if (n < 2) return;
    uint32_t *x = (uint32_t *)a, *t = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)n);
    if (!t) { /* no scratch: an insertion-free fallback keeps the result */
        qsort(a, (size_t)n, sizeof(int), icmp_slow);
        return;
    }
    for (int64_t i = 0; i < n; i++) x[i] ^= 0x80000000u;
    uint32_t *src = x, *dst = t;
    for (int pass = 0; pass < 3; pass++) {
        const int sh = 11 * pass;
        int64_t cnt[2049] = {0};
        for (int64_t i = 0; i < n; i++) cnt[((src[i] >> sh) & 2047) + 1]++;
        for (int b = 0; b < 2048; b++) cnt[b + 1] += cnt[b];
        for (int64_t i = 0; i < n; i++) dst[cnt[(src[i] >> sh) & 2047]++] = src[i];
        uint32_t *sw = src;
        src = dst;
        dst = sw;
    }
    /* three passes: the sorted data is in t */
    for (int64_t i = 0; i < n; i++) x[i] = src[i] ^ 0x80000000u;
    free(t);
}

int grom_insert_stats(bgzf_reader *r, double prob2, int *lseq, int *imin, int *imax, long *mapped, int min_mapq) {
    const int cap = 10000000; /* insert_sample_size, GROM.c:913 */
    int *ins = malloc(sizeof(int) * cap), *lq = malloc(sizeof(int) * cap);
    int n = 0;
    long m = 0;
    bam_rec b;
    memset(&b, 0, sizeof(b));
    while (n < cap && bam_read_rec(r, &b) > 0) {
        if ((b.flag & GF_UNMAP) || (b.flag & GF_DUP)) continue;
        if (!(b.flag & GF_PAIRED)) {
            ins[n] = b.l_qseq;
            lq[n++] = b.l_qseq;
        } else if (!(b.flag & GF_MUNMAP) && b.tid == b.mtid && b.pos < b.mpos && (b.flag & GF_PROPER) && b.isize > 0) {
            ins[n] = b.isize;
            lq[n++] = b.l_qseq;
        }
        if (b.mapq >= min_mapq) m += b.l_qseq;
    }
    bam_free_rec(&b);
    if (n == 0) { free(ins); free(lq); return -1; }
    grom_sort_ints(ins, n);
    int mean = ins[n / 2], lim = mean * 5, end = 0; /* g_insert_max_mult = 5 */
    for (int a = n - 1; a >= 0; a--)
        if (ins[a] <= lim) { end = a; break; }
    end += 1;
    mean = ins[end / 2];
    int lo = (int)(prob2 * end / 2);
    *imin = ins[lo];
    *imax = ins[end - lo < n ? end - lo : n - 1];
    grom_sort_ints(lq, n);
    *lseq = lq[n / 2];
    if (mapped) *mapped = m;
    free(ins);
    free(lq);
    return mean;
}

/* ---------------- batches ---------------- */


void grom_batch_init(grom_batch *b, int32_t tid, int read_name_len) {
    memset(b, 0, sizeof(*b));
    b->tid = tid;
    b->p_last = -1;
    b->read_name_len = read_name_len;
    b->splitread = 1;
    b->target_name = "";
}

void grom_batch_set_sv(grom_batch *b, const char *target_name, int splitread) {
    b->target_name = target_name ? target_name : "";
    b->splitread = splitread;
}

void grom_batch_end_record(grom_batch *b, const bam_rec *r) { b->lseq_tail = r->l_qseq; }

/* The SA CIGAR's leading/trailing 'S' and I-D balance (GROM.c:6683-6733):
 * digits accumulate until a letter closes an op. */
static void aux_cigar(const char *cig, grom_aux *o) {
    char num[1001];
    int nl = 0, n = 0;
    char first = 0, last = 0;
    int first_len = 0, last_len = 0;
    o->start_adj = o->end_adj = o->end_adj_indel = 0;
    for (const char *c = cig; *c; c++) {
        if (*c >= '0' && *c <= '9') {
            if (nl < 1000) num[nl++] = *c;
        } else if ((*c >= 'A' && *c <= 'Z') || (*c >= 'a' && *c <= 'z')) {
            num[nl] = 0;
            int len = (int)strtol(num, NULL, 10);
            if (n == 0) { first = *c; first_len = len; }
            last = *c;
            last_len = len;
            if (*c == 'I') o->end_adj_indel += len;
            else if (*c == 'D') o->end_adj_indel -= len;
            n++;
            nl = 0;
            if (n >= 1000) break;
        }
    }
    if (n == 0) return;
    if (first == 'S') o->start_adj = first_len;
    if (last == 'S') o->end_adj = last_len;
}

int grom_parse_aux(const bam_rec *r, const char *target_name, grom_aux *out) {
    const int l_aux = bam_l_aux(r);
    if (!(l_aux > 0 && l_aux < 100)) return 0; /* aux_str_len, GROM.c:643, 5763 */
    int is_xp = 1;
    const uint8_t *a = bam_aux_find(r, "XP");
    if (!a) { is_xp = 0; a = bam_aux_find(r, "SA"); }
    if (!a) return 0;
    char buf[128];
    const uint8_t *src = (a[0] == 'Z') ? a + 1 : a, *end = r->data + r->data_len;
    int k = 0;
    while (src + k < end && src[k] && k < (int)sizeof(buf) - 1) { buf[k] = (char)src[k]; k++; }
    buf[k] = 0;
    char *save = NULL;
    char *chr = strtok_r(buf, ",", &save);
    char *t1 = strtok_r(NULL, ",", &save);
    memset(out, 0, sizeof(*out));
    char *cig, *mq;
    if (is_xp) { /* XP:Z:chr,+pos,CIGAR,mapq (GROM.c:5776-5790) */
        if (!t1) return 0;
        out->strand = (t1[0] == '+') ? 0 : 1;
        out->pos = atoi(t1 + 1);
        cig = strtok_r(NULL, ",", &save);
        mq = strtok_r(NULL, ",", &save);
    } else { /* SA:Z:chr,pos,strand,CIGAR,mapq,NM; (GROM.c:5806-5820) */
        char *t2 = strtok_r(NULL, ",", &save);
        if (!t1 || !t2) return 0;
        out->pos = atoi(t1);
        out->strand = (t2[0] == '+') ? 0 : 1;
        cig = strtok_r(NULL, ",", &save);
        mq = strtok_r(NULL, ",", &save);
    }
    if (!chr || !cig) return 0;
    out->mq = (int16_t)(mq ? atoi(mq) : 0);
    out->same_chr = strncmp(target_name, chr, strlen(target_name)) == 0;
    aux_cigar(cig, out);
    return 1;
}

void grom_batch_free(grom_batch *b) {
    free(b->aux_idx); free(b->aux); free(b->drop_pos); free(b->drop_lq); free(b->drop_before);
    free(b->pos); free(b->flag); free(b->mapq); free(b->mtid); free(b->mpos); free(b->isize); free(b->l_qseq);
    free(b->cigar_off); free(b->cigar); free(b->base_off); free(b->seq); free(b->qual); free(b->name_id);
    free(b->nkeys);
    free(b->nhash);
    free(b->nids);
    free(b->narena);
    memset(b, 0, sizeof(*b));
}

static uint64_t hash_name(const char *s, size_t *len) {
    uint64_t h = 0xcbf29ce484222325ULL;
    const char *p = s;
    for (; *p; p++) h = (h ^ (unsigned char)*p) * 0x100000001b3ULL;
    *len = (size_t)(p - s);
    return h;
}

/* read name -> 32-bit id, equal names <=> equal ids (names of read_name_len
 * or more characters are never stored: id 0, GROM.c:6813).  Names live in one
 * growing arena, so interning a new name is a copy, not an allocation. */
static uint32_t intern(grom_batch *b, const char *s) {
    size_t L;
    const uint64_t h = hash_name(s, &L);
    if (L == 0 || L >= (size_t)b->read_name_len) return 0;
    if (2 * (b->nn + 1) > b->ncap) {
        int64_t nc = b->ncap ? 2 * b->ncap : 65536;
        int64_t *nk = calloc(nc, sizeof(int64_t));
        uint64_t *nh = malloc(sizeof(uint64_t) * nc);
        uint32_t *ni = malloc(sizeof(uint32_t) * nc);
        for (int64_t i = 0; i < b->ncap; i++)
            if (b->nkeys[i]) {
                int64_t j = (int64_t)(b->nhash[i] & (uint64_t)(nc - 1));
                while (nk[j]) j = (j + 1) & (nc - 1);
                nk[j] = b->nkeys[i];
                nh[j] = b->nhash[i];
                ni[j] = b->nids[i];
            }
        free(b->nkeys);
        free(b->nhash);
        free(b->nids);
        b->nkeys = nk;
        b->nhash = nh;
        b->nids = ni;
        b->ncap = nc;
    }
    int64_t j = (int64_t)(h & (uint64_t)(b->ncap - 1));
    while (b->nkeys[j]) {
        if (b->nhash[j] == h && strcmp(b->narena + b->nkeys[j] - 1, s) == 0) return b->nids[j];
        j = (j + 1) & (b->ncap - 1);
    }
    if (b->narena_len + (int64_t)L + 1 > b->narena_cap) {
        int64_t nc = b->narena_cap ? 2 * b->narena_cap : (1 << 22);
        while (nc < b->narena_len + (int64_t)L + 1) nc *= 2;
        b->narena = realloc(b->narena, nc);
        b->narena_cap = nc;
    }
    memcpy(b->narena + b->narena_len, s, L + 1);
    b->nkeys[j] = b->narena_len + 1;
    b->narena_len += (int64_t)L + 1;
    b->nhash[j] = h;
    b->nids[j] = (uint32_t)(++b->nn);
    return b->nids[j];
}

void grom_batch_add(grom_batch *b, const bam_rec *r, int32_t index_start) {
    /* which fetch site loaded this record: the scan start (GROM.c:5743) and
     * the skip branch (14861) parse SA/XP always, the ingest loop (10968)
     * only without -S */
    const int parse_aux = (b->n_seen == 0) || b->prev_skipped || b->splitread;
    b->n_seen++;
    if (r->pos < index_start && !b->any_ingested) { /* skip branch, GROM.c:14859-14969 */
        b->n_skip++;
        b->prev_skipped = 1;
        return;
    }
    b->prev_skipped = 0;
    b->any_ingested = 1;
    b->last_pos = r->pos;
    b->lseq_tail = r->l_qseq; /* at end of file the last record's length (plus hard clips, below) */
    if ((r->flag & GF_UNMAP) || (r->flag & GF_DUP)) { /* GROM.c:6418 */
        if (b->n_drop + 1 > b->cap_drop) {
            int64_t nc = b->cap_drop ? 2 * b->cap_drop : 1024;
            b->drop_pos = realloc(b->drop_pos, sizeof(int32_t) * nc);
            b->drop_lq = realloc(b->drop_lq, sizeof(int32_t) * nc);
            b->drop_before = realloc(b->drop_before, sizeof(int64_t) * nc);
            b->cap_drop = nc;
        }
        b->drop_pos[b->n_drop] = r->pos;
        b->drop_lq[b->n_drop] = r->l_qseq;
        b->drop_before[b->n_drop] = b->n;
        b->n_drop++;
        return;
    }
    int64_t i = b->n;
    if (i + 1 > b->cap) {
        int64_t nc = b->cap ? b->cap * 2 : 1024;
        b->pos = realloc(b->pos, sizeof(int32_t) * nc);
        b->flag = realloc(b->flag, sizeof(uint16_t) * nc);
        b->mapq = realloc(b->mapq, nc);
        b->mtid = realloc(b->mtid, sizeof(int32_t) * nc);
        b->mpos = realloc(b->mpos, sizeof(int32_t) * nc);
        b->isize = realloc(b->isize, sizeof(int32_t) * nc);
        b->l_qseq = realloc(b->l_qseq, sizeof(int32_t) * nc);
        b->cigar_off = realloc(b->cigar_off, sizeof(uint32_t) * (nc + 1));
        b->base_off = realloc(b->base_off, sizeof(int64_t) * nc);
        b->name_id = realloc(b->name_id, sizeof(uint32_t) * nc);
        b->aux_idx = realloc(b->aux_idx, sizeof(int32_t) * nc);
        b->cap = nc;
    }
    {
        grom_aux ax;
        b->aux_idx[i] = -1;
        if (parse_aux && grom_parse_aux(r, b->target_name, &ax)) {
            if (b->n_aux + 1 > b->cap_aux) {
                int64_t nc = b->cap_aux ? 2 * b->cap_aux : 1024;
                b->aux = realloc(b->aux, sizeof(grom_aux) * nc);
                b->cap_aux = nc;
            }
            b->aux_idx[i] = (int32_t)b->n_aux;
            b->aux[b->n_aux++] = ax;
        }
    }
    b->pos[i] = r->pos;
    b->flag[i] = r->flag;
    b->mapq[i] = r->mapq;
    b->mtid[i] = r->mtid;
    b->mpos[i] = r->mpos;
    b->isize[i] = r->isize;
    b->l_qseq[i] = r->l_qseq;
    if (i == 0) b->cigar_off[0] = 0;
    if (b->n_cig + r->n_cigar > b->cap_cig) {
        int64_t nc = b->cap_cig ? b->cap_cig : 4096;
        while (nc < b->n_cig + r->n_cigar) nc *= 2;
        b->cigar = realloc(b->cigar, sizeof(uint32_t) * nc);
        b->cap_cig = nc;
    }
    memcpy(b->cigar + b->n_cig, bam_cigar(r), sizeof(uint32_t) * r->n_cigar);
    const uint32_t *cg = b->cigar + b->n_cig;  /* the aligned copy */
    int32_t span = 0;
    for (int k = 0; k < r->n_cigar; k++) {
        int op = cg[k] & 0xf;
        if (op == GC_MATCH || op == GC_DEL || op == GC_REF_SKIP || op == GC_EQUAL || op == GC_DIFF) span += (int32_t)(cg[k] >> 4);
    }
    if (span > b->max_ref_span) b->max_ref_span = span;
    for (int k = 0; k < r->n_cigar; k++) /* the ingest adds hard clips to cdp_lseq, GROM.c:6997-7000 */
        if ((cg[k] & 0xf) == GC_HARD_CLIP) b->lseq_tail += (int32_t)(cg[k] >> 4);
    b->n_cig += r->n_cigar;
    b->cigar_off[i + 1] = (uint32_t)b->n_cig;
    int64_t L = r->l_qseq, Lp = (L + 1) & ~1LL; /* keep every read's first base on a byte */
    int64_t need = b->n_bases + Lp;
    if (need > b->cap_bases) {
        int64_t nc = b->cap_bases ? b->cap_bases : 1 << 20;
        while (nc < need) nc *= 2;
        b->qual = realloc(b->qual, nc);
        b->seq = realloc(b->seq, nc / 2);
        b->cap_bases = nc;
    }
    b->base_off[i] = b->n_bases;
    memcpy(b->seq + b->n_bases / 2, bam_seq(r), (size_t)((L + 1) / 2));
    memcpy(b->qual + b->n_bases, bam_qual(r), (size_t)L);
    if (Lp > L) b->qual[b->n_bases + L] = 0;
    b->n_bases = need;
    b->name_id[i] = intern(b, bam_qname(r));
    b->n = i + 1;
}

void grom_batch_finish(grom_batch *b, int32_t index_start, int32_t overlap_mult, int32_t insert_max) {
    if (!b->any_ingested) { b->p_last = -1; return; }
    int32_t p = b->last_pos - overlap_mult * insert_max;
    b->p_last = p > index_start ? p : index_start;
}

void grom_batch_view(const grom_batch *b, grom_reads *o) {
    memset(o, 0, sizeof(*o));
    o->n = b->n;
    o->n_cigar_ops = b->n_cig;
    o->n_bases = b->n_bases;
    o->pos = b->pos;
    o->flag = b->flag;
    o->mapq = b->mapq;
    o->mtid = b->mtid;
    o->mpos = b->mpos;
    o->isize = b->isize;
    o->l_qseq = b->l_qseq;
    o->cigar_off = b->cigar_off;
    o->cigar = b->cigar;
    o->base_off = b->base_off;
    o->seq = b->seq;
    o->qual = b->qual;
    o->name_id = b->name_id;
    o->n_aux = b->n_aux;
    o->aux_idx = b->aux_idx;
    o->aux = b->aux;
    o->n_drop = b->n_drop;
    o->drop_pos = b->drop_pos;
    o->drop_lq = b->drop_lq;
    o->drop_before = b->drop_before;
}

/* ---------------- serial stream planner ---------------- */

void grom_planner_init(grom_planner *p, const int32_t *order, int n_order) {
    memset(p, 0, sizeof(*p));
    p->order = order;
    p->n_order = n_order;
}

int grom_planner_feed(grom_planner *p, int32_t tid) {
    if (p->k >= p->n_order) return -1;
    switch (p->state) {
    case 0: /* outer loop of count_discordant_pairs, GROM.c:5740 / 17549 */
        if (tid == p->order[p->k]) { p->state = 1; return p->k; }
        return -1;
    case 1: /* inner walk: a foreign record ends the chromosome (begin=2) ... */
        if (tid == p->order[p->k]) return p->k;
        p->state = 2;
        return -1;
    default: /* ... and the outer `while` condition reads one more (Q1) */
        p->state = 0;
        p->k++;
        return -1;
    }
}
