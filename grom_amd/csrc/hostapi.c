/*
 * hostapi.c -- host conveniences for tests and benchmarks: a synthetic
 * chromosome turned straight into the read batch its scan ingests, without a
 * BAM round trip (the SoA the BAM decoder would have produced).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/grom_amd.h"
#include "stream.h"
#include "pdecode.h"
#include "synth.h"

struct grom_batch_handle {
    grom_batch b;
    char *ref;
    int64_t len;
    int32_t tid;
    char name[48];
    /* insert statistics sample (find_insert_mean's rule) */
    int *ins, *lq;
    int64_t n_ins, cap_ins;
};

static void on_record(void *ctx, const bam_rec *r) {
    struct grom_batch_handle *h = (struct grom_batch_handle *)ctx;
    if (!(r->flag & GF_UNMAP) && !(r->flag & GF_DUP) && h->n_ins < 10000000) {
        int take = 0, v = 0;
        if (!(r->flag & GF_PAIRED)) { take = 1; v = r->l_qseq; }
        else if (!(r->flag & GF_MUNMAP) && r->tid == r->mtid && r->pos < r->mpos && (r->flag & GF_PROPER) && r->isize > 0) {
            take = 1;
            v = r->isize;
        }
        if (take) {
            if (h->n_ins == h->cap_ins) {
                h->cap_ins = h->cap_ins ? 2 * h->cap_ins : 1 << 16;
                h->ins = realloc(h->ins, sizeof(int) * h->cap_ins);
                h->lq = realloc(h->lq, sizeof(int) * h->cap_ins);
            }
            h->ins[h->n_ins] = v;
            h->lq[h->n_ins++] = r->l_qseq;
        }
    }
    grom_batch_add(&h->b, r, 0); /* the skip prefix is trimmed once index_start is known */
}


/* find_insert_mean's statistics (GROM.c:1276-1310) from the sampled pairs */
static void insert_stats(struct grom_batch_handle *h, grom_params *P) {
    grom_sort_ints(h->ins, h->n_ins);
    int64_t n = h->n_ins;
    int mean = h->ins[n / 2], lim = mean * 5;
    int64_t end = 0;
    for (int64_t a = n - 1; a >= 0; a--)
        if (h->ins[a] <= lim) { end = a; break; }
    end += 1;
    mean = h->ins[end / 2];
    int lo = (int)(grom_prob2(3.0) * end / 2);
    int imin = h->ins[lo], imax = h->ins[end - lo < n ? end - lo : n - 1];
    grom_sort_ints(h->lq, n);
    grom_params_set_insert(P, mean, imin, imax, h->lq[n / 2]);
}

/* drop the leading records with pos < s0 (the walk's skip branch) */
static void trim_prefix(grom_batch *b, int32_t s0, int64_t *n_dropped_mapped) {
    int64_t k = 0;
    while (k < b->n && b->pos[k] < s0) k++;
    *n_dropped_mapped = k;
    if (k == 0) return;
    int64_t n = b->n - k;
    int64_t c0 = b->cigar_off[k], bo0 = b->base_off[k];
    memmove(b->pos, b->pos + k, sizeof(int32_t) * n);
    memmove(b->flag, b->flag + k, sizeof(uint16_t) * n);
    memmove(b->mapq, b->mapq + k, n);
    memmove(b->mtid, b->mtid + k, sizeof(int32_t) * n);
    memmove(b->mpos, b->mpos + k, sizeof(int32_t) * n);
    memmove(b->isize, b->isize + k, sizeof(int32_t) * n);
    memmove(b->l_qseq, b->l_qseq + k, sizeof(int32_t) * n);
    memmove(b->name_id, b->name_id + k, sizeof(uint32_t) * n);
    memmove(b->aux_idx, b->aux_idx + k, sizeof(int32_t) * n);
    /* dropped (unmapped / duplicate) records of the prefix go with it */
    int64_t nd = 0;
    for (int64_t d = 0; d < b->n_drop; d++) {
        if (b->drop_pos[d] < s0) continue;
        b->drop_pos[nd] = b->drop_pos[d];
        b->drop_lq[nd] = b->drop_lq[d];
        b->drop_before[nd] = b->drop_before[d] > k ? b->drop_before[d] - k : 0;
        nd++;
    }
    b->n_drop = nd;
    for (int64_t i = 0; i <= n; i++) b->cigar_off[i] = b->cigar_off[i + k] - (uint32_t)c0;
    memmove(b->cigar, b->cigar + c0, sizeof(uint32_t) * (b->n_cig - c0));
    b->n_cig -= c0;
    for (int64_t i = 0; i < n; i++) b->base_off[i] = b->base_off[i + k] - bo0;
    memmove(b->qual, b->qual + bo0, b->n_bases - bo0);
    memmove(b->seq, b->seq + bo0 / 2, (b->n_bases - bo0) / 2);
    b->n_bases -= bo0;
    b->n = n;
}

grom_batch_handle *grom_synth_batch(int64_t chr_len, double coverage, int32_t read_len, double insert_mean,
                                    double insert_sd, uint64_t seed, grom_params *P) {
    synth_cfg c;
    synth_default_cfg(&c);
    c.n_chr = 1;
    c.chr_len[0] = chr_len;
    snprintf(c.chr_name[0], sizeof(c.chr_name[0]), "chr1");
    c.coverage = coverage;
    c.read_len = read_len;
    c.insert_mean = insert_mean;
    c.insert_sd = insert_sd;
    c.seed = seed;
    c.munmap_frac = 0.0; /* every ingested record is a placed, mapped read */
    struct grom_batch_handle *h = calloc(1, sizeof(*h));
    h->len = chr_len;
    snprintf(h->name, sizeof(h->name), "chr1");
    h->ref = synth_reference(&c, 0);
    grom_batch_init(&h->b, 0, P->read_name_len);
    synth_reads(&c, 0, h->ref, on_record, h);
    if (h->n_ins == 0) { grom_batch_release(h); return NULL; }
    insert_stats(h, P);
    int32_t s0 = P->one_base_rd_len / 4 + 1;
    int64_t dropped = 0;
    trim_prefix(&h->b, s0, &dropped);
    h->b.n_skip = (int32_t)dropped;
    h->b.any_ingested = h->b.n > 0;
    if (h->b.n > 0) h->b.last_pos = h->b.pos[h->b.n - 1];
    grom_batch_finish(&h->b, s0, P->overlap_mult, P->insert_max_size);
    return h;
}

/* records straight into the batch with the walk's skip rule applied
 * (index_start known up front: the insert statistics are already set) */
struct direct_ctx { grom_batch *b; int32_t s0; };
static void on_record_direct(void *ctx, const bam_rec *r) {
    struct direct_ctx *d = (struct direct_ctx *)ctx;
    grom_batch_add(d->b, r, d->s0);
}

/* the stream of one chromosome inside a whole genome's BAM (every chromosome
 * processed, in order): the previous chromosome's loop took its first two
 * records (GROM.c:5740, 14960-14976) */
struct stream_ctx { grom_batch *b; int32_t s0; int64_t drop; };
static void on_record_stream(void *ctx, const bam_rec *r) {
    struct stream_ctx *d = (struct stream_ctx *)ctx;
    if (d->drop > 0) { d->drop--; return; }
    grom_batch_add(d->b, r, d->s0);
}
static void on_first_record(void *ctx, const bam_rec *r) { *(int32_t *)ctx = r->l_qseq; }

static grom_batch_handle *synth_chrom(const grom_synth_spec *sp, grom_params *P, int stream);

grom_batch_handle *grom_synth_chrom(const grom_synth_spec *sp, grom_params *P) { return synth_chrom(sp, P, 0); }

grom_batch_handle *grom_synth_chrom_stream(const grom_synth_spec *sp, grom_params *P) {
    if (!P || P->half_one_base_rd_len <= 0) {
        grom_set_last_error("grom_synth_chrom_stream: set the insert statistics first (grom_params_set_insert)");
        return NULL;
    }
    return synth_chrom(sp, P, 1);
}

static grom_batch_handle *synth_chrom(const grom_synth_spec *sp, grom_params *P, int stream) {
    if (!sp || !P || sp->n_chr < 1 || sp->n_chr > SYNTH_MAX_CHR || sp->chrom < 0 || sp->chrom >= sp->n_chr ||
        !sp->chr_len)
        return NULL;
    synth_cfg c;
    synth_default_cfg(&c);
    c.n_chr = sp->n_chr;
    for (int i = 0; i < c.n_chr; i++) {
        c.chr_len[i] = sp->chr_len[i];
        snprintf(c.chr_name[i], sizeof(c.chr_name[i]), "chr%d", i + 1);
    }
    if (sp->names) { /* comma-separated, as grom_synth -n */
        const char *q = sp->names;
        for (int i = 0; i < c.n_chr && *q; i++) {
            const char *e = strchr(q, ',');
            size_t l = e ? (size_t)(e - q) : strlen(q);
            if (l >= sizeof(c.chr_name[i])) l = sizeof(c.chr_name[i]) - 1;
            memcpy(c.chr_name[i], q, l);
            c.chr_name[i][l] = 0;
            if (!e) break;
            q = e + 1;
        }
    }
    if (sp->coverage > 0) c.coverage = sp->coverage;
    if (sp->read_len > 0) c.read_len = sp->read_len;
    if (sp->ploidy > 0) c.ploidy = sp->ploidy;
    if (sp->insert_mean > 0) c.insert_mean = sp->insert_mean;
    if (sp->insert_sd > 0) c.insert_sd = sp->insert_sd;
    c.dup_frac = sp->dup_frac;
    c.sv_per_mb = sp->sv_per_mb;
    c.cnv_rate = sp->cnv_rate;
    if (sp->cnv_min > 0) c.cnv_min = sp->cnv_min;
    if (sp->cnv_max > 0) c.cnv_max = sp->cnv_max;
    if (sp->chr_cov)
        for (int i = 0; i < c.n_chr; i++) c.chr_cov[i] = sp->chr_cov[i];
    c.munmap_frac = sp->munmap_frac;
    c.seed = sp->seed;
    const int ci = sp->chrom;
    struct grom_batch_handle *h = calloc(1, sizeof(*h));
    if (!h) return NULL;
    h->len = c.chr_len[ci];
    h->tid = ci;
    snprintf(h->name, sizeof(h->name), "%s", c.chr_name[ci]);
    /* the scan takes the lower-cased FASTA name (GROM.c:20893-20906) */
    for (char *q = h->name; *q; q++)
        if (*q >= 'A' && *q <= 'Z') *q = (char)(*q + 32);
    h->ref = synth_reference(&c, ci);
    grom_batch_init(&h->b, ci, P->read_name_len);
    grom_batch_set_sv(&h->b, c.chr_name[ci], P->splitread);
    if (stream) {
        struct stream_ctx d = {&h->b, P->one_base_rd_len / 4 + 1, ci > 0 ? 2 : 0};
        synth_reads(&c, ci, h->ref, on_record_stream, &d);
        if (ci + 1 < c.n_chr) { /* the record that ends the stream: the next chromosome's first */
            synth_cfg c1 = c;
            c1.max_emit = 1;
            char *r1 = synth_reference(&c1, ci + 1);
            int32_t lq = -1;
            if (r1 && synth_reads(&c1, ci + 1, r1, on_first_record, &lq) == 1 && h->b.n_seen > 0) h->b.lseq_tail = lq;
            free(r1);
        }
    } else if (P->half_one_base_rd_len > 0) {
        struct direct_ctx d = {&h->b, P->one_base_rd_len / 4 + 1};
        synth_reads(&c, ci, h->ref, on_record_direct, &d);
    } else {
        synth_reads(&c, ci, h->ref, on_record, h);
        if (h->n_ins == 0) { grom_batch_release(h); return NULL; }
        insert_stats(h, P);
        int64_t dropped = 0;
        trim_prefix(&h->b, P->one_base_rd_len / 4 + 1, &dropped);
        h->b.n_skip = (int32_t)dropped;
        h->b.any_ingested = h->b.n > 0;
        if (h->b.n > 0) h->b.last_pos = h->b.pos[h->b.n - 1];
    }
    grom_batch_finish(&h->b, P->one_base_rd_len / 4 + 1, P->overlap_mult, P->insert_max_size);
    return h;
}

uint64_t grom_reads_digest(const grom_reads *r) { return pd_digest(r); }

int grom_batch_get(grom_batch_handle *h, grom_chrom *ch, grom_reads *rd) {
    if (!h) return GROM_E_ARG;
    ch->ref = h->ref;
    ch->len = h->len;
    ch->name = h->name;
    ch->tid = h->tid;
    ch->n_skip = h->b.n_skip;
    ch->p_last = h->b.p_last;
    ch->cnv = 1;
    ch->seed = 1;
    ch->lseq_tail = h->b.lseq_tail;
    ch->pad = 0;
    grom_batch_view(&h->b, rd);
    return GROM_OK;
}

void grom_batch_release(grom_batch_handle *h) {
    if (!h) return;
    grom_batch_free(&h->b);
    free(h->ref);
    free(h->ins);
    free(h->lq);
    free(h);
}

/* ---------------- BAM index entry points ---------------- */
int grom_bai_build(const char *bam_path) { return bai_build(bam_path) == 0 ? 0 : GROM_E_ARG; }

int grom_bai_summary(const char *bai_path, int64_t out[5]) {
    bai_index idx;
    if (bai_load(bai_path, &idx) != 0) return GROM_E_ARG;
    int64_t bins = 0, chunks = 0, intv = 0;
    for (int t = 0; t < idx.n_ref; t++) {
        bins += idx.ref[t].n_bin;
        intv += idx.ref[t].n_intv;
        for (int i = 0; i < idx.ref[t].n_bin; i++) chunks += idx.ref[t].bin[i].n_chunk;
    }
    out[0] = idx.n_ref;
    out[1] = bins;
    out[2] = chunks;
    out[3] = intv;
    out[4] = idx.has_no_coor ? (int64_t)idx.n_no_coor : -1;
    bai_free(&idx);
    return 0;
}

typedef struct {
    uint64_t hash;
    int64_t n;
} fetch_acc;

/* an order-free digest of a record set: sum of per-record hashes */
static uint64_t rec_hash(const bam_rec *b) {
    uint64_t h = 1469598103934665603ull ^ ((uint64_t)(uint32_t)b->tid << 32 | (uint32_t)b->pos);
    for (int i = 0; i < b->data_len; i++) h = (h ^ b->data[i]) * 1099511628211ull;
    return h ^ ((uint64_t)b->flag << 48);
}

static void fetch_visit(void *ctx, const bam_rec *b) {
    fetch_acc *a = (fetch_acc *)ctx;
    a->hash += rec_hash(b);
    a->n++;
}

int64_t grom_bai_selftest(const char *bam_path, int64_t n_queries, uint64_t seed, int64_t *visited) {
    char bai[4096];
    snprintf(bai, sizeof(bai), "%s.bai", bam_path);
    bai_index idx;
    if (bai_load(bai, &idx) != 0) return GROM_E_ARG;
    bgzf_reader r;
    bam_hdr h;
    if (bgzf_open_read(&r, bam_path) != 0 || bam_read_header(&r, &h) != 0) {
        bai_free(&idx);
        return GROM_E_ARG;
    }
    /* every placed record once: tid, pos, end, hash */
    int64_t n = 0, cap = 1 << 16;
    int32_t *tp = (int32_t *)malloc(sizeof(int32_t) * 3 * cap);
    uint64_t *hs = (uint64_t *)malloc(sizeof(uint64_t) * cap);
    bam_rec b;
    memset(&b, 0, sizeof(b));
    while (bam_read_rec(&r, &b) == 1) {
        if (b.tid < 0) continue;
        if (n == cap) {
            cap *= 2;
            tp = (int32_t *)realloc(tp, sizeof(int32_t) * 3 * cap);
            hs = (uint64_t *)realloc(hs, sizeof(uint64_t) * cap);
        }
        tp[3 * n] = b.tid;
        tp[3 * n + 1] = b.pos;
        tp[3 * n + 2] = bam_end_pos(&b);
        hs[n] = rec_hash(&b);
        n++;
    }
    uint64_t s = seed ? seed : 1;
    int64_t bad = 0, seen = 0;
    for (int64_t q = 0; q < n_queries && h.n_ref > 0; q++) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        const int tid = (int)(s % (uint64_t)h.n_ref);
        const int32_t L = h.ref_len[tid] > 0 ? h.ref_len[tid] : 1;
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        const int32_t beg = (int32_t)(s % (uint64_t)L);
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        /* point, short, medium and long regions; every fifth query a whole
         * chromosome or more (100 Mb: more bins than any fixed list holds) */
        const int32_t span = (q % 5 == 4) ? (q % 2 ? L : 100000000)
                             : (q % 4 == 0) ? 1 : (int32_t)(1 + s % (q % 4 == 1 ? 200u : q % 4 == 2 ? 40000u : 3000000u));
        const int32_t b0 = (q % 5 == 4) ? 0 : beg;
        const int32_t end = (int32_t)((int64_t)b0 + span > INT32_MAX ? INT32_MAX : b0 + span);
        fetch_acc want = {0, 0}, got = {0, 0};
        for (int64_t i = 0; i < n; i++)
            if (tp[3 * i] == tid && tp[3 * i + 1] < end && tp[3 * i + 2] > b0) {
                want.hash += hs[i];
                want.n++;
            }
        if (bam_fetch(&r, &idx, tid, b0, end, fetch_visit, &got) < 0) { bad = GROM_E_ARG; break; }
        seen += got.n;
        if (got.n != want.n || got.hash != want.hash) bad++;
    }
    if (visited) *visited = seen;
    bam_free_rec(&b);
    free(tp);
    free(hs);
    bam_free_header(&h);
    bgzf_close_read(&r);
    bai_free(&idx);
    return bad;
}
