/*
 * hostapi.c -- host conveniences for tests and benchmarks: a synthetic
 * chromosome turned straight into the read batch its scan ingests, without a
 * BAM round trip (the SoA the BAM decoder would have produced).
 */
#include <stdlib.h>
#include <string.h>

#include "../../include/grom_amd.h"
#include "stream.h"
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

static int icmp(const void *a, const void *b) { return *(const int *)a - *(const int *)b; }

/* find_insert_mean's statistics (GROM.c:1276-1310) from the sampled pairs */
static void insert_stats(struct grom_batch_handle *h, grom_params *P) {
    qsort(h->ins, h->n_ins, sizeof(int), icmp);
    int64_t n = h->n_ins;
    int mean = h->ins[n / 2], lim = mean * 5;
    int64_t end = 0;
    for (int64_t a = n - 1; a >= 0; a--)
        if (h->ins[a] <= lim) { end = a; break; }
    end += 1;
    mean = h->ins[end / 2];
    int lo = (int)(grom_prob2(3.0) * end / 2);
    int imin = h->ins[lo], imax = h->ins[end - lo < n ? end - lo : n - 1];
    qsort(h->lq, n, sizeof(int), icmp);
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

grom_batch_handle *grom_synth_chrom(const grom_synth_spec *sp, grom_params *P) {
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
    if (P->half_one_base_rd_len > 0) {
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
