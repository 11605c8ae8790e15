/*
 * pdecode.c -- parallel BAM decode into pinned pieces, streamed to device
 * stages in file order (see pdecode.h).
 *
 * Threads: n decoder threads take pieces in file order (at most `window`
 * pieces ahead of the uploader) and inflate + parse each into a pinned
 * buffer; one uploader thread takes finished pieces in file order,
 * accumulates find_insert_mean's sample, applies the order-dependent fix-ups
 * and appends the piece to its chromosome's stage (async copies); chromosomes
 * are finalised in plan order once the walk parameters are known and handed
 * to the caller through pd_stream_chrom.
 */
#define _GNU_SOURCE
#include "pdecode.h"

#include <dlfcn.h>
#include <stddef.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>
#include <zlib.h>

#include "ddecode.h"
#include "stream.h"

#define PD_INSERT_CAP 10000000 /* insert_sample_size, GROM.c:913 */
#define PD_PIECE_RECS 65536    /* target records per piece */
#define PD_LOWPOS_LIMIT (1 << 22) /* the skip prefix is resolved below this position */
#define PD_MAX_REC (256 << 20)    /* a record larger than this is taken as a bad offset */

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static uint16_t ld16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }
static uint32_t ld32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static int32_t ldi32(const uint8_t *p) { int32_t v; memcpy(&v, p, 4); return v; }

/* ---------------- inflate: libdeflate when the image has it, else zlib ---------------- */
typedef void *(*ld_alloc_fn)(void);
typedef int (*ld_dec_fn)(void *, const void *, size_t, void *, size_t, size_t *);
typedef void (*ld_free_fn)(void *);
static ld_alloc_fn ld_alloc;
static ld_dec_fn ld_dec;
static ld_free_fn ld_free;
static pthread_once_t ld_once = PTHREAD_ONCE_INIT;

static void ld_init(void) {
    if (getenv("GROM_NO_LIBDEFLATE")) return;
    void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    ld_alloc_fn a = (ld_alloc_fn)dlsym(h, "libdeflate_alloc_decompressor");
    ld_dec_fn d = (ld_dec_fn)dlsym(h, "libdeflate_deflate_decompress");
    ld_free_fn f = (ld_free_fn)dlsym(h, "libdeflate_free_decompressor");
    if (a && d && f) { ld_alloc = a; ld_dec = d; ld_free = f; }
}

typedef struct {
    void *ld;
    z_stream zs;
    int zinit;
} pd_inflater;

static void inf_init(pd_inflater *f) {
    memset(f, 0, sizeof(*f));
    pthread_once(&ld_once, ld_init);
    if (ld_alloc) f->ld = ld_alloc();
}

static void inf_free(pd_inflater *f) {
    if (f->ld) ld_free(f->ld);
    if (f->zinit) inflateEnd(&f->zs);
    memset(f, 0, sizeof(*f));
}

/* raw deflate data -> exactly isize bytes; 0 or -1 */
static int inf_block(pd_inflater *f, const uint8_t *c, size_t clen, uint8_t *out, uint32_t isize) {
    if (isize == 0) return 0;
    if (f->ld) {
        size_t got = 0;
        if (ld_dec(f->ld, c, clen, out, isize, &got) != 0 || got != isize) return -1;
        return 0;
    }
    if (!f->zinit) {
        if (inflateInit2(&f->zs, -15) != Z_OK) return -1;
        f->zinit = 1;
    } else if (inflateReset(&f->zs) != Z_OK) {
        return -1;
    }
    f->zs.next_in = (uint8_t *)c;
    f->zs.avail_in = (uInt)clen;
    f->zs.next_out = out;
    f->zs.avail_out = isize;
    int rc = inflate(&f->zs, Z_FINISH);
    return (rc == Z_STREAM_END && f->zs.total_out == isize) ? 0 : -1;
}

/* ---------------- a reader over [vbeg, vend) of the decompressed stream ---------------- */
typedef struct {
    int fd;
    int64_t file_size;
    uint8_t *cbuf;
    int64_t cbuf_cap, cbuf_off, cbuf_len; /* cbuf holds file bytes [cbuf_off, cbuf_off + cbuf_len) */
    int64_t next_coff;                     /* the next block to inflate */
    uint8_t *ub;
    int64_t ub_cap, ub_len, ub_pos;
    int64_t stop_at;                       /* ub offset where parsing stops, -1 unknown */
    int64_t stop_coff;                     /* -1: read to end of file */
    int stop_uoff, no_more;
    pd_inflater inf;
    int64_t inflated, compressed;
    double t_inflate, t_io;
} pd_reader;

static int rd_fetch(pd_reader *r, int64_t off, int64_t need) {
    if (off >= r->cbuf_off && off + need <= r->cbuf_off + r->cbuf_len) return 0;
    int64_t want = need > (4 << 20) ? need : (4 << 20);
    if (want > r->cbuf_cap) {
        uint8_t *nb = (uint8_t *)realloc(r->cbuf, (size_t)want);
        if (!nb) return -1;
        r->cbuf = nb;
        r->cbuf_cap = want;
    }
    if (off + want > r->file_size) want = r->file_size - off;
    if (want < need) return -1;
    int64_t got = 0;
    const double t0 = now_s();
    while (got < want) {
        ssize_t k = pread(r->fd, r->cbuf + got, (size_t)(want - got), (off_t)(off + got));
        if (k <= 0) break;
        got += k;
    }
    r->t_io += now_s() - t0;
    if (got < need) return -1;
    r->cbuf_off = off;
    r->cbuf_len = got;
    return 0;
}

static int rd_reserve(pd_reader *r, int64_t cap) {
    if (cap <= r->ub_cap) return 0;
    int64_t nc = r->ub_cap ? r->ub_cap : (1 << 20);
    while (nc < cap) nc *= 2;
    uint8_t *nb = (uint8_t *)realloc(r->ub, (size_t)nc);
    if (!nb) return -1;
    r->ub = nb;
    r->ub_cap = nc;
    return 0;
}

/* inflate the next block onto ub: 1, 0 when there is nothing more, -1 error */
static int rd_next_block(pd_reader *r) {
    for (;;) {
        if (r->no_more) return 0;
        if (r->stop_coff >= 0 && r->next_coff > r->stop_coff) return -1; /* the stop offset is not a block start */
        if (r->next_coff == r->stop_coff && r->stop_uoff == 0) {
            r->stop_at = r->ub_len;
            r->no_more = 1;
            return 0;
        }
        if (r->next_coff >= r->file_size) {
            if (r->stop_coff >= 0) return -1;
            r->no_more = 1;
            return 0;
        }
        if (rd_fetch(r, r->next_coff, 18)) return -1;
        const uint8_t *h = r->cbuf + (r->next_coff - r->cbuf_off);
        if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || !(h[3] & 4)) return -1;
        const int xlen = ld16(h + 10);
        if (rd_fetch(r, r->next_coff, 12 + xlen)) return -1;
        h = r->cbuf + (r->next_coff - r->cbuf_off);
        int bsize = -1;
        for (int o = 0; o + 4 <= xlen;) {
            const int sl = ld16(h + 12 + o + 2);
            if (h[12 + o] == 'B' && h[12 + o + 1] == 'C' && sl == 2) { bsize = ld16(h + 12 + o + 4); break; }
            o += 4 + sl;
        }
        if (bsize < 0) return -1;
        const int64_t blen = (int64_t)bsize + 1;
        if (blen < 12 + xlen + 8 || rd_fetch(r, r->next_coff, blen)) return -1;
        h = r->cbuf + (r->next_coff - r->cbuf_off);
        const uint32_t isize = ld32(h + blen - 4);
        if (isize > 65536) return -1;
        if (rd_reserve(r, r->ub_len + isize + 64)) return -1;
        const double t0 = now_s();
        if (inf_block(&r->inf, h + 12 + xlen, (size_t)(blen - 12 - xlen - 8), r->ub + r->ub_len, isize)) return -1;
        r->t_inflate += now_s() - t0;
        if (r->next_coff == r->stop_coff) {
            r->stop_at = r->ub_len + r->stop_uoff;
            r->no_more = 1;
        }
        r->ub_len += isize;
        r->next_coff += blen;
        r->inflated += isize;
        r->compressed += blen;
        if (isize > 0 || r->no_more) return 1;
    }
}

static int rd_open(pd_reader *r, int fd, int64_t file_size, uint64_t vbeg, uint64_t vend) {
    r->fd = fd;
    r->file_size = file_size;
    r->cbuf_off = r->cbuf_len = 0;
    r->ub_len = r->ub_pos = 0;
    r->stop_at = -1;
    r->no_more = 0;
    r->stop_coff = vend == UINT64_MAX ? -1 : (int64_t)(vend >> 16);
    r->stop_uoff = vend == UINT64_MAX ? 0 : (int)(vend & 0xffff);
    r->next_coff = (int64_t)(vbeg >> 16);
    const int uoff = (int)(vbeg & 0xffff);
    if (uoff > 0 || r->next_coff != r->stop_coff) {
        int k = rd_next_block(r);
        if (k < 0) return -1;
        if (uoff > r->ub_len) return -1;
    }
    r->ub_pos = uoff;
    return 0;
}

/* make at least `need` bytes available at ub_pos: 1, 0 if the range/file
 * ended first, -1 on error */
static int rd_avail(pd_reader *r, int64_t need) {
    while (r->ub_len - r->ub_pos < need) {
        if (r->ub_pos > 0) {
            memmove(r->ub, r->ub + r->ub_pos, (size_t)(r->ub_len - r->ub_pos));
            r->ub_len -= r->ub_pos;
            if (r->stop_at >= 0) r->stop_at -= r->ub_pos;
            r->ub_pos = 0;
        }
        int k = rd_next_block(r);
        if (k < 0) return -1;
        if (k == 0) return 0;
    }
    return 1;
}

static void rd_free(pd_reader *r) {
    free(r->cbuf);
    free(r->ub);
    inf_free(&r->inf);
    memset(r, 0, sizeof(*r));
}

/* ---------------- piece buffers ---------------- */
typedef struct pd_buf {
    /* pinned, appended to the stage: one block holds every part at its first
     * capacity (a part that outgrows it gets a block of its own) */
    char *base;
    size_t base_len;
    int64_t cap;
    void *rec_mem;
    int32_t *pos, *mtid, *mpos, *isize, *lq, *aidx;
    uint16_t *flag;
    uint8_t *mapq;
    uint32_t *coff, *nid;
    int64_t *boff;
    int64_t cap_cig;
    uint32_t *cig;
    int64_t cap_b;
    uint8_t *qual, *seq;
    int64_t cap_aux;
    grom_aux *aux;
    /* pageable */
    int32_t *end, *hclip;
    int64_t cap_drop;
    int32_t *dpos, *dlq;
    int64_t *dbef;
    /* read names: open-addressing table of local ids, arena offsets per id */
    uint32_t *nt_id;
    uint64_t *nt_hash;
    int64_t nt_cap;
    uint32_t *id_off;
    int64_t cap_ids;
    char *arena;
    int64_t arena_len, arena_cap;
    /* counts */
    int64_t n, n_cig, n_b, n_aux, n_drop, n_names;
    /* after the append: which copy must finish before reuse */
    grom_stage *stage;
    int64_t ticket;
    struct pd_buf *next;
} pd_buf;

typedef struct {
    int run;
    uint64_t vbeg, vend;
    int full;             /* decode into a buffer (a processed chromosome's run) */
    volatile int state;   /* 0 pending, 1 busy, 2 done, 3 skipped, 4 error */
    pd_buf *buf;
    int stats;            /* the sample arrays below were collected */
    int32_t *st_ins, *st_lq;
    int64_t *st_m;
    int64_t st_n, st_cap, m_total;
    int64_t n_rec;
    int sorted;           /* positions non-decreasing inside the piece */
    int32_t first_pos;    /* first record's position */
    int32_t last_pos, last_lq, last_hclip, last_kept;
    double secs;
    char err[200];
} pd_piece;

typedef struct {
    int32_t tid;
    int64_t count;        /* -1: unknown (unplaced reads without the index's count) */
    uint64_t vbeg, vend;
    int chrom;            /* plan index taking this run, -1 none */
    int64_t j0;           /* leading records consumed by the previous chromosome (Q1) */
    int first_piece, n_pieces;
    int has_next;         /* a record follows this run in the file */
    int32_t next_lq;      /* its l_qseq (grom_batch_end_record) */
} pd_run;

/* T: reads of earlier pieces of the chromosome that can still overlap a read */
typedef struct {
    uint32_t gid;
    int32_t end;
    int64_t name_off;
} tail_ent;

typedef struct {
    tail_ent *e;
    int64_t n, cap;
    char *arena;
    int64_t arena_len, arena_cap;
    int64_t *ht; /* index+1 into e, 0 empty */
    uint64_t *hh;
    int64_t ht_cap;
    int32_t max_end;
} tail_set;

typedef struct {
    int32_t pos;
    int32_t lq;
    int64_t before;
} drop_rec;

typedef struct {
    int64_t idx;
    grom_aux a;
} saux_rec;

/* per processed chromosome: upload progress and its stream facts */
typedef struct {
    int run;              /* -1: no records */
    int device;
    grom_stage *stage;
    int begun, uploaded, final, handed;
    int64_t j_left;
    int64_t n_kept, n_cig, n_bases, n_aux, n_names;
    int64_t n_seen;       /* stream records after the Q1 drops */
    int32_t last_pos, last_lq, last_hclip, last_kept;
    int32_t prev_pos;     /* sortedness check across pieces */
    drop_rec *drops;
    int64_t n_drops, cap_drops;
    int32_t *lowpos;      /* kept positions < PD_LOWPOS_LIMIT, stream order */
    int64_t n_low, cap_low;
    saux_rec *saux;       /* -S: every kept read's split alignment, resolved at the end */
    int64_t n_saux, cap_saux;
    int kept;             /* in the final plan */
    pd_chrom_facts facts;
    int rc;
    /* host mirror (plan-only) */
    grom_batch mirror;
    int mirror_used;
} pd_chrom;

struct pd_session {
    int fd;
    int64_t file_size;
    int n_plan;
    pd_chrom_in *plan;
    pd_chrom *ch;
    pd_run *runs;
    int n_runs;
    pd_piece *pieces;
    int n_pieces;
    int splitread, read_name_len, min_mapq_stats;
    /* threads */
    int n_threads, window;
    pthread_t *thr;
    pthread_t upl;
    int upl_started;
    pthread_mutex_t mu;
    pthread_cond_t cv;     /* pieces, buffers, window, chromosomes, stats */
    int next_piece, head, abort, stop;
    char abort_msg[300];
    int abort_soft;        /* the index plan was contradicted: read serially */
    /* buffers */
    pd_buf *free_bufs, *inflight_head, *inflight_tail;
    int n_bufs, max_bufs, buf_waiters;
    void **old_pinned;     /* replaced pinned blocks, freed at close */
    int n_old, cap_old;
    /* stats */
    int stats_done, stats_collect;
    int32_t *s_ins, *s_lq;
    int64_t s_n, s_m;
    int walk_set, final_pending, final_applied;
    int next_final, finalizing; /* the uploader's finalisation cursor */
    int *keep;             /* final plan (per preliminary chromosome) */
    int *want;             /* scanned by this process (GROM_CHROMS): unwanted plan chromosomes keep their
                              place in the serial stream's plan but are neither decoded nor staged */
    int32_t index_start, overlap_mult, insert_max;
    /* devices and stages (pd_stream_chrom's caller owns the stages) */
    int plan_only, no_mirror;
    int n_dev;
    int *dev_of;           /* plan index -> device */
    grom_stage **stages;   /* pool: n_stage, each with its device and busy flag */
    int *stage_dev, *stage_busy, *stage_owner; /* owner: the chromosome using it */
    int *stage_mine;       /* made here (freed by pd_close), not by the caller */
    int n_stage, cap_stage, extra_stages;
    /* counters */
    int64_t c_records, c_inflated, c_compressed, c_h2d;
    double c_dec_s, c_upl_s, c_wait_s, c_inflate_s, c_io_s;
    /* GROM_TRACE */
    char *trace_path;
    double t0;
    struct { double t; int64_t a, b; int ev, thr; } *tr;
    int64_t tr_n, tr_cap;
    int test_soft_abort;   /* GROM_TEST_SOFT_ABORT=<piece>: contradict the plan at that piece (tests) */
    /* device mode (pd_start with GROM_DEVICE_DECODE): whole runs inflated and
     * parsed on the GPUs (ddecode.hip) by one worker thread per device */
    int dev_mode;
    uint64_t **lin;        /* per target: the BAI's linear index (record starts every 16 kb) */
    int *n_lin;
    int n_tgt;
    pthread_t *dw;
    int n_dw, dw_started;
    double c_gpu_ms[4];    /* inflate, record walk, parse (HIP events, summed); buffer growth (wall) */
    int64_t c_reclaimed;   /* idle stage blocks freed for a waiting allocation */
    int64_t c_stats_only;  /* device mode: runs decoded for the statistics alone */
    int stats_given;       /* the insert statistics come from <bam>.mean (pd_stats_given) */
    int fetch_mode;        /* GROM -P n: every chromosome its own records (bam_fetch), pd_set_fetch_mode */
    int reclaim_on;        /* pd_reclaim_stages is registered (devmem.h) */
    int64_t c_rewalk, c_subchunks; /* record walk: sub-chunks re-walked / all */
    int io_threads;
    int64_t insert_cap;    /* PD_INSERT_CAP (GROM_TEST_INSERT_CAP: tests of both decoders against each other) */
    int64_t prefix_records; /* GROM_TEST_PREFIX_RECORDS: the stats prefix's record target (tests) */
    /* uploader scratch */
    uint32_t *remap;
    int64_t remap_cap;
    tail_set T;
};

static __thread int tls_thread_id = -1;
static int g_thread_ids;

void pd_trace(pd_session *s, int ev, int64_t a, int64_t b) {
    if (!s || !s->tr) return;
    if (tls_thread_id < 0) tls_thread_id = __sync_fetch_and_add(&g_thread_ids, 1);
    const int64_t i = __sync_fetch_and_add(&s->tr_n, 1);
    if (i >= s->tr_cap) return;
    s->tr[i].t = now_s() - s->t0;
    s->tr[i].ev = ev;
    s->tr[i].a = a;
    s->tr[i].b = b;
    s->tr[i].thr = tls_thread_id;
}

static void sess_abort(pd_session *s, int soft, const char *msg) {
    pthread_mutex_lock(&s->mu);
    if (!s->abort) {
        s->abort = 1;
        s->abort_soft = soft;
        snprintf(s->abort_msg, sizeof(s->abort_msg), "%s", msg);
    }
    pthread_cond_broadcast(&s->cv);
    pthread_mutex_unlock(&s->mu);
}

/* ---- pinned buffer growth ---- */
static void *pin_alloc(pd_session *s, size_t bytes, int pinned) {
    (void)s;
    return pinned ? grom_pinned_alloc(bytes) : malloc(bytes ? bytes : 16);
}

static void pin_retire(pd_session *s, const pd_buf *b, void *p, int pinned) {
    if (!p) return;
    if (b->base && (char *)p >= b->base && (char *)p < b->base + b->base_len) return; /* part of the block */
    if (!pinned) { free(p); return; }
    pthread_mutex_lock(&s->mu);
    if (s->n_old == s->cap_old) {
        s->cap_old = s->cap_old ? 2 * s->cap_old : 64;
        s->old_pinned = (void **)realloc(s->old_pinned, sizeof(void *) * s->cap_old);
    }
    s->old_pinned[s->n_old++] = p;
    pthread_mutex_unlock(&s->mu);
}

/* the per-read arrays as one block: grow to hold `need` reads */
static int buf_grow_recs(pd_session *s, pd_buf *b, int64_t need) {
    if (need <= b->cap) return 0;
    int64_t nc = b->cap ? b->cap : PD_PIECE_RECS + PD_PIECE_RECS / 2;
    while (nc < need) nc *= 2;
    /* pos mtid mpos isize lq aidx (6 x 4) + flag 2 + mapq 1 + coff (n+1)x4 + nid 4 + boff 8 */
    const size_t per = 6 * 4 + 2 + 1 + 4 + 4 + 8;
    const size_t bytes = per * (size_t)nc + 4 + 8 * 64;
    char *m = (char *)pin_alloc(s, bytes, !s->plan_only);
    int32_t *end = (int32_t *)malloc(sizeof(int32_t) * (size_t)nc), *hc = (int32_t *)malloc(sizeof(int32_t) * (size_t)nc);
    if (!m || !end || !hc) { free(end); free(hc); return -1; }
    size_t o = 0;
#define CARVE(field, type, count)                                                                 \
    do {                                                                                           \
        type *p_ = (type *)(m + o);                                                                \
        if (b->n) memcpy(p_, b->field, sizeof(type) * (size_t)(b->n + ((count) > nc ? 1 : 0)));    \
        b->field = p_;                                                                             \
        o += ((sizeof(type) * (size_t)(count)) + 63) & ~(size_t)63;                                \
    } while (0)
    CARVE(boff, int64_t, nc);
    CARVE(pos, int32_t, nc);
    CARVE(mtid, int32_t, nc);
    CARVE(mpos, int32_t, nc);
    CARVE(isize, int32_t, nc);
    CARVE(lq, int32_t, nc);
    CARVE(aidx, int32_t, nc);
    CARVE(coff, uint32_t, nc + 1);
    CARVE(nid, uint32_t, nc);
    CARVE(flag, uint16_t, nc);
    CARVE(mapq, uint8_t, nc);
#undef CARVE
    if (b->n) {
        memcpy(end, b->end, sizeof(int32_t) * (size_t)b->n);
        memcpy(hc, b->hclip, sizeof(int32_t) * (size_t)b->n);
    }
    free(b->end);
    free(b->hclip);
    b->end = end;
    b->hclip = hc;
    pin_retire(s, b, b->rec_mem, !s->plan_only);
    b->rec_mem = m;
    b->cap = nc;
    return 0;
}

static int buf_grow_cig(pd_session *s, pd_buf *b, int64_t need) {
    if (need <= b->cap_cig) return 0;
    int64_t nc = b->cap_cig ? b->cap_cig : 4 * PD_PIECE_RECS;
    while (nc < need) nc *= 2;
    uint32_t *p = (uint32_t *)pin_alloc(s, sizeof(uint32_t) * (size_t)nc, !s->plan_only);
    if (!p) return -1;
    if (b->n_cig) memcpy(p, b->cig, sizeof(uint32_t) * (size_t)b->n_cig);
    pin_retire(s, b, b->cig, !s->plan_only);
    b->cig = p;
    b->cap_cig = nc;
    return 0;
}

static int buf_grow_bases(pd_session *s, pd_buf *b, int64_t need) {
    if (need <= b->cap_b) return 0;
    int64_t nc = b->cap_b ? b->cap_b : (int64_t)200 * PD_PIECE_RECS;
    while (nc < need) nc *= 2;
    /* qual then seq (nc/2) in one block, seq 16-byte aligned */
    uint8_t *p = (uint8_t *)pin_alloc(s, (size_t)nc + (size_t)nc / 2 + 64, !s->plan_only);
    if (!p) return -1;
    uint8_t *q = p, *sq = p + ((nc + 15) & ~(int64_t)15);
    if (b->n_b) {
        memcpy(q, b->qual, (size_t)b->n_b);
        memcpy(sq, b->seq, (size_t)b->n_b / 2);
    }
    pin_retire(s, b, b->qual, !s->plan_only);
    b->qual = q;
    b->seq = sq;
    b->cap_b = nc;
    return 0;
}

static int buf_grow_aux(pd_session *s, pd_buf *b, int64_t need) {
    if (need <= b->cap_aux) return 0;
    int64_t nc = b->cap_aux ? 2 * b->cap_aux : 1024;
    while (nc < need) nc *= 2;
    grom_aux *p = (grom_aux *)pin_alloc(s, sizeof(grom_aux) * (size_t)nc, !s->plan_only);
    if (!p) return -1;
    if (b->n_aux) memcpy(p, b->aux, sizeof(grom_aux) * (size_t)b->n_aux);
    pin_retire(s, b, b->aux, !s->plan_only);
    b->aux = p;
    b->cap_aux = nc;
    return 0;
}

static int buf_grow_drop(pd_buf *b, int64_t need) {
    if (need <= b->cap_drop) return 0;
    int64_t nc = b->cap_drop ? 2 * b->cap_drop : 4096;
    while (nc < need) nc *= 2;
    int32_t *a = (int32_t *)realloc(b->dpos, sizeof(int32_t) * (size_t)nc);
    if (!a) return -1;
    b->dpos = a;
    a = (int32_t *)realloc(b->dlq, sizeof(int32_t) * (size_t)nc);
    if (!a) return -1;
    b->dlq = a;
    int64_t *c = (int64_t *)realloc(b->dbef, sizeof(int64_t) * (size_t)nc);
    if (!c) return -1;
    b->dbef = c;
    b->cap_drop = nc;
    return 0;
}

static void buf_reset(pd_buf *b) {
    b->n = b->n_cig = b->n_b = b->n_aux = b->n_drop = b->n_names = 0;
    b->arena_len = 0;
    b->stage = NULL;
    b->ticket = -1;
    if (b->nt_cap) memset(b->nt_id, 0, sizeof(uint32_t) * (size_t)b->nt_cap);
}

static void buf_destroy(pd_buf *b, int pinned) {
    void *parts[5] = {b->rec_mem, b->cig, b->qual, b->aux, b->base};
    for (int i = 0; i < 5; i++) {
        void *q = parts[i];
        if (!q || (i < 4 && b->base && (char *)q >= b->base && (char *)q < b->base + b->base_len)) continue;
        if (pinned) grom_pinned_free(q);
        else free(q);
    }
    free(b->end);
    free(b->hclip);
    free(b->dpos);
    free(b->dlq);
    free(b->dbef);
    free(b->nt_id);
    free(b->nt_hash);
    free(b->id_off);
    free(b->arena);
    free(b);
}

static uint64_t fnv(const char *p, size_t *len) {
    uint64_t h = 0xcbf29ce484222325ULL;
    const char *q = p;
    for (; *q; q++) h = (h ^ (unsigned char)*q) * 0x100000001b3ULL;
    *len = (size_t)(q - p);
    return h;
}

/* local read-name id (1..), 0 for names the reference never stores
 * (empty or >= read_name_len characters, GROM.c:6813) */
static int64_t buf_intern(pd_buf *b, const char *name, int read_name_len) {
    size_t L;
    const uint64_t h = fnv(name, &L);
    if (L == 0 || L >= (size_t)read_name_len) return 0;
    if (2 * (b->n_names + 1) > b->nt_cap) {
        int64_t nc = b->nt_cap ? 2 * b->nt_cap : 2 * PD_PIECE_RECS;
        uint32_t *ni = (uint32_t *)calloc((size_t)nc, sizeof(uint32_t));
        uint64_t *nh = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)nc);
        if (!ni || !nh) { free(ni); free(nh); return -1; }
        for (int64_t i = 0; i < b->nt_cap; i++)
            if (b->nt_id[i]) {
                int64_t j = (int64_t)(b->nt_hash[i] & (uint64_t)(nc - 1));
                while (ni[j]) j = (j + 1) & (nc - 1);
                ni[j] = b->nt_id[i];
                nh[j] = b->nt_hash[i];
            }
        free(b->nt_id);
        free(b->nt_hash);
        b->nt_id = ni;
        b->nt_hash = nh;
        b->nt_cap = nc;
    }
    int64_t j = (int64_t)(h & (uint64_t)(b->nt_cap - 1));
    while (b->nt_id[j]) {
        if (b->nt_hash[j] == h && strcmp(b->arena + b->id_off[b->nt_id[j]], name) == 0) return b->nt_id[j];
        j = (j + 1) & (b->nt_cap - 1);
    }
    if (b->arena_len + (int64_t)L + 1 > b->arena_cap) {
        int64_t nc = b->arena_cap ? 2 * b->arena_cap : (1 << 22);
        while (nc < b->arena_len + (int64_t)L + 1) nc *= 2;
        char *na = (char *)realloc(b->arena, (size_t)nc);
        if (!na) return -1;
        b->arena = na;
        b->arena_cap = nc;
    }
    if (b->n_names + 2 > b->cap_ids) {
        int64_t nc = b->cap_ids ? 2 * b->cap_ids : PD_PIECE_RECS;
        uint32_t *no = (uint32_t *)realloc(b->id_off, sizeof(uint32_t) * (size_t)nc);
        if (!no) return -1;
        b->id_off = no;
        b->cap_ids = nc;
    }
    memcpy(b->arena + b->arena_len, name, L + 1);
    const uint32_t id = (uint32_t)(++b->n_names);
    b->id_off[id] = (uint32_t)b->arena_len;
    b->arena_len += (int64_t)L + 1;
    b->nt_id[j] = id;
    b->nt_hash[j] = h;
    return id;
}

/* ---------------- decoding one piece ---------------- */
static int stat_push(pd_piece *p, int32_t ins, int32_t lq, int64_t m) {
    if (p->st_n == p->st_cap) {
        int64_t nc = p->st_cap ? 2 * p->st_cap : 16384;
        int32_t *a = (int32_t *)realloc(p->st_ins, sizeof(int32_t) * (size_t)nc);
        if (!a) return -1;
        p->st_ins = a;
        a = (int32_t *)realloc(p->st_lq, sizeof(int32_t) * (size_t)nc);
        if (!a) return -1;
        p->st_lq = a;
        int64_t *c = (int64_t *)realloc(p->st_m, sizeof(int64_t) * (size_t)nc);
        if (!c) return -1;
        p->st_m = c;
        p->st_cap = nc;
    }
    p->st_ins[p->st_n] = ins;
    p->st_lq[p->st_n] = lq;
    p->st_m[p->st_n] = m;
    p->st_n++;
    return 0;
}

static int decode_piece(pd_session *s, pd_reader *r, pd_piece *p, pd_buf *b) {
    const pd_run *run = &s->runs[p->run];
    const char *target = (run->chrom >= 0 && s->plan[run->chrom].target_name) ? s->plan[run->chrom].target_name : "";
    if (rd_open(r, s->fd, s->file_size, p->vbeg, p->vend)) {
        snprintf(p->err, sizeof(p->err), "piece at voffset %llu: bad block", (unsigned long long)p->vbeg);
        return -1;
    }
    const int collect = p->stats;
    int64_t m = 0;
    int32_t prev = INT32_MIN;
    p->sorted = 1;
    p->n_rec = 0;
    p->last_kept = -1;
    for (;;) {
        if (r->stop_at >= 0 && r->ub_pos >= r->stop_at) break;
        int k = rd_avail(r, 4);
        if (k < 0) goto bad;
        if (k == 0) {
            if (r->ub_len - r->ub_pos == 0) break;
            goto bad;
        }
        if (r->stop_at >= 0 && r->ub_pos >= r->stop_at) break;
        const uint32_t bs = ld32(r->ub + r->ub_pos);
        if (bs < 32 || bs > PD_MAX_REC) goto bad;
        if ((k = rd_avail(r, 4 + (int64_t)bs)) <= 0) goto bad;
        const uint8_t *q = r->ub + r->ub_pos + 4;
        const int32_t tid = ldi32(q), pos = ldi32(q + 4);
        const int l_qname = q[8], mapq = q[9];
        const int n_cigar = ld16(q + 12), flag = ld16(q + 14);
        const int32_t lq = ldi32(q + 16), mtid = ldi32(q + 20), mpos = ldi32(q + 24), isz = ldi32(q + 28);
        if (lq < 0 || l_qname < 1 || 32 + (int64_t)l_qname + 4 * (int64_t)n_cigar + (lq + 1) / 2 + lq > (int64_t)bs ||
            tid != run->tid)
            goto bad;
        if (p->n_rec == 0) p->first_pos = pos;
        if (pos < prev) p->sorted = 0;
        prev = pos;
        p->n_rec++;
        const int dropped = (flag & GF_UNMAP) || (flag & GF_DUP);
        if (collect && !dropped) { /* find_insert_mean, GROM.c:1226-1317 */
            int take = 0;
            int32_t v = 0;
            if (!(flag & GF_PAIRED)) { take = 1; v = lq; }
            else if (!(flag & GF_MUNMAP) && tid == mtid && pos < mpos && (flag & GF_PROPER) && isz > 0) { take = 1; v = isz; }
            if (mapq >= s->min_mapq_stats) m += lq;
            if (take && stat_push(p, v, lq, m)) goto oom;
        }
        p->last_pos = pos;
        p->last_lq = lq;
        p->last_hclip = 0;
        if (!b) { /* stats only */
            p->last_kept = !dropped;
            r->ub_pos += 4 + (int64_t)bs;
            continue;
        }
        if (dropped) { /* GROM.c:6418: skipped by the ingest, kept for the breakpoint tests */
            if (buf_grow_drop(b, b->n_drop + 1)) goto oom;
            b->dpos[b->n_drop] = pos;
            b->dlq[b->n_drop] = lq;
            b->dbef[b->n_drop] = b->n;
            b->n_drop++;
            p->last_kept = 0;
            r->ub_pos += 4 + (int64_t)bs;
            continue;
        }
        const int64_t i = b->n;
        if (buf_grow_recs(s, b, i + 1) || buf_grow_cig(s, b, b->n_cig + n_cigar) ||
            buf_grow_bases(s, b, b->n_b + lq + 2))
            goto oom;
        const uint8_t *data = q + 32;
        b->pos[i] = pos;
        b->flag[i] = (uint16_t)flag;
        b->mapq[i] = (uint8_t)mapq;
        b->mtid[i] = mtid;
        b->mpos[i] = mpos;
        b->isize[i] = isz;
        b->lq[i] = lq;
        if (i == 0) b->coff[0] = (uint32_t)b->n_cig;
        const uint8_t *cg = data + l_qname;
        memcpy(b->cig + b->n_cig, cg, 4 * (size_t)n_cigar);
        int32_t span = 0, hc = 0;
        for (int c = 0; c < n_cigar; c++) {
            const uint32_t op = ld32(cg + 4 * c);
            const int o = op & 0xf;
            if (o == GC_MATCH || o == GC_DEL || o == GC_REF_SKIP || o == GC_EQUAL || o == GC_DIFF) span += (int32_t)(op >> 4);
            else if (o == GC_HARD_CLIP) hc += (int32_t)(op >> 4);
        }
        b->n_cig += n_cigar;
        b->coff[i + 1] = (uint32_t)b->n_cig;
        const int64_t Lp = ((int64_t)lq + 1) & ~1LL;
        b->boff[i] = b->n_b;
        const uint8_t *sq = cg + 4 * n_cigar;
        memcpy(b->seq + b->n_b / 2, sq, (size_t)(lq + 1) / 2);
        memcpy(b->qual + b->n_b, sq + (lq + 1) / 2, (size_t)lq);
        if (Lp > lq) b->qual[b->n_b + lq] = 0;
        b->n_b += Lp;
        b->end[i] = pos + span + lq + hc + 1; /* covers every base the read can touch */
        b->hclip[i] = hc;
        p->last_hclip = hc;
        p->last_kept = 1;
        int64_t id = buf_intern(b, (const char *)data, s->read_name_len);
        if (id < 0) goto oom;
        b->nid[i] = (uint32_t)id;
        {
            bam_rec rv;
            memset(&rv, 0, sizeof(rv));
            rv.tid = tid;
            rv.pos = pos;
            rv.l_qname = (uint8_t)l_qname;
            rv.n_cigar = (uint16_t)n_cigar;
            rv.l_qseq = lq;
            rv.data = (uint8_t *)data;
            rv.data_len = (int32_t)bs - 32;
            grom_aux ax;
            b->aidx[i] = -1;
            if (grom_parse_aux(&rv, target, &ax)) {
                if (buf_grow_aux(s, b, b->n_aux + 1)) goto oom;
                b->aidx[i] = (int32_t)b->n_aux;
                b->aux[b->n_aux++] = ax;
            }
        }
        b->n = i + 1;
        r->ub_pos += 4 + (int64_t)bs;
    }
    p->m_total = m;
    return 0;
bad:
    snprintf(p->err, sizeof(p->err), "piece [%llu, %llu) of target %d does not decode as records of that target",
             (unsigned long long)p->vbeg, (unsigned long long)p->vend, run->tid);
    return -2;
oom:
    snprintf(p->err, sizeof(p->err), "out of host memory decoding a piece");
    return -1;
}

/* ---------------- buffer pool ---------------- */
/* a new buffer: every part carved from one block at its first capacity */
static int buf_block(pd_session *s, pd_buf *b) {
    const int64_t nr = PD_PIECE_RECS + PD_PIECE_RECS / 2, ncig = 4 * PD_PIECE_RECS, nb = (int64_t)160 * PD_PIECE_RECS,
                  naux = 1024;
    const size_t rec = (6 * 4 + 2 + 1 + 4 + 4 + 8) * (size_t)nr + 4 + 8 * 64;
    const size_t sz[4] = {rec, 4 * (size_t)ncig, (size_t)nb + (size_t)nb / 2 + 64, sizeof(grom_aux) * (size_t)naux};
    size_t off[4], tot = 0;
    for (int i = 0; i < 4; i++) {
        off[i] = tot;
        tot += (sz[i] + 255) & ~(size_t)255;
    }
    b->base = (char *)pin_alloc(s, tot, !s->plan_only);
    if (!b->base) return -1;
    b->base_len = tot;
    /* the growth functions carve from a part pointer that they then retire:
     * point them at the block and let them "grow" from zero */
    char *m = b->base + off[0];
    size_t o = 0;
#define CARVE0(field, type, count)                                                                \
    do {                                                                                          \
        b->field = (type *)(m + o);                                                               \
        o += ((sizeof(type) * (size_t)(count)) + 63) & ~(size_t)63;                               \
    } while (0)
    CARVE0(boff, int64_t, nr);
    CARVE0(pos, int32_t, nr);
    CARVE0(mtid, int32_t, nr);
    CARVE0(mpos, int32_t, nr);
    CARVE0(isize, int32_t, nr);
    CARVE0(lq, int32_t, nr);
    CARVE0(aidx, int32_t, nr);
    CARVE0(coff, uint32_t, nr + 1);
    CARVE0(nid, uint32_t, nr);
    CARVE0(flag, uint16_t, nr);
    CARVE0(mapq, uint8_t, nr);
#undef CARVE0
    b->rec_mem = m;
    b->cap = nr;
    b->end = (int32_t *)malloc(sizeof(int32_t) * (size_t)nr);
    b->hclip = (int32_t *)malloc(sizeof(int32_t) * (size_t)nr);
    if (!b->end || !b->hclip) return -1;
    b->cig = (uint32_t *)(b->base + off[1]);
    b->cap_cig = ncig;
    b->qual = (uint8_t *)(b->base + off[2]);
    b->seq = b->qual + ((nb + 15) & ~(int64_t)15);
    b->cap_b = nb;
    b->aux = (grom_aux *)(b->base + off[3]);
    b->cap_aux = naux;
    return 0;
}

static pd_buf *pool_get(pd_session *s) {
    pthread_mutex_lock(&s->mu);
    for (;;) {
        if (s->abort) { pthread_mutex_unlock(&s->mu); return NULL; }
        if (s->free_bufs) {
            pd_buf *b = s->free_bufs;
            s->free_bufs = b->next;
            pthread_mutex_unlock(&s->mu);
            buf_reset(b);
            return b;
        }
        if (s->n_bufs < s->max_bufs) {
            s->n_bufs++;
            pthread_mutex_unlock(&s->mu);
            pd_buf *b = (pd_buf *)calloc(1, sizeof(pd_buf));
            if (b && buf_block(s, b)) { buf_destroy(b, !s->plan_only); b = NULL; }
            if (b) buf_reset(b);
            return b;
        }
        s->buf_waiters++;
        pthread_cond_broadcast(&s->cv);
        pthread_cond_wait(&s->cv, &s->mu);
        s->buf_waiters--;
    }
}

/* uploader: buffers whose copies finished go back to the free list (force:
 * wait for the oldest one if decoders are starved) */
static void pool_reclaim(pd_session *s, int force) {
    for (;;) {
        pd_buf *b = s->inflight_head;
        if (!b) return;
        if (!grom_stage_ticket_done(b->stage, b->ticket)) {
            if (!force) return;
            (void)grom_stage_ticket_wait(b->stage, b->ticket);
        }
        force = 0;
        s->inflight_head = b->next;
        if (!s->inflight_head) s->inflight_tail = NULL;
        pthread_mutex_lock(&s->mu);
        b->next = s->free_bufs;
        s->free_bufs = b;
        pthread_cond_broadcast(&s->cv);
        pthread_mutex_unlock(&s->mu);
    }
}

static void pool_put_now(pd_session *s, pd_buf *b) {
    pthread_mutex_lock(&s->mu);
    b->next = s->free_bufs;
    s->free_bufs = b;
    pthread_cond_broadcast(&s->cv);
    pthread_mutex_unlock(&s->mu);
}

static void pool_put_inflight(pd_session *s, pd_buf *b) {
    b->next = NULL;
    if (s->inflight_tail) s->inflight_tail->next = b;
    else s->inflight_head = b;
    s->inflight_tail = b;
}

/* ---------------- decoder threads ---------------- */
static void *decoder_main(void *arg) {
    pd_session *s = (pd_session *)arg;
    pd_reader r;
    memset(&r, 0, sizeof(r));
    inf_init(&r.inf);
    int64_t recs = 0;
    double secs = 0;
    for (;;) {
        pthread_mutex_lock(&s->mu);
        while (!s->abort && !s->stop && s->next_piece < s->n_pieces && s->next_piece >= s->head + s->window)
            pthread_cond_wait(&s->cv, &s->mu);
        if (s->abort || s->stop || s->next_piece >= s->n_pieces) {
            pthread_mutex_unlock(&s->mu);
            break;
        }
        const int idx = s->next_piece++;
        pd_piece *p = &s->pieces[idx];
        const int need_stats = !s->stats_done;
        const int full = p->full;
        p->state = 1;
        pthread_mutex_unlock(&s->mu);
        const double t0 = now_s();
        int rc = 0;
        pd_trace(s, PD_EV_DECODE, idx, 0);
        if (!full && !need_stats) {
            pthread_mutex_lock(&s->mu);
            p->state = 3;
            pthread_cond_broadcast(&s->cv);
            pthread_mutex_unlock(&s->mu);
            continue;
        }
        p->stats = need_stats;
        pd_buf *b = NULL;
        if (full) {
            b = pool_get(s);
            if (!b) { rc = -1; snprintf(p->err, sizeof(p->err), "no piece buffer"); }
        }
        if (rc == 0) rc = decode_piece(s, &r, p, b);
        p->buf = b;
        pd_trace(s, PD_EV_DECODE, idx, 1);
        p->secs = now_s() - t0;
        secs += p->secs;
        recs += p->n_rec;
        pthread_mutex_lock(&s->mu);
        p->state = rc == 0 ? 2 : 4;
        pthread_cond_broadcast(&s->cv);
        pthread_mutex_unlock(&s->mu);
        if (rc != 0) sess_abort(s, rc == -2, p->err);
    }
    pthread_mutex_lock(&s->mu);
    s->c_dec_s += secs;
    s->c_inflated += r.inflated;
    s->c_inflate_s += r.t_inflate;
    s->c_io_s += r.t_io;
    s->c_compressed += r.compressed;
    pthread_mutex_unlock(&s->mu);
    rd_free(&r);
    return NULL;
}

/* ---------------- the tail set of read names ---------------- */
static void tail_reset(tail_set *T) {
    T->n = 0;
    T->arena_len = 0;
    T->max_end = INT32_MIN;
    if (T->ht_cap) memset(T->ht, 0, sizeof(int64_t) * (size_t)T->ht_cap);
}

static void tail_rehash(tail_set *T, int64_t want) {
    int64_t nc = 64;
    while (nc < 4 * want) nc *= 2;
    if (nc != T->ht_cap) {
        free(T->ht);
        free(T->hh);
        T->ht = (int64_t *)calloc((size_t)nc, sizeof(int64_t));
        T->hh = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)nc);
        T->ht_cap = nc;
    } else {
        memset(T->ht, 0, sizeof(int64_t) * (size_t)nc);
    }
    for (int64_t i = 0; i < T->n; i++) {
        size_t L;
        const uint64_t h = fnv(T->arena + T->e[i].name_off, &L);
        int64_t j = (int64_t)(h & (uint64_t)(T->ht_cap - 1));
        while (T->ht[j]) j = (j + 1) & (T->ht_cap - 1);
        T->ht[j] = i + 1;
        T->hh[j] = h;
    }
}

/* keep the entries that can still overlap a read at or after p0 */
static void tail_filter(tail_set *T, int32_t p0) {
    int64_t k = 0, al = 0;
    int32_t mx = INT32_MIN;
    for (int64_t i = 0; i < T->n; i++) {
        if (T->e[i].end <= p0) continue;
        const char *nm = T->arena + T->e[i].name_off;
        const size_t L = strlen(nm);
        memmove(T->arena + al, nm, L + 1);
        T->e[k] = T->e[i];
        T->e[k].name_off = al;
        al += (int64_t)L + 1;
        if (T->e[k].end > mx) mx = T->e[k].end;
        k++;
    }
    T->n = k;
    T->arena_len = al;
    T->max_end = mx;
    tail_rehash(T, k + 64);
}

static int64_t tail_find(const tail_set *T, const char *name) {
    if (!T->n) return -1;
    size_t L;
    const uint64_t h = fnv(name, &L);
    int64_t j = (int64_t)(h & (uint64_t)(T->ht_cap - 1));
    while (T->ht[j]) {
        const int64_t i = T->ht[j] - 1;
        if (T->hh[j] == h && strcmp(T->arena + T->e[i].name_off, name) == 0) return i;
        j = (j + 1) & (T->ht_cap - 1);
    }
    return -1;
}

static void tail_add(tail_set *T, const char *name, uint32_t gid, int32_t end) {
    const int64_t f = tail_find(T, name);
    if (f >= 0) {
        if (end > T->e[f].end) T->e[f].end = end;
        if (end > T->max_end) T->max_end = end;
        return;
    }
    const size_t L = strlen(name);
    if (T->n == T->cap) {
        T->cap = T->cap ? 2 * T->cap : 256;
        T->e = (tail_ent *)realloc(T->e, sizeof(tail_ent) * (size_t)T->cap);
    }
    if (T->arena_len + (int64_t)L + 1 > T->arena_cap) {
        T->arena_cap = T->arena_cap ? 2 * T->arena_cap : 16384;
        while (T->arena_len + (int64_t)L + 1 > T->arena_cap) T->arena_cap *= 2;
        T->arena = (char *)realloc(T->arena, (size_t)T->arena_cap);
    }
    memcpy(T->arena + T->arena_len, name, L + 1);
    T->e[T->n].gid = gid;
    T->e[T->n].end = end;
    T->e[T->n].name_off = T->arena_len;
    T->arena_len += (int64_t)L + 1;
    T->n++;
    if (end > T->max_end) T->max_end = end;
    if (4 * T->n > T->ht_cap) tail_rehash(T, T->n);
    else {
        uint64_t h;
        size_t LL;
        h = fnv(name, &LL);
        int64_t j = (int64_t)(h & (uint64_t)(T->ht_cap - 1));
        while (T->ht[j]) j = (j + 1) & (T->ht_cap - 1);
        T->ht[j] = T->n;
        T->hh[j] = h;
    }
}

/* ---------------- host mirror (plan-only / tests) ---------------- */
static int mirror_append(grom_batch *m, const grom_reads *p) {
    const int64_t n = m->n + p->n;
    if (n + 1 > m->cap) {
        int64_t nc = m->cap ? 2 * m->cap : 4096;
        while (nc < n + 1) nc *= 2;
#define RA(f, t) m->f = (t *)realloc(m->f, sizeof(t) * (size_t)nc)
        RA(pos, int32_t); RA(flag, uint16_t); RA(mapq, uint8_t); RA(mtid, int32_t); RA(mpos, int32_t);
        RA(isize, int32_t); RA(l_qseq, int32_t); RA(base_off, int64_t); RA(name_id, uint32_t); RA(aux_idx, int32_t);
#undef RA
        m->cigar_off = (uint32_t *)realloc(m->cigar_off, sizeof(uint32_t) * (size_t)(nc + 1));
        m->cap = nc;
    }
    if (m->n_cig + p->n_cigar_ops > m->cap_cig) {
        int64_t nc = m->cap_cig ? m->cap_cig : 4096;
        while (nc < m->n_cig + p->n_cigar_ops) nc *= 2;
        m->cigar = (uint32_t *)realloc(m->cigar, sizeof(uint32_t) * (size_t)nc);
        m->cap_cig = nc;
    }
    if (m->n_bases + p->n_bases > m->cap_bases) {
        int64_t nc = m->cap_bases ? m->cap_bases : 1 << 20;
        while (nc < m->n_bases + p->n_bases) nc *= 2;
        m->qual = (uint8_t *)realloc(m->qual, (size_t)nc);
        m->seq = (uint8_t *)realloc(m->seq, (size_t)nc / 2);
        m->cap_bases = nc;
    }
    if (m->n_aux + p->n_aux > m->cap_aux) {
        int64_t nc = m->cap_aux ? 2 * m->cap_aux : 1024;
        while (nc < m->n_aux + p->n_aux) nc *= 2;
        m->aux = (grom_aux *)realloc(m->aux, sizeof(grom_aux) * (size_t)nc);
        m->cap_aux = nc;
    }
    if (m->n_drop + p->n_drop > m->cap_drop) {
        int64_t nc = m->cap_drop ? 2 * m->cap_drop : 1024;
        while (nc < m->n_drop + p->n_drop) nc *= 2;
        m->drop_pos = (int32_t *)realloc(m->drop_pos, sizeof(int32_t) * (size_t)nc);
        m->drop_lq = (int32_t *)realloc(m->drop_lq, sizeof(int32_t) * (size_t)nc);
        m->drop_before = (int64_t *)realloc(m->drop_before, sizeof(int64_t) * (size_t)nc);
        m->cap_drop = nc;
    }
    const int64_t k = p->n, o = m->n;
    if (k > 0) {
        memcpy(m->pos + o, p->pos, 4 * (size_t)k);
        memcpy(m->flag + o, p->flag, 2 * (size_t)k);
        memcpy(m->mapq + o, p->mapq, (size_t)k);
        memcpy(m->mtid + o, p->mtid, 4 * (size_t)k);
        memcpy(m->mpos + o, p->mpos, 4 * (size_t)k);
        memcpy(m->isize + o, p->isize, 4 * (size_t)k);
        memcpy(m->l_qseq + o, p->l_qseq, 4 * (size_t)k);
        memcpy(m->cigar_off + o, p->cigar_off, 4 * (size_t)(k + 1));
        memcpy(m->base_off + o, p->base_off, 8 * (size_t)k);
        memcpy(m->name_id + o, p->name_id, 4 * (size_t)k);
        if (p->aux_idx) memcpy(m->aux_idx + o, p->aux_idx, 4 * (size_t)k);
        else memset(m->aux_idx + o, 0xff, 4 * (size_t)k);
        memcpy(m->cigar + m->n_cig, p->cigar, 4 * (size_t)p->n_cigar_ops);
        memcpy(m->qual + m->n_bases, p->qual, (size_t)p->n_bases);
        memcpy(m->seq + m->n_bases / 2, p->seq, (size_t)p->n_bases / 2);
    }
    if (p->n_aux > 0) memcpy(m->aux + m->n_aux, p->aux, sizeof(grom_aux) * (size_t)p->n_aux);
    if (p->n_drop > 0) {
        memcpy(m->drop_pos + m->n_drop, p->drop_pos, 4 * (size_t)p->n_drop);
        memcpy(m->drop_lq + m->n_drop, p->drop_lq, 4 * (size_t)p->n_drop);
        memcpy(m->drop_before + m->n_drop, p->drop_before, 8 * (size_t)p->n_drop);
    }
    m->n = n;
    m->n_cig += p->n_cigar_ops;
    m->n_bases += p->n_bases;
    m->n_aux += p->n_aux;
    m->n_drop += p->n_drop;
    if (m->n == 0) {
        if (!m->cigar_off) m->cigar_off = (uint32_t *)calloc(1, sizeof(uint32_t));
    }
    return 0;
}

/* ---------------- the uploader ---------------- */
static void apply_final(pd_session *s, int idx);

/* A stage for chromosome k on GPU `dev`.  Waiting for a busy one is safe
 * only when every busy stage belongs to a chromosome already finalised (the
 * scans release those); a stage held by a chromosome still waiting for its
 * finalisation -- which this same thread does -- would never come back, so
 * then one more stage is made instead. */
static int stage_acquire(pd_session *s, int dev, int k, grom_stage **out) {
    pd_trace(s, PD_EV_STAGE, k, 0);
    pthread_mutex_lock(&s->mu);
    for (;;) {
        if (s->abort) { pthread_mutex_unlock(&s->mu); return -1; }
        for (int i = 0; i < s->n_stage; i++)
            if (!s->stage_busy[i] && s->stage_dev[i] == dev) {
                s->stage_busy[i] = 1;
                s->stage_owner[i] = k;
                *out = s->stages[i];
                pthread_mutex_unlock(&s->mu);
                pd_trace(s, PD_EV_STAGE, k, 1);
                return 0;
            }
        int reserving = 0;
        for (int i = 0; i < s->n_stage; i++) reserving |= s->stage_busy[i] && s->stage_owner[i] == -2;
        if (reserving) { /* stres_main is growing this device's stages: wait for them */
            pthread_cond_wait(&s->cv, &s->mu);
            continue;
        }
        int unsafe = s->n_stage < 1;
        for (int i = 0; i < s->n_stage && !unsafe; i++)
            if (s->stage_busy[i] && (s->stage_owner[i] < 0 || !s->ch[s->stage_owner[i]].final)) unsafe = 1;
        if (unsafe) {
            pthread_mutex_unlock(&s->mu);
            grom_stage *st = grom_stage_new(dev);
            if (!st) return -1;
            pthread_mutex_lock(&s->mu);
            if (s->n_stage == s->cap_stage) {
                s->cap_stage = s->cap_stage ? 2 * s->cap_stage : 16;
                s->stages = (grom_stage **)realloc(s->stages, sizeof(grom_stage *) * s->cap_stage);
                s->stage_dev = (int *)realloc(s->stage_dev, sizeof(int) * s->cap_stage);
                s->stage_busy = (int *)realloc(s->stage_busy, sizeof(int) * s->cap_stage);
                s->stage_owner = (int *)realloc(s->stage_owner, sizeof(int) * s->cap_stage);
                s->stage_mine = (int *)realloc(s->stage_mine, sizeof(int) * s->cap_stage);
            }
            s->stages[s->n_stage] = st;
            s->stage_dev[s->n_stage] = dev;
            s->stage_busy[s->n_stage] = 1;
            s->stage_owner[s->n_stage] = k;
            s->stage_mine[s->n_stage] = 1;
            s->n_stage++;
            s->extra_stages++;
            *out = st;
            pthread_mutex_unlock(&s->mu);
            pd_trace(s, PD_EV_STAGE, k, 2);
            return 0;
        }
        pthread_cond_wait(&s->cv, &s->mu);
    }
}

static void stats_take(pd_session *s, pd_piece *p) {
    if (s->stats_done || !p->stats) return;
    for (int64_t i = 0; i < p->st_n && s->s_n < s->insert_cap; i++) {
        s->s_ins[s->s_n] = p->st_ins[i];
        s->s_lq[s->s_n] = p->st_lq[i];
        s->s_n++;
        if (s->s_n == s->insert_cap) s->s_m += p->st_m[i];
    }
    if (s->s_n < s->insert_cap) s->s_m += p->m_total;
}

static void piece_free_stats(pd_piece *p) {
    free(p->st_ins);
    free(p->st_lq);
    free(p->st_m);
    p->st_ins = p->st_lq = NULL;
    p->st_m = NULL;
    p->st_n = p->st_cap = 0;
}

static void mark_stats_done(pd_session *s) {
    pd_trace(s, PD_EV_STATS, 0, 0);
    pthread_mutex_lock(&s->mu);
    s->stats_done = 1;
    pthread_cond_broadcast(&s->cv);
    pthread_mutex_unlock(&s->mu);
}

static int finalize_ready(pd_session *s);

static int chrom_begin(pd_session *s, int k, const pd_buf *first) {
    pd_chrom *c = &s->ch[k];
    c->begun = 1;
    if (s->plan_only) return 0;
    /* earlier chromosomes first: their stages can then go back to the pool */
    if (finalize_ready(s)) return -1;
    if (stage_acquire(s, c->device, k, &c->stage)) return -1;
    grom_stage_sizes est;
    memset(&est, 0, sizeof(est));
    if (c->run >= 0) {
        const pd_run *r = &s->runs[c->run];
        const int64_t cnt = r->count > 0 ? r->count : 1;
        est.n = cnt;
        est.n_drop = first && first->n_drop ? (int64_t)((double)first->n_drop / (first->n + first->n_drop + 1) * cnt * 1.5) + 1024 : 1024;
        if (first && first->n > 0) {
            est.n_cigar_ops = (int64_t)((double)first->n_cig / first->n * cnt * 1.15) + 4096;
            est.n_bases = ((int64_t)((double)first->n_b / first->n * cnt * 1.15) + 65536) & ~1LL;
            est.n_aux = (int64_t)((double)first->n_aux / first->n * cnt * 1.5) + 1024;
        }
    }
    return grom_stage_begin(c->stage, &est) == GROM_OK ? 0 : -1;
}

static int upload_piece(pd_session *s, pd_piece *p) {
    const pd_run *run = &s->runs[p->run];
    pd_chrom *c = &s->ch[run->chrom];
    pd_buf *b = p->buf;
    if (!c->begun && chrom_begin(s, run->chrom, b)) return -1;
    const int64_t n = b->n, nd = b->n_drop;
    /* the records the previous chromosome's walk consumed (Q1): the stream's
     * first j0 records, in stream order (a dropped record with before == k
     * precedes kept read k) */
    int64_t k0 = 0, d0 = 0;
    while (c->j_left > 0 && (k0 < n || d0 < nd)) {
        if (d0 < nd && b->dbef[d0] == k0) d0++;
        else k0++;
        c->j_left--;
    }
    const int64_t seen = (n - k0) + (nd - d0);
    if (seen > 0) {
        if (!p->sorted) { sess_abort(s, 1, "records are not sorted by position"); return -1; }
        const int32_t first_pos = (k0 < n && (d0 >= nd || b->dbef[d0] > k0)) ? b->pos[k0] : b->dpos[d0];
        if (c->n_seen > 0 && first_pos < c->prev_pos) { sess_abort(s, 1, "records are not sorted by position"); return -1; }
        c->prev_pos = p->last_pos;
        c->n_seen += seen;
        c->last_pos = p->last_pos;
        c->last_lq = p->last_lq;
        c->last_hclip = p->last_hclip;
        c->last_kept = p->last_kept;
    }
    /* drops: to the chromosome's host list (uploaded when it is finalised) */
    for (int64_t d = d0; d < nd; d++) {
        if (c->n_drops == c->cap_drops) {
            c->cap_drops = c->cap_drops ? 2 * c->cap_drops : 4096;
            c->drops = (drop_rec *)realloc(c->drops, sizeof(drop_rec) * (size_t)c->cap_drops);
            if (!c->drops) return -1;
        }
        drop_rec *q = &c->drops[c->n_drops++];
        q->pos = b->dpos[d];
        q->lq = b->dlq[d];
        q->before = c->n_kept + (b->dbef[d] - k0);
    }
    const int64_t m = n - k0;
    if (m > 0) {
        /* read-name ids: piece-local -> chromosome ids, equal for equal names
         * of reads that can share a base (T holds the earlier pieces' reads
         * that reach this far) */
        if (s->remap_cap < b->n_names + 1) {
            s->remap_cap = b->n_names + 1 + 1024;
            s->remap = (uint32_t *)realloc(s->remap, sizeof(uint32_t) * (size_t)s->remap_cap);
            if (!s->remap) return -1;
        }
        s->remap[0] = 0;
        for (int64_t l = 1; l <= b->n_names; l++) s->remap[l] = (uint32_t)(c->n_names + l);
        tail_filter(&s->T, b->pos[k0]);
        for (int64_t i = k0; i < n && b->pos[i] < s->T.max_end; i++) {
            const uint32_t l = b->nid[i];
            if (!l) continue;
            const int64_t f = tail_find(&s->T, b->arena + b->id_off[l]);
            if (f >= 0) s->remap[l] = s->T.e[f].gid;
        }
        c->n_names += b->n_names;
        for (int64_t i = k0; i < n; i++) {
            const uint32_t l = b->nid[i];
            if (l && b->end[i] > p->last_pos) tail_add(&s->T, b->arena + b->id_off[l], s->remap[l], b->end[i]);
        }
        for (int64_t i = k0; i < n; i++) b->nid[i] = s->remap[b->nid[i]];
        /* kept positions that may lie in the walk's skip prefix */
        for (int64_t i = k0; i < n && b->pos[i] < PD_LOWPOS_LIMIT; i++) {
            if (c->n_low == c->cap_low) {
                c->cap_low = c->cap_low ? 2 * c->cap_low : 65536;
                c->lowpos = (int32_t *)realloc(c->lowpos, sizeof(int32_t) * (size_t)c->cap_low);
                if (!c->lowpos) return -1;
            }
            c->lowpos[c->n_low++] = b->pos[i];
        }
        /* global offsets */
        const uint32_t c0 = b->coff[k0];
        const int64_t b0 = b->boff[k0];
        for (int64_t i = k0; i <= n; i++) b->coff[i] = b->coff[i] - c0 + (uint32_t)c->n_cig;
        for (int64_t i = k0; i < n; i++) b->boff[i] = b->boff[i] - b0 + c->n_bases;
        int64_t a0 = b->n_aux;
        for (int64_t i = k0; i < n; i++)
            if (b->aidx[i] >= 0) { a0 = b->aidx[i]; break; }
        grom_reads v;
        memset(&v, 0, sizeof(v));
        v.n = m;
        v.pos = b->pos + k0;
        v.flag = b->flag + k0;
        v.mapq = b->mapq + k0;
        v.mtid = b->mtid + k0;
        v.mpos = b->mpos + k0;
        v.isize = b->isize + k0;
        v.l_qseq = b->lq + k0;
        v.cigar_off = b->coff + k0;
        v.cigar = b->cig + c0 - 0; /* c0 was the piece-local offset of read k0 */
        v.n_cigar_ops = (int64_t)b->n_cig - (int64_t)c0;
        v.base_off = b->boff + k0;
        v.seq = b->seq + b0 / 2;
        v.qual = b->qual + b0;
        v.n_bases = b->n_b - b0;
        v.name_id = b->nid + k0;
        if (s->splitread) {
            for (int64_t i = k0; i < n; i++)
                if (b->aidx[i] >= 0) b->aidx[i] = (int32_t)(b->aidx[i] - a0 + c->n_aux);
            v.aux_idx = b->aidx + k0;
            v.aux = b->aux + a0;
            v.n_aux = b->n_aux - a0;
        } else {
            /* -S: only the walk's first ingested read keeps its SA/XP (Q13),
             * known when the chromosome is finalised */
            for (int64_t i = k0; i < n; i++)
                if (b->aidx[i] >= 0) {
                    if (c->n_saux == c->cap_saux) {
                        c->cap_saux = c->cap_saux ? 2 * c->cap_saux : 1024;
                        c->saux = (saux_rec *)realloc(c->saux, sizeof(saux_rec) * (size_t)c->cap_saux);
                        if (!c->saux) return -1;
                    }
                    c->saux[c->n_saux].idx = c->n_kept + (i - k0);
                    c->saux[c->n_saux].a = b->aux[b->aidx[i]];
                    c->n_saux++;
                }
            v.aux_idx = NULL;
            v.n_aux = 0;
        }
        if (s->plan_only) {
            if (!s->no_mirror) mirror_append(&c->mirror, &v);
            c->mirror_used = 1;
        } else {
            const int64_t t = grom_stage_append(c->stage, &v);
            if (t < 0) return -1;
            b->stage = c->stage;
            b->ticket = t;
        }
        c->n_kept += m;
        c->n_cig += v.n_cigar_ops;
        c->n_bases += v.n_bases;
        c->n_aux += v.n_aux;
    }
    return 0;
}

/* the walk's facts and the trims that need the insert statistics
 * (grom_batch_add's skip branch and grom_batch_finish, GROM.c:14859-14969,
 * 5842, 6406-6412) */
static int chrom_finalize(pd_session *s, int k) {
    pd_chrom *c = &s->ch[k];
    if (!c->begun && chrom_begin(s, k, NULL)) return -1;
    const int32_t s0 = s->index_start;
    if (s0 > PD_LOWPOS_LIMIT) { sess_abort(s, 1, "walk index start beyond the streamed prefix limit"); return -1; }
    int64_t sk = 0, sd = 0;
    for (int64_t i = 0; i < c->n_low; i++) sk += c->lowpos[i] < s0;
    while (sd < c->n_drops && c->drops[sd].pos < s0) sd++;
    const int any = (c->n_kept + c->n_drops) > (sk + sd);
    pd_chrom_facts *f = &c->facts;
    memset(f, 0, sizeof(*f));
    f->n_skip = (int32_t)(sk + sd);
    f->n_reads = c->n_kept - sk;
    f->n_drop = c->n_drops - sd;
    if (any) {
        const int32_t p = c->last_pos - s->overlap_mult * s->insert_max;
        f->p_last = p > s0 ? p : s0;
    } else {
        f->p_last = -1;
    }
    /* (-P: the chromosome's stream ends at its own last record) */
    if (c->n_seen > 0 && c->run >= 0 && s->runs[c->run].has_next && !s->fetch_mode) f->lseq_tail = s->runs[c->run].next_lq;
    else if (any) f->lseq_tail = c->last_lq + (c->last_kept == 1 ? c->last_hclip : 0);
    else f->lseq_tail = 0;
    /* drops after the prefix, counting kept reads after the trim */
    grom_reads dv;
    memset(&dv, 0, sizeof(dv));
    const int64_t ndr = c->n_drops - sd;
    int32_t *dp = NULL, *dl = NULL;
    int64_t *db = NULL;
    if (ndr > 0) {
        dp = s->plan_only ? (int32_t *)malloc(4 * (size_t)ndr) : (int32_t *)grom_pinned_alloc(4 * (size_t)ndr);
        dl = s->plan_only ? (int32_t *)malloc(4 * (size_t)ndr) : (int32_t *)grom_pinned_alloc(4 * (size_t)ndr);
        db = s->plan_only ? (int64_t *)malloc(8 * (size_t)ndr) : (int64_t *)grom_pinned_alloc(8 * (size_t)ndr);
        if (!dp || !dl || !db) {
            if (s->plan_only) { free(dp); free(dl); free(db); }
            else { grom_pinned_free(dp); grom_pinned_free(dl); grom_pinned_free(db); }
            return -1;
        }
        for (int64_t d = 0; d < ndr; d++) {
            const drop_rec *q = &c->drops[sd + d];
            dp[d] = q->pos;
            dl[d] = q->lq;
            db[d] = q->before >= sk ? q->before - sk : 0;
        }
        dv.n_drop = ndr;
        dv.drop_pos = dp;
        dv.drop_lq = dl;
        dv.drop_before = db;
    }
    /* -S: the first ingested record, if it is a kept read, keeps its SA/XP */
    int64_t patch = -1;
    grom_aux pa;
    memset(&pa, 0, sizeof(pa));
    if (!s->splitread && any) {
        const int first_is_drop = sd < c->n_drops && c->drops[sd].before == sk;
        if (!first_is_drop)
            for (int64_t i = 0; i < c->n_saux; i++)
                if (c->saux[i].idx == sk) { patch = sk; pa = c->saux[i].a; break; }
    }
    int rc = 0;
    if (s->plan_only) {
        grom_batch *m = &c->mirror;
        if (patch >= 0) {
            grom_reads one;
            memset(&one, 0, sizeof(one));
            one.n_aux = 1;
            one.aux = &pa;
            mirror_append(m, &one);
            m->aux_idx[patch] = (int32_t)(m->n_aux - 1);
        }
        if (ndr > 0) mirror_append(m, &dv);
        if (sk > 0) { /* drop the prefix from the front (the device uses a trimmed view) */
            const int64_t r = m->n - sk;
            memmove(m->pos, m->pos + sk, 4 * (size_t)r);
            memmove(m->flag, m->flag + sk, 2 * (size_t)r);
            memmove(m->mapq, m->mapq + sk, (size_t)r);
            memmove(m->mtid, m->mtid + sk, 4 * (size_t)r);
            memmove(m->mpos, m->mpos + sk, 4 * (size_t)r);
            memmove(m->isize, m->isize + sk, 4 * (size_t)r);
            memmove(m->l_qseq, m->l_qseq + sk, 4 * (size_t)r);
            memmove(m->cigar_off, m->cigar_off + sk, 4 * (size_t)(r + 1));
            memmove(m->base_off, m->base_off + sk, 8 * (size_t)r);
            memmove(m->name_id, m->name_id + sk, 4 * (size_t)r);
            memmove(m->aux_idx, m->aux_idx + sk, 4 * (size_t)r);
            m->n = r;
        }
        if (!m->cigar_off) m->cigar_off = (uint32_t *)calloc(1, sizeof(uint32_t));
        free(dp);
        free(dl);
        free(db);
    } else {
        if (patch >= 0 && grom_stage_patch_aux(c->stage, patch, &pa) != GROM_OK) rc = -1;
        if (rc == 0 && ndr > 0) {
            const int64_t t = grom_stage_append(c->stage, &dv);
            /* the copies read these arrays: wait for them before they go */
            if (t < 0 || grom_stage_ticket_wait(c->stage, t) != GROM_OK) rc = -1;
        }
        if (rc == 0 && grom_stage_trim(c->stage, sk) != GROM_OK) rc = -1;
        s->c_h2d += grom_stage_bytes(c->stage);
        grom_pinned_free(dp);
        grom_pinned_free(dl);
        grom_pinned_free(db);
    }
    free(c->drops);
    c->drops = NULL;
    free(c->lowpos);
    c->lowpos = NULL;
    free(c->saux);
    c->saux = NULL;
    return rc;
}

/* finalise, in plan order, every chromosome whose records are all staged
 * (uploader thread only); 0, or -1 after an abort */
static int finalize_ready(pd_session *s) {
    if (s->finalizing) return 0;
    s->finalizing = 1;
    int rc = 0;
    for (;;) {
        pthread_mutex_lock(&s->mu);
        while (s->next_final < s->n_plan && s->final_applied &&
               (!s->ch[s->next_final].kept || !s->want[s->next_final]))
            s->next_final++;
        const int k = s->next_final;
        const int ok = !s->abort && k < s->n_plan && s->stats_done && s->final_applied &&
                       (s->ch[k].run < 0 || s->ch[k].uploaded);
        pthread_mutex_unlock(&s->mu);
        if (!ok) break;
        const double t0 = now_s();
        const int r = chrom_finalize(s, k);
        s->c_upl_s += now_s() - t0;
        pthread_mutex_lock(&s->mu);
        s->ch[k].rc = r;
        s->ch[k].final = 1;
        pd_trace(s, PD_EV_FINAL, k, 0);
        pthread_cond_broadcast(&s->cv);
        pthread_mutex_unlock(&s->mu);
        if (r) {
            sess_abort(s, 0, "finalising a chromosome failed");
            rc = -1;
            break;
        }
        s->next_final++;
    }
    s->finalizing = 0;
    return rc;
}

static void *uploader_main(void *arg) {
    pd_session *s = (pd_session *)arg;
    int cur_chrom = -1;
    for (int idx = 0; idx <= s->n_pieces; idx++) {
        pthread_mutex_lock(&s->mu);
        const int pend = s->final_pending && !s->final_applied;
        pthread_mutex_unlock(&s->mu);
        if (pend) apply_final(s, idx < s->n_pieces ? idx : s->n_pieces);
        if (finalize_ready(s)) break;
        if (idx == s->n_pieces) {
            if (!s->stats_done) mark_stats_done(s);
            /* the walk parameters may still be on their way */
            pthread_mutex_lock(&s->mu);
            while (!s->abort && s->next_final < s->n_plan && !s->walk_set) pthread_cond_wait(&s->cv, &s->mu);
            while (s->next_final < s->n_plan && s->final_applied &&
                   (!s->ch[s->next_final].kept || !s->want[s->next_final]))
                s->next_final++;
            const int more = !s->abort && s->next_final < s->n_plan;
            pthread_mutex_unlock(&s->mu);
            if (more) { idx--; continue; } /* loop back to finalise */
            break;
        }
        pd_piece *p = &s->pieces[idx];
        if (s->test_soft_abort >= 0 && idx == s->test_soft_abort && idx > 0) { /* test hook: a late contradiction */
            sess_abort(s, 1, "test hook: the index plan is contradicted here (GROM_TEST_SOFT_ABORT)");
            break;
        }
        const double tw = now_s();
        pthread_mutex_lock(&s->mu);
        while (!s->abort && (p->state == 0 || p->state == 1)) {
            if (s->buf_waiters > 0 && s->inflight_head) {
                pthread_mutex_unlock(&s->mu);
                pool_reclaim(s, 1);
                pthread_mutex_lock(&s->mu);
                continue;
            }
            struct timespec ts;
            clock_gettime(CLOCK_REALTIME, &ts);
            ts.tv_nsec += 2000000;
            if (ts.tv_nsec >= 1000000000) { ts.tv_sec++; ts.tv_nsec -= 1000000000; }
            pthread_cond_timedwait(&s->cv, &s->mu, &ts);
            if (s->inflight_head) {
                pthread_mutex_unlock(&s->mu);
                pool_reclaim(s, 0);
                pthread_mutex_lock(&s->mu);
            }
        }
        const int aborted = s->abort;
        pthread_mutex_unlock(&s->mu);
        s->c_wait_s += now_s() - tw;
        if (aborted) break;
        const double t0 = now_s();
        if (p->state == 2) {
            s->c_records += p->n_rec;
            stats_take(s, p);
            piece_free_stats(p);
            if (!s->stats_done && s->s_n >= s->insert_cap) mark_stats_done(s);
        }
        const pd_run *run = &s->runs[p->run];
        if (p->buf && run->chrom < 0) { /* decoded for a chromosome the final plan dropped */
            pool_put_now(s, p->buf);
            p->buf = NULL;
        }
        if (p->buf && p->state == 2) {
            if (run->chrom != cur_chrom) {
                cur_chrom = run->chrom;
                tail_reset(&s->T);
            }
            pd_trace(s, PD_EV_UPLOAD, idx, 0);
            const int urc = upload_piece(s, p);
            pd_trace(s, PD_EV_UPLOAD, idx, 1);
            if (urc) {
                sess_abort(s, 0, grom_last_error());
                break;
            }
            if (s->plan_only || p->buf->ticket < 0) pool_put_now(s, p->buf);
            else pool_put_inflight(s, p->buf);
            p->buf = NULL;
        }
        /* a run's records all decoded: check them against the index's count */
        if (idx == run->first_piece + run->n_pieces - 1) {
            int64_t got = 0;
            int all = 1;
            for (int q = run->first_piece; q <= idx; q++) {
                if (s->pieces[q].state != 2) all = 0;
                got += s->pieces[q].n_rec;
            }
            if (all && run->count >= 0 && got != run->count) {
                char msg[200];
                snprintf(msg, sizeof(msg), "target %d: %lld records decoded, the index counts %lld", run->tid,
                         (long long)got, (long long)run->count);
                sess_abort(s, 1, msg);
                break;
            }
            if (run->chrom >= 0) {
                pthread_mutex_lock(&s->mu);
                s->ch[run->chrom].uploaded = 1;
                pthread_mutex_unlock(&s->mu);
            }
        }
        s->c_upl_s += now_s() - t0;
        pthread_mutex_lock(&s->mu);
        s->head = idx + 1;
        pthread_cond_broadcast(&s->cv);
        pthread_mutex_unlock(&s->mu);
        pool_reclaim(s, 0);
    }
    /* wake everyone: the plan is done (or aborted) */
    pthread_mutex_lock(&s->mu);
    s->stop = 1;
    if (!s->stats_done) s->stats_done = 1;
    pthread_cond_broadcast(&s->cv);
    pthread_mutex_unlock(&s->mu);
    return NULL;
}

/* ---------------- session ---------------- */
/* The serial record stream over the runs (grom_planner_feed's state machine,
 * GROM.c:5740, 11075-11083, 14960-14976): which run each kept plan
 * chromosome consumes, after how many of its records (the two records the
 * previous chromosome's loop reads past its end, Q1); a chromosome whose
 * target has no records left starves every later one (Q21). */
static void plan_runs(const pd_session *s, const int *keep, int *rc, int64_t *rj, int *chr) {
    for (int i = 0; i < s->n_runs; i++) {
        rc[i] = -1;
        rj[i] = 0;
    }
    if (s->fetch_mode) {
        /* -P: each chromosome reads its own target's records through
         * bam_fetch (GROM.c:21051-21064, 304-324): its whole run, nothing
         * consumed by the chromosome before it, nothing starved */
        for (int k = 0; k < s->n_plan; k++) {
            chr[k] = -1;
            if (keep && !keep[k]) continue;
            for (int i = 0; i < s->n_runs && s->plan[k].tid >= 0; i++)
                if (s->runs[i].tid == s->plan[k].tid) {
                    if (rc[i] < 0) {
                        rc[i] = k;
                        chr[k] = i;
                    }
                    break;
                }
        }
        return;
    }
    int cr = 0, stuck = 0;
    int64_t co = 0;
    for (int k = 0; k < s->n_plan; k++) {
        chr[k] = -1;
        if ((keep && !keep[k]) || stuck) continue;
        int R = -1;
        for (int i = 0; i < s->n_runs && s->plan[k].tid >= 0; i++)
            if (s->runs[i].tid == s->plan[k].tid) { R = i; break; }
        if (R < 0 || R < cr || rc[R] >= 0 || (R == cr && s->runs[R].count >= 0 && co >= s->runs[R].count)) {
            stuck = 1;
            continue;
        }
        const int64_t j0 = (R == cr) ? co : 0;
        rc[R] = k;
        rj[R] = j0;
        chr[k] = R;
        /* the foreign record and one more are consumed (Q1) */
        int r = R + 1;
        int64_t off = 0, drop = 2;
        while (drop > 0 && r < s->n_runs) {
            const int64_t cnt = s->runs[r].count >= 0 ? s->runs[r].count : INT64_MAX;
            const int64_t take = drop < cnt - off ? drop : cnt - off;
            off += take;
            drop -= take;
            if (off == cnt) { r++; off = 0; }
        }
        cr = r;
        co = off;
    }
}

/* the final plan (uploader thread, before piece `idx`): runs already being
 * uploaded must keep their assignment, runs a decoder already took must keep
 * whether they are decoded into buffers */
static void apply_final(pd_session *s, int idx) {
    int *rc = (int *)malloc(sizeof(int) * (size_t)(s->n_runs + 1));
    int64_t *rj = (int64_t *)malloc(sizeof(int64_t) * (size_t)(s->n_runs + 1));
    int *chr = (int *)malloc(sizeof(int) * (size_t)(s->n_plan + 1));
    plan_runs(s, s->keep, rc, rj, chr);
    pthread_mutex_lock(&s->mu);
    int bad = 0;
    for (int i = 0; i < s->n_runs && !bad; i++) {
        const pd_run *r = &s->runs[i];
        if (r->first_piece < idx && (rc[i] != r->chrom || rj[i] != r->j0)) bad = 1;
        if (r->first_piece < s->next_piece && ((rc[i] >= 0) != (r->chrom >= 0))) bad = 1;
    }
    for (int k = 0; k < s->n_plan && !bad; k++)
        if (!s->keep[k] && s->ch[k].begun) bad = 1;
    if (!bad) {
        for (int i = 0; i < s->n_runs; i++) {
            pd_run *r = &s->runs[i];
            r->chrom = rc[i];
            r->j0 = rj[i];
            for (int q = r->first_piece; q < r->first_piece + r->n_pieces; q++)
                if (q >= s->next_piece) s->pieces[q].full = rc[i] >= 0 && s->want[rc[i]];
        }
        for (int k = 0; k < s->n_plan; k++) {
            pd_chrom *c = &s->ch[k];
            c->kept = s->keep[k];
            if (!c->begun) {
                c->run = chr[k];
                c->j_left = chr[k] >= 0 ? rj[chr[k]] : 0;
            }
        }
        s->final_applied = 1;
        pthread_cond_broadcast(&s->cv);
    }
    pthread_mutex_unlock(&s->mu);
    free(rc);
    free(rj);
    free(chr);
    if (bad) sess_abort(s, 1, "the final chromosome plan differs where decoding already began");
}

static int read_first_lq(int fd, int64_t fsize, uint64_t voff, int32_t *lq) {
    pd_reader r;
    memset(&r, 0, sizeof(r));
    inf_init(&r.inf);
    int rc = -1;
    if (rd_open(&r, fd, fsize, voff, UINT64_MAX) == 0 && rd_avail(&r, 36) == 1) {
        *lq = ldi32(r.ub + r.ub_pos + 4 + 16);
        rc = 0;
    }
    rd_free(&r);
    return rc;
}

static int cmp_run(const void *a, const void *b) {
    const pd_run *x = (const pd_run *)a, *y = (const pd_run *)b;
    return x->vbeg < y->vbeg ? -1 : x->vbeg > y->vbeg;
}

pd_session *pd_open(const char *bam_path, const bam_hdr *hdr, const pd_chrom_in *plan, int n_plan, int splitread,
                    int read_name_len, int n_threads, char *why, int why_len) {
#define FAIL(...)                                                   \
    do {                                                            \
        if (why) snprintf(why, (size_t)why_len, __VA_ARGS__);       \
        goto fail;                                                  \
    } while (0)
    pd_session *s = (pd_session *)calloc(1, sizeof(pd_session));
    bai_index idx;
    memset(&idx, 0, sizeof(idx));
    int have_idx = 0;
    if (!s) return NULL;
    s->fd = -1;
    {
        char path[4096];
        snprintf(path, sizeof(path), "%s.bai", bam_path);
        if (access(path, R_OK) != 0) {
            size_t L = strlen(bam_path);
            if (L > 4 && strcmp(bam_path + L - 4, ".bam") == 0) snprintf(path, sizeof(path), "%.*s.bai", (int)(L - 4), bam_path);
        }
        if (bai_load(path, &idx) != 0) FAIL("index does not load");
        have_idx = 1;
    }
    if (idx.n_ref != hdr->n_ref) FAIL("index has %d references, BAM header %d", idx.n_ref, hdr->n_ref);
    s->fd = open(bam_path, O_RDONLY);
    if (s->fd < 0) FAIL("cannot open BAM");
    {
        struct stat st;
        if (fstat(s->fd, &st) != 0) FAIL("cannot stat BAM");
        s->file_size = (int64_t)st.st_size;
    }
    /* runs of records per reference from the pseudo-bins */
    s->runs = (pd_run *)calloc((size_t)hdr->n_ref + 1, sizeof(pd_run));
    uint64_t max_end = 0;
    int any_bins = 0;
    for (int t = 0; t < idx.n_ref; t++) {
        const bai_ref *R = &idx.ref[t];
        const bai_bin *meta = NULL;
        int n_real = 0;
        for (int i = 0; i < R->n_bin; i++) {
            if (R->bin[i].bin == 37450u) meta = &R->bin[i];
            else if (R->bin[i].n_chunk > 0) n_real++;
        }
        if (!meta) {
            if (n_real > 0) FAIL("index has no pseudo-bin for target %d", t);
            continue;
        }
        if (meta->n_chunk != 2) FAIL("malformed pseudo-bin for target %d", t);
        any_bins = 1;
        const int64_t cnt = (int64_t)(meta->chunk[1].beg + meta->chunk[1].end);
        if (cnt <= 0) continue;
        pd_run *r = &s->runs[s->n_runs++];
        r->tid = t;
        r->count = cnt;
        r->vbeg = meta->chunk[0].beg;
        r->vend = meta->chunk[0].end;
        r->chrom = -1;
        if (r->vend > max_end) max_end = r->vend;
    }
    if (!any_bins && idx.n_ref > 0) FAIL("index has no pseudo-bins");
    qsort(s->runs, (size_t)s->n_runs, sizeof(pd_run), cmp_run);
    for (int i = 0; i < s->n_runs; i++) {
        if (i > 0 && (s->runs[i].tid <= s->runs[i - 1].tid || s->runs[i].vbeg < s->runs[i - 1].vend))
            FAIL("index runs are not in target order");
        if (s->runs[i].vend <= s->runs[i].vbeg) FAIL("empty run in the index");
    }
    /* unplaced reads after the placed ones (their count when the index has it) */
    if (!(idx.has_no_coor && idx.n_no_coor == 0)) {
        pd_run *r = &s->runs[s->n_runs];
        r->tid = -1;
        r->count = idx.has_no_coor ? (int64_t)idx.n_no_coor : -1;
        if (max_end == 0) {
            bgzf_reader br;
            bam_hdr h2;
            if (bgzf_open_read(&br, bam_path) != 0 || bam_read_header(&br, &h2) != 0) FAIL("cannot read header");
            max_end = (uint64_t)bgzf_tell(&br);
            bam_free_header(&h2);
            bgzf_close_read(&br);
        }
        r->vbeg = max_end;
        r->vend = UINT64_MAX;
        r->chrom = -1;
        s->n_runs++;
    }
    /* the record after each run (the one that ends a chromosome's stream) */
    for (int i = 0; i + 1 < s->n_runs; i++) {
        s->runs[i].has_next = 1;
        if (read_first_lq(s->fd, s->file_size, s->runs[i + 1].vbeg, &s->runs[i].next_lq) != 0) {
            if (s->runs[i + 1].tid < 0 && s->runs[i + 1].count < 0) s->runs[i].has_next = 0; /* no unplaced reads */
            else FAIL("cannot read the record after target %d", s->runs[i].tid);
        }
    }
    s->n_plan = n_plan;
    s->plan = (pd_chrom_in *)calloc((size_t)(n_plan > 0 ? n_plan : 1), sizeof(pd_chrom_in));
    s->ch = (pd_chrom *)calloc((size_t)(n_plan > 0 ? n_plan : 1), sizeof(pd_chrom));
    s->keep = (int *)calloc((size_t)(n_plan > 0 ? n_plan : 1), sizeof(int));
    s->want = (int *)calloc((size_t)(n_plan > 0 ? n_plan : 1), sizeof(int));
    for (int k = 0; k < n_plan; k++) s->want[k] = 1;
    memcpy(s->plan, plan, sizeof(pd_chrom_in) * (size_t)n_plan);
    {
        int *rc = (int *)malloc(sizeof(int) * (size_t)(s->n_runs + 1));
        int64_t *rj = (int64_t *)malloc(sizeof(int64_t) * (size_t)(s->n_runs + 1));
        int *chr = (int *)malloc(sizeof(int) * (size_t)(n_plan + 1));
        plan_runs(s, NULL, rc, rj, chr);
        for (int i = 0; i < s->n_runs; i++) {
            s->runs[i].chrom = rc[i];
            s->runs[i].j0 = rj[i];
        }
        for (int k = 0; k < n_plan; k++) {
            pd_chrom *c = &s->ch[k];
            grom_batch_init(&c->mirror, plan[k].tid, read_name_len);
            c->run = chr[k];
            c->j_left = chr[k] >= 0 ? rj[chr[k]] : 0;
            c->kept = 1;
            s->keep[k] = 1;
        }
        free(rc);
        free(rj);
        free(chr);
    }
    /* pieces: each run cut at linear-index offsets into ~PD_PIECE_RECS records */
    {
        int cap = 1024;
        s->pieces = (pd_piece *)calloc((size_t)cap, sizeof(pd_piece));
        for (int i = 0; i < s->n_runs; i++) {
            pd_run *r = &s->runs[i];
            r->first_piece = s->n_pieces;
            uint64_t cut[4096 + 2];
            int nc = 0;
            cut[nc++] = r->vbeg;
            if (r->tid >= 0) {
                const bai_ref *R = &idx.ref[r->tid];
                const int64_t nw = R->n_intv > 0 ? R->n_intv : 1;
                const double per_w = (double)r->count / (double)nw;
                const char *pr = getenv("GROM_PIECE_RECS"); /* test hook: smaller pieces, more borders */
                const double target = pr && atof(pr) > 0 ? atof(pr) : (double)PD_PIECE_RECS;
                int64_t wpp = per_w > 0 ? (int64_t)(target / per_w) : nw;
                if (wpp < 1) wpp = 1;
                while (nw / wpp > 4096) wpp *= 2;
                for (int64_t w = wpp; w < R->n_intv; w += wpp) {
                    const uint64_t v = R->ioff[w];
                    if (v > cut[nc - 1] && v < r->vend) cut[nc++] = v;
                }
            }
            cut[nc] = r->vend;
            for (int j = 0; j < nc; j++) {
                if (s->n_pieces == cap) {
                    cap *= 2;
                    s->pieces = (pd_piece *)realloc(s->pieces, sizeof(pd_piece) * (size_t)cap);
                    memset(s->pieces + cap / 2, 0, sizeof(pd_piece) * (size_t)(cap / 2));
                }
                pd_piece *p = &s->pieces[s->n_pieces++];
                p->run = i;
                p->vbeg = cut[j];
                p->vend = cut[j + 1];
                p->full = r->chrom >= 0;
            }
            r->n_pieces = s->n_pieces - r->first_piece;
        }
    }
    /* device mode cuts runs at the linear index's record starts: keep it */
    s->n_tgt = idx.n_ref;
    s->lin = (uint64_t **)calloc((size_t)(idx.n_ref > 0 ? idx.n_ref : 1), sizeof(uint64_t *));
    s->n_lin = (int *)calloc((size_t)(idx.n_ref > 0 ? idx.n_ref : 1), sizeof(int));
    for (int t = 0; t < idx.n_ref; t++) {
        const bai_ref *R = &idx.ref[t];
        if (R->n_intv > 0) {
            s->lin[t] = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)R->n_intv);
            if (s->lin[t]) {
                memcpy(s->lin[t], R->ioff, sizeof(uint64_t) * (size_t)R->n_intv);
                s->n_lin[t] = R->n_intv;
            }
        }
    }
    bai_free(&idx);
    have_idx = 0;
    s->splitread = splitread;
    s->read_name_len = read_name_len;
    s->n_threads = n_threads < 1 ? 1 : n_threads;
    s->window = 2 * s->n_threads + 4;
    s->max_bufs = s->window + s->n_threads / 2 + 8;
    s->insert_cap = PD_INSERT_CAP;
    if (getenv("GROM_TEST_INSERT_CAP") && atoll(getenv("GROM_TEST_INSERT_CAP")) > 0)
        s->insert_cap = atoll(getenv("GROM_TEST_INSERT_CAP"));
    if (getenv("GROM_TEST_PREFIX_RECORDS")) s->prefix_records = atoll(getenv("GROM_TEST_PREFIX_RECORDS"));
    s->s_ins = (int32_t *)malloc(sizeof(int32_t) * (size_t)s->insert_cap);
    s->s_lq = (int32_t *)malloc(sizeof(int32_t) * (size_t)s->insert_cap);
    if (!s->s_ins || !s->s_lq) FAIL("out of memory");
    pthread_mutex_init(&s->mu, NULL);
    pthread_cond_init(&s->cv, NULL);
    s->t0 = now_s();
    if (getenv("GROM_TRACE")) {
        s->trace_path = strdup(getenv("GROM_TRACE"));
        s->tr_cap = 8 * (int64_t)s->n_pieces + 16 * (int64_t)n_plan + 4096;
        s->tr = calloc((size_t)s->tr_cap, sizeof(*s->tr));
    }
    return s;
fail:
    if (have_idx) bai_free(&idx);
    if (s->fd >= 0) close(s->fd);
    if (s->ch)
        for (int k = 0; k < n_plan; k++) grom_batch_free(&s->ch[k].mirror);
    free(s->ch);
    free(s->plan);
    free(s->keep);
    free(s->want);
    free(s->runs);
    free(s->pieces);
    free(s->s_ins);
    free(s->s_lq);
    free(s);
    return NULL;
#undef FAIL
}

void pd_set_device_mode(pd_session *s, int on) { s->dev_mode = on; }

void pd_set_fetch_mode(pd_session *s, int on) {
    s->fetch_mode = on != 0;
    /* the initial plan again (pd_open made the serial stream's) */
    int *rc = (int *)malloc(sizeof(int) * (size_t)(s->n_runs + 1));
    int64_t *rj = (int64_t *)malloc(sizeof(int64_t) * (size_t)(s->n_runs + 1));
    int *chr = (int *)malloc(sizeof(int) * (size_t)(s->n_plan + 1));
    plan_runs(s, NULL, rc, rj, chr);
    for (int i = 0; i < s->n_runs; i++) {
        s->runs[i].chrom = rc[i];
        s->runs[i].j0 = rj[i];
    }
    for (int k = 0; k < s->n_plan; k++) {
        s->ch[k].run = chr[k];
        s->ch[k].j_left = chr[k] >= 0 ? rj[chr[k]] : 0;
    }
    for (int i = 0; i < s->n_runs; i++) {
        const pd_run *r = &s->runs[i];
        for (int q = r->first_piece; q < r->first_piece + r->n_pieces; q++)
            s->pieces[q].full = r->chrom >= 0 && s->want[r->chrom];
    }
    free(rc);
    free(rj);
    free(chr);
}
int pd_device_mode(const pd_session *s) { return s->dev_mode; }

void pd_set_wanted(pd_session *s, const int *want) {
    for (int k = 0; k < s->n_plan; k++) s->want[k] = want ? (want[k] != 0) : 1;
    for (int i = 0; i < s->n_runs; i++) {
        const pd_run *r = &s->runs[i];
        for (int q = r->first_piece; q < r->first_piece + r->n_pieces; q++)
            s->pieces[q].full = r->chrom >= 0 && s->want[r->chrom];
    }
}

/* ================= device mode: whole runs decoded on the GPUs ================= */
/* A worker's compressed runs are read one ahead by its prefetch thread: the
 * run's bytes by pread into a pinned slot, its block table and record starts
 * on the host, and the copy to the device slot of the same number started on
 * the decode context's copy stream -- all while the GPU decodes the run
 * before it.  The worker takes a slot, decodes the run piece by piece
 * (dd_run_decode) and releases it; a run nobody takes is simply read again
 * when needed. */
/* PF_HELD: read, and promised to the worker's next dw_decode (its first piece
 * is already loading on the device, dd_run_req.next_cb) */
enum { PF_FREE = 0, PF_WANTED = 1, PF_READY = 2, PF_USED = 3, PF_HELD = 4 };
typedef struct {
    int ri, state, rc;
    char err[200];
    int64_t len;             /* the compressed run's bytes (copied to the device slot of the same number) */
    DdBlock *blk;
    int64_t blk_cap, nb, ub;
    int64_t *starts;
    int64_t starts_cap, m, u_end;
    double t_io;
} pf_slot;

typedef struct {
    pd_session *s;
    int device, first;       /* first: this worker also gathers the insert statistics */
    int sub, nsub;           /* this device's chromosomes taken in turn by nsub workers */
    dd_ctx *dd;
    pf_slot slot[2];
    pthread_mutex_t mu;
    pthread_cond_t cv;
    pthread_t pf_thr;
    int pf_started, pf_stop;
    uint8_t *ring[2];        /* pinned read ring of the prefetch thread (PF_CHUNK bytes each) */
    int test_abort, n_done;  /* GROM_TEST_DD_ABORT=n: -2 at the n-th chromosome (tests) */
} dd_worker;

#define PF_CHUNK ((int64_t)128 << 20)

typedef struct {
    int fd;
    uint8_t *buf;
    int64_t len, off;
    int ok;
} pread_part;

static void *pread_main(void *arg) {
    pread_part *p = (pread_part *)arg;
    int64_t got = 0;
    while (got < p->len) {
        const ssize_t k = pread(p->fd, p->buf + got, (size_t)(p->len - got), (off_t)(p->off + got));
        if (k <= 0) break;
        got += k;
    }
    p->ok = got == p->len;
    return NULL;
}

/* read [off, off+len) on up to nt threads */
static int pread_par(int fd, uint8_t *buf, int64_t len, int64_t off, int nt) {
    if (nt < 1) nt = 1;
    if (len < ((int64_t)8 << 20)) nt = 1;
    pread_part parts[32];
    pthread_t th[32];
    if (nt > 32) nt = 32;
    const int64_t step = (len + nt - 1) / nt;
    int started = 0;
    for (int t = 0; t < nt; t++) {
        const int64_t a = t * step, b = a + step < len ? a + step : len;
        parts[t].fd = fd;
        parts[t].buf = buf + a;
        parts[t].len = b > a ? b - a : 0;
        parts[t].off = off + a;
        parts[t].ok = 0;
        if (t == nt - 1 || pthread_create(&th[t], NULL, pread_main, &parts[t]) != 0) pread_main(&parts[t]);
        else started |= 1 << t;
    }
    int ok = 1;
    for (int t = 0; t < nt; t++) {
        if (started & (1 << t)) pthread_join(th[t], NULL);
        ok &= parts[t].ok;
    }
    return ok ? 0 : -1;
}

static int cmp_i64(const void *a, const void *b) {
    const int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
    return x < y ? -1 : x > y;
}

/* a run's compressed bytes into a pinned slot, its block table and record
 * starts, and the slot's copy to the device started (prefetch thread) */
static int pf_read(dd_worker *w, pf_slot *sl, int slot_no, int ri, char *err, int errlen) {
    pd_session *s = w->s;
    const pd_run *r = &s->runs[ri];
    const uint64_t vend = r->vend;
    const int64_t c0 = (int64_t)(r->vbeg >> 16);
    int64_t c1;
    if (vend == UINT64_MAX) {
        c1 = s->file_size;
    } else {
        c1 = (int64_t)(vend >> 16);
        if ((vend & 0xffff) != 0) { /* the block holding the end is part of the range */
            uint8_t h[18];
            if (pread(s->fd, h, 18, (off_t)c1) != 18) { snprintf(err, (size_t)errlen, "cannot read a block header"); return -2; }
            const int xlen = h[10] | (h[11] << 8);
            if (xlen < 6 || h[12] != 'B' || h[13] != 'C') { snprintf(err, (size_t)errlen, "not a BGZF block at %lld", (long long)c1); return -2; }
            c1 += (int64_t)(h[16] | (h[17] << 8)) + 1;
        }
    }
    const int64_t len = c1 - c0;
    if (len <= 0 || c1 > s->file_size) { snprintf(err, (size_t)errlen, "bad run range"); return -2; }
    /* the compressed run in chunks of whole blocks through a ring of two
     * pinned buffers (PF_CHUNK each: pinning a whole 1.6 GB run per process
     * cost ~0.4 s and held up the device allocations made meanwhile), each
     * copied to the device slot while the next is read; the block table is
     * built chunk by chunk */
    for (int k = 0; k < 2; k++)
        if (!w->ring[k]) {
            w->ring[k] = (uint8_t *)grom_pinned_alloc(PF_CHUNK);
            if (!w->ring[k]) { snprintf(err, (size_t)errlen, "no pinned memory for the read ring"); return -1; }
        }
    if (dd_comp_begin(w->dd, slot_no, len, err, errlen)) return -1;
    const double t0 = now_s();
    int64_t off = 0, ub = 0, nb = 0;
    for (int ring = 0; off < len; ring ^= 1) {
        const int64_t want = len - off < PF_CHUNK ? len - off : PF_CHUNK;
        if (dd_comp_ring_wait(w->dd, ring)) { snprintf(err, (size_t)errlen, "device copy failed"); return -1; }
        if (pread_par(s->fd, w->ring[ring], want, c0 + off, s->io_threads)) {
            snprintf(err, (size_t)errlen, "reading the BAM failed");
            return -1;
        }
        int64_t used = 0, cb = 0;
        const int64_t n = dd_block_table_prefix(w->ring[ring], want, NULL, 0, &cb, &used);
        if (n <= 0 || (off + want == len && used != want)) {
            snprintf(err, (size_t)errlen, "the run is not whole BGZF blocks");
            return -2;
        }
        if (nb + n > sl->blk_cap) {
            sl->blk_cap = (nb + n) + (nb + n) / 2 + 16;
            DdBlock *nbk = (DdBlock *)realloc(sl->blk, sizeof(DdBlock) * (size_t)sl->blk_cap);
            if (!nbk) { sl->blk_cap = 0; return -1; }
            sl->blk = nbk;
        }
        dd_block_table_prefix(w->ring[ring], used, sl->blk + nb, n, &cb, NULL);
        for (int64_t k = nb; k < nb + n; k++) { /* offsets in the whole run */
            sl->blk[k].in_off += off;
            sl->blk[k].c_off += off;
            sl->blk[k].out_off += ub;
        }
        if (dd_comp_chunk(w->dd, slot_no, ring, w->ring[ring], off, used, err, errlen)) return -1;
        nb += n;
        ub += cb;
        off += used;
    }
    sl->t_io = now_s() - t0;
    /* record starts: the run's first record, then every linear-index offset inside the run */
    const int64_t u0 = (int64_t)(r->vbeg & 0xffff);
    int64_t u_end = ub;
    if (vend != UINT64_MAX && (vend & 0xffff) != 0) u_end = sl->blk[nb - 1].out_off + (int64_t)(vend & 0xffff);
    const int nl = (r->tid >= 0 && r->tid < s->n_tgt) ? s->n_lin[r->tid] : 0;
    if (nl + 2 > sl->starts_cap) {
        free(sl->starts);
        sl->starts_cap = nl + 64;
        sl->starts = (int64_t *)malloc(sizeof(int64_t) * (size_t)sl->starts_cap);
        if (!sl->starts) { sl->starts_cap = 0; return -1; }
    }
    int64_t ns = 0;
    sl->starts[ns++] = u0;
    for (int k = 0; k < nl; k++) {
        const uint64_t v = s->lin[r->tid][k];
        if (v < r->vbeg || v >= vend) continue;
        const int64_t cb = (int64_t)(v >> 16) - c0;
        int64_t lo = 0, hi = nb - 1; /* the block starting at cb */
        while (lo < hi) {
            const int64_t mid = (lo + hi + 1) / 2;
            if (sl->blk[mid].c_off <= cb) lo = mid;
            else hi = mid - 1;
        }
        if (sl->blk[lo].c_off != cb) continue;
        const int64_t u = sl->blk[lo].out_off + (int64_t)(v & 0xffff);
        if (u > u0 && u < u_end) sl->starts[ns++] = u;
    }
    qsort(sl->starts, (size_t)ns, sizeof(int64_t), cmp_i64);
    int64_t m = 0;
    for (int64_t k = 0; k < ns; k++)
        if (m == 0 || sl->starts[k] != sl->starts[m - 1]) sl->starts[m++] = sl->starts[k];
    sl->starts[m] = u_end; /* (dd_run_req: the run's end after its starts) */
    sl->len = len;
    sl->nb = nb;
    sl->ub = ub;
    sl->m = m;
    sl->u_end = u_end;
    return dd_comp_end(w->dd, slot_no, len, err, errlen) ? -1 : 0;
}

static void *pf_main(void *arg) {
    dd_worker *w = (dd_worker *)arg;
    pthread_mutex_lock(&w->mu);
    for (;;) {
        int q = -1;
        for (int k = 0; k < 2 && q < 0; k++)
            if (w->slot[k].state == PF_WANTED) q = k;
        if (q < 0) {
            if (w->pf_stop) break;
            pthread_cond_wait(&w->cv, &w->mu);
            continue;
        }
        pf_slot *sl = &w->slot[q];
        const int ri = sl->ri;
        pthread_mutex_unlock(&w->mu);
        char err[200] = "";
        pd_trace(w->s, PD_EV_PHASE, 101, 0);
        const int rc = pf_read(w, sl, q, ri, err, (int)sizeof(err));
        pd_trace(w->s, PD_EV_PHASE, 101, 1);
        pthread_mutex_lock(&w->mu);
        sl->rc = rc;
        snprintf(sl->err, sizeof(sl->err), "%s", err);
        sl->state = PF_READY;
        pthread_cond_broadcast(&w->cv);
    }
    pthread_mutex_unlock(&w->mu);
    return NULL;
}

/* ask for run ri to be read ahead (no-op when it is already asked for or no
 * slot is free) */
static void pf_want(dd_worker *w, int ri) {
    if (ri < 0) return;
    pthread_mutex_lock(&w->mu);
    int have = 0, q = -1;
    for (int k = 0; k < 2; k++) {
        if (w->slot[k].ri == ri && w->slot[k].state != PF_FREE) have = 1;
        if (q < 0 && (w->slot[k].state == PF_FREE || w->slot[k].state == PF_READY)) q = k;
    }
    if (!have && q >= 0) {
        w->slot[q].ri = ri;
        w->slot[q].state = PF_WANTED;
        pthread_cond_broadcast(&w->cv);
    }
    pthread_mutex_unlock(&w->mu);
}

/* the slot holding run ri, read (waits); NULL with err set on failure */
static pf_slot *pf_take(dd_worker *w, int ri, int *slot_no, int *rc, char *err, int errlen) {
    pthread_mutex_lock(&w->mu);
    int q = -1;
    for (;;) {
        q = -1;
        for (int k = 0; k < 2; k++)
            if (w->slot[k].ri == ri &&
                (w->slot[k].state == PF_WANTED || w->slot[k].state == PF_READY || w->slot[k].state == PF_HELD))
                q = k;
        if (q >= 0) break;
        for (int k = 0; k < 2 && q < 0; k++)
            if (w->slot[k].state == PF_FREE || w->slot[k].state == PF_READY) q = k;
        if (q >= 0) {
            w->slot[q].ri = ri;
            w->slot[q].state = PF_WANTED;
            pthread_cond_broadcast(&w->cv);
            break;
        }
        pthread_cond_wait(&w->cv, &w->mu); /* both slots busy: wait for a release */
    }
    while (w->slot[q].state == PF_WANTED) pthread_cond_wait(&w->cv, &w->mu);
    pf_slot *sl = &w->slot[q];
    sl->state = PF_USED;
    *rc = sl->rc;
    if (sl->rc) snprintf(err, (size_t)errlen, "%s", sl->err);
    pthread_mutex_unlock(&w->mu);
    *slot_no = q;
    return sl;
}

static void pf_release(dd_worker *w, pf_slot *sl) {
    pthread_mutex_lock(&w->mu);
    sl->state = PF_FREE;
    sl->ri = -1;
    pthread_cond_broadcast(&w->cv);
    pthread_mutex_unlock(&w->mu);
}

/* dd_run_decode's next_cb: run `next` of this worker, if its slot is read
 * (without waiting), held for the worker's next dw_decode */
typedef struct {
    dd_worker *w;
    int next;
} dw_next_arg;

static int dw_next_cb(void *arg, dd_run_req *nq) {
    const dw_next_arg *a = (const dw_next_arg *)arg;
    dd_worker *w = a->w;
    if (a->next < 0) return 0;
    int got = 0;
    pthread_mutex_lock(&w->mu);
    for (int k = 0; k < 2 && !got; k++) {
        pf_slot *sl = &w->slot[k];
        if (sl->ri != a->next || sl->state != PF_READY || sl->rc != 0) continue;
        const pd_run *r = &w->s->runs[a->next];
        sl->state = PF_HELD;
        nq->slot = k;
        nq->comp_len = sl->len;
        nq->blk = sl->blk;
        nq->nblk = sl->nb;
        nq->starts = sl->starts;
        nq->n_starts = sl->m;
        nq->u_end = sl->u_end;
        nq->tid = r->tid;
        nq->count = r->count;
        got = 1;
    }
    pthread_mutex_unlock(&w->mu);
    return got;
}

/* the statistics' progress (dd_run_decode's callback, the first worker):
 * find_insert_mean's sample grows by `taken` pairs; complete: the cap */
static void dw_stats_cb(void *arg, int64_t taken, int64_t m, int complete) {
    pd_session *s = (pd_session *)arg;
    pthread_mutex_lock(&s->mu);
    s->s_n += taken;
    s->s_m += m;
    pthread_mutex_unlock(&s->mu);
    if (complete) mark_stats_done(s);
}

/* run ri decoded on the device from the prefetcher's compressed bytes (then
 * `next`, the run this worker needs after it, -1 none, is asked for): parsed
 * into `stage` (NULL: the insert statistics only), the statistics' sample
 * taken from it while `stats` and the cap is not reached */
static int dw_decode(dd_worker *w, int ri, int next, grom_stage *stage, int64_t j0, int64_t ref_len, int stats,
                     dd_parse_out *po, int64_t *n_rec, char *err, int errlen) {
    pd_session *s = w->s;
    const pd_run *r = &s->runs[ri];
    int q = 0, rc = 0;
    const double tw = now_s();
    pf_slot *sl = pf_take(w, ri, &q, &rc, err, errlen);
    const double t1 = now_s();
    if (rc) { pf_release(w, sl); return rc; }
    pf_want(w, next);
    dd_run_req rq;
    memset(&rq, 0, sizeof(rq));
    rq.slot = q;
    rq.comp_len = sl->len;
    rq.blk = sl->blk;
    rq.nblk = sl->nb;
    rq.starts = sl->starts;
    rq.n_starts = sl->m;
    rq.u_end = sl->u_end;
    rq.tid = r->tid;
    rq.j0 = j0;
    rq.read_name_len = s->read_name_len;
    rq.ref_len = ref_len;
    rq.count = r->count;
    rq.stage = stage;
    if (stats && !s->stats_done) {
        rq.stats_left = s->insert_cap - s->s_n;
        rq.min_mapq = s->min_mapq_stats;
        rq.h_ins = s->s_ins + s->s_n;
        rq.h_lq = s->s_lq + s->s_n;
        rq.stats_cb = dw_stats_cb;
        rq.stats_arg = s;
    }
    dw_next_arg na = {w, next};
    /* the next run's first piece loads while this one finishes (not in the
     * statistics-only pass: the run after it is not necessarily the next
     * one this worker decodes, and a held slot reads nothing ahead) */
    if (stage && !getenv("GROM_DD_NO_AHEAD")) {
        rq.next_cb = dw_next_cb;
        rq.next_arg = &na;
    }
    int64_t R = 0;
    pd_trace(s, PD_EV_PHASE, 102, 0);
    rc = dd_run_decode(w->dd, &rq, po, &R, err, errlen);
    pd_trace(s, PD_EV_PHASE, 102, 1);
    const double tdec = now_s() - t1;
    const int64_t len = sl->len, ub = sl->ub;
    const double tio = sl->t_io;
    pf_release(w, sl);
    if (rc) return rc;
    if (stage && r->count >= 0 && R != r->count) {
        snprintf(err, (size_t)errlen, "target %d: %lld records decoded, the index counts %lld", r->tid, (long long)R,
                 (long long)r->count);
        return -2;
    }
    pthread_mutex_lock(&s->mu);
    s->c_records += stage ? R : 0;
    s->c_inflated += ub;
    s->c_compressed += len;
    s->c_io_s += tio;
    s->c_wait_s += t1 - tw;
    s->c_dec_s += tdec;
    pthread_mutex_unlock(&s->mu);
    *n_rec = R;
    return 0;
}

static int next_placed_run(const pd_session *s, int ri);

/* Stages reserved ahead: the first chromosomes' stages would otherwise be
 * allocated (hipMalloc of ~15 GB each at 30x) on the decode's critical path.
 * The decode hands chromosomes out longest first and a stage's later
 * chromosomes are never larger than its first, so stage i is sized for the
 * i-th largest run of this device: its record count from the index, bases and
 * CIGAR words per record from the first 2,000 records of the file, and that
 * chromosome's reference. */
typedef struct {
    pd_session *s;
    int device;
} stres_job;

static void *stres_body(stres_job *j);

static void *stres_main(void *arg) {
    stres_job *j = (stres_job *)arg;
    pd_trace(j->s, PD_EV_PHASE, 105, 0);
    void *r = stres_body(j);
    pd_trace(j->s, PD_EV_PHASE, 105, 1);
    return r;
}

static void *stres_body(stres_job *j) {
    pd_session *s = j->s;
    /* this device's wanted chromosomes by record count, largest first */
    int64_t recs[64], refl[64];
    int nw = 0;
    for (int k = 0; k < s->n_plan; k++) {
        if (s->ch[k].device != j->device || !s->want[k] || s->ch[k].run < 0) continue;
        const int64_t c = s->runs[s->ch[k].run].count;
        if (c <= 0) continue;
        /* insertion into the top 64 (more stages than that are never made) */
        int at = nw;
        if (nw == 64) {
            if (recs[63] >= c) continue;
            at = 63;
        } else {
            nw++;
        }
        for (; at > 0 && recs[at - 1] < c; at--) {
            recs[at] = recs[at - 1];
            refl[at] = refl[at - 1];
        }
        recs[at] = c;
        refl[at] = s->plan[k].len;
    }
    int64_t ref_max = 0;
    for (int k = 0; k < s->n_plan; k++)
        if (s->ch[k].device == j->device && s->want[k] && s->plan[k].len > ref_max) ref_max = s->plan[k].len;
    const int r0 = next_placed_run(s, -1);
    if (nw == 0 || r0 < 0) return NULL;
    pd_reader r;
    memset(&r, 0, sizeof(r));
    inf_init(&r.inf);
    int64_t n = 0, lq = 0, nc = 0;
    if (rd_open(&r, s->fd, s->file_size, s->runs[r0].vbeg, UINT64_MAX) == 0) {
        while (n < 2000 && rd_avail(&r, 4) == 1) {
            const int32_t bs = ldi32(r.ub + r.ub_pos);
            if (bs < 32 || rd_avail(&r, 4 + (int64_t)bs) != 1) break;
            const uint8_t *q = r.ub + r.ub_pos + 4;
            lq += ldi32(q + 16) > 0 ? ldi32(q + 16) : 0;
            nc += ld16(q + 12);
            n++;
            r.ub_pos += 4 + (int64_t)bs;
        }
    }
    rd_free(&r);
    if (n == 0) return NULL;
    pthread_mutex_lock(&s->mu);
    int ns = s->n_stage;
    grom_stage *mine[64];
    int mi[64], m = 0;
    /* the stages being reserved are busy (owner -2) until their blocks exist:
     * a worker's stage_acquire waits for them (a second worker on
     * the device could otherwise fill a stage this thread is growing) */
    for (int i = 0; i < ns && m < 64; i++)
        if (s->stage_dev[i] == j->device && !s->stage_busy[i]) {
            s->stage_busy[i] = 1;
            s->stage_owner[i] = -2;
            mi[m] = i;
            mine[m++] = s->stages[i];
        }
    pthread_mutex_unlock(&s->mu);
    for (int i = 0; i < m; i++) {
        const int64_t rc = recs[i < nw ? i : nw - 1];
        grom_stage_sizes est;
        memset(&est, 0, sizeof(est));
        est.n = rc;
        est.n_drop = rc / 4 + 1024;
        est.n_bases = (int64_t)((double)rc * ((double)lq / (double)n + 1.0) * 1.05);
        est.n_cigar_ops = (int64_t)((double)rc * (double)nc / (double)n * 1.1) + 1024;
        est.n_aux = rc / 16 + 1024;
        /* the reference: this chromosome's, at least the largest's share that
         * a later, shorter run with a longer sequence would need */
        est.ref_len = refl[i < nw ? i : nw - 1] > ref_max / 2 ? refl[i < nw ? i : nw - 1] : ref_max / 2;
        (void)grom_stage_begin(mine[i], &est);
    }
    pthread_mutex_lock(&s->mu);
    for (int i = 0; i < m; i++) {
        s->stage_busy[mi[i]] = 0;
        s->stage_owner[mi[i]] = -1;
    }
    pthread_cond_broadcast(&s->cv);
    pthread_mutex_unlock(&s->mu);
    return NULL;
}

/* The decode buffers sized once, while the first run is read: the largest
 * record count the index gives for a run this worker may load, and its
 * largest compressed span times the inflate ratio of the BAM's first blocks
 * (+4%): the piece slots and the chromosome-wide name arrays (dd_reserve).
 * A run beyond the estimate still grows the buffers. */
static int dw_reserve(dd_worker *w, char *err, int errlen) {
    pd_session *s = w->s;
    int64_t recs = 0, span = 0;
    for (int i = 0; i < s->n_runs; i++) {
        const pd_run *r = &s->runs[i];
        if (r->tid < 0) continue;
        if (r->count > recs) recs = r->count;
        const int64_t c1 = r->vend == UINT64_MAX ? s->file_size : (int64_t)(r->vend >> 16) + 65536;
        const int64_t sp = c1 - (int64_t)(r->vbeg >> 16);
        if (sp > span) span = sp;
    }
    if (recs == 0 || span == 0) return 0;
    /* the inflate ratio of up to 1 MB of whole blocks from the first run's start */
    const int r0 = next_placed_run(s, -1);
    if (r0 < 0) return 0;
    const int64_t c0 = (int64_t)(s->runs[r0].vbeg >> 16);
    int64_t n = s->file_size - c0 < ((int64_t)1 << 20) ? s->file_size - c0 : ((int64_t)1 << 20);
    uint8_t *b = (uint8_t *)malloc((size_t)n);
    if (!b) return 0;
    int64_t got = pread(s->fd, b, (size_t)n, (off_t)c0), csum = 0, usum = 0;
    for (int64_t o = 0; got > 0 && o + 18 <= got;) {
        const uint8_t *h = b + o;
        if (h[0] != 0x1f || h[1] != 0x8b || h[12] != 'B' || h[13] != 'C') break;
        const int64_t bl = (int64_t)(h[16] | (h[17] << 8)) + 1;
        if (o + bl > got) break;
        csum += bl;
        usum += (int64_t)((uint32_t)b[o + bl - 4] | (uint32_t)b[o + bl - 3] << 8 | (uint32_t)b[o + bl - 2] << 16 |
                          (uint32_t)b[o + bl - 1] << 24);
        o += bl;
    }
    free(b);
    if (csum <= 0 || usum <= 0) return 0;
    const int64_t ub = (int64_t)((double)span * (double)usum / (double)csum * 1.04);
    int64_t nst = 0;
    for (int t = 0; t < s->n_tgt; t++)
        if (s->n_lin[t] > nst) nst = s->n_lin[t];
    return dd_reserve(w->dd, span, ub, recs + recs / 20, nst + 2, err, errlen);
}

/* the next run (tid >= 0) after ri in file order, -1 none */
static int next_placed_run(const pd_session *s, int ri) {
    for (int i = ri + 1; i < s->n_runs; i++)
        if (s->runs[i].tid >= 0) return i;
    return -1;
}

/* find_insert_mean's sample from the runs in file order, from run `from`,
 * until the cap (the first worker, when the statistics' runs are not among
 * the ones it parses): pieces of each run, the statistics only */
static int dw_stats_only(dd_worker *w, int from, char *err, int errlen) {
    pd_session *s = w->s;
    for (int i = from; i >= 0 && i < s->n_runs && !s->stats_done && !s->abort; i = next_placed_run(s, i)) {
        dd_parse_out po;
        int64_t R = 0;
        pd_trace(s, PD_EV_PHASE, 103, i);
        const int rc = dw_decode(w, i, next_placed_run(s, i), NULL, 0, 0, 1, &po, &R, err, errlen);
        if (rc) return rc;
        pthread_mutex_lock(&s->mu);
        s->c_stats_only++;
        pthread_mutex_unlock(&s->mu);
    }
    if (!s->stats_done) mark_stats_done(s);
    return 0;
}

static void dw_final(pd_session *s);

/* one processed chromosome: its run parsed into a stage, the split-read
 * alignments parsed on the host, the walk's trims (chrom_finalize's facts) */
static int dw_chrom(dd_worker *w, int k, int next_run, int stats, char *err, int errlen) {
    pd_session *s = w->s;
    pd_chrom *c = &s->ch[k];
    /* test hook: the plan contradicted at this worker's n-th chromosome */
    if (w->test_abort >= 0 && w->n_done++ == w->test_abort) {
        snprintf(err, (size_t)errlen, "test: the device decode plan contradicted (GROM_TEST_DD_ABORT)");
        return -2;
    }
    if (stage_acquire(s, w->device, k, &c->stage)) { snprintf(err, (size_t)errlen, "no stage"); return -1; }
    const int ri = c->run;
    dd_parse_out po;
    memset(&po, 0, sizeof(po));
    int64_t j0 = 0;
    if (ri >= 0) {
        j0 = s->runs[ri].j0;
        int64_t R = 0;
        int rc = dw_decode(w, ri, next_run, c->stage, j0, s->plan[k].len, stats, &po, &R, err, errlen);
        if (rc) return rc;
        /* the cap not reached in this run: the runs after it in file order */
        if (stats && !s->stats_done && (rc = dw_stats_only(w, next_placed_run(s, ri), err, errlen))) return rc;
    } else {
        grom_stage_sizes sz;
        grom_reads dv;
        memset(&sz, 0, sizeof(sz));
        sz.ref_len = s->plan[k].len;
        if (grom_stage_fill_begin(c->stage, &sz, &dv) != GROM_OK) { snprintf(err, (size_t)errlen, "%s", grom_last_error()); return -1; }
    }
    /* the split-read alignments, parsed as decode_piece parses them */
    const char *target = s->plan[k].target_name ? s->plan[k].target_name : "";
    grom_aux *ax = NULL;
    int64_t *ak = NULL, na = 0;
    if (po.n_auxc > 0) {
        ax = (grom_aux *)malloc(sizeof(grom_aux) * (size_t)po.n_auxc);
        ak = (int64_t *)malloc(sizeof(int64_t) * (size_t)po.n_auxc);
        if (!ax || !ak) { free(ax); free(ak); return -1; }
        for (int64_t a = 0; a < po.n_auxc; a++) {
            const uint8_t *q = po.aux_bytes + po.aux_off[a] + 4;
            const int32_t bs = (int32_t)(po.aux_off[a + 1] - po.aux_off[a] - 4);
            bam_rec rv;
            memset(&rv, 0, sizeof(rv));
            rv.tid = ldi32(q);
            rv.pos = ldi32(q + 4);
            rv.l_qname = q[8];
            rv.n_cigar = ld16(q + 12);
            rv.l_qseq = ldi32(q + 16);
            rv.data = (uint8_t *)q + 32;
            rv.data_len = bs - 32;
            if (grom_parse_aux(&rv, target, &ax[na])) ak[na++] = po.aux_kidx[a];
        }
    }
    int rc = 0;
    if (s->splitread && na > 0 && grom_stage_put_aux(c->stage, ax, ak, na) != GROM_OK) rc = -1;
    /* the walk's facts: wait for the insert statistics and the final plan */
    dw_final(s);
    if (s->abort) { free(ax); free(ak); return -3; }
    const int32_t s0 = s->index_start;
    int64_t sk = 0, sd = 0;
    if (rc == 0 && ri >= 0 && dd_stage_prefix(w->dd, c->stage, s0, &sk, &sd)) rc = -1;
    /* -S: the first ingested record keeps its SA/XP if it is a kept read */
    int64_t first_drop_before = -1;
    if (rc == 0 && !s->splitread && sd < po.n_drop) {
        grom_reads dv;
        grom_stage_dev_reads(c->stage, &dv);
        if (dd_copy_d2h(w->dd, &first_drop_before, dv.drop_before + sd, sizeof(int64_t))) rc = -1;
    }
    if (rc == 0 && ri >= 0 && grom_stage_trim_drops(c->stage, sd, sk) != GROM_OK) rc = -1;
    if (rc == 0 && grom_stage_trim(c->stage, sk) != GROM_OK) rc = -1;
    const int any = (po.n_kept + po.n_drop) > (sk + sd);
    pd_chrom_facts *f = &c->facts;
    memset(f, 0, sizeof(*f));
    f->n_skip = (int32_t)(sk + sd);
    f->n_reads = po.n_kept - sk;
    f->n_drop = po.n_drop - sd;
    if (any) {
        const int32_t p = po.last_pos - s->overlap_mult * s->insert_max;
        f->p_last = p > s0 ? p : s0;
    } else {
        f->p_last = -1;
    }
    const int64_t n_seen = ri >= 0 ? po.n_rec - j0 : 0;
    if (n_seen > 0 && s->runs[ri].has_next && !s->fetch_mode) f->lseq_tail = s->runs[ri].next_lq;
    else if (any) f->lseq_tail = po.last_lq + (po.last_kept ? po.last_hclip : 0);
    else f->lseq_tail = 0;
    if (rc == 0 && !s->splitread && any) {
        const int first_is_drop = sd < po.n_drop && first_drop_before == sk;
        if (!first_is_drop)
            for (int64_t a = 0; a < na; a++)
                if (ak[a] == sk) {
                    if (grom_stage_patch_aux(c->stage, sk, &ax[a]) != GROM_OK) rc = -1;
                    break;
                }
    }
    free(ax);
    free(ak);
    pthread_mutex_lock(&s->mu);
    s->c_h2d += 0;
    pthread_mutex_unlock(&s->mu);
    return rc;
}

/* wait for the walk's facts (the CLI's pd_set_walk, after the insert
 * statistics) and apply the final plan once */
static void dw_final(pd_session *s) {
    pthread_mutex_lock(&s->mu);
    while (!s->abort && !s->walk_set) pthread_cond_wait(&s->cv, &s->mu);
    const int need = !s->abort && !s->final_applied;
    pthread_mutex_unlock(&s->mu);
    if (need) apply_final(s, 0);
}

static void *dw_main(void *arg) {
    dd_worker *w = (dd_worker *)arg;
    pd_session *s = w->s;
    char err[300] = "";
    int rc = 0;
    pd_trace(s, PD_EV_PHASE, 100, 0);
    w->dd = dd_ctx_new(w->device);
    pd_trace(s, PD_EV_PHASE, 100, 1);
    if (!w->dd) { rc = -1; snprintf(err, sizeof(err), "device decode: no context on device %d", w->device); }
    if (rc == 0) w->pf_started = pthread_create(&w->pf_thr, NULL, pf_main, w) == 0;
    if (rc == 0 && !w->pf_started) { rc = -1; snprintf(err, sizeof(err), "device decode: no prefetch thread"); }
    /* this worker's chromosomes, longest first (the CLI hands them to the
     * scans in the same order, so the last scans are the short chromosomes';
     * the final plan's keep[] only drops some) */
    int *mine = (int *)malloc(sizeof(int) * (size_t)(s->n_plan > 0 ? s->n_plan : 1)), n_mine = 0;
    int *lo = (int *)malloc(sizeof(int) * (size_t)(s->n_plan > 0 ? s->n_plan : 1)), n_lo = 0;
    for (int k = 0; k < s->n_plan; k++)
        if (s->want[k] && s->ch[k].device == w->device) lo[n_lo++] = k;
    for (int a = 1; a < n_lo; a++) /* insertion sort: length descending, plan order on ties */
        for (int b = a; b > 0 && s->plan[lo[b]].len > s->plan[lo[b - 1]].len; b--) {
            const int t = lo[b];
            lo[b] = lo[b - 1];
            lo[b - 1] = t;
        }
    for (int a = 0; a < n_lo; a++)
        if (a % w->nsub == w->sub) mine[n_mine++] = lo[a];
    free(lo);
    /* The insert statistics (the first worker): find_insert_mean's sample is
     * the first records in file order, so the chromosome of the first placed
     * run is decoded first and the sample taken from its pieces as they are
     * decoded; a worker that does not parse that run reads the statistics
     * from it (and the runs after it) alone first. */
    const int stats_here = w->first && !s->stats_given;
    const int r0 = stats_here ? next_placed_run(s, -1) : -1;
    int k0 = -1;
    for (int i = 0; r0 >= 0 && i < n_mine && k0 < 0; i++)
        if (s->ch[mine[i]].run == r0) {
            k0 = mine[i];
            for (int j = i; j > 0; j--) mine[j] = mine[j - 1];
            mine[0] = k0;
        }
    const int stats_pass = stats_here && r0 >= 0 && k0 < 0;
    if (rc == 0) pf_want(w, stats_pass ? r0 : (n_mine > 0 ? s->ch[mine[0]].run : -1));
    pd_trace(s, PD_EV_PHASE, 104, 0);
    if (rc == 0 && dw_reserve(w, err, (int)sizeof(err))) rc = -1;
    pd_trace(s, PD_EV_PHASE, 104, 1);
    /* (after the worker's own buffers: a small allocation waits behind any
     * large one in flight; a stage being reserved makes stage_acquire wait) */
    pthread_t stres_thr;
    stres_job sj = {s, w->device};
    const char *nsr = getenv("GROM_NO_STAGE_RESERVE");
    const int stres = rc == 0 && w->sub == 0 && !(nsr && atoi(nsr) == 1) &&
                      pthread_create(&stres_thr, NULL, stres_main, &sj) == 0;
    if (rc == 0 && stats_pass) rc = dw_stats_only(w, r0, err, (int)sizeof(err));
    else if (rc == 0 && w->first && (!stats_here || r0 < 0)) mark_stats_done(s);
    for (int i = 0; rc == 0 && i < n_mine && !s->abort; i++) {
        const int k = mine[i];
        pd_chrom *c = &s->ch[k];
        const int with_stats = stats_here && k == k0;
        /* the final plan (which chromosomes, which records each one's run
         * starts with) needs the statistics: the statistics' own chromosome
         * is decoded before it (its run starts with its first record in
         * any plan) */
        if (!with_stats) {
            dw_final(s);
            if (s->abort) break;
            if (!s->keep[k]) continue;
        }
        int next_run = -1;
        for (int j = i + 1; j < n_mine && next_run < 0; j++)
            if (!s->final_applied || s->keep[mine[j]]) next_run = s->ch[mine[j]].run;
        const double t0 = now_s();
        pd_trace(s, PD_EV_UPLOAD, k, 0);
        rc = dw_chrom(w, k, next_run, with_stats, err, (int)sizeof(err));
        pd_trace(s, PD_EV_UPLOAD, k, 1);
        if (rc == 0 && with_stats) {
            dw_final(s);
            if (!s->abort && !s->keep[k]) { /* the final plan drops it: nobody scans it */
                pd_release_stage(s, c->stage);
                c->stage = NULL;
            }
        }
        pthread_mutex_lock(&s->mu);
        s->c_upl_s += now_s() - t0;
        if ((rc == -2 || rc == -1) && !s->abort) {
            /* the session's abort is published with the chromosome's final
             * state, under one lock: a waiter on this chromosome sees the
             * abort (soft for -2: the serial reader reruns), never a bare rc */
            s->abort = 1;
            s->abort_soft = rc == -2;
            snprintf(s->abort_msg, sizeof(s->abort_msg), "%s", err);
        }
        c->rc = rc;
        c->final = 1;
        c->begun = 1;
        pd_trace(s, PD_EV_FINAL, k, 0);
        pthread_cond_broadcast(&s->cv);
        pthread_mutex_unlock(&s->mu);
    }
    if (stres) pthread_join(stres_thr, NULL);
    if (rc == -2 || rc == -1) sess_abort(s, rc == -2, err);
    if (w->dd) {
        double ms[4];
        dd_ctx_times(w->dd, ms);
        pthread_mutex_lock(&s->mu);
        for (int q = 0; q < 3; q++) s->c_gpu_ms[q] += ms[q];
        s->c_gpu_ms[3] = ms[3];
        int64_t rw = 0, sc = 0;
        dd_ctx_counts(w->dd, &rw, &sc);
        s->c_rewalk += rw;
        s->c_subchunks += sc;
        pthread_mutex_unlock(&s->mu);
    }
    free(mine);
    if (w->pf_started) {
        pthread_mutex_lock(&w->mu);
        w->pf_stop = 1;
        pthread_cond_broadcast(&w->cv);
        pthread_mutex_unlock(&w->mu);
        pthread_join(w->pf_thr, NULL);
    }
    /* the scans may still read the stages; the decode context goes now */
    dd_ctx_free(w->dd);
    for (int q = 0; q < 2; q++) {
        grom_pinned_free(w->ring[q]);
        free(w->slot[q].blk);
        free(w->slot[q].starts);
    }
    pthread_mutex_destroy(&w->mu);
    pthread_cond_destroy(&w->cv);
    free(w);
    return NULL;
}

int pd_dd_workers(void) {
    const char *ws = getenv("GROM_DD_WORKERS");
    int per = ws && atoi(ws) > 0 ? atoi(ws) : 1;
    return per > 8 ? 8 : per;
}

static int pd_start_device(pd_session *s) {
    int devs[64], nd = 0;
    for (int k = 0; k < s->n_plan; k++) {
        int seen = 0;
        for (int q = 0; q < nd; q++) seen |= devs[q] == s->ch[k].device;
        if (!seen && nd < 64) devs[nd++] = s->ch[k].device;
    }
    if (nd == 0) devs[nd++] = 0;
    /* GROM_DD_WORKERS per GPU (one reads a run while another's is on the GPU) */
    const int per = pd_dd_workers();
    const char *it = getenv("GROM_DECODE_THREADS");
    /* the read-ahead's pread threads per worker: 16 read chr1's 1.75 GB in
     * 0.18 s from the page cache against 0.28 s with 8 (profiles/r05aa) */
    s->io_threads = it && atoi(it) > 0 ? atoi(it) / (nd * per) : 16;
    if (s->io_threads < 1) s->io_threads = 1;
    if (s->io_threads > 16) s->io_threads = 16;
    s->dw = (pthread_t *)calloc((size_t)(nd * per), sizeof(pthread_t));
    for (int q = 0; q < nd * per; q++) {
        dd_worker *w = (dd_worker *)calloc(1, sizeof(dd_worker));
        w->s = s;
        w->device = devs[q / per];
        w->sub = q % per;
        w->nsub = per;
        w->first = q == 0;
        w->test_abort = getenv("GROM_TEST_DD_ABORT") ? atoi(getenv("GROM_TEST_DD_ABORT")) : -1;
        w->slot[0].ri = w->slot[1].ri = -1;
        pthread_mutex_init(&w->mu, NULL);
        pthread_cond_init(&w->cv, NULL);
        if (pthread_create(&s->dw[q], NULL, dw_main, w) != 0) {
            free(w);
            sess_abort(s, 0, "cannot start device decode workers");
            return -1;
        }
        s->dw_started = q + 1;
    }
    s->n_threads = 0;
    return 0;
}

static int64_t pd_reclaim_stages(void *arg, int device, size_t want);

int pd_start(pd_session *s, int min_mapq, int n_dev, const int *dev_of, int plan_only) {
    s->min_mapq_stats = min_mapq;
    s->plan_only = plan_only;
    s->test_soft_abort = getenv("GROM_TEST_SOFT_ABORT") ? atoi(getenv("GROM_TEST_SOFT_ABORT")) : -1;
    s->no_mirror = plan_only && getenv("GROM_DECODE_ONLY") != NULL; /* time the decode alone */
    s->n_dev = n_dev < 1 ? 1 : n_dev;
    for (int k = 0; k < s->n_plan; k++) s->ch[k].device = dev_of ? dev_of[k] : 0;
    if (!plan_only) { /* an allocation short of device memory may take idle stages' blocks */
        grom_dev_add_reclaim(pd_reclaim_stages, s);
        s->reclaim_on = 1;
    }
    if (!plan_only && s->dev_mode) return pd_start_device(s);
    s->thr = (pthread_t *)calloc((size_t)s->n_threads, sizeof(pthread_t));
    for (int t = 0; t < s->n_threads; t++)
        if (pthread_create(&s->thr[t], NULL, decoder_main, s) != 0) {
            s->n_threads = t;
            break;
        }
    if (s->n_threads == 0 || pthread_create(&s->upl, NULL, uploader_main, s) != 0) {
        sess_abort(s, 0, "cannot start decoder threads");
        return -1;
    }
    s->upl_started = 1;
    return 0;
}

int pd_insert_stats(pd_session *s, double prob2, int min_mapq, int *lseq, int *imin, int *imax, long *mapped) {
    (void)min_mapq;
    pthread_mutex_lock(&s->mu);
    while (!s->stats_done && !s->abort) pthread_cond_wait(&s->cv, &s->mu);
    const int ab = s->abort;
    pthread_mutex_unlock(&s->mu);
    if (ab) return -2;
    const int64_t n = s->s_n;
    if (n == 0) return -1;
    /* find_insert_mean's arithmetic, as grom_insert_stats */
    grom_sort_ints(s->s_ins, n);
    int mean = s->s_ins[n / 2], lim = mean * 5, end = 0;
    for (int64_t a = n - 1; a >= 0; a--)
        if (s->s_ins[a] <= lim) { end = (int)a; break; }
    end += 1;
    mean = s->s_ins[end / 2];
    int lo = (int)(prob2 * end / 2);
    *imin = s->s_ins[lo];
    *imax = s->s_ins[end - lo < n ? end - lo : n - 1];
    grom_sort_ints(s->s_lq, n);
    *lseq = s->s_lq[n / 2];
    if (mapped) *mapped = (long)s->s_m;
    return mean;
}

void pd_stats_given(pd_session *s) { s->stats_given = 1; }

void pd_set_walk(pd_session *s, int32_t index_start, int32_t overlap_mult, int32_t insert_max, const int *keep) {
    pthread_mutex_lock(&s->mu);
    for (int k = 0; k < s->n_plan; k++) s->keep[k] = keep ? (keep[k] != 0) : 1;
    s->final_pending = 1;
    s->index_start = index_start;
    s->overlap_mult = overlap_mult;
    s->insert_max = insert_max;
    s->walk_set = 1;
    pthread_cond_broadcast(&s->cv);
    pthread_mutex_unlock(&s->mu);
}

int pd_wait_chrom(pd_session *s, int k, grom_stage **stage, pd_chrom_facts *facts) {
    pthread_mutex_lock(&s->mu);
    while (!s->abort && !s->ch[k].final) pthread_cond_wait(&s->cv, &s->mu);
    const int ab = s->abort, soft = s->abort_soft;
    pthread_mutex_unlock(&s->mu);
    if (ab) return soft ? 1 : GROM_E_ARG;
    if (s->ch[k].rc) return GROM_E_ARG;
    if (stage) *stage = s->ch[k].stage;
    if (facts) *facts = s->ch[k].facts;
    s->ch[k].handed = 1;
    return 0;
}

void pd_release_stage(pd_session *s, grom_stage *st) {
    pthread_mutex_lock(&s->mu);
    for (int i = 0; i < s->n_stage; i++)
        if (s->stages[i] == st) { s->stage_busy[i] = 0; s->stage_owner[i] = -1; }
    pthread_cond_broadcast(&s->cv);
    pthread_mutex_unlock(&s->mu);
    grom_dev_release_notify(); /* an allocation waiting for memory may take its block */
}

/* devmem.h reclaim hook: the blocks of this device's idle stages (no
 * chromosome holds them), largest first, until `want` bytes are free */
static int64_t pd_reclaim_stages(void *arg, int device, size_t want) {
    pd_session *s = (pd_session *)arg;
    int64_t got = 0;
    for (;;) {
        pthread_mutex_lock(&s->mu);
        int pick = -1;
        for (int i = 0; i < s->n_stage; i++)
            if (!s->stage_busy[i] && s->stage_dev[i] == device && grom_stage_held(s->stages[i]) > 0 &&
                (pick < 0 || grom_stage_held(s->stages[i]) > grom_stage_held(s->stages[pick])))
                pick = i;
        if (pick >= 0) {
            s->stage_busy[pick] = 1;
            s->stage_owner[pick] = -3;
        }
        pthread_mutex_unlock(&s->mu);
        if (pick < 0) break;
        got += grom_stage_drop(s->stages[pick]);
        pthread_mutex_lock(&s->mu);
        s->stage_busy[pick] = 0;
        s->stage_owner[pick] = -1;
        s->c_reclaimed++;
        pthread_cond_broadcast(&s->cv);
        pthread_mutex_unlock(&s->mu);
        if (got >= (int64_t)want) break;
    }
    return got;
}

int pd_add_stage(pd_session *s, grom_stage *st, int device) {
    pthread_mutex_lock(&s->mu);
    if (s->n_stage == s->cap_stage) {
        s->cap_stage = s->cap_stage ? 2 * s->cap_stage : 16;
        s->stages = (grom_stage **)realloc(s->stages, sizeof(grom_stage *) * s->cap_stage);
        s->stage_dev = (int *)realloc(s->stage_dev, sizeof(int) * s->cap_stage);
        s->stage_busy = (int *)realloc(s->stage_busy, sizeof(int) * s->cap_stage);
        s->stage_owner = (int *)realloc(s->stage_owner, sizeof(int) * s->cap_stage);
        s->stage_mine = (int *)realloc(s->stage_mine, sizeof(int) * s->cap_stage);
    }
    s->stages[s->n_stage] = st;
    s->stage_dev[s->n_stage] = device;
    s->stage_busy[s->n_stage] = 0;
    s->stage_owner[s->n_stage] = -1;
    s->stage_mine[s->n_stage] = 0;
    s->n_stage++;
    pthread_cond_broadcast(&s->cv);
    pthread_mutex_unlock(&s->mu);
    return 0;
}

const char *pd_error(pd_session *s) { return s->abort_msg; }

int pd_mirror_view(pd_session *s, int k, grom_reads *out) {
    if (k < 0 || k >= s->n_plan) return -1;
    grom_batch_view(&s->ch[k].mirror, out);
    return 0;
}

void pd_get_counters(pd_session *s, pd_counters *c) {
    memset(c, 0, sizeof(*c));
    pthread_mutex_lock(&s->mu);
    c->records = s->c_records;
    c->pieces = s->n_pieces;
    c->inflated_bytes = s->c_inflated;
    c->compressed_bytes = s->c_compressed;
    c->decode_thread_s = s->c_dec_s;
    c->h2d_bytes = s->c_h2d;
    c->inflate_s = s->c_inflate_s;
    c->device = s->dev_mode;
    for (int q = 0; q < 4; q++) c->gpu_ms[q] = s->c_gpu_ms[q];
    c->rewalked = s->c_rewalk;
    c->subchunks = s->c_subchunks;
    c->io_s = s->c_io_s;
    c->upload_s = s->c_upl_s;
    c->reclaimed = s->c_reclaimed;
    c->dd_workers = s->dw_started;
    c->stats_only_runs = s->c_stats_only;
    c->wait_s = s->c_wait_s;
    c->threads = s->n_threads;
    pthread_mutex_unlock(&s->mu);
    pthread_once(&ld_once, ld_init);
    c->libdeflate = ld_alloc != NULL;
}

void pd_close(pd_session *s) {
    if (!s) return;
    if (s->reclaim_on) grom_dev_remove_reclaim(pd_reclaim_stages, s);
    if (s->tr && s->trace_path) {
        FILE *f = fopen(s->trace_path, "w");
        if (f) {
            static const char *names[] = {"", "decode", "upload", "final", "stats", "stage", "scan", "handed", "phase"};
            fprintf(f, "t,thread,event,a,b\n");
            const int64_t n = s->tr_n < s->tr_cap ? s->tr_n : s->tr_cap;
            for (int64_t i = 0; i < n; i++)
                fprintf(f, "%.6f,%d,%s,%lld,%lld\n", s->tr[i].t, s->tr[i].thr,
                        s->tr[i].ev >= 1 && s->tr[i].ev <= 8 ? names[s->tr[i].ev] : "?", (long long)s->tr[i].a,
                        (long long)s->tr[i].b);
            fclose(f);
        }
    }
    free(s->tr);
    s->tr = NULL;
    free(s->trace_path);
    pthread_mutex_lock(&s->mu);
    s->stop = 1;
    if (!s->abort) s->abort = 1; /* wake and stop everyone */
    pthread_cond_broadcast(&s->cv);
    pthread_mutex_unlock(&s->mu);
    for (int t = 0; t < s->n_threads && s->thr; t++) pthread_join(s->thr[t], NULL);
    if (s->upl_started) pthread_join(s->upl, NULL);
    for (int t = 0; t < s->dw_started; t++) pthread_join(s->dw[t], NULL);
    /* buffers: wait for their copies, then free */
    while (s->inflight_head) {
        pd_buf *b = s->inflight_head;
        (void)grom_stage_ticket_wait(b->stage, b->ticket);
        s->inflight_head = b->next;
        buf_destroy(b, !s->plan_only);
    }
    while (s->free_bufs) {
        pd_buf *b = s->free_bufs;
        s->free_bufs = b->next;
        buf_destroy(b, !s->plan_only);
    }
    for (int i = 0; i < s->n_pieces; i++) {
        if (s->pieces[i].buf) buf_destroy(s->pieces[i].buf, !s->plan_only);
        piece_free_stats(&s->pieces[i]);
    }
    for (int i = 0; i < s->n_old; i++) grom_pinned_free(s->old_pinned[i]);
    free(s->old_pinned);
    for (int k = 0; k < s->n_plan; k++) {
        grom_batch_free(&s->ch[k].mirror);
        free(s->ch[k].drops);
        free(s->ch[k].lowpos);
        free(s->ch[k].saux);
    }
    for (int t = 0; t < s->n_tgt && s->lin; t++) free(s->lin[t]);
    free(s->lin);
    free(s->n_lin);
    free(s->dw);
    free(s->T.e);
    free(s->T.arena);
    free(s->T.ht);
    free(s->T.hh);
    free(s->remap);
    for (int i = 0; i < s->n_stage; i++)
        if (s->stage_mine[i]) grom_stage_free(s->stages[i]);
    free(s->stages);
    free(s->stage_dev);
    free(s->stage_busy);
    free(s->stage_owner);
    free(s->stage_mine);
    free(s->thr);
    free(s->ch);
    free(s->plan);
    free(s->keep);
    free(s->want);
    free(s->runs);
    free(s->pieces);
    free(s->s_ins);
    free(s->s_lq);
    if (s->fd >= 0) close(s->fd);
    pthread_mutex_destroy(&s->mu);
    pthread_cond_destroy(&s->cv);
    free(s);
}

/* ---------------- digest of a read batch (tests) ---------------- */
static uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

static uint64_t hbytes(uint64_t h, const void *p, size_t n) {
    const uint8_t *q = (const uint8_t *)p;
    for (size_t i = 0; i < n; i++) h = (h ^ q[i]) * 0x100000001b3ULL;
    return h;
}

static int32_t ref_span(const grom_reads *r, int64_t i) {
    int32_t span = 0;
    for (uint32_t c = r->cigar_off[i]; c < r->cigar_off[i + 1]; c++) {
        const int o = r->cigar[c] & 0xf;
        if (o == GC_MATCH || o == GC_DEL || o == GC_REF_SKIP || o == GC_EQUAL || o == GC_DIFF) span += (int32_t)(r->cigar[c] >> 4);
    }
    return span;
}

uint64_t pd_digest(const grom_reads *r) {
    uint64_t h = mix64((uint64_t)r->n * 31 + (uint64_t)r->n_drop);
    int32_t max_span = 0;
    for (int64_t i = 0; i < r->n; i++) {
        const int32_t sp = ref_span(r, i);
        if (sp > max_span) max_span = sp;
    }
    for (int64_t i = 0; i < r->n; i++) {
        uint64_t x = 0xcbf29ce484222325ULL;
        x = hbytes(x, &r->pos[i], 4);
        x = hbytes(x, &r->flag[i], 2);
        x = hbytes(x, &r->mapq[i], 1);
        x = hbytes(x, &r->mtid[i], 4);
        x = hbytes(x, &r->mpos[i], 4);
        x = hbytes(x, &r->isize[i], 4);
        x = hbytes(x, &r->l_qseq[i], 4);
        const uint32_t c0 = r->cigar_off[i], c1 = r->cigar_off[i + 1];
        x = hbytes(x, r->cigar + c0, 4 * (size_t)(c1 - c0));
        const int64_t L = r->l_qseq[i];
        x = hbytes(x, r->qual + r->base_off[i], (size_t)L);
        x = hbytes(x, r->seq + r->base_off[i] / 2, (size_t)(L + 1) / 2);
        if (r->aux_idx && r->aux_idx[i] >= 0 && r->aux) {
            const grom_aux *a = &r->aux[r->aux_idx[i]];
            x = hbytes(x, a, offsetof(grom_aux, pad));
        } else {
            x = hbytes(x, "-", 1);
        }
        h += mix64(x + (uint64_t)i * 0x9e3779b97f4a7c15ULL);
        /* earlier reads sharing a base with this one, with the same name id
         * (the relation the pileup's read-name de-duplication reads) */
        if (r->name_id[i]) {
            for (int64_t j = i - 1; j >= 0 && (int64_t)r->pos[j] + max_span > r->pos[i]; j--) {
                if (r->name_id[j] == r->name_id[i] && r->pos[j] + ref_span(r, j) > r->pos[i])
                    h += mix64(((uint64_t)i << 32) ^ (uint64_t)j ^ 0x5bd1e995ULL);
            }
        }
    }
    for (int64_t d = 0; d < r->n_drop; d++) {
        uint64_t x = 0x84222325cbf29ce4ULL;
        x = hbytes(x, &r->drop_pos[d], 4);
        x = hbytes(x, &r->drop_lq[d], 4);
        x = hbytes(x, &r->drop_before[d], 8);
        h += mix64(x + (uint64_t)d * 0x632be59bd9b4e019ULL);
    }
    return h;
}
