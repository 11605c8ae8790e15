/*
 * bamio.c -- BGZF/BAM reader and writer on zlib (see bamio.h).
 */
#include "bamio.h"

#include <dlfcn.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>
#include <unistd.h>

#define BGZF_MAX_BLOCK 65536
#define BGZF_WRITE_PAYLOAD 0xff00

const char grom_nt16_rev[16] = {'=', 'A', 'C', 'M', 'G', 'R', 'S', 'V',
                                'T', 'W', 'Y', 'H', 'K', 'D', 'B', 'N'};

static const unsigned char BGZF_EOF_BLOCK[28] = {
    0x1f, 0x8b, 0x08, 0x04, 0x00, 0x00, 0x00, 0x00, 0x00, 0xff, 0x06, 0x00, 0x42, 0x43,
    0x02, 0x00, 0x1b, 0x00, 0x03, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00};

static uint16_t rd16(const unsigned char *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static uint32_t rd32(const unsigned char *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static void wr16(unsigned char *p, uint16_t v) { p[0] = v & 0xff; p[1] = v >> 8; }
static void wr32(unsigned char *p, uint32_t v) {
    p[0] = v & 0xff; p[1] = (v >> 8) & 0xff; p[2] = (v >> 16) & 0xff; p[3] = v >> 24;
}

int bgzf_open_read(bgzf_reader *r, const char *path) {
    memset(r, 0, sizeof(*r));
    r->fp = fopen(path, "rb");
    if (!r->fp) return -1;
    r->blk = (unsigned char *)malloc(BGZF_MAX_BLOCK);
    r->cbuf = (unsigned char *)malloc(BGZF_MAX_BLOCK);
    if (!r->blk || !r->cbuf) return -1;
    return 0;
}

/* ---- multi-threaded inflate: the caller reads compressed blocks in file
 * order into a ring of slots, workers inflate them, the caller consumes the
 * slots in order (so the byte stream is the same as the serial reader's) ---- */
enum { SLOT_FREE = 0, SLOT_QUEUED, SLOT_BUSY, SLOT_DONE };
typedef struct {
    unsigned char *cbuf, *blk;
    int clen, len, rc, state;
    uint32_t isize;
} bgzf_slot;

struct bgzf_mt {
    int n_thr, n_slot;
    bgzf_slot *slot;
    long head, tail; /* next slot to consume / to fill */
    int file_eof, file_err;
    int stop;
    pthread_t *thr;
    pthread_mutex_t mu;
    pthread_cond_t work, done;
};

static int inflate_block(const unsigned char *cbuf, int clen, uint32_t isize, unsigned char *out) {
    if (isize == 0) return 0;
    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    if (inflateInit2(&zs, -15) != Z_OK) return -1;
    zs.next_in = (unsigned char *)cbuf;
    zs.avail_in = clen - 8;
    zs.next_out = out;
    zs.avail_out = BGZF_MAX_BLOCK;
    int rc = inflate(&zs, Z_FINISH);
    inflateEnd(&zs);
    if (rc != Z_STREAM_END || zs.total_out != isize) return -1;
    return (int)isize;
}

/* one compressed block: header parsed, deflate data + trailer into cbuf;
 * returns 1, 0 at EOF, -1 on error */
static int read_cblock(FILE *fp, unsigned char *cbuf, int *clen_out, uint32_t *isize_out) {
    unsigned char hdr[18];
    size_t got = fread(hdr, 1, 18, fp);
    if (got == 0) return 0;
    if (got != 18 || hdr[0] != 0x1f || hdr[1] != 0x8b || hdr[3] != 0x04) return -1;
    uint16_t xlen = rd16(hdr + 10);
    /* locate the BC subfield; hdr holds the first 6 bytes of the extra field */
    unsigned char extra[1024];
    if (xlen > sizeof(extra) || xlen < 6) return -1;
    memcpy(extra, hdr + 12, 6);
    if (xlen > 6 && fread(extra + 6, 1, xlen - 6, fp) != (size_t)(xlen - 6)) return -1;
    int bsize = -1;
    for (int o = 0; o + 4 <= xlen;) {
        int sl = rd16(extra + o + 2);
        if (extra[o] == 'B' && extra[o + 1] == 'C' && sl == 2) { bsize = rd16(extra + o + 4); break; }
        o += 4 + sl;
    }
    if (bsize < 0) return -1;
    int clen = bsize + 1 - 12 - xlen; /* deflate data + 8-byte trailer */
    if (clen < 8 || clen > BGZF_MAX_BLOCK) return -1;
    if (fread(cbuf, 1, clen, fp) != (size_t)clen) return -1;
    uint32_t isize = rd32(cbuf + clen - 4);
    if (isize > BGZF_MAX_BLOCK) return -1;
    *clen_out = clen;
    *isize_out = isize;
    return 1;
}

static void *bgzf_worker(void *arg) {
    struct bgzf_mt *m = (struct bgzf_mt *)arg;
    pthread_mutex_lock(&m->mu);
    for (;;) {
        bgzf_slot *s = NULL;
        while (!m->stop) {
            for (long k = m->head; k < m->tail; k++)
                if (m->slot[k % m->n_slot].state == SLOT_QUEUED) { s = &m->slot[k % m->n_slot]; break; }
            if (s) break;
            pthread_cond_wait(&m->work, &m->mu);
        }
        if (m->stop) break;
        s->state = SLOT_BUSY;
        pthread_mutex_unlock(&m->mu);
        const int rc = inflate_block(s->cbuf, s->clen, s->isize, s->blk);
        pthread_mutex_lock(&m->mu);
        s->rc = rc;
        s->len = rc;
        s->state = SLOT_DONE;
        pthread_cond_broadcast(&m->done);
    }
    pthread_mutex_unlock(&m->mu);
    return NULL;
}

static void bgzf_mt_free(struct bgzf_mt *m);

int bgzf_set_threads(bgzf_reader *r, int n) {
    if (n <= 1 || r->mt) return 0;
    struct bgzf_mt *m = (struct bgzf_mt *)calloc(1, sizeof(*m));
    if (!m) return -1;
    m->n_thr = 0; /* threads actually started (the only ones joined) */
    m->n_slot = 4 * n;
    m->slot = (bgzf_slot *)calloc(m->n_slot, sizeof(bgzf_slot));
    m->thr = (pthread_t *)calloc(n, sizeof(pthread_t));
    int ok = m->slot && m->thr;
    for (int k = 0; ok && k < m->n_slot; k++) {
        m->slot[k].cbuf = (unsigned char *)malloc(BGZF_MAX_BLOCK);
        m->slot[k].blk = (unsigned char *)malloc(BGZF_MAX_BLOCK);
        if (!m->slot[k].cbuf || !m->slot[k].blk) ok = 0;
    }
    if (!ok) {
        for (int k = 0; m->slot && k < m->n_slot; k++) { free(m->slot[k].cbuf); free(m->slot[k].blk); }
        free(m->slot);
        free(m->thr);
        free(m);
        return -1;
    }
    pthread_mutex_init(&m->mu, NULL);
    pthread_cond_init(&m->work, NULL);
    pthread_cond_init(&m->done, NULL);
    for (int t = 0; t < n; t++) {
        if (pthread_create(&m->thr[t], NULL, bgzf_worker, m) != 0) break;
        m->n_thr++;
    }
    if (m->n_thr == 0) { /* no worker: the serial reader */
        bgzf_mt_free(m);
        return 0;
    }
    r->mt = m;
    return 0;
}

static void bgzf_mt_free(struct bgzf_mt *m) {
    if (!m) return;
    pthread_mutex_lock(&m->mu);
    m->stop = 1;
    pthread_cond_broadcast(&m->work);
    pthread_mutex_unlock(&m->mu);
    for (int t = 0; t < m->n_thr; t++) pthread_join(m->thr[t], NULL);
    for (int k = 0; k < m->n_slot; k++) {
        free(m->slot[k].cbuf);
        free(m->slot[k].blk);
    }
    pthread_mutex_destroy(&m->mu);
    pthread_cond_destroy(&m->work);
    pthread_cond_destroy(&m->done);
    free(m->slot);
    free(m->thr);
    free(m);
}

/* the next block in file order through the pipeline: 1, 0 at EOF, -1 error */
static int bgzf_mt_next(bgzf_reader *r) {
    struct bgzf_mt *m = r->mt;
    pthread_mutex_lock(&m->mu);
    /* top up the read-ahead: compressed blocks are read here, in file order,
     * into slots that are free (consumed) */
    while (!m->file_eof && !m->file_err && m->tail - m->head < m->n_slot) {
        bgzf_slot *s = &m->slot[m->tail % m->n_slot];
        pthread_mutex_unlock(&m->mu);
        const int rc = read_cblock(r->fp, s->cbuf, &s->clen, &s->isize);
        pthread_mutex_lock(&m->mu);
        if (rc <= 0) {
            if (rc < 0) m->file_err = 1;
            else m->file_eof = 1;
            break;
        }
        s->state = SLOT_QUEUED;
        m->tail++;
        pthread_cond_signal(&m->work);
    }
    if (m->head == m->tail) {
        const int err = m->file_err;
        pthread_mutex_unlock(&m->mu);
        if (err) return -1;
        r->eof = 1;
        return 0;
    }
    bgzf_slot *s = &m->slot[m->head % m->n_slot];
    while (s->state != SLOT_DONE) pthread_cond_wait(&m->done, &m->mu);
    m->head++;
    pthread_mutex_unlock(&m->mu);
    if (s->rc < 0) return -1;
    /* hand the block over by swapping buffers (the slot is refilled later) */
    unsigned char *t = r->blk;
    r->blk = s->blk;
    s->blk = t;
    s->state = SLOT_FREE;
    r->blk_len = s->len;
    r->blk_off = 0;
    return 1;
}

void bgzf_close_read(bgzf_reader *r) {
    bgzf_mt_free(r->mt);
    if (r->fp) fclose(r->fp);
    free(r->blk);
    free(r->cbuf);
    memset(r, 0, sizeof(*r));
}

/* the next block into r->blk; returns 1, 0 at EOF, -1 error */
static int bgzf_next_block(bgzf_reader *r) {
    if (r->mt) return bgzf_mt_next(r);
    int clen = 0;
    uint32_t isize = 0;
    r->blk_coff = r->next_coff;
    const int rc = read_cblock(r->fp, r->cbuf, &clen, &isize);
    r->next_coff = (int64_t)ftell(r->fp);
    if (rc == 0) { r->eof = 1; return 0; }
    if (rc < 0) return -1;
    const int n = inflate_block(r->cbuf, clen, isize, r->blk);
    if (n < 0) return -1;
    r->blk_len = n;
    r->blk_off = 0;
    return 1;
}

int bgzf_read(bgzf_reader *r, void *dst, int n) {
    unsigned char *d = (unsigned char *)dst;
    int done = 0;
    while (done < n) {
        if (r->blk_off >= r->blk_len) {
            int rc = bgzf_next_block(r);
            if (rc < 0) return -1;
            if (rc == 0) return done == 0 ? 0 : -1;
            continue;
        }
        int take = r->blk_len - r->blk_off;
        if (take > n - done) take = n - done;
        memcpy(d + done, r->blk + r->blk_off, take);
        r->blk_off += take;
        done += take;
    }
    return done;
}

int bgzf_open_write(bgzf_writer *w, const char *path, int level) {
    memset(w, 0, sizeof(*w));
    w->fp = fopen(path, "wb");
    if (!w->fp) return -1;
    w->buf = (unsigned char *)malloc(BGZF_MAX_BLOCK);
    w->level = level;
    return w->buf ? 0 : -1;
}

/* ---- block compression: libdeflate when the image has it, else zlib ---- */
typedef void *(*ldc_alloc_fn)(int);
typedef size_t (*ldc_comp_fn)(void *, const void *, size_t, void *, size_t);
typedef void (*ldc_free_fn)(void *);
static ldc_alloc_fn ldc_alloc;
static ldc_comp_fn ldc_comp;
static ldc_free_fn ldc_free;
static pthread_once_t ldc_once = PTHREAD_ONCE_INIT;
/* one compressor per thread, freed when the thread exits */
typedef struct {
    void *cmp;
    int level;
} ldc_tls;
static pthread_key_t ldc_key;
static int ldc_key_ok;
static void ldc_tls_free(void *p) {
    ldc_tls *t = (ldc_tls *)p;
    if (t && t->cmp) ldc_free(t->cmp);
    free(t);
}
static void ldc_init(void) {
    if (getenv("GROM_NO_LIBDEFLATE")) return;
    ldc_key_ok = pthread_key_create(&ldc_key, ldc_tls_free) == 0;
    if (!ldc_key_ok) return;
    void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    ldc_alloc_fn a = (ldc_alloc_fn)dlsym(h, "libdeflate_alloc_compressor");
    ldc_comp_fn c = (ldc_comp_fn)dlsym(h, "libdeflate_deflate_compress");
    ldc_free_fn f = (ldc_free_fn)dlsym(h, "libdeflate_free_compressor");
    if (a && c && f) { ldc_alloc = a; ldc_comp = c; ldc_free = f; }
}

int bgzf_block_compress(const unsigned char *in, int len, unsigned char *out, int level) {
    pthread_once(&ldc_once, ldc_init);
    int clen = -1;
    const int room = BGZF_MAX_BLOCK - 18 - 8;
    if (ldc_alloc) {
        ldc_tls *t = (ldc_tls *)pthread_getspecific(ldc_key);
        if (!t && (t = (ldc_tls *)calloc(1, sizeof(ldc_tls))) != NULL) {
            t->level = -1;
            if (pthread_setspecific(ldc_key, t) != 0) {
                free(t);
                t = NULL;
            }
        }
        if (t && (!t->cmp || t->level != level)) {
            if (t->cmp) ldc_free(t->cmp);
            t->cmp = ldc_alloc(level < 1 ? 1 : level);
            t->level = level;
        }
        if (t && t->cmp) {
            const size_t k = ldc_comp(t->cmp, in, (size_t)len, out + 18, (size_t)room);
            if (k > 0) clen = (int)k;
        }
    }
    if (clen < 0) {
        z_stream zs;
        memset(&zs, 0, sizeof(zs));
        if (deflateInit2(&zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return -1;
        zs.next_in = (unsigned char *)in;
        zs.avail_in = (uInt)len;
        zs.next_out = out + 18;
        zs.avail_out = (uInt)room;
        int rc = deflate(&zs, Z_FINISH);
        clen = (int)zs.total_out;
        deflateEnd(&zs);
        if (rc != Z_STREAM_END) return -1;
    }
    static const unsigned char h[12] = {0x1f, 0x8b, 0x08, 0x04, 0, 0, 0, 0, 0, 0xff, 0x06, 0x00};
    memcpy(out, h, 12);
    out[12] = 'B'; out[13] = 'C';
    wr16(out + 14, 2);
    wr16(out + 16, (uint16_t)(18 + clen + 8 - 1));
    uint32_t crc = crc32(0L, in, (uInt)len);
    wr32(out + 18 + clen, crc);
    wr32(out + 18 + clen + 4, (uint32_t)len);
    return 18 + clen + 8;
}

int bgzf_flush_block(bgzf_writer *w) {
    if (w->len == 0) return 0;
    unsigned char out[BGZF_MAX_BLOCK + 64];
    const int n = bgzf_block_compress(w->buf, w->len, out, w->level);
    if (n < 0) return -1;
    if (fwrite(out, 1, n, w->fp) != (size_t)n) return -1;
    w->len = 0;
    return 0;
}

const unsigned char *bgzf_eof_block(void) { return BGZF_EOF_BLOCK; }

int bgzf_write(bgzf_writer *w, const void *src, int n) {
    const unsigned char *s = (const unsigned char *)src;
    while (n > 0) {
        int take = BGZF_WRITE_PAYLOAD - w->len;
        if (take > n) take = n;
        memcpy(w->buf + w->len, s, take);
        w->len += take;
        s += take;
        n -= take;
        if (w->len >= BGZF_WRITE_PAYLOAD && bgzf_flush_block(w) != 0) return -1;
    }
    return 0;
}

int bgzf_close_write(bgzf_writer *w) {
    int rc = bgzf_flush_block(w);
    if (fwrite(BGZF_EOF_BLOCK, 1, 28, w->fp) != 28) rc = -1;
    if (fclose(w->fp) != 0) rc = -1;
    free(w->buf);
    memset(w, 0, sizeof(*w));
    return rc;
}

int bam_read_header(bgzf_reader *r, bam_hdr *h) {
    memset(h, 0, sizeof(*h));
    unsigned char b4[4];
    if (bgzf_read(r, b4, 4) != 4 || memcmp(b4, "BAM\1", 4) != 0) return -1;
    if (bgzf_read(r, b4, 4) != 4) return -1;
    h->l_text = (int32_t)rd32(b4);
    h->text = (char *)calloc((size_t)h->l_text + 1, 1);
    if (h->l_text && bgzf_read(r, h->text, h->l_text) != h->l_text) return -1;
    if (bgzf_read(r, b4, 4) != 4) return -1;
    h->n_ref = (int32_t)rd32(b4);
    h->ref_name = (char **)calloc(h->n_ref > 0 ? h->n_ref : 1, sizeof(char *));
    h->ref_len = (int32_t *)calloc(h->n_ref > 0 ? h->n_ref : 1, sizeof(int32_t));
    for (int i = 0; i < h->n_ref; i++) {
        if (bgzf_read(r, b4, 4) != 4) return -1;
        int32_t ln = (int32_t)rd32(b4);
        h->ref_name[i] = (char *)calloc((size_t)ln + 1, 1);
        if (bgzf_read(r, h->ref_name[i], ln) != ln) return -1;
        if (bgzf_read(r, b4, 4) != 4) return -1;
        h->ref_len[i] = (int32_t)rd32(b4);
    }
    return 0;
}

void bam_free_header(bam_hdr *h) {
    for (int i = 0; i < h->n_ref; i++) free(h->ref_name[i]);
    free(h->ref_name);
    free(h->ref_len);
    free(h->text);
    memset(h, 0, sizeof(*h));
}

int bam_read_rec(bgzf_reader *r, bam_rec *b) {
    unsigned char c[36];
    int got = bgzf_read(r, c, 4);
    if (got == 0) return 0;
    if (got != 4) return -1;
    int32_t block = (int32_t)rd32(c);
    if (block < 32) return -1;
    if (bgzf_read(r, c + 4, 32) != 32) return -1;
    b->tid = (int32_t)rd32(c + 4);
    b->pos = (int32_t)rd32(c + 8);
    b->l_qname = c[12];
    b->mapq = c[13];
    b->bin = rd16(c + 14);
    b->n_cigar = rd16(c + 16);
    b->flag = rd16(c + 18);
    b->l_qseq = (int32_t)rd32(c + 20);
    b->mtid = (int32_t)rd32(c + 24);
    b->mpos = (int32_t)rd32(c + 28);
    b->isize = (int32_t)rd32(c + 32);
    b->data_len = block - 32;
    if (b->data_len > b->m_data) {
        b->m_data = (b->data_len + 255) & ~255;
        b->data = (uint8_t *)realloc(b->data, b->m_data);
        if (!b->data) return -1;
    }
    if (bgzf_read(r, b->data, b->data_len) != b->data_len) return -1;
    return 1;
}

void bam_free_rec(bam_rec *b) {
    free(b->data);
    memset(b, 0, sizeof(*b));
}

int bam_write_header(bgzf_writer *w, const bam_hdr *h) {
    unsigned char b4[4];
    if (bgzf_write(w, "BAM\1", 4)) return -1;
    wr32(b4, (uint32_t)h->l_text);
    if (bgzf_write(w, b4, 4)) return -1;
    if (h->l_text && bgzf_write(w, h->text, h->l_text)) return -1;
    wr32(b4, (uint32_t)h->n_ref);
    if (bgzf_write(w, b4, 4)) return -1;
    for (int i = 0; i < h->n_ref; i++) {
        int32_t ln = (int32_t)strlen(h->ref_name[i]) + 1;
        wr32(b4, (uint32_t)ln);
        if (bgzf_write(w, b4, 4) || bgzf_write(w, h->ref_name[i], ln)) return -1;
        wr32(b4, (uint32_t)h->ref_len[i]);
        if (bgzf_write(w, b4, 4)) return -1;
    }
    return 0;
}

int bam_write_rec(bgzf_writer *w, const bam_rec *b) {
    unsigned char c[36];
    wr32(c, (uint32_t)(32 + b->data_len));
    wr32(c + 4, (uint32_t)b->tid);
    wr32(c + 8, (uint32_t)b->pos);
    c[12] = b->l_qname;
    c[13] = b->mapq;
    wr16(c + 14, b->bin);
    wr16(c + 16, b->n_cigar);
    wr16(c + 18, b->flag);
    wr32(c + 20, (uint32_t)b->l_qseq);
    wr32(c + 24, (uint32_t)b->mtid);
    wr32(c + 28, (uint32_t)b->mpos);
    wr32(c + 32, (uint32_t)b->isize);
    /* keep a record inside one block when it fits, as htslib does */
    if (w->len + 36 + b->data_len > BGZF_WRITE_PAYLOAD && w->len > 0) {
        if (bgzf_flush_block(w)) return -1;
    }
    if (bgzf_write(w, c, 36)) return -1;
    return bgzf_write(w, b->data, b->data_len);
}

/* size in bytes of one aux value of type t (not B/Z/H) */
static int aux_type_size(uint8_t t) {
    switch (t) {
    case 'A': case 'c': case 'C': return 1;
    case 's': case 'S': return 2;
    case 'i': case 'I': case 'f': return 4;
    case 'd': return 8;
    default: return -1;
    }
}

uint8_t *bam_aux_find(const bam_rec *b, const char tag[2]) {
    uint8_t *s = bam_aux(b);
    uint8_t *end = b->data + b->data_len;
    while (s + 3 <= end) {
        int hit = (s[0] == (uint8_t)tag[0] && s[1] == (uint8_t)tag[1]);
        uint8_t t = s[2];
        if (hit) return s + 2;
        s += 3;
        if (t == 'Z' || t == 'H') {
            while (s < end && *s) s++;
            s++;
        } else if (t == 'B') {
            if (s + 5 > end) return NULL;
            int sz = aux_type_size(s[0]);
            uint32_t n = rd32(s + 1);
            if (sz < 0) return NULL;
            s += 5 + (size_t)sz * n;
        } else {
            int sz = aux_type_size(t);
            if (sz < 0) return NULL;
            s += sz;
        }
    }
    return NULL;
}

int bam_reg2bin(int beg, int end) {
    --end;
    if (beg >> 14 == end >> 14) return ((1 << 15) - 1) / 7 + (beg >> 14);
    if (beg >> 17 == end >> 17) return ((1 << 12) - 1) / 7 + (beg >> 17);
    if (beg >> 20 == end >> 20) return ((1 << 9) - 1) / 7 + (beg >> 20);
    if (beg >> 23 == end >> 23) return ((1 << 6) - 1) / 7 + (beg >> 23);
    if (beg >> 26 == end >> 26) return ((1 << 3) - 1) / 7 + (beg >> 26);
    return 0;
}

int bai_write_minimal(const char *bam_path, int32_t n_ref) {
    char path[4096];
    snprintf(path, sizeof(path), "%s.bai", bam_path);
    FILE *f = fopen(path, "wb");
    if (!f) return -1;
    unsigned char b4[4];
    fwrite("BAI\1", 1, 4, f);
    wr32(b4, (uint32_t)n_ref);
    fwrite(b4, 1, 4, f);
    wr32(b4, 0);
    for (int i = 0; i < n_ref; i++) {
        fwrite(b4, 1, 4, f); /* n_bin */
        fwrite(b4, 1, 4, f); /* n_intv */
    }
    return fclose(f);
}

int bai_loads(const char *bam_path) {
    char path[4096];
    bai_index idx;
    snprintf(path, sizeof(path), "%s.bai", bam_path);
    if (access(path, R_OK) != 0) {
        size_t n = strlen(bam_path);
        if (n <= 4 || strcmp(bam_path + n - 4, ".bam") != 0) return 0;
        snprintf(path, sizeof(path), "%.*s.bai", (int)(n - 4), bam_path);
    }
    if (bai_load(path, &idx) != 0) return 0;
    bai_free(&idx);
    return 1;
}

int bai_exists(const char *bam_path) {
    char path[4096];
    snprintf(path, sizeof(path), "%s.bai", bam_path);
    if (access(path, R_OK) == 0) return 1;
    size_t n = strlen(bam_path);
    if (n > 4 && strcmp(bam_path + n - 4, ".bam") == 0) {
        snprintf(path, sizeof(path), "%.*s.bai", (int)(n - 4), bam_path);
        if (access(path, R_OK) == 0) return 1;
    }
    return 0;
}

/* ---------------- virtual offsets and the BAI index ---------------- */

int64_t bgzf_tell(const bgzf_reader *r) {
    if (r->mt) return -1;
    if (r->blk_off >= r->blk_len) return r->next_coff << 16;
    return (r->blk_coff << 16) | r->blk_off;
}

int bgzf_seek(bgzf_reader *r, int64_t voff) {
    if (r->mt) return -1;
    const int64_t coff = voff >> 16;
    const int uoff = (int)(voff & 0xffff);
    if (fseek(r->fp, (long)coff, SEEK_SET) != 0) return -1;
    r->next_coff = coff;
    r->blk_len = r->blk_off = 0;
    r->eof = 0;
    if (uoff == 0) return 0;  /* the block is read on demand */
    if (bgzf_next_block(r) != 1 || uoff > r->blk_len) return -1;
    r->blk_off = uoff;
    return 0;
}

int32_t bam_end_pos(const bam_rec *b) {
    int32_t len = 0;
    if (!(b->flag & 4)) {
        for (int i = 0; i < b->n_cigar; i++) {
            const uint32_t c = bam_cigar_op(b, i);
            const int op = c & 15;
            if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) len += (int32_t)(c >> 4);
        }
    }
    return b->pos + (len > 0 ? len : 1);
}

/* growable per-reference index under construction */
typedef struct {
    uint32_t bin;
    int32_t n, cap;
    bai_chunk *c;
} bin_acc;
struct bai_racc {
    bin_acc *bins;
    int32_t n_bins, cap_bins;
    uint64_t *lin;
    int32_t n_lin;
    uint64_t off_beg, off_end, n_mapped, n_unmapped;
    int any;
    /* the current run of records with one bin (a chunk is flushed when it ends) */
    int in_run;
    uint32_t run_bin;
    uint64_t run_beg, run_end;
};

static bin_acc *acc_bin(bai_racc *R, uint32_t bin) {
    for (int i = R->n_bins - 1; i >= 0; i--)  /* bins recur close together in sorted input */
        if (R->bins[i].bin == bin) return &R->bins[i];
    if (R->n_bins == R->cap_bins) {
        R->cap_bins = R->cap_bins ? 2 * R->cap_bins : 64;
        R->bins = (bin_acc *)realloc(R->bins, sizeof(bin_acc) * R->cap_bins);
    }
    bin_acc *b = &R->bins[R->n_bins++];
    memset(b, 0, sizeof(*b));
    b->bin = bin;
    return b;
}

static void acc_chunk(bai_racc *R, uint32_t bin, uint64_t beg, uint64_t end) {
    bin_acc *b = acc_bin(R, bin);
    if (b->n > 0 && b->c[b->n - 1].end >> 16 == beg >> 16) {  /* adjacent within a block: extend */
        if (end > b->c[b->n - 1].end) b->c[b->n - 1].end = end;
        return;
    }
    if (b->n == b->cap) {
        b->cap = b->cap ? 2 * b->cap : 4;
        b->c = (bai_chunk *)realloc(b->c, sizeof(bai_chunk) * b->cap);
    }
    b->c[b->n].beg = beg;
    b->c[b->n].end = end;
    b->n++;
}

bai_racc *bai_racc_new(void) { return (bai_racc *)calloc(1, sizeof(bai_racc)); }

void bai_racc_free(bai_racc *R) {
    if (!R) return;
    for (int i = 0; i < R->n_bins; i++) free(R->bins[i].c);
    free(R->bins);
    free(R->lin);
    free(R);
}

void bai_racc_push(bai_racc *A, int32_t beg, int32_t end, uint64_t voff_beg, uint64_t voff_end, int unmapped) {
    if (beg < 0) beg = 0;
    const uint32_t bin = (uint32_t)bam_reg2bin(beg, end);
    if (A->in_run && A->run_bin != bin) acc_chunk(A, A->run_bin, A->run_beg, A->run_end);
    if (!A->in_run || A->run_bin != bin) {
        A->in_run = 1;
        A->run_bin = bin;
        A->run_beg = voff_beg;
    }
    A->run_end = voff_end;
    /* linear index: the first record overlapping each 16 kb window */
    const int w0 = beg >> 14, w1 = (end - 1) >> 14;
    if (w1 >= A->n_lin) {
        A->lin = (uint64_t *)realloc(A->lin, sizeof(uint64_t) * (w1 + 1));
        for (int w = A->n_lin; w <= w1; w++) A->lin[w] = UINT64_MAX;
        A->n_lin = w1 + 1;
    }
    for (int w = w0; w <= w1; w++)
        if (A->lin[w] == UINT64_MAX) A->lin[w] = voff_beg;
    if (!A->any) A->off_beg = voff_beg;
    A->any = 1;
    A->off_end = voff_end;
    if (unmapped) A->n_unmapped++;
    else A->n_mapped++;
}

void bai_racc_flush(bai_racc *A) {
    if (A->in_run) acc_chunk(A, A->run_bin, A->run_beg, A->run_end);
    A->in_run = 0;
}

static int cmp_bin_acc(const void *a, const void *b) {
    const uint32_t x = ((const bin_acc *)a)->bin, y = ((const bin_acc *)b)->bin;
    return x < y ? -1 : x > y;
}

static void put32(FILE *f, uint32_t v) {
    unsigned char b[4];
    wr32(b, v);
    fwrite(b, 1, 4, f);
}
static void put64(FILE *f, uint64_t v) {
    put32(f, (uint32_t)v);
    put32(f, (uint32_t)(v >> 32));
}

static uint64_t map_id(void *ctx, int ref, uint64_t v) { (void)ctx; (void)ref; return v; }

int bai_write_racc(const char *path, bai_racc **R, int n_ref, uint64_t n_no_coor,
                   uint64_t (*map)(void *ctx, int ref, uint64_t voff), void *ctx) {
    if (!map) map = map_id;
    FILE *f = fopen(path, "wb");
    if (!f) return -1;
    fwrite("BAI\1", 1, 4, f);
    put32(f, (uint32_t)n_ref);
    for (int t = 0; t < n_ref; t++) {
        bai_racc *A = R[t];
        if (!A) { put32(f, 0); put32(f, 0); continue; }
        bai_racc_flush(A);
        qsort(A->bins, A->n_bins, sizeof(bin_acc), cmp_bin_acc);
        put32(f, (uint32_t)(A->n_bins + (A->any ? 1 : 0)));
        for (int i = 0; i < A->n_bins; i++) {
            put32(f, A->bins[i].bin);
            put32(f, (uint32_t)A->bins[i].n);
            for (int c = 0; c < A->bins[i].n; c++) {
                put64(f, map(ctx, t, A->bins[i].c[c].beg));
                put64(f, map(ctx, t, A->bins[i].c[c].end));
            }
        }
        if (A->any) {  /* pseudo-bin 37450: offset span, mapped/unmapped counts */
            put32(f, 37450u);
            put32(f, 2u);
            put64(f, map(ctx, t, A->off_beg));
            put64(f, map(ctx, t, A->off_end));
            put64(f, A->n_mapped);
            put64(f, A->n_unmapped);
        }
        /* empty windows take the offset of the window before them
         * (a smaller offset only makes a query read more) */
        uint64_t prev = A->n_lin > 0 && A->lin[0] != UINT64_MAX ? A->lin[0] : 0;
        for (int w = 0; w < A->n_lin; w++) {
            if (A->lin[w] == UINT64_MAX) A->lin[w] = prev;
            prev = A->lin[w];
        }
        put32(f, (uint32_t)A->n_lin);
        for (int w = 0; w < A->n_lin; w++) put64(f, map(ctx, t, A->lin[w]));
    }
    put64(f, n_no_coor);
    return fclose(f) != 0 ? -1 : 0;
}

int bai_build(const char *bam_path) {
    bgzf_reader r;
    bam_hdr h;
    if (bgzf_open_read(&r, bam_path) != 0) return -1;
    if (bam_read_header(&r, &h) != 0) { bgzf_close_read(&r); return -1; }
    bai_racc **R = (bai_racc **)calloc(h.n_ref > 0 ? h.n_ref : 1, sizeof(bai_racc *));
    for (int t = 0; t < h.n_ref; t++) R[t] = bai_racc_new();
    bam_rec b;
    memset(&b, 0, sizeof(b));
    uint64_t n_no_coor = 0;
    int rc = 0, last_tid = -1, seen_unplaced = 0;
    int32_t last_pos = -1;
    int64_t off = bgzf_tell(&r);
    for (;;) {
        const int k = bam_read_rec(&r, &b);
        if (k < 0) { rc = -1; break; }
        const int64_t end_off = bgzf_tell(&r);
        if (k == 0) break;
        if (b.tid < 0) {  /* unplaced reads sort last */
            n_no_coor++;
            seen_unplaced = 1;
            off = end_off;
            continue;
        }
        /* a placed record after an unplaced one, or out of order: unsorted */
        if (seen_unplaced || b.tid >= h.n_ref || b.tid < last_tid || (b.tid == last_tid && b.pos < last_pos)) {
            rc = -1;
            break;
        }
        if (b.tid != last_tid && last_tid >= 0) bai_racc_flush(R[last_tid]);
        last_tid = b.tid;
        last_pos = b.pos;
        bai_racc_push(R[b.tid], b.pos < 0 ? 0 : b.pos, bam_end_pos(&b), (uint64_t)off, (uint64_t)end_off,
                      (b.flag & 4) != 0);
        off = end_off;
    }
    bam_free_rec(&b);
    bgzf_close_read(&r);
    if (rc == 0) {
        char path[4096];
        snprintf(path, sizeof(path), "%s.bai", bam_path);
        rc = bai_write_racc(path, R, h.n_ref, n_no_coor, NULL, NULL);
    }
    for (int t = 0; t < h.n_ref; t++) bai_racc_free(R[t]);
    free(R);
    bam_free_header(&h);
    return rc;
}

static int get32(FILE *f, uint32_t *v) {
    unsigned char b[4];
    if (fread(b, 1, 4, f) != 4) return -1;
    *v = rd32(b);
    return 0;
}
static int get64(FILE *f, uint64_t *v) {
    uint32_t lo, hi;
    if (get32(f, &lo) || get32(f, &hi)) return -1;
    *v = ((uint64_t)hi << 32) | lo;
    return 0;
}

void bai_free(bai_index *idx) {
    for (int t = 0; t < idx->n_ref; t++) {
        for (int i = 0; i < idx->ref[t].n_bin; i++) free(idx->ref[t].bin[i].chunk);
        free(idx->ref[t].bin);
        free(idx->ref[t].ioff);
    }
    free(idx->ref);
    memset(idx, 0, sizeof(*idx));
}

int bai_load(const char *bai_path, bai_index *idx) {
    memset(idx, 0, sizeof(*idx));
    FILE *f = fopen(bai_path, "rb");
    if (!f) return -1;
    char magic[4];
    uint32_t u;
    int rc = -1;
    if (fread(magic, 1, 4, f) != 4 || memcmp(magic, "BAI\1", 4) != 0 || get32(f, &u) || u > (1u << 24)) goto out;
    idx->n_ref = (int32_t)u;
    idx->ref = (bai_ref *)calloc(idx->n_ref ? idx->n_ref : 1, sizeof(bai_ref));
    for (int t = 0; t < idx->n_ref; t++) {
        bai_ref *R = &idx->ref[t];
        if (get32(f, &u) || u > (1u << 20)) goto out;
        R->bin = (bai_bin *)calloc(u ? u : 1, sizeof(bai_bin));
        R->n_bin = (int32_t)u;
        for (int i = 0; i < R->n_bin; i++) {
            uint32_t nc;
            if (get32(f, &R->bin[i].bin) || get32(f, &nc) || nc > (1u << 26)) goto out;
            R->bin[i].chunk = (bai_chunk *)malloc(sizeof(bai_chunk) * (nc ? nc : 1));
            R->bin[i].n_chunk = (int32_t)nc;
            for (uint32_t c = 0; c < nc; c++)
                if (get64(f, &R->bin[i].chunk[c].beg) || get64(f, &R->bin[i].chunk[c].end)) goto out;
        }
        if (get32(f, &u) || u > (1u << 20)) goto out;
        R->ioff = (uint64_t *)malloc(sizeof(uint64_t) * (u ? u : 1));
        R->n_intv = (int32_t)u;
        for (int w = 0; w < R->n_intv; w++)
            if (get64(f, &R->ioff[w])) goto out;
    }
    idx->has_no_coor = get64(f, &idx->n_no_coor) == 0;
    rc = 0;
out:
    fclose(f);
    if (rc) bai_free(idx);
    return rc;
}

static int cmp_chunk(const void *a, const void *b) {
    const uint64_t x = ((const bai_chunk *)a)->beg, y = ((const bai_chunk *)b)->beg;
    return x < y ? -1 : x > y;
}

int bai_query(const bai_index *idx, int tid, int beg, int end, bai_chunk **out) {
    *out = NULL;
    if (tid < 0 || tid >= idx->n_ref || end <= beg) return 0;
    if (beg < 0) beg = 0;
    const bai_ref *R = &idx->ref[tid];
    /* reg2bins (SAM v1 section 5.3): a bin of level l (first bin number
     * off[l], 2^shift[l] bases each) overlaps [beg, end) iff its index lies
     * between beg >> shift and (end - 1) >> shift -- tested per bin, so no
     * span is too long */
    static const uint32_t lv_off[6] = {0, 1, 9, 73, 585, 4681};
    static const int lv_shift[6] = {29, 26, 23, 20, 17, 14};
    const int e = end - 1;
    const uint64_t min_off = R->n_intv > 0 ? R->ioff[(beg >> 14) < R->n_intv ? (beg >> 14) : R->n_intv - 1] : 0;
    int n = 0, cap = 16;
    bai_chunk *c = (bai_chunk *)malloc(sizeof(bai_chunk) * cap);
    for (int i = 0; i < R->n_bin; i++) {
        const uint32_t bn = R->bin[i].bin;
        if (bn >= 37450u) continue;
        int l = 5;
        while (l > 0 && bn < lv_off[l]) l--;
        const uint32_t k = bn - lv_off[l];
        if (!(k >= (uint32_t)(beg >> lv_shift[l]) && k <= (uint32_t)(e >> lv_shift[l]))) continue;
        for (int q = 0; q < R->bin[i].n_chunk; q++) {
            if (R->bin[i].chunk[q].end <= min_off) continue;
            if (n == cap) {
                cap *= 2;
                c = (bai_chunk *)realloc(c, sizeof(bai_chunk) * cap);
            }
            c[n++] = R->bin[i].chunk[q];
        }
    }
    qsort(c, n, sizeof(bai_chunk), cmp_chunk);
    int m = 0;
    for (int i = 0; i < n; i++) {
        if (m > 0 && c[i].beg <= c[m - 1].end) {
            if (c[i].end > c[m - 1].end) c[m - 1].end = c[i].end;
        } else {
            c[m++] = c[i];
        }
    }
    *out = c;
    return m;
}

long bam_fetch(bgzf_reader *r, const bai_index *idx, int tid, int beg, int end,
               void (*visit)(void *ctx, const bam_rec *b), void *ctx) {
    bai_chunk *c = NULL;
    const int n = bai_query(idx, tid, beg, end, &c);
    if (n < 0) return -1;
    bam_rec b;
    memset(&b, 0, sizeof(b));
    long seen = 0;
    int rc = 0;
    for (int i = 0; i < n && rc == 0; i++) {
        if (bgzf_seek(r, (int64_t)c[i].beg) != 0) { rc = -1; break; }
        while ((uint64_t)bgzf_tell(r) < c[i].end) {
            const int k = bam_read_rec(r, &b);
            if (k <= 0) { rc = k; break; }
            if (b.tid != tid || b.pos >= end) { i = n; break; }  /* sorted: nothing later overlaps */
            if (bam_end_pos(&b) > beg) {
                visit(ctx, &b);
                seen++;
            }
        }
    }
    free(c);
    bam_free_rec(&b);
    return rc < 0 ? -1 : seen;
}
