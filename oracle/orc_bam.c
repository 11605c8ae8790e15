/*
 * orc_bam.c -- TEST INFRASTRUCTURE ONLY.  The oracle's own BAM reader (see
 * orc_bam.h): the file as one gzip stream (zlib gzread), records cut from it
 * by their block_size, little-endian fields decoded byte by byte.
 */
#include "orc_bam.h"

#include <stdlib.h>
#include <string.h>
#include <unistd.h>

const char grom_nt16_rev[16] = "=ACMGRSVTWYHKDBN";

static int32_t le32(const uint8_t *p) {
    return (int32_t)((uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24);
}
static uint16_t le16(const uint8_t *p) { return (uint16_t)(p[0] | p[1] << 8); }

/* exactly n bytes from the stream: n, 0 at a clean end, -1 otherwise */
static int take(bgzf_reader *r, void *dst, int n) {
    int got = 0;
    while (got < n) {
        int k = gzread(r->gz, (char *)dst + got, (unsigned)(n - got));
        if (k < 0) return -1;
        if (k == 0) return got == 0 ? 0 : -1;
        got += k;
    }
    return n;
}

int bgzf_open_read(bgzf_reader *r, const char *path) {
    r->gz = gzopen(path, "rb");
    if (!r->gz) return -1;
    gzbuffer(r->gz, 1 << 20);
    return 0;
}

void bgzf_close_read(bgzf_reader *r) {
    if (r->gz) gzclose(r->gz);
    r->gz = NULL;
}

/* magic, l_text + text, n_ref, then per reference l_name + name + l_ref */
int bam_read_header(bgzf_reader *r, bam_hdr *h) {
    memset(h, 0, sizeof(*h));
    uint8_t v[4];
    char magic[4];
    if (take(r, magic, 4) != 4 || memcmp(magic, "BAM\001", 4) != 0) return -1;
    if (take(r, v, 4) != 4) return -1;
    int32_t l_text = le32(v);
    if (l_text < 0) return -1;
    char *text = (char *)malloc((size_t)l_text + 1);
    if (!text || (l_text && take(r, text, l_text) != l_text)) { free(text); return -1; }
    free(text);
    if (take(r, v, 4) != 4) return -1;
    h->n_ref = le32(v);
    if (h->n_ref < 0) return -1;
    h->ref_name = (char **)calloc((size_t)h->n_ref + 1, sizeof(char *));
    h->ref_len = (int32_t *)calloc((size_t)h->n_ref + 1, sizeof(int32_t));
    for (int32_t i = 0; i < h->n_ref; i++) {
        if (take(r, v, 4) != 4) return -1;
        int32_t l_name = le32(v);
        if (l_name < 1) return -1;
        h->ref_name[i] = (char *)malloc((size_t)l_name + 1);
        if (take(r, h->ref_name[i], l_name) != l_name) return -1;
        h->ref_name[i][l_name] = 0;
        if (take(r, v, 4) != 4) return -1;
        h->ref_len[i] = le32(v);
    }
    return 0;
}

void bam_free_header(bam_hdr *h) {
    for (int32_t i = 0; i < h->n_ref; i++) free(h->ref_name[i]);
    free(h->ref_name);
    free(h->ref_len);
    memset(h, 0, sizeof(*h));
}

/* block_size, then refID pos l_read_name mapq bin n_cigar_op flag l_seq
 * next_refID next_pos tlen (32 bytes), then the variable part */
int bam_read_rec(bgzf_reader *r, bam_rec *b) {
    uint8_t f[36];
    const int k = take(r, f, 4);
    if (k == 0) return 0;
    if (k < 0) return -1;
    const int32_t block = le32(f);
    if (block < 32 || take(r, f + 4, 32) != 32) return -1;
    b->tid = le32(f + 4);
    b->pos = le32(f + 8);
    b->l_qname = f[12];
    b->mapq = f[13];
    b->bin = le16(f + 14);
    b->n_cigar = le16(f + 16);
    b->flag = le16(f + 18);
    b->l_qseq = le32(f + 20);
    b->mtid = le32(f + 24);
    b->mpos = le32(f + 28);
    b->isize = le32(f + 32);
    b->data_len = block - 32;
    if (b->data_len > b->m_data) {
        uint8_t *d = (uint8_t *)realloc(b->data, (size_t)b->data_len);
        if (!d) return -1;
        b->data = d;
        b->m_data = b->data_len;
    }
    return take(r, b->data, b->data_len) == b->data_len ? 1 : -1;
}

void bam_free_rec(bam_rec *b) {
    free(b->data);
    memset(b, 0, sizeof(*b));
}

/* bytes of one value of an aux type (SAM v1 section 4.2.4) */
static int aux_width(uint8_t t) {
    switch (t) {
    case 'A': case 'c': case 'C': return 1;
    case 's': case 'S': return 2;
    case 'i': case 'I': case 'f': return 4;
    case 'd': return 8;
    default: return -1;
    }
}

uint8_t *bam_aux_find(const bam_rec *b, const char tag[2]) {
    const int n = bam_l_aux(b);
    uint8_t *a = b->data + (b->data_len - n), *end = b->data + b->data_len;
    while (end - a >= 3) {
        uint8_t *type = a + 2;
        if (a[0] == (uint8_t)tag[0] && a[1] == (uint8_t)tag[1]) return type;
        uint8_t *v = type + 1;
        if (*type == 'Z' || *type == 'H') {
            uint8_t *z = (uint8_t *)memchr(v, 0, (size_t)(end - v));
            if (!z) return NULL;
            a = z + 1;
        } else if (*type == 'B') {
            if (end - v < 5) return NULL;
            const int w = aux_width(v[0]);
            if (w < 0) return NULL;
            a = v + 5 + (size_t)w * (uint32_t)le32(v + 1);
        } else {
            const int w = aux_width(*type);
            if (w < 0) return NULL;
            a = v + w;
        }
    }
    return NULL;
}

int bai_exists(const char *bam_path) {
    size_t n = strlen(bam_path);
    char *p = (char *)malloc(n + 8);
    if (!p) return 0;
    strcpy(p, bam_path);
    strcat(p, ".bai");
    int ok = access(p, R_OK) == 0;
    if (!ok && n > 4 && strcmp(bam_path + n - 4, ".bam") == 0) {
        strcpy(p + n - 4, ".bai");
        ok = access(p, R_OK) == 0;
    }
    free(p);
    return ok;
}
