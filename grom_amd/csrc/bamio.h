/*
 * bamio.h -- self-contained BGZF/BAM reader and writer on zlib.
 *
 * GROM links samtools/htslib 1.3.1 (Makefile:3-8) for `samopen`, `samread`,
 * `bam_aux_get` and `bam_index_load`; that source is absent from this image, so
 * the BAM layer is written here from the SAM/BAM specification.  Only what the
 * per-chromosome scan needs is provided: sequential record decode (the serial
 * `samread` stream of GROM.c:981-992), aux-tag lookup with htslib's skip rules,
 * and -- for the synthetic-data generator -- a BGZF/BAM writer and a minimal
 * BAI (GROM.c:22128-22138 only checks that an index loads).
 */
#ifndef GROM_AMD_BAMIO_H
#define GROM_AMD_BAMIO_H

#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* BAM flag bits (SAM spec section 1.4) */
#define GF_PAIRED 0x1
#define GF_PROPER 0x2
#define GF_UNMAP 0x4
#define GF_MUNMAP 0x8
#define GF_REVERSE 0x10
#define GF_MREVERSE 0x20
#define GF_READ1 0x40
#define GF_READ2 0x80
#define GF_SECONDARY 0x100
#define GF_QCFAIL 0x200
#define GF_DUP 0x400
#define GF_SUPPL 0x800

/* CIGAR op codes (BAM encoding) */
#define GC_MATCH 0
#define GC_INS 1
#define GC_DEL 2
#define GC_REF_SKIP 3
#define GC_SOFT_CLIP 4
#define GC_HARD_CLIP 5
#define GC_PAD 6
#define GC_EQUAL 7
#define GC_DIFF 8

struct bgzf_mt;
typedef struct bgzf_reader {
    FILE *fp;
    unsigned char *blk;     /* decompressed block */
    int blk_len, blk_off;
    unsigned char *cbuf;    /* compressed block */
    int eof;
    struct bgzf_mt *mt;     /* multi-threaded inflate (bgzf_set_threads), or NULL */
    int64_t blk_coff;       /* file offset of the current block (serial mode) */
    int64_t next_coff;      /* file offset of the block after it */
} bgzf_reader;

typedef struct bgzf_writer {
    FILE *fp;
    unsigned char *buf;
    int len;
    int level;
} bgzf_writer;

typedef struct bam_hdr {
    int32_t n_ref;
    char **ref_name;
    int32_t *ref_len;
    char *text;
    int32_t l_text;
} bam_hdr;

/* One decoded record.  `data` holds read_name, cigar, seq, qual, aux exactly as
 * in the BAM record (the htslib bam1_t data block). */
typedef struct bam_rec {
    int32_t tid, pos;
    uint8_t l_qname, mapq;
    uint16_t bin, n_cigar, flag;
    int32_t l_qseq, mtid, mpos, isize;
    int32_t data_len, m_data;
    uint8_t *data;
} bam_rec;

static inline char *bam_qname(const bam_rec *b) { return (char *)b->data; }
/* the CIGAR starts right after the read name, at any byte offset: read its
 * operations through bam_cigar_op (an unaligned uint32_t load is undefined) */
static inline const uint8_t *bam_cigar(const bam_rec *b) { return b->data + b->l_qname; }
static inline uint32_t bam_cigar_op(const bam_rec *b, int i) {
    uint32_t v;
    memcpy(&v, b->data + b->l_qname + 4 * (size_t)i, 4);
    return v;
}
static inline uint8_t *bam_seq(const bam_rec *b) { return b->data + b->l_qname + 4 * b->n_cigar; }
static inline uint8_t *bam_qual(const bam_rec *b) { return bam_seq(b) + ((b->l_qseq + 1) >> 1); }
static inline uint8_t *bam_aux(const bam_rec *b) { return bam_qual(b) + b->l_qseq; }
/* htslib bam_get_l_aux */
static inline int bam_l_aux(const bam_rec *b) { return b->data_len - (int)(bam_aux(b) - b->data); }
static inline int bam_seqi(const uint8_t *s, int i) { return (s[i >> 1] >> ((~i & 1) << 2)) & 0xf; }

/* htslib bam_nt16_rev_table: 4-bit code -> IUPAC char */
extern const char grom_nt16_rev[16];

int bgzf_open_read(bgzf_reader *r, const char *path);
void bgzf_close_read(bgzf_reader *r);
/* read exactly n bytes; returns n, 0 at clean EOF, -1 on error/truncation */
int bgzf_read(bgzf_reader *r, void *dst, int n);
/* inflate blocks on n worker threads (n <= 1: in the caller), read ahead in
 * file order and consumed in order; call before the first read.  0 on success. */
int bgzf_set_threads(bgzf_reader *r, int n);

int bgzf_open_write(bgzf_writer *w, const char *path, int level);
int bgzf_write(bgzf_writer *w, const void *src, int n);
int bgzf_flush_block(bgzf_writer *w);
int bgzf_close_write(bgzf_writer *w); /* writes the EOF marker block */
/* one BGZF block of `len` (<= 0xff00) payload bytes into out (room for
 * 65536 bytes); returns its size or -1.  Thread-safe. */
int bgzf_block_compress(const unsigned char *in, int len, unsigned char *out, int level);
/* the 28-byte BGZF end-of-file marker */
const unsigned char *bgzf_eof_block(void);
#define BGZF_PAYLOAD 0xff00

int bam_read_header(bgzf_reader *r, bam_hdr *h);
void bam_free_header(bam_hdr *h);
/* returns 1 on success, 0 at EOF, -1 on error (mirrors samread's >0 test) */
int bam_read_rec(bgzf_reader *r, bam_rec *b);
void bam_free_rec(bam_rec *b);

int bam_write_header(bgzf_writer *w, const bam_hdr *h);
int bam_write_rec(bgzf_writer *w, const bam_rec *b);

/* htslib bam_aux_get: pointer to the type byte of tag, or NULL */
uint8_t *bam_aux_find(const bam_rec *b, const char tag[2]);

/* virtual offset (compressed block offset << 16 | offset in the block) of
 * the next byte, canonical at block ends as htslib's bgzf_tell; -1 with
 * threaded inflate */
int64_t bgzf_tell(const bgzf_reader *r);
/* position the (serial) reader at a virtual offset: 0, or -1 */
int bgzf_seek(bgzf_reader *r, int64_t voff);

/* writes <bam>.bai with n_ref empty references (enough for GROM's serial mode) */
int bai_write_minimal(const char *bam_path, int32_t n_ref);

/* ---- BAI (SAM v1 section 5.2): the binning index with 16 kb linear index ---- */
typedef struct { uint64_t beg, end; } bai_chunk;
typedef struct {
    uint32_t bin;
    int32_t n_chunk;
    bai_chunk *chunk;
} bai_bin;
typedef struct {
    int32_t n_bin;
    bai_bin *bin;
    int32_t n_intv;
    uint64_t *ioff;
} bai_ref;
typedef struct {
    int32_t n_ref;
    bai_ref *ref;
    int has_no_coor;
    uint64_t n_no_coor;
} bai_index;

/* index a coordinate-sorted BAM as samtools index does: per reference the
 * bins with their chunks (adjacent chunks merged), the pseudo-bin 37450
 * (offset span, mapped/unmapped counts), the linear index, then the count of
 * unplaced reads; writes <bam>.bai.  0, or -1 (unsorted input, I/O error). */
int bai_build(const char *bam_path);
/* the same index built incrementally: one accumulator per reference fed
 * its records in file order (start/end virtual offsets of each record),
 * written with an optional offset map (the parallel writer records offsets
 * as block index << 16 | offset in block and maps them once the compressed
 * block sizes are known) */
typedef struct bai_racc bai_racc;
bai_racc *bai_racc_new(void);
void bai_racc_push(bai_racc *A, int32_t beg, int32_t end, uint64_t voff_beg, uint64_t voff_end, int unmapped);
void bai_racc_flush(bai_racc *A);
void bai_racc_free(bai_racc *A);
/* R[t] may be NULL (no records); 0 or -1 */
int bai_write_racc(const char *path, bai_racc **R, int n_ref, uint64_t n_no_coor,
                   uint64_t (*map)(void *ctx, int ref, uint64_t voff), void *ctx);
/* parse an index file; 0, or -1 */
int bai_load(const char *bai_path, bai_index *idx);
void bai_free(bai_index *idx);
/* the chunks that can hold records of tid overlapping [beg, end) (0-based),
 * sorted and merged; *out is malloc'd.  Returns the count, or -1. */
int bai_query(const bai_index *idx, int tid, int beg, int end, bai_chunk **out);
/* visit every record of tid overlapping [beg, end) through the index, in
 * file order; returns the number visited, or -1 */
long bam_fetch(bgzf_reader *r, const bai_index *idx, int tid, int beg, int end,
               void (*visit)(void *ctx, const bam_rec *b), void *ctx);
/* reference span of a record from its CIGAR (M/D/N/=/X), bam_endpos */
int32_t bam_end_pos(const bam_rec *b);
/* 1 if an index file for bam_path exists (<bam>.bai or <stem>.bai) */
int bai_exists(const char *bam_path);
/* 1 if that index file parses (bam_index_load's test, GROM.c:22128-22138) */
int bai_loads(const char *bam_path);

/* reg2bin from the SAM spec (0-based, end exclusive) */
int bam_reg2bin(int beg, int end);

#ifdef __cplusplus
}
#endif
#endif
