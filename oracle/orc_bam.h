/*
 * orc_bam.h -- TEST INFRASTRUCTURE ONLY.  The oracle's own BAM reader.
 *
 * The oracle must not share the product's decoder (grom_amd/csrc/bamio.c): a
 * decoding bug there would otherwise reach both sides of every parity test.
 * This reader is written independently from the SAM/BAM specification (v1,
 * sections 4.1-4.2) and takes another route through the file: BGZF is a
 * concatenation of gzip members, so the whole BAM is read as one gzip stream
 * with zlib's gzread (which walks the members itself), and records are cut
 * from that byte stream.  The product parses BGZF blocks (BSIZE field) and
 * inflates each raw deflate payload; nothing below is taken from it.
 *
 * It exposes what grom_oracle.c reads from a record, under the names the
 * oracle uses (the htslib accessor names: bam_qname, bam_cigar, ...), which
 * mirror htslib's bam1_t layout that GROM.c reads (GROM.c:981-992).
 */
#ifndef ORC_BAM_H
#define ORC_BAM_H

#include <stdint.h>
#include <zlib.h>

/* FLAG bits, SAM v1 section 1.4 */
enum {
    GF_PAIRED = 0x1, GF_PROPER = 0x2, GF_UNMAP = 0x4, GF_MUNMAP = 0x8, GF_REVERSE = 0x10, GF_MREVERSE = 0x20,
    GF_READ1 = 0x40, GF_READ2 = 0x80, GF_SECONDARY = 0x100, GF_QCFAIL = 0x200, GF_DUP = 0x400, GF_SUPPL = 0x800
};
/* CIGAR operation codes "MIDNSHP=X" -> 0..8, BAM v1 section 4.2 */
enum { GC_MATCH = 0, GC_INS, GC_DEL, GC_REF_SKIP, GC_SOFT_CLIP, GC_HARD_CLIP, GC_PAD, GC_EQUAL, GC_DIFF };

typedef struct {
    gzFile gz;
} bgzf_reader;

typedef struct {
    int32_t n_ref;
    char **ref_name;
    int32_t *ref_len;
} bam_hdr;

typedef struct {
    int32_t tid, pos;
    uint8_t l_qname, mapq;
    uint16_t bin, n_cigar, flag;
    int32_t l_qseq, mtid, mpos, isize;
    int32_t data_len, m_data;
    uint8_t *data; /* read_name, cigar, seq, qual, aux (the variable part of the record) */
} bam_rec;

/* "=ACMGRSVTWYHKDBN": the 4-bit base codes of BAM v1 section 4.2.3 */
extern const char grom_nt16_rev[16];

int bgzf_open_read(bgzf_reader *r, const char *path);
void bgzf_close_read(bgzf_reader *r);
int bam_read_header(bgzf_reader *r, bam_hdr *h);
void bam_free_header(bam_hdr *h);
/* 1: a record, 0: end of file, -1: error */
int bam_read_rec(bgzf_reader *r, bam_rec *b);
void bam_free_rec(bam_rec *b);
/* the type byte of aux tag `tag`, or NULL (htslib bam_aux_get's result) */
uint8_t *bam_aux_find(const bam_rec *b, const char tag[2]);
/* 1 if <bam>.bai or <stem>.bai is readable (GROM.c:22128-22138 only loads it) */
int bai_exists(const char *bam_path);

static inline char *bam_qname(const bam_rec *b) { return (char *)b->data; }
static inline uint32_t *bam_cigar(const bam_rec *b) { return (uint32_t *)(b->data + b->l_qname); }
static inline uint8_t *bam_seq(const bam_rec *b) { return b->data + b->l_qname + 4 * (int)b->n_cigar; }
static inline uint8_t *bam_qual(const bam_rec *b) { return bam_seq(b) + (b->l_qseq + 1) / 2; }
static inline int bam_l_aux(const bam_rec *b) { return b->data_len - (b->l_qname + 4 * (int)b->n_cigar + (b->l_qseq + 1) / 2 + b->l_qseq); }
/* base i of a packed sequence: high nibble first */
static inline int bam_seqi(const uint8_t *s, int i) { return (i % 2 == 0) ? (s[i / 2] >> 4) : (s[i / 2] & 15); }

#endif
