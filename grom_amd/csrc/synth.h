/*
 * synth.h -- deterministic synthetic genome + paired-end read generator.
 *
 * The bundled tilapia BAM of the reference is a missing blob,
 * so every benchmark and parity case is built from seeded synthetic data:
 * a FASTA with isochore GC, N telomeres, soft-masked stretches and
 * dinucleotide repeats; a diploid donor with SNVs and small indels; and
 * coordinate-sorted 2xL paired-end reads with sequencing errors, low base
 * qualities, low-MAPQ reads, soft clips, unmapped mates and PCR duplicates
 * (the knobs listed in SURVEY.md §8d).
 */
#ifndef GROM_AMD_SYNTH_H
#define GROM_AMD_SYNTH_H

#include <stdint.h>
#include "bamio.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SYNTH_MAX_CHR 64
#define SYNTH_MAX_PLOIDY 8

typedef struct synth_cfg {
    int n_chr;
    long chr_len[SYNTH_MAX_CHR];
    char chr_name[SYNTH_MAX_CHR][48];
    double coverage;      /* mean depth */
    double chr_cov[SYNTH_MAX_CHR]; /* per-chromosome depth; < 0 means `coverage` */
    int read_len;
    double insert_mean, insert_sd;
    double snv_rate, indel_rate;
    int max_indel;
    double err_rate;      /* per-base substitution error */
    double lowq_frac;     /* fraction of bases at lo_q */
    int hi_q, lo_q;
    double lowmapq_frac;  /* fraction of reads with MAPQ 0..19 */
    double softclip_frac; /* fraction of reads with a 5..30 bp soft clip */
    double munmap_frac;   /* fraction of pairs whose right read is unmapped */
    double dup_frac;      /* fraction of fragments emitted twice */
    int telomere_n;       /* N bases at both chromosome ends */
    double lower_frac;    /* fraction of reference in soft-masked blocks */
    double gc_lo, gc_hi;  /* isochore GC range */
    double repeat_rate;   /* dinucleotide repeat runs per base */
    int fasta_line;       /* FASTA line width */
    double cnv_rate;      /* copy-number regions per base (0 = none) */
    double multi_indel;   /* fraction of indels whose second haplotype carries
                             a different length (exercises the evidence
                             "other" slots); 0 keeps the random stream as is */
    long cnv_min, cnv_max;/* copy-number region length range */
    double sv_per_mb;     /* breakpoint SVs per Mb (DEL, DUP, INV, INS, and
                             CTX with the next chromosome), each with its
                             discordant pairs, split reads (SA:Z tags), soft
                             clips and unmapped mates; 0 = none */
    double sv_evidence;   /* evidence depth: pairs per breakpoint as a
                             fraction of the spanning-fragment depth */
    const char *ref_fasta; /* non-NULL: the chromosomes are this FASTA's records
                             (names, lengths and bases, case kept; written out
                             byte for byte), reads simulated from them */
    int ref_period;       /* > 0: the reference repeats one random pattern of
                             this length (every window has the same GC: one
                             GC bin takes every CNV depth sample) */
    int ploidy;           /* donor haplotypes (2; 4 for the -p 4 configuration):
                             variants sit on a random non-empty subset, so
                             allele fractions are k/ploidy */
    uint64_t seed;
    long max_emit;        /* > 0: synth_reads stops after this many records
                             (the first records of a chromosome, cheaply) */
} synth_cfg;

void synth_default_cfg(synth_cfg *c);
/* names and lengths of an existing FASTA's records into c (-F); 0 or -1 */
int synth_cfg_from_fasta(synth_cfg *c, const char *path);

/* Generate chromosome i's reference sequence (chr_len bytes, not NUL-terminated,
 * returned buffer has one extra NUL). Deterministic in (seed, i). */
char *synth_reference(const synth_cfg *c, int i);

typedef void (*synth_emit_fn)(void *ctx, const bam_rec *b);

/* Emit chromosome i's records in coordinate order (ties in generation order).
 * `ref` is the sequence from synth_reference.  Returns number of records. */
long synth_reads(const synth_cfg *c, int i, const char *ref, synth_emit_fn emit, void *ctx);

/* Write FASTA, BAM and minimal BAI for the whole genome. 0 on success. */
int synth_write_files(const synth_cfg *c, const char *fasta_path, const char *bam_path);

#ifdef __cplusplus
}
#endif
#endif
