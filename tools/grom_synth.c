/*
 * grom_synth -- command-line front end of the synthetic data generator
 * (grom_amd/csrc/synth.c).  Writes FASTA + BAM + minimal BAI.
 *
 *   grom_synth -o prefix [-L len[,len...]] [-c cov] [-l readlen] [-m mean] [-d sd]
 *              [-s seed] [-e err] [-Q lowmapq_frac] [-C clip_frac] [-U munmap_frac]
 *              [-D dup_frac] [-S snv_rate] [-I indel_rate] [-T telomere_n] [-n names]
 *              [-X sv_per_mb] [-E sv_evidence] [-P ploidy] [-R ref_period] [-F ref.fa]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "../grom_amd/csrc/synth.h"

int main(int argc, char **argv) {
    synth_cfg c;
    synth_default_cfg(&c);
    const char *prefix = NULL;
    const char *names = NULL, *ref_fasta = NULL;
    int opt;
    while ((opt = getopt(argc, argv, "o:L:c:l:m:d:s:e:Q:C:U:D:S:I:T:n:q:M:V:W:J:X:E:P:R:F:")) != -1) {
        switch (opt) {
        case 'o': prefix = optarg; break;
        case 'L': {
            c.n_chr = 0;
            char *s = strdup(optarg), *tok = strtok(s, ",");
            while (tok && c.n_chr < SYNTH_MAX_CHR) { c.chr_len[c.n_chr++] = atol(tok); tok = strtok(NULL, ","); }
            free(s);
            break;
        }
        case 'c': {
            /* one depth for all chromosomes, or a comma list per chromosome */
            char *d = strdup(optarg), *tok = strtok(d, ",");
            int k = 0;
            c.coverage = atof(optarg);
            while (tok && k < SYNTH_MAX_CHR) { c.chr_cov[k++] = atof(tok); tok = strtok(NULL, ","); }
            if (k == 1) c.chr_cov[0] = -1.0;
            free(d);
            break;
        }
        case 'l': c.read_len = atoi(optarg); break;
        case 'm': c.insert_mean = atof(optarg); break;
        case 'd': c.insert_sd = atof(optarg); break;
        case 's': c.seed = strtoull(optarg, NULL, 10); break;
        case 'e': c.err_rate = atof(optarg); break;
        case 'Q': c.lowmapq_frac = atof(optarg); break;
        case 'C': c.softclip_frac = atof(optarg); break;
        case 'U': c.munmap_frac = atof(optarg); break;
        case 'D': c.dup_frac = atof(optarg); break;
        case 'S': c.snv_rate = atof(optarg); break;
        case 'I': c.indel_rate = atof(optarg); break;
        case 'T': c.telomere_n = atoi(optarg); break;
        case 'n': names = optarg; break;
        case 'q': c.lowq_frac = atof(optarg); break;
        case 'M': c.lower_frac = atof(optarg); break;
        case 'P': c.ploidy = atoi(optarg); break;
        case 'R': c.ref_period = atoi(optarg); break;               /* periodic reference (one GC bin) */
        case 'F': ref_fasta = optarg; break;                        /* reads from an existing FASTA */                   /* donor haplotypes (allele fractions k/P) */
        case 'J': c.multi_indel = atof(optarg); break;              /* multi-allelic indel fraction */
        case 'X': c.sv_per_mb = atof(optarg); break;                /* breakpoint SVs per Mb */
        case 'E': c.sv_evidence = atof(optarg); break;              /* SV evidence depth factor */
        case 'V': c.cnv_rate = atof(optarg); break;                 /* CNV regions per base */
        case 'W': sscanf(optarg, "%ld,%ld", &c.cnv_min, &c.cnv_max); break; /* CNV length range */
        default:
            fprintf(stderr, "usage: grom_synth -o prefix [-L len,...] [-c cov] ...\n");
            return 2;
        }
    }
    if (!prefix) { fprintf(stderr, "grom_synth: -o prefix required\n"); return 2; }
    for (int i = 0; i < c.n_chr; i++) snprintf(c.chr_name[i], sizeof(c.chr_name[i]), "chr%d", i + 1);
    if (ref_fasta && synth_cfg_from_fasta(&c, ref_fasta) != 0) {
        fprintf(stderr, "grom_synth: cannot read %s\n", ref_fasta);
        return 1;
    }
    if (names) {
        char *s = strdup(names), *tok = strtok(s, ",");
        for (int i = 0; tok && i < c.n_chr; i++) {
            snprintf(c.chr_name[i], sizeof(c.chr_name[i]), "%s", tok);
            tok = strtok(NULL, ",");
        }
        free(s);
    }
    char fa[4096], bam[4096];
    snprintf(fa, sizeof(fa), "%s.fa", prefix);
    snprintf(bam, sizeof(bam), "%s.bam", prefix);
    if (synth_write_files(&c, fa, bam) != 0) { fprintf(stderr, "grom_synth: write failed\n"); return 1; }
    return 0;
}
