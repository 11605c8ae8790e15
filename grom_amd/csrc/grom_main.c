/*
 * grom_main.c -- `grom`, the drop-in command line for GROM's scan.
 *
 * Mirrors GROM's main (GROM.c:21865-22781) and find_disc_svs
 * (GROM.c:20440-21129): the same getopt string and defaults, the same output
 * files (OUT and OUT's .ctx.vcf sibling), the same chromosome selection and
 * order.  The per-chromosome scan (count_discordant_pairs, GROM.c:1432) runs
 * on the GPU through include/grom_amd.h.
 *
 * Not yet restated (the build reports them rather than guessing): -f
 * (tab-separated output).  Options that steer parts of the reference outside
 * the implemented scan rows are accepted and recorded.
 */
#include <ctype.h>
#include <dirent.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <execinfo.h>
#include <signal.h>
#include <time.h>
#include <unistd.h>
#include <sys/mman.h>

#include "../../include/grom_amd.h"
#include "bamio.h"
#include "ddecode.h"
#include "stream.h"
#include "pdecode.h"
#include "ddecode.h"

static const char *VERSION = "GROM, Version 1.0.1\n"; /* g_version_name, GROM.c:690 */

static void print_help(void) {
    /* GROM.c:1125-1181 */
    printf("\n%s", VERSION);
    printf("\nUsage: GROM -i <BAM input file> -r <REFERENCE input file> -o <output file> [optional parameters]\n");
    printf("\nRequired Parameters:\n");
    printf("\t-i \tBAM input file\n");
    printf("\t-r \tREFERENCE input file (fasta)\n");
    printf("\t-o \tSTRUCTURAL VARIANT output file\n");
    printf("\nOptional Parameters:\n");
    printf("\t-P \tthreads [1]\n");
    printf("\t-M \tturn on GROM's duplicate read filtering\n");
    printf("\t-q \tmapping quality threshold [35]\n");
    printf("\t-s \tminimum standard deviations for discordance [3]\n");
    printf("\t-v \tprobability threshold [0.001]\n");
    printf("\t-g \tgender (0=female,1=male) [0]\n");
    printf("\t-d \tminimum discordant pairs [3]\n");
    printf("\t-b \tbase phred quality score threshold [35]\n");
    printf("\t-n \tminimum SNV bases [3]\n");
    printf("\t-a \tminimum SNV ratio [0.2]\n");
    printf("\t-y \tmaximum unmapped gap or overlap for split reads [20]\n");
    printf("\t-z \tminimum split read mapped length (each split) [30]\n");
    printf("\t-S \tturn off split-read detection\n");
    printf("\t-p \tploidy [2]\n");
    printf("\t-e \tinsertion probability threshold [0.0000000001]\n");
    printf("\t-j \tminimum SV ratio [0.05]\n");
    printf("\t-k \tmaximum homopolymer (indels) [0.05]\n");
    printf("\t-m \tminimum indel ratio [0.125]\n");
    printf("\t-u \tmaximum evidence ratio (SV except insertion) [0.25]\n");
    printf("\t-A \tsampling rate [2]\n");
    printf("\t-V \tread depth p-value threshold [0.000001]\n");
    printf("\t-W \twindow minimum size [100]\n");
    printf("\t-X \twindow maximum size [10000]\n");
    printf("\t-Y \tminimum number of blocks [4]\n");
    printf("\t-Z \tblock minimum size [10000]\n");
    printf("\t-U \texcessive coverage threshold [2]\n");
    printf("\t-B \tchromosome maximum length [300000000]\n");
    printf("\t-D \tdinucleotide repeat minimum length [20]\n");
    printf("\t-E \tdinucleotide repeat minimum standard deviation [1.5]\n");
    printf("\t-K \tranks (0=no ranking,1=use ranks) [1]\n");
    printf("\t-L \tduplication coverage threshold [2]\n");
    printf("\nSee README file for additional help.\n");
    printf("\n");
}

static void header(FILE *f, const char *fasta_name, int ctx) {
    /* GROM.c:20517-20565 (main VCF) and GROM.c:22612-22651 (.ctx.vcf) */
    const char *pin = getenv("GROM_FILEDATE");
    fprintf(f, "##fileformat=VCFv4.2\n");
    if (pin) {
        fprintf(f, "##fileDate=%s\n", pin);
    } else {
        time_t t = time(NULL);
        struct tm tm = *localtime(&t);
        fprintf(f, "##fileDate=%d%d%d\n", tm.tm_year + 1900, tm.tm_mon + 1, tm.tm_mday);
    }
    fprintf(f, "##reference=%s\n", fasta_name);
    fprintf(f, "##ALT=<ID=DEL,Description=\"Deletion\">\n");
    fprintf(f, "##ALT=<ID=DUP,Description=\"Duplication\">\n");
    fprintf(f, "##ALT=<ID=INS,Description=\"Insertion\">\n");
    fprintf(f, "##ALT=<ID=INV,Description=\"Inversion\">\n");
    fprintf(f, "##INFO=<ID=END,Number=1,Type=Integer,Description=\"End position of the structural variant\">\n");
    if (!ctx) fprintf(f, "##FORMAT=<ID=GT,Number=1,Type=String,Description=\"Genotype\">\n");
    static const char *fmt_lines[][2] = {
        {"SPR", "Float\",Description=\"Probability of start breakpoint evidence occurring by chance"},
        {"EPR", "Float\",Description=\"Probability of end breakpoint evidence occurring by chance"},
        {"SEV", "Integer\",Description=\"Evidence supporting variant at start breakpoint"},
        {"EEV", "Integer\",Description=\"Evidence supporting variant at end breakpoint"},
        {"SRD", "Integer\",Description=\"Physical read depth at start breakpoint"},
        {"ERD", "Integer\",Description=\"Physical read depth at end breakpoint"},
        {"SCO", "Integer\",Description=\"Concordant pairs at start breakpoint"},
        {"ECO", "Integer\",Description=\"Concordant pairs at end breakpoint"},
        {"SOT", "Integer\",Description=\"Count of distinct SVs with evidence at start breakpoint"},
        {"EOT", "Integer\",Description=\"Count of distinct SVs with evidence at end breakpoint"},
        {"SSC", "Integer\",Description=\"Soft-clipped reads at start breakpoint"},
        {"ESC", "Integer\",Description=\"Soft-clipped at end breakpoint"},
        {"SFR", "Integer\",Description=\"Position of first read supporting start breakpoint"},
        {"SLR", "Integer\",Description=\"Position of last read supporting start breakpoint"},
        {"EFR", "Integer\",Description=\"Position of first read supporting end breakpoint"},
        {"ELR", "Integer\",Description=\"Position of last read supporting end breakpoint"},
        {"AF", "Float\",Description=\"Allele frequency (high mapping quality reads)"},
        {"PR", "Float\",Description=\"Probability of SNV evidence occurring by chance"},
        {"A", "Integer\",Description=\"A nucleotides (high mapping quality reads)"},
        {"C", "Integer\",Description=\"C nucleotides (high mapping quality reads)"},
        {"G", "Integer\",Description=\"G nucleotides (high mapping quality reads)"},
        {"T", "Integer\",Description=\"T nucleotides (high mapping quality reads)"},
        {"AL", "Integer\",Description=\"A nucleotides (low mapping quality reads)"},
        {"CL", "Integer\",Description=\"C nucleotides (low mapping quality reads)"},
        {"GL", "Integer\",Description=\"G nucleotides (low mapping quality reads)"},
        {"TL", "Integer\",Description=\"T nucleotides (low mapping quality reads)"},
        {"BQ", "Float\",Description=\"Average base quality (all reads)"},
        {"MQ", "Float\",Description=\"Average mapping quality (all reads)"},
        {"PIR", "Float\",Description=\"Average distance of SNV from DNA fragment end)"},
        {"FS", "Integer\",Description=\"SNV reads mapped to forward strand)"},
    };
    for (size_t i = 0; i < sizeof(fmt_lines) / sizeof(fmt_lines[0]); i++) {
        /* the Type= value is unquoted in GROM's text; rebuild it exactly */
        const char *rest = fmt_lines[i][1];
        const char *q = strchr(rest, '"');
        fprintf(f, "##FORMAT=<ID=%s,Number=1,Type=%.*s%s\">\n", fmt_lines[i][0], (int)(q - rest), rest, q + 1);
    }
    if (!ctx) {
        fprintf(f, "##FORMAT=<ID=SD,Number=1,Type=Float,Description=\"CNV standard deviation\"\n");
        fprintf(f, "##FORMAT=<ID=Z,Number=1,Type=Float,Description=\"CNV probability score\"\n");
        fprintf(f, "##FORMAT=<ID=CN,Number=1,Type=Float,Description=\"CNV copy number\"\n");
        fprintf(f, "##FORMAT=<ID=CS,Number=1,Type=Float,Description=\"CNV copy number standard deviation\"\n");
    }
    fprintf(f, "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\n");
}

/* -f: the insert statistics and the column header instead of the VCF header
 * (GROM.c:20566-20671) */
static const char TAB_COLUMNS[] =
    "SV\tChromosome\tStart (Tumor)\tEnd (Tumor)\tLength (Tumor)\tP-val (Start, Tumor)\t"
    "P-val (End, Tumor)\tConcordant Pairs (Start, Tumor)\tConcordant Pairs (End, Tumor)\t"
    "Start or End?\tRead Depth (High MapQ, Normal)\tRead Depth (Low MapQ, Normal)\t"
    "Concordant Pairs (Normal)\tINS (Normal)\tDEL (For, Normal)\tDEL (Rev, Normal)\t"
    "DEL (For, Length, Normal)\tDEL (Rev, Length, Normal)\tDUP (Rev, Normal)\tDUP (For, Normal)\t"
    "DUP (Rev, Length, Normal)\tDUP (For, Length, Normal)\tINV (For, Start, Normal)\t"
    "INV (Rev, Start, Normal)\tINV (For, End, Normal)\tINV (Rev, End, Normal)\t"
    "INV (For, Start, Length, Normal)\tINV (Rev, Start, Length, Normal)\t"
    "INV (For, End, Length, Normal)\tINV (Rev, End, Length, Normal)\tUnmapped Mate (For, Normal)\t"
    "Unmapped Mate (Rev, Normal)\tSoft-clipping (Left, Normal)\tSoft-clipping (Right, Normal)\t"
    "Soft-clipping Read Depth (Left, Normal)\tSoft-clipping Read Depth (Right, Normal)\t"
    "Soft-clipping Read Depth (Left+Right, Normal)\tINS Indel (Normal)\tDEL Indel (Start, Normal)\t"
    "DEL Indel (End, Normal)\tDEL Indel (Start, Length, Normal)\tDEL Indel (End, Length, Normal)\t"
    "CTX Soft-clipping (Left, Normal)\tCTX Soft-clipping (Right, Normal)\t"
    "CTX Soft-clipping Read Depth (Left, Normal)\tCTX Soft-clipping Read Depth (Right, Normal)\t"
    "CTX Soft-clipping Read Depth (Left+Right, Normal)\tIndel Soft-clipping (Left, Normal)\t"
    "Indel Soft-clipping (Right, Normal)\tIndel Soft-clipping Read Depth (Left, Normal)\t"
    "Indel Soft-clipping Read Depth (Right, Normal)\t"
    "Indel Soft-clipping Read Depth (Left+Right, Normal)\t"
    "Soft-clipping (Left Max including CTX, Normal)\t"
    "Soft-clipping (Right Max including CTX, Normal)\tOther (Number of Non-Empty, Normal)\t"
    "CTX (For, Normal)\tCTX (Rev, Normal)\tSV Overlap (Normal)\tOther (Number of Non-Empty, Tumor)\t"
    "Read Start (Start, Tumor)\tRead End (Start, Tumor)\tRead Start (End, Tumor)\t"
    "Read End (End, Tumor)\tDEL Read Start (For/Rev, Normal)\tDEL Read End (For/Rev, Normal)\t"
    "DUP Read Start (Rev/For, Normal)\tDUP Read End (Rev/For, Normal)\tINV Read Start (For, Normal)\t"
    "INV Read End (For, Normal)\tINV Read Start (Rev, Normal)\tINV Read End (Rev, Normal)\t"
    "CTX Read Start (For, Normal)\tCTX Read End (For, Normal)\tCTX Read Start (Rev, Normal)\t"
    "CTX Read End (Rev, Normal)\tMate Chr (CTX only, Tumor)\tMate Pos (CTX only, Tumor)\t"
    "Mate Chr (For, Normal)\tMate Pos (For, Normal)\tMate Chr (Rev, Normal)\tMate Pos (Rev, Normal)\t"
    "Reference Base\tSNV Base (Tumor)\tSNV Ratio (Tumor)\tSNV Count (A, Tumor)\t"
    "SNV Count (C, Tumor)\tSNV Count (G, Tumor)\tSNV Count (T, Tumor)\tSNV Count (A, Normal)\t"
    "SNV Count (C, Normal)\tSNV Count (G, Normal)\tSNV Count (T, Normal)\t\n";
static void tab_header(FILE *f, const grom_params *P) {
    fprintf(f, "%d\t%d\t%d\t%d\n", P->insert_mean, P->insert_min_size, P->insert_max_size, P->lseq);
    fputs(TAB_COLUMNS, f);
}

typedef struct {
    int fasta_idx;
    int32_t tid;
    char *ref;
    long len;
    char name[GROM_MAX_CHR_NAME_LEN + 1];
    char *target; /* BAM name the SA/XP chromosome test compares with (GROM.c:1894-1961, 7431) */
} chrom_plan;

static int g_plan_only = 0; /* GROM_PLAN_ONLY: report the record plan, no GPU */
static const char *g_side_base; /* -o name: the -N side files are named after it */

static double clock_gettime_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* seconds from this process's start (the kernel's start time, clock ticks
 * since boot) to now: what loading the program and the library took before
 * the CLI's first line; -1 when /proc does not say */
static double since_process_start(void) {
    FILE *f = fopen("/proc/self/stat", "r");
    if (!f) return -1.0;
    char buf[2048];
    const size_t n = fread(buf, 1, sizeof(buf) - 1, f);
    fclose(f);
    buf[n] = 0;
    const char *p = strrchr(buf, ')'); /* (the command name may hold spaces) */
    if (!p) return -1.0;
    unsigned long long start = 0;
    int field = 2;
    for (const char *q = p + 1; *q && field < 22; q++)
        if (*q == ' ') {
            field++;
            if (field == 22) start = strtoull(q + 1, NULL, 10);
        }
    struct timespec t;
    clock_gettime(CLOCK_BOOTTIME, &t);
    const long hz = sysconf(_SC_CLK_TCK);
    if (start == 0 || hz <= 0) return -1.0;
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec - (double)start / (double)hz;
}

typedef struct {
    char *p;
    size_t len, cap;
} textbuf;

static void textbuf_add(textbuf *t, const char *s, size_t n) {
    if (t->len + n + 1 > t->cap) {
        size_t nc = t->cap ? 2 * t->cap : 1 << 16;
        while (nc < t->len + n + 1) nc *= 2;
        t->p = realloc(t->p, nc);
        t->cap = nc;
    }
    memcpy(t->p + t->len, s, n);
    t->len += n;
    t->p[t->len] = 0;
}

/* main's translocation post-pass (GROM.c:22400-22770): the raw CTX rows of
 * every chromosome are read back, each breakpoint is paired with a mate row
 * (its chromosome and mate chromosome swapped, positions within
 * insert_max - 2*lseq, orientations consistent), the weaker of two nearby
 * paired rows is dropped with its mate, and the rest are written as BND rows. */
typedef struct {
    int type, chr, pos, rd, conc, other, mchr, mpos, rs, re, mateid, keep;
    double binom, ev, hez;
} ctx_row_t;

static void ctx_postpass(const char *raw, size_t raw_len, const bam_hdr *hdr, int Mx, int glseq, int vcf, FILE *out) {
    int n_t = hdr->n_ref;
    char **lc = calloc(n_t > 0 ? n_t : 1, sizeof(char *));
    for (int a = 0; a < n_t; a++) {
        size_t L = strlen(hdr->ref_name[a]);
        lc[a] = malloc(L + 1);
        for (size_t b = 0; b <= L; b++) lc[a][b] = (char)tolower((unsigned char)hdr->ref_name[a][b]);
    }
    int n = 0, cap = 1024;
    ctx_row_t *rw = calloc(cap, sizeof(ctx_row_t));
    size_t off = 0;
    while (raw && off < raw_len) {
        const char *e = memchr(raw + off, '\n', raw_len - off);
        size_t ll = e ? (size_t)(e - (raw + off)) : raw_len - off;
        char *line = malloc(ll + 1);
        memcpy(line, raw + off, ll);
        line[ll] = 0;
        off += ll + (e ? 1 : 0);
        if (n == cap) { cap *= 2; rw = realloc(rw, cap * sizeof(ctx_row_t)); }
        ctx_row_t *q = &rw[n++];
        memset(q, 0, sizeof(*q));
        char *save = NULL, *t = strtok_r(line, "\t", &save);
        q->type = t ? (strcmp(t, "CTX_F") == 0 ? 6 : strcmp(t, "CTX_R") == 0 ? 7 : -1) : -1; /* g_sv_types */
        t = strtok_r(NULL, "\t", &save);
        q->chr = -1;
        if (t) {
            char tl[1024];
            size_t L = strlen(t);
            if (L > sizeof(tl) - 1) L = sizeof(tl) - 1;
            for (size_t b = 0; b < L; b++) tl[b] = (char)tolower((unsigned char)t[b]);
            tl[L] = 0;
            for (int a = 0; a < n_t; a++)
                if (strcmp(lc[a], tl) == 0) { q->chr = a; break; }
        }
        int *ifld[] = {&q->pos, NULL, NULL, &q->rd, &q->conc, &q->other, &q->mchr, &q->mpos, &q->rs, &q->re, NULL};
        double *dfld[] = {NULL, &q->binom, &q->ev, NULL, NULL, NULL, NULL, NULL, NULL, NULL, &q->hez};
        for (int k = 0; k < 11; k++) {
            t = strtok_r(NULL, "\t", &save);
            if (ifld[k]) *ifld[k] = t ? atoi(t) : 0;
            else *dfld[k] = t ? atof(t) : 0;
        }
        free(line);
    }
    const int span = Mx - 2 * glseq;
    for (int b = 0; b < n; b++) { rw[b].keep = 0; rw[b].mateid = -1; }
    for (int b = 0; b < n; b++)
        for (int c = 0; c < n; c++) {
            if (!(rw[b].chr == rw[c].mchr && rw[c].chr == rw[b].mchr)) continue;
            if (!(abs(rw[b].pos - abs(rw[c].mpos)) < span && abs(rw[c].pos - abs(rw[b].mpos)) < span)) continue;
            const int bo = (rw[b].type == 6 && rw[c].mpos >= 0) || (rw[b].type == 7 && rw[c].mpos < 0);
            const int co = (rw[c].type == 6 && rw[b].mpos >= 0) || (rw[c].type == 7 && rw[b].mpos < 0);
            if (bo && co) {
                rw[b].keep = 1;
                rw[b].mateid = c;
                rw[b].mpos = rw[b].mpos < 0 ? -rw[c].pos : rw[c].pos;
            }
        }
    for (int b = 0; b < n; b++)
        for (int c = 0; c < n; c++) {
            if (b == c || rw[b].chr != rw[c].chr || rw[b].mchr != rw[c].mchr) continue;
            if (!(abs(rw[b].pos - rw[c].pos) < span && abs(abs(rw[b].mpos) - abs(rw[c].mpos)) < span)) continue;
            if (rw[b].keep == 1 && rw[c].keep == 1 && (rw[b].binom > rw[c].binom || (rw[b].binom == rw[c].binom && b > c))) {
                rw[b].keep = 0;
                if (rw[b].mateid >= 0) rw[rw[b].mateid].keep = 0;
            }
        }
    printf("Translocations before filter: %d\n", n);
    int n2 = 0;
    for (int b = 0; b < n; b++) {
        const ctx_row_t *q = &rw[b];
        if (q->keep != 1) continue;
        n2++;
        char bnd[64];
        const char *mn = (q->mchr >= 0 && q->mchr < n_t) ? lc[q->mchr] : "";
        if (!vcf) { /* -f rows, GROM.c:22734 (g_sv_types[6] "CTX_F", [7] "CTX_R", GROM.c:867) */
            fprintf(out, "%s\t%s\t%d\t%d\t%d\t%e\t%.1f\t%d\t%d\t%d\t%s\t%d\t%d\t%d\t%e\n", q->type == 6 ? "CTX_F" : "CTX_R",
                    (q->chr >= 0 && q->chr < n_t) ? lc[q->chr] : "", q->pos, b, q->mateid, q->binom, q->ev, q->rd, q->conc,
                    q->other, mn, q->mpos, q->rs, q->re, q->hez);
            continue;
        }
        const int am = abs(q->mpos);
        if (q->type == 6) snprintf(bnd, sizeof(bnd), q->mpos < 0 ? "N[%s:%d[" : "N]%s:%d]", mn, am);
        else snprintf(bnd, sizeof(bnd), q->mpos < 0 ? "[%s:%d[N" : "]%s:%d]N", mn, am);
        fprintf(out, "%s\t%d\t%d\tN\t%s\t.\t.\tSVTYPE=BND;MATEID=%d\tSPR:SEV:SRD:SCO:SOT:SFR:SLR:SHPR\t%e:%.1f:%d:%d:%d:%d:%d:%e\n",
                (q->chr >= 0 && q->chr < n_t) ? lc[q->chr] : "", q->pos + 1, b, bnd, q->mateid, q->binom, q->ev, q->rd,
                q->conc, q->other, q->rs + 1, q->re + 1, q->hez);
    }
    printf("Translocations after filter: %d\n", n2);
    for (int a = 0; a < n_t; a++) free(lc[a]);
    free(lc);
    free(rw);
}

int grom_ctx_postpass(const char *raw, size_t raw_len, const char *const *target_names, int32_t n_targets,
                      int32_t insert_max, int32_t lseq, grom_out *out) {
    if (!out || n_targets < 0 || (n_targets > 0 && !target_names)) {
        grom_set_last_error("grom_ctx_postpass: bad argument");
        return GROM_E_ARG;
    }
    bam_hdr h;
    memset(&h, 0, sizeof(h));
    h.n_ref = n_targets;
    h.ref_name = (char **)target_names;
    char *buf = NULL;
    size_t len = 0;
    FILE *f = open_memstream(&buf, &len);
    if (!f) { grom_set_last_error("grom_ctx_postpass: no memory"); return GROM_E_NOMEM; }
    ctx_postpass(raw, raw_len, &h, insert_max, lseq, 1, f);
    fclose(f);
    if (out->ctx_len + len + 1 > out->ctx_cap) {
        size_t nc = out->ctx_cap ? out->ctx_cap : 4096;
        while (nc < out->ctx_len + len + 1) nc *= 2;
        char *p = realloc(out->ctx, nc);
        if (!p) { free(buf); grom_set_last_error("grom_ctx_postpass: no memory"); return GROM_E_NOMEM; }
        out->ctx = p;
        out->ctx_cap = nc;
    }
    memcpy(out->ctx + out->ctx_len, buf, len);
    out->ctx_len += len;
    out->ctx[out->ctx_len] = 0;
    free(buf);
    return GROM_OK;
}

/* ---- one chromosome's scan, from either input path ----
 * serial path: `batch` holds the chromosome's records in host memory;
 * streamed path: `stage` holds them in HBM (pdecode.c) and `facts` the
 * serial stream's facts about them. */
typedef struct {
    chrom_plan *cp;
    grom_batch batch;
    int has_batch;
    grom_stage *stage;
    pd_chrom_facts facts;
    pd_session *pd;        /* releases the stage after the scan */
    int stage_released;    /* the scan gave the stage back before its CNV path */
    int k;                 /* plan index (trace) */
    int device;            /* the GPU the stage lives on, -1: any */
    char *text, *ctx_text;
    size_t text_len, ctx_len;
    int rc, ready, done, taken;
    char err[512];
} grom_job;

static void write_dumps(int slot, const chrom_plan *cp, const grom_chrom *ch, const grom_reads *host_rd,
                        grom_stage *stage, const grom_params *P) {
    /* test hook: per-base counters and caf depth, same files as the oracle's */
    const char *dump = getenv("GROM_DUMP");
    int32_t first = 0;
    int32_t lo = P->one_base_rd_len / 4 + 1;
    if (lo < 2 * P->insert_max_size + 1) lo = 2 * P->insert_max_size + 1;
    int64_t n_eval = (ch->p_last >= lo) ? (int64_t)ch->p_last - lo + 1 : 0;
    int32_t *cnt = malloc(sizeof(int32_t) * GROM_NCOUNT * (n_eval > 0 ? n_eval : 1));
    int32_t *caf = malloc(sizeof(int32_t) * 3 * cp->len);
    int rc = stage ? grom_debug_counts_staged(slot, stage, ch, &first, cnt, GROM_NCOUNT * n_eval, caf)
                   : grom_debug_counts(slot, ch, host_rd, &first, cnt, GROM_NCOUNT * n_eval, caf);
    if (rc == GROM_OK) {
        char path[4096];
        snprintf(path, sizeof(path), "%s.%s.cnt", dump, cp->name);
        FILE *f = fopen(path, "wb");
        if (f) { fwrite(cnt, sizeof(int32_t) * GROM_NCOUNT, n_eval, f); fclose(f); }
        snprintf(path, sizeof(path), "%s.%s.caf", dump, cp->name);
        f = fopen(path, "wb");
        if (f) { fwrite(caf, sizeof(int32_t), 3 * cp->len, f); fclose(f); }
        /* indel evidence of the same scan (row A7) */
        int64_t n_ind = grom_debug_indels(slot, NULL, 0);
        grom_indel_rec *ind = n_ind > 0 ? malloc(sizeof(grom_indel_rec) * n_ind) : NULL;
        if (n_ind >= 0 && (n_ind == 0 || (ind && grom_debug_indels(slot, ind, n_ind) == n_ind))) {
            snprintf(path, sizeof(path), "%s.%s.ind", dump, cp->name);
            f = fopen(path, "wb");
            if (f) { if (n_ind) fwrite(ind, sizeof(grom_indel_rec), n_ind, f); fclose(f); }
        } else {
            fprintf(stderr, "grom: indel dump of %s failed: %s\n", cp->name, grom_last_error());
        }
        free(ind);
        /* breakpoint cluster records (rows A8/A9; the scan keeps them when
         * GROM_SV_DEBUG is set) */
        int64_t n_sv = grom_debug_sv(slot, NULL, 0);
        grom_sv_rec *svr = n_sv > 0 ? malloc(sizeof(grom_sv_rec) * n_sv) : NULL;
        if (n_sv >= 0 && (n_sv == 0 || (svr && grom_debug_sv(slot, svr, n_sv) == n_sv))) {
            snprintf(path, sizeof(path), "%s.%s.sv", dump, cp->name);
            f = fopen(path, "wb");
            if (f) { if (n_sv) fwrite(svr, sizeof(grom_sv_rec), n_sv, f); fclose(f); }
        }
        free(svr);
    } else {
        fprintf(stderr, "grom: counter dump of %s failed: %s\n", cp->name, grom_last_error());
    }
    free(cnt);
    free(caf);
}

static int chrom_wanted(const char *name);

static uint32_t chrom_seed(void) {
    /* srand(time()) per chromosome, GROM.c:1584; GROM_SEED pins it */
    const char *e = getenv("GROM_SEED");
    return e ? (uint32_t)strtoul(e, NULL, 10) : (uint32_t)time(NULL);
}

/* test hook (GROM_STAGE_DIGEST): the staged input of a chromosome, copied
 * back to the host, as the plan-only line prints it (the device decoder's
 * output against the host decoder's, tests/test_gpu_parity.py) */
static void stage_digest_line(grom_stage *st, const grom_chrom *ch, int device) {
    grom_chrom dc;
    grom_reads d, h;
    if (grom_stage_view(st, ch, &dc, &d) != GROM_OK) return;
    memset(&h, 0, sizeof(h));
    h.n = d.n;
    h.n_cigar_ops = d.n_cigar_ops;
    h.n_bases = d.n_bases;
    h.n_aux = d.n_aux;
    h.n_drop = d.n_drop;
    const int64_t n = d.n, nd = d.n_drop;
#define DL(f, T, cnt)                                                                     \
    T *f##_h = (T *)malloc(sizeof(T) * (size_t)((cnt) > 0 ? (cnt) : 1));                   \
    if ((cnt) > 0 && d.f) grom_copy_d2h(f##_h, d.f, sizeof(T) * (size_t)(cnt), device);   \
    h.f = f##_h;
    DL(pos, int32_t, n) DL(flag, uint16_t, n) DL(mapq, uint8_t, n) DL(mtid, int32_t, n) DL(mpos, int32_t, n)
    DL(isize, int32_t, n) DL(l_qseq, int32_t, n) DL(cigar_off, uint32_t, n + 1) DL(base_off, int64_t, n)
    DL(name_id, uint32_t, n) DL(drop_pos, int32_t, nd) DL(drop_lq, int32_t, nd) DL(drop_before, int64_t, nd)
    /* absolute offsets: the whole CIGAR / base arrays */
    DL(cigar, uint32_t, d.n_cigar_ops) DL(qual, uint8_t, d.n_bases) DL(seq, uint8_t, d.n_bases / 2)
    DL(aux, grom_aux, d.n_aux)
#undef DL
    int32_t *ai = NULL;
    if (d.aux_idx) {
        ai = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
        if (n > 0) grom_copy_d2h(ai, d.aux_idx, sizeof(int32_t) * (size_t)n, device);
        h.aux_idx = ai;
    }
    printf("stage %s tid=%d reads=%lld n_skip=%d p_last=%d lseq_tail=%d digest=%016llx\n", ch->name, ch->tid,
           (long long)n, ch->n_skip, ch->p_last, ch->lseq_tail, (unsigned long long)pd_digest(&h));
    free((void *)h.pos); free((void *)h.flag); free((void *)h.mapq); free((void *)h.mtid); free((void *)h.mpos);
    free((void *)h.isize); free((void *)h.l_qseq); free((void *)h.cigar_off); free((void *)h.base_off);
    free((void *)h.name_id); free((void *)h.drop_pos); free((void *)h.drop_lq); free((void *)h.drop_before);
    free((void *)h.cigar); free((void *)h.qual); free((void *)h.seq); free((void *)h.aux); free(ai);
}

/* Scan one chromosome on context `slot`; its VCF rows go to j->text (malloc'd). */
/* the scan no longer reads the job's stage: the decoder may refill it while
 * the CNV path runs (grom_stage_on_consumed) */
static void job_stage_consumed(void *arg, grom_stage *st) {
    grom_job *j = (grom_job *)arg;
    j->stage_released = 1;
    pd_release_stage(j->pd, st);
}

static int scan_job(int slot, grom_job *j, const grom_params *P, int verbose) {
    chrom_plan *cp = j->cp;
    j->text = j->ctx_text = NULL;
    j->text_len = j->ctx_len = 0;
    if (!chrom_wanted(cp->name)) return GROM_OK; /* serial path: another rank's chromosome */
    grom_chrom ch;
    memset(&ch, 0, sizeof(ch));
    grom_reads rd;
    memset(&rd, 0, sizeof(rd));
    int64_t n_reads;
    if (j->has_batch) {
        grom_batch *b = &j->batch;
        grom_batch_finish(b, P->one_base_rd_len / 4 + 1, P->overlap_mult, P->insert_max_size);
        if (g_plan_only) {
            grom_batch_view(b, &rd);
            printf("plan %s tid=%d reads=%lld n_skip=%d p_last=%d lseq_tail=%d digest=%016llx\n", cp->name, cp->tid,
                   (long long)b->n, b->n_skip, b->p_last, b->lseq_tail, (unsigned long long)pd_digest(&rd));
            return GROM_OK;
        }
        ch.lseq_tail = b->lseq_tail;
        ch.n_skip = b->n_skip;
        ch.p_last = b->p_last;
        grom_batch_view(b, &rd);
        n_reads = b->n;
    } else {
        if (g_plan_only) { /* streamed plan-only (host tests): the decoder's host mirror */
            pd_mirror_view(j->pd, j->k, &rd);
            printf("plan %s tid=%d reads=%lld n_skip=%d p_last=%d lseq_tail=%d digest=%016llx\n", cp->name, cp->tid,
                   (long long)j->facts.n_reads, j->facts.n_skip, j->facts.p_last, j->facts.lseq_tail,
                   (unsigned long long)pd_digest(&rd));
            return GROM_OK;
        }
        ch.lseq_tail = j->facts.lseq_tail;
        ch.n_skip = j->facts.n_skip;
        ch.p_last = j->facts.p_last;
        n_reads = j->facts.n_reads;
    }
    ch.ref = cp->ref;
    ch.len = cp->len;
    ch.name = cp->name;
    ch.tid = cp->tid;
    ch.cnv = cp->tid >= 0; /* detect_del_dup runs for a matched target, GROM.c:16633 */
    ch.seed = chrom_seed();
    if (!j->has_batch && getenv("GROM_STAGE_DIGEST")) stage_digest_line(j->stage, &ch, j->device);
    grom_out out = {0};
    grom_stats st = {0};
    /* the pileup's input sizes (the verbose line) before the stage is given back */
    int64_t n_cig = rd.n_cigar_ops, n_b = rd.n_bases;
    if (!j->has_batch) {
        grom_chrom dc;
        grom_reads dr;
        if (grom_stage_view(j->stage, &ch, &dc, &dr) == GROM_OK) {
            n_cig = dr.n_cigar_ops;
            n_b = dr.n_bases;
        }
        /* (GROM_DUMP reads the stage after the scan: it keeps it) */
        grom_stage_on_consumed(j->stage, j->pd && !getenv("GROM_DUMP") ? job_stage_consumed : NULL, j);
    }
    if (j->pd) pd_trace(j->pd, PD_EV_SCAN, j->k, 0);
    int rc = j->has_batch ? grom_scan_chrom(slot, &ch, &rd, &out, &st)
                          : grom_scan_chrom_staged(slot, j->stage, &ch, &out, &st);
    if (j->pd) pd_trace(j->pd, PD_EV_SCAN, j->k, 1);
    if (rc != GROM_OK) {
        fprintf(stderr, "grom: scan of %s failed: %s\n", cp->name, grom_last_error());
        grom_out_free(&out);
        return rc;
    }
    j->text = out.vcf;
    j->text_len = out.vcf_len;
    j->ctx_text = out.ctx; /* raw CTX rows for the translocation post-pass */
    j->ctx_len = out.ctx_len;
    if (out.side_written && g_side_base) { /* -N: <results>.1000gen.<chr>, GROM.c:20246-20267 */
        char *fn = malloc(strlen(g_side_base) + strlen(cp->name) + 16);
        sprintf(fn, "%s.1000gen.%s", g_side_base, cp->name);
        FILE *f = fopen(fn, "w");
        if (!f) {
            printf("\nCould not open %s\n", fn);
            free(fn);
            free(out.side);
            return GROM_E_ARG;
        }
        if (out.side_len) fwrite(out.side, 1, out.side_len, f);
        fclose(f);
        free(fn);
    }
    free(out.side);
    if (getenv("GROM_DUMP")) write_dumps(slot, cp, &ch, &rd, j->has_batch ? NULL : j->stage, P);
    if (verbose) {
        /* the pileup kernel's launch and its inputs' sizes (bench.py's roofline) */
        printf("%s: %lld reads, %.3f ms on GPU (%.2f Mbases/s); pileup %.3f ms, cnv %.3f ms, cigar_ops %lld, "
               "bases %lld, len %ld\n", cp->name, (long long)n_reads, st.ms_total,
               st.ms_total > 0 ? cp->len / (st.ms_total * 1e3) : 0.0, st.ms_pileup, st.ms_cnv, (long long)n_cig,
               (long long)n_b, (long)cp->len);
    }
    return GROM_OK;
}

/* ---- multi-GPU: chromosomes shard across devices ----
 * The reference's -P forks one process per chromosome (GROM.c:328-624).  Here
 * -P n (or GROM_DEVICES) runs GROM_SCANS_PER_GPU worker threads per GPU, each
 * with its own library context.  Streamed input: every chromosome is staged
 * on the GPU chosen for it (longest-processing-time over the index's record
 * counts) and scanned by one of that GPU's workers.  Rows are written in
 * chromosome order, so the VCF is the same bytes as a one-GPU run. */

/* GROM_VCF_SEGS (a multi-GPU rank's run): where each chromosome's rows lie
 * in the VCF, "chromosome<TAB>offset<TAB>bytes" per line, so a merge of the
 * ranks' files copies byte ranges without reading the rows
 * (grom_amd.shard.merge_rank_outputs_parallel) */
static textbuf g_vcf_segs;

/* a finished chromosome: its VCF rows go out, its raw CTX rows are kept */
static void take_rows(grom_job *j, FILE *vcf, textbuf *ctx_all) {
    if (j->text_len && getenv("GROM_VCF_SEGS")) {
        const char *tab = memchr(j->text, '\t', j->text_len);
        char line[320];
        const int nl = tab ? (int)(tab - j->text) : 0;
        const int k = snprintf(line, sizeof(line), "%.*s\t%ld\t%zu\n", nl < 256 ? nl : 256, j->text, ftell(vcf),
                               (size_t)j->text_len);
        if (k > 0) textbuf_add(&g_vcf_segs, line, (size_t)k);
    }
    if (j->text_len) fwrite(j->text, 1, j->text_len, vcf);
    free(j->text);
    j->text = NULL;
    if (j->ctx_len) textbuf_add(ctx_all, j->ctx_text, j->ctx_len);
    free(j->ctx_text);
    j->ctx_text = NULL;
}

typedef struct {
    pthread_mutex_t mu;
    pthread_cond_t cv;
    grom_job *jobs;
    int n_jobs, closing;
    const grom_params *P;
    int verbose;
    const int *pos; /* pos[k]: the job of the k-th chromosome in BAM order (NULL: job k) */
} grom_pool;

typedef struct {
    grom_pool *pool;
    int slot;   /* the worker's own library context (grom_ctx_init) */
    int device; /* its GPU */
} grom_worker;

static void *grom_worker_main(void *arg) {
    grom_worker *w = (grom_worker *)arg;
    grom_pool *pl = w->pool;
    int cur = 0; /* jobs before `cur` are taken or belong to other GPUs */
    for (;;) {
        pthread_mutex_lock(&pl->mu);
        grom_job *j = NULL;
        for (;;) {
            while (cur < pl->n_jobs && pl->jobs[cur].ready &&
                   (pl->jobs[cur].taken || (pl->jobs[cur].device >= 0 && pl->jobs[cur].device != w->device)))
                cur++;
            if (cur < pl->n_jobs && pl->jobs[cur].ready) { j = &pl->jobs[cur]; break; }
            if (pl->closing) break;
            pthread_cond_wait(&pl->cv, &pl->mu);
        }
        if (!j) {
            pthread_mutex_unlock(&pl->mu);
            break;
        }
        j->taken = 1;
        pthread_mutex_unlock(&pl->mu);
        /* contexts are independent: workers sharing a GPU scan concurrently */
        int rc = scan_job(w->slot, j, pl->P, pl->verbose);
        if (rc != GROM_OK) snprintf(j->err, sizeof(j->err), "%s: %s", j->cp->name, grom_last_error());
        free(j->cp->ref);
        j->cp->ref = NULL;
        if (j->has_batch) grom_batch_free(&j->batch);
        if (j->stage && j->pd && !j->stage_released) pd_release_stage(j->pd, j->stage);
        j->stage = NULL;
        pthread_mutex_lock(&pl->mu);
        j->rc = rc;
        j->done = 1;
        pthread_cond_broadcast(&pl->cv);
        pthread_mutex_unlock(&pl->mu);
    }
    return NULL;
}

/* everything the two input paths share */
typedef struct {
    grom_params P;
    const char *bam_name, *fasta_name, *out_name;
    long max_chr_len;
    double num_sd;
    int device, verbose, n_dev;
    bam_hdr hdr;
    grom_fasta fa;
    double *hez, *mq;
    pthread_t tables_thr;
    int tables_started;
    chrom_plan *plan; /* candidates in BAM order (preliminary: before the length test) */
    int n_cand;
    char ctx_name[4096];
    int wdev[64], n_work, n_init;
    double t_cli0, t_cand; /* CLI start, candidates (FASTA lengths) done */
    double t_load;         /* process start to the CLI's start (program and library loading) */
    double t_scans, t_pdclose, t_outputs; /* scans done, decoder closed, outputs written */
    double t_decclose;                     /* the decoder's host side closed */
    pthread_t hip_thr;     /* HIP runtime start-up, beside the header/FASTA/index work */
    int hip_started;
    /* -P n (1..256, GROM.c:21923-21927): every chromosome reads its own
     * target's records (bam_fetch, GROM.c:21051-21064 and the -c children of
     * GROM.c:549-599) -- pd_set_fetch_mode; GROM_P_SERIAL=1 keeps the serial
     * stream's input (a one-process run's rows) on n GPUs */
    int fetch;
    /* -c chr,sub,start,end (GROM.c:21928-21930): one child of a -P n run --
     * BAM target `one_chrom` alone, read through bam_fetch, its rows to
     * OUT.<target>-<sub> and its raw CTX rows to OUT.<target>-<sub>.ctx, no
     * header, no translocation post-pass (the parent concatenates and pairs,
     * GROM.c:603-624, 22400), the insert statistics from <bam>.mean
     * (GROM.c:22253-22257).  Whole chromosomes only (start 0, end at or past
     * the chromosome's end: the children -P n forks without -R). */
    int one_chrom, sub_child, sub_start, sub_end;
    char part_name[4096];
} cli_state;

/* Peak device memory of this process (GROM_VERBOSE): the kernel driver's
 * per-process VRAM count (/sys/class/kfd/kfd/proc/<pid>/vram_<gpu>), sampled
 * every 5 ms; without it, the device-wide use above the start's.  Printed as
 * the "footprint:" line, which bench.py reports. */
typedef struct {
    pthread_t thr;
    int started, stop, device, kfd;
    int64_t peak, base;
    double t_peak;
    pthread_mutex_t mu;
    pthread_cond_t cv;
} fp_sampler;

static int64_t fp_kfd_bytes(void) {
    char dir[96], path[384], buf[64];
    snprintf(dir, sizeof(dir), "/sys/class/kfd/kfd/proc/%d", (int)getpid());
    DIR *d = opendir(dir);
    if (!d) return -1;
    int64_t tot = 0;
    int any = 0;
    struct dirent *e;
    while ((e = readdir(d)) != NULL) {
        if (strncmp(e->d_name, "vram_", 5) != 0) continue;
        snprintf(path, sizeof(path), "%s/%s", dir, e->d_name);
        FILE *f = fopen(path, "r");
        if (!f) continue;
        if (fgets(buf, sizeof(buf), f)) { tot += atoll(buf); any = 1; }
        fclose(f);
    }
    closedir(d);
    return any ? tot : -1;
}

static int64_t fp_sample(fp_sampler *F) {
    if (F->kfd) return fp_kfd_bytes();
    const int64_t fr = grom_device_mem_free(F->device);
    return fr < 0 ? -1 : F->base - fr; /* base: free bytes at the start */
}

static void *fp_main(void *arg) {
    fp_sampler *F = (fp_sampler *)arg;
    F->kfd = fp_kfd_bytes() >= 0;
    if (!F->kfd) F->base = grom_device_mem_free(F->device);
    const double t0 = clock_gettime_s();
    pthread_mutex_lock(&F->mu);
    while (!F->stop) {
        pthread_mutex_unlock(&F->mu);
        const int64_t v = fp_sample(F);
        pthread_mutex_lock(&F->mu);
        if (v > F->peak) { F->peak = v; F->t_peak = clock_gettime_s() - t0; }
        struct timespec ts;
        clock_gettime(CLOCK_REALTIME, &ts);
        ts.tv_nsec += 5000000;
        if (ts.tv_nsec >= 1000000000) { ts.tv_sec++; ts.tv_nsec -= 1000000000; }
        if (!F->stop) pthread_cond_timedwait(&F->cv, &F->mu, &ts);
    }
    pthread_mutex_unlock(&F->mu);
    return NULL;
}

static void fp_start(fp_sampler *F, int device) {
    memset(F, 0, sizeof(*F));
    F->device = device;
    pthread_mutex_init(&F->mu, NULL);
    pthread_cond_init(&F->cv, NULL);
    F->started = pthread_create(&F->thr, NULL, fp_main, F) == 0;
}

static void fp_stop(fp_sampler *F, double since_start) {
    if (!F->started) return;
    pthread_mutex_lock(&F->mu);
    F->stop = 1;
    pthread_cond_broadcast(&F->cv);
    pthread_mutex_unlock(&F->mu);
    pthread_join(F->thr, NULL);
    int64_t pk[GROM_DEVCAT_N + 1], nw = 0, ns = 0;
    double sw = 0, ss = 0;
    grom_dev_peaks(pk, NULL);
    grom_dev_waits(&nw, &sw);
    grom_dev_slow(&ns, &ss);
    printf("footprint: peak %.2f GB of device memory (%s), at %.3f s of %.3f s; buffers: peak %.2f GB together, "
           "per kind scan %.2f, breakpoint %.2f, CNV %.2f, stages %.2f, decode %.2f, phase arenas %.2f GB; %lld "
           "allocations waited %.3f s for memory; %lld slow hipMalloc calls %.3f s\n", F->peak / 1e9,
           F->kfd ? "this process, kfd" : "device-wide use above the start's", F->t_peak, since_start,
           pk[GROM_DEVCAT_N] / 1e9, pk[GROM_DEVCAT_SCAN] / 1e9, pk[GROM_DEVCAT_SV] / 1e9, pk[GROM_DEVCAT_CNV] / 1e9,
           pk[GROM_DEVCAT_STAGE] / 1e9, pk[GROM_DEVCAT_DECODE] / 1e9, pk[GROM_DEVCAT_ARENA] / 1e9, (long long)nw, sw,
           (long long)ns, ss);
    pthread_mutex_destroy(&F->mu);
    pthread_cond_destroy(&F->cv);
    F->started = 0;
}

static void *hip_init_main(void *arg) {
    const int device = *(const int *)arg;
    (void)grom_device_count();
    if (getenv("GROM_NO_WARM") == NULL) dd_device_warm(device);
    /* the device decoder's first context, made while the host reads the
     * FASTA lengths and the BAI (GROM_NO_CTX_PREPARE=1: made by the worker).
     * One context is prepared: with several decode workers per GPU
     * (GROM_DD_WORKERS > 1) the first to start takes it, the others make
     * their own */
    const char *dd = getenv("GROM_DEVICE_DECODE"), *np = getenv("GROM_NO_CTX_PREPARE");
    if (!(dd && atoi(dd) == 0) && !(np && atoi(np) == 1)) dd_ctx_prepare(device);
    return NULL;
}

static void hip_ready(cli_state *S) {
    if (S->hip_started) pthread_join(S->hip_thr, NULL);
    S->hip_started = 0;
}

#define CLI_FALLBACK 99 /* the streamed path could not be used: read serially */

static void *tables_main(void *arg) {
    cli_state *S = (cli_state *)arg;
    grom_build_tables(S->P.min_mapq, S->hez, S->mq); /* read_binom_tables, GROM.c:22234 */
    return NULL;
}

static void tables_join(cli_state *S) {
    if (S->tables_started) pthread_join(S->tables_thr, NULL);
    S->tables_started = 0;
}

/* worker contexts: GROM_SCANS_PER_GPU (default 2) per GPU, so two
 * chromosomes are in flight on every GPU; GROM_WORKER_DEVICES=0,0,0 runs
 * three workers on device 0 (test hook) */
static int setup_workers(cli_state *S) {
    grom_params *P = &S->P;
    if (getenv("GROM_DEVICES")) S->n_dev = atoi(getenv("GROM_DEVICES"));
    if (S->n_dev < 1) S->n_dev = 1;
    if (!g_plan_only && S->n_dev > 1) {
        int avail = grom_device_count();
        if (avail < 1) { fprintf(stderr, "grom: no GPU\n"); return -1; }
        if (S->n_dev > avail - S->device) S->n_dev = avail - S->device;
        if (S->n_dev < 1) S->n_dev = 1;
    }
    int per_gpu = getenv("GROM_SCANS_PER_GPU") ? atoi(getenv("GROM_SCANS_PER_GPU")) : 2;
    if (S->n_dev > 64) S->n_dev = 64;
    if (per_gpu < 1) per_gpu = 1;
    if (per_gpu * S->n_dev > 64) per_gpu = 64 / S->n_dev;
    if (per_gpu < 1) per_gpu = 1;
    /* a second context per GPU doubles the scan's device buffers: keep it
     * only when the free HBM holds per_gpu scans of the longest chromosome
     * (about 64 B per base at 30x) */
    if (per_gpu > 1 && !g_plan_only) {
        long longest = 0;
        for (int i = 0; i < S->fa.n; i++)
            if (S->fa.len[i] > longest) longest = S->fa.len[i];
        const double need = 64.0 * (double)longest;
        for (int d = 0; d < S->n_dev; d++) {
            int64_t fr = grom_device_mem_free(S->device + d);
            if (fr >= 0 && (double)fr < need * per_gpu) {
                int fit = (int)((double)fr / need);
                per_gpu = fit < 1 ? 1 : (fit < per_gpu ? fit : per_gpu);
            }
        }
    }
    S->n_work = S->n_dev * per_gpu;
    for (int d = 0; d < 64; d++) S->wdev[d] = S->device + d % S->n_dev;
    if (getenv("GROM_WORKER_DEVICES")) {
        char *sdup = strdup(getenv("GROM_WORKER_DEVICES")), *tok = strtok(sdup, ",");
        S->n_work = 0;
        while (tok && S->n_work < 64) { S->wdev[S->n_work++] = atoi(tok); tok = strtok(NULL, ","); }
        free(sdup);
        if (S->n_work < 1) { S->wdev[0] = S->device; S->n_work = 1; }
    }
    tables_join(S);
    hip_ready(S);
    int rc = GROM_OK;
    for (int d = 0; d < S->n_work && !g_plan_only && rc == GROM_OK; d++) {
        rc = grom_ctx_init(d, S->wdev[d], P, S->hez, S->mq);
        if (rc == GROM_OK) S->n_init = d + 1;
    }
    if (rc != GROM_OK) { fprintf(stderr, "grom: %s\n", grom_last_error()); return -1; }
    return 0;
}

/* set once the streamed run printed the insert lines: a serial rerun after
 * a late fallback (the index plan contradicted mid-file) does not print them
 * again, so stdout reads as one run */
static __thread int t_insert_printed;

static void print_insert(cli_state *S, int imean, int lseq, int imin, int imax, long mapped) {
    const int quiet = t_insert_printed;
    t_insert_printed = 1;
    if (!quiet) printf("insert_min_size, insert_max_size %d %d\n", imin, imax);
    char mean_name[4096];
    snprintf(mean_name, sizeof(mean_name), "%s.mean", S->bam_name);
    FILE *mf = fopen(mean_name, "w"); /* save_insert_mean, GROM.c:994-1008 */
    if (mf) {
        if (!quiet) printf("Saving insert_mean et al to %s\n", mean_name);
        fprintf(mf, "%d %d %d %d %ld\n", imean, lseq, imin, imax, mapped);
        fclose(mf);
    }
    grom_params_set_insert(&S->P, imean, imin, imax, lseq);
    if (quiet) return;
    printf("insert mean, insert minimum, insert maximum: %d %d %d\n", S->P.insert_mean, imin, imax);
    printf("median read length: %d\n", lseq);
}

/* find_disc_svs' length test (GROM.c:20826-21050), needs the insert size */
static int passes_length(const cli_state *S, const chrom_plan *c) {
    const int32_t s0 = S->P.one_base_rd_len / 4 + 1;
    if (c->len > S->max_chr_len)
        printf("ERROR: Reference chromosome length exceeds maximum allowed chromosome size (%ld)\n", S->max_chr_len);
    if (!(c->len > s0 + (long)S->P.overlap_mult * S->P.insert_max_size)) return 0;
    if (!(c->len > 0 && c->len <= S->max_chr_len)) return 0;
    return 1;
}

static void finish_outputs(cli_state *S, textbuf *ctx_all) {
    const char *segs = getenv("GROM_VCF_SEGS");
    if (segs) {
        FILE *f = fopen(segs, "w");
        if (f) {
            if (g_vcf_segs.len) fwrite(g_vcf_segs.p, 1, g_vcf_segs.len, f);
            fclose(f);
        }
        free(g_vcf_segs.p);
        memset(&g_vcf_segs, 0, sizeof(g_vcf_segs));
    }
    if (S->one_chrom >= 0) { /* -c: the raw CTX rows; the parent pairs them (GROM.c:22400) */
        FILE *f = fopen(S->ctx_name, "w");
        if (f) {
            if (ctx_all->len) fwrite(ctx_all->p, 1, ctx_all->len, f);
            fclose(f);
        }
        return;
    }
    const char *raw = getenv("GROM_CTX_RAW"); /* the raw CTX rows, for a merge of several ranks' runs */
    if (raw) {
        FILE *f = fopen(raw, "w");
        if (f) {
            if (ctx_all->len) fwrite(ctx_all->p, 1, ctx_all->len, f);
            fclose(f);
        }
    }
    /* CTX post-pass (GROM.c:22400-22770): pair the translocation rows of all
     * chromosomes with their mates and write them under the header */
    FILE *ctx = fopen(S->ctx_name, "w");
    if (ctx) {
        if (S->P.vcf == 1) header(ctx, S->fasta_name, 1);
        else /* the trimmed file's column header, GROM.c:22652-22700 */
            fputs("SV\tChromosome\tStart\tID\tMate ID\tBinom Prob (Start)\tCTX evidence\tRead Depth (High MapQ)\t"
                  "Concordant Pairs\tOther (Number of Non-Empty)\tMate Chr\tMate Pos\tRead Start\tRead End\t"
                  "Hez binom prob\n", ctx);
        ctx_postpass(ctx_all->p, ctx_all->len, &S->hdr, S->P.insert_max_size, S->P.lseq, S->P.vcf == 1, ctx);
        fclose(ctx);
    }
}

/* rows of finished jobs, in chromosome order (caller holds pool.mu) */
static void drain_rows(grom_pool *pool, int *next_write, int upto, FILE *vcf, textbuf *ctx_all, int *status) {
    while (*next_write < upto && pool->jobs[pool->pos ? pool->pos[*next_write] : *next_write].done) {
        grom_job *j = &pool->jobs[pool->pos ? pool->pos[*next_write] : *next_write];
        (*next_write)++;
        pthread_mutex_unlock(&pool->mu);
        if (j->rc != GROM_OK) *status = 1;
        take_rows(j, vcf, ctx_all);
        pthread_mutex_lock(&pool->mu);
    }
}

static void pool_start(grom_pool *pool, cli_state *S, int n_jobs, grom_worker **workers, pthread_t **tids) {
    memset(pool, 0, sizeof(*pool));
    pthread_mutex_init(&pool->mu, NULL);
    pthread_cond_init(&pool->cv, NULL);
    pool->jobs = calloc(n_jobs > 0 ? n_jobs : 1, sizeof(grom_job));
    pool->n_jobs = n_jobs;
    pool->P = &S->P;
    pool->verbose = S->verbose;
    *workers = calloc(S->n_work, sizeof(grom_worker));
    *tids = calloc(S->n_work, sizeof(pthread_t));
    for (int d = 0; d < S->n_work; d++) {
        (*workers)[d].pool = pool;
        (*workers)[d].slot = d;
        (*workers)[d].device = S->wdev[d];
        pthread_create(&(*tids)[d], NULL, grom_worker_main, &(*workers)[d]);
    }
}

/* close the pool: wait for every job, write the remaining rows */
static void pool_finish(grom_pool *pool, cli_state *S, grom_worker *workers, pthread_t *tids, int *next_write,
                        FILE *vcf, textbuf *ctx_all, int *status) {
    pthread_mutex_lock(&pool->mu);
    pool->closing = 1;
    pthread_cond_broadcast(&pool->cv);
    for (;;) {
        drain_rows(pool, next_write, pool->n_jobs, vcf, ctx_all, status);
        int busy = 0;
        for (int j = 0; j < pool->n_jobs; j++)
            if (pool->jobs[j].ready && !pool->jobs[j].done) busy = 1;
        if (!busy) break;
        pthread_cond_wait(&pool->cv, &pool->mu);
    }
    pthread_mutex_unlock(&pool->mu);
    for (int d = 0; d < S->n_work; d++) pthread_join(tids[d], NULL);
    for (int j = 0; j < pool->n_jobs; j++)
        if (pool->jobs[j].ready && pool->jobs[j].rc != GROM_OK) { grom_set_last_error(pool->jobs[j].err); *status = 1; break; }
    free(tids);
    free(workers);
    free(pool->jobs);
    pthread_mutex_destroy(&pool->mu);
    pthread_cond_destroy(&pool->cv);
}

/* ---------------- serial input: one pass over the record stream ---------------- */
static int run_serial(cli_state *S) {
    grom_params *P = &S->P;
    bgzf_reader br;
    if (bgzf_open_read(&br, S->bam_name) != 0) return 1;
    {
        bam_hdr h2;
        if (bam_read_header(&br, &h2) != 0) { bgzf_close_read(&br); return 1; }
        bam_free_header(&h2);
    }
    /* insert-size pre-pass on the first records (GROM.c:22255) */
    int lseq = 0, imin = 0, imax = 0;
    long mapped = 0;
    int imean = grom_insert_stats(&br, grom_prob2(S->num_sd), &lseq, &imin, &imax, &mapped, P->min_mapq);
    bgzf_close_read(&br);
    if (imean < 0) { printf("ERROR: no reads to estimate the insert size from\n"); return 1; }
    print_insert(S, imean, lseq, imin, imax, mapped);
    if (setup_workers(S)) return 1;
    /* the final plan: candidates that pass the length test */
    const int32_t s0 = P->one_base_rd_len / 4 + 1;
    chrom_plan **plan = calloc(S->n_cand > 0 ? S->n_cand : 1, sizeof(chrom_plan *));
    int32_t *order = calloc(S->n_cand > 0 ? S->n_cand : 1, sizeof(int32_t));
    int n_plan = 0;
    for (int c = 0; c < S->n_cand; c++)
        if (passes_length(S, &S->plan[c])) {
            order[n_plan] = S->plan[c].tid;
            plan[n_plan++] = &S->plan[c];
        }
    FILE *vcf = fopen(S->out_name, "w");
    if (!vcf) { printf("Error opening file %s\n", S->out_name); free(plan); free(order); return 1; }
    if (S->one_chrom < 0) { /* (-c: rows only, the parent wrote the header) */
        if (P->vcf == 1) header(vcf, S->fasta_name, 0);
        else tab_header(vcf, P);
    }
    /* one serial pass over the records, split per chromosome (stream.h);
     * finished chromosomes go to the GPU workers, rows are written in order */
    if (bgzf_open_read(&br, S->bam_name) != 0) { fclose(vcf); free(plan); free(order); return 1; }
    {
        /* BGZF blocks inflate on GROM_DECODE_THREADS threads (default 4) while
         * this thread parses records in order (htslib's bgzf_mt) */
        const char *dt = getenv("GROM_DECODE_THREADS");
        const int n_dec = dt ? atoi(dt) : 4;
        if (bgzf_set_threads(&br, n_dec) != 0) { bgzf_close_read(&br); fclose(vcf); free(plan); free(order); return 1; }
    }
    {
        bam_hdr h2;
        if (bam_read_header(&br, &h2) != 0) { bgzf_close_read(&br); fclose(vcf); free(plan); free(order); return 1; }
        bam_free_header(&h2);
    }
    grom_planner pl;
    grom_planner_init(&pl, order, n_plan);
    grom_batch batch;
    int cur = 0;
    int batch_ended = 0; /* the record after the chromosome's last one was seen */
    if (n_plan > 0) {
        grom_batch_init(&batch, order[0], P->read_name_len);
        grom_batch_set_sv(&batch, plan[0]->target, P->splitread);
    }
    bam_rec rec;
    memset(&rec, 0, sizeof(rec));
    int status = 0, next_write = 0;
    grom_pool pool;
    grom_worker *workers;
    pthread_t *tids;
    pool_start(&pool, S, n_plan, &workers, &tids);
    textbuf ctx_all = {0};
    /* hand chromosome `cur` (its batch complete) to the workers; at most one
     * decoded chromosome waits beyond those being scanned */
    #define SUBMIT_CUR()                                                                           \
        do {                                                                                       \
            plan[cur]->ref = malloc(plan[cur]->len + 1);                                           \
            grom_fasta_load(&S->fa, plan[cur]->fasta_idx, plan[cur]->ref, plan[cur]->len);         \
            pthread_mutex_lock(&pool.mu);                                                          \
            pool.jobs[cur].cp = plan[cur];                                                         \
            pool.jobs[cur].batch = batch;                                                          \
            pool.jobs[cur].has_batch = 1;                                                          \
            pool.jobs[cur].device = -1;                                                            \
            pool.jobs[cur].ready = 1;                                                              \
            pthread_cond_broadcast(&pool.cv);                                                      \
            for (;;) {                                                                             \
                drain_rows(&pool, &next_write, cur + 1, vcf, &ctx_all, &status);                   \
                if (cur + 1 - next_write < S->n_work + 1) break;                                   \
                pthread_cond_wait(&pool.cv, &pool.mu);                                             \
            }                                                                                      \
            pthread_mutex_unlock(&pool.mu);                                                        \
            cur++;                                                                                 \
            if (cur < n_plan) {                                                                    \
                grom_batch_init(&batch, order[cur], P->read_name_len);                             \
                grom_batch_set_sv(&batch, plan[cur]->target, P->splitread);                        \
                batch_ended = 0;                                                                   \
            }                                                                                      \
        } while (0)
    while (S->fetch && cur < n_plan && bam_read_rec(&br, &rec) > 0) {
        /* -P: chromosome `cur` is given its own target's placed records
         * (bam_fetch over [0, MAX_REGION), GROM.c:320) and its stream ends at
         * its last one; a record of a later plan chromosome completes every
         * chromosome before it.  The file is coordinate-sorted (bam_fetch's
         * precondition): a record of an earlier target cannot follow. */
        if (rec.pos < 0 || rec.pos >= 300000000) continue;
        int k = -1;
        for (int j = cur; j < n_plan && k < 0; j++)
            if (order[j] == rec.tid) k = j;
        if (k < 0) {
            for (int j = 0; j < cur; j++)
                if (order[j] == rec.tid) {
                    fprintf(stderr, "grom: -P needs a coordinate-sorted BAM (target %d after a later one)\n", rec.tid);
                    status = 1;
                }
            if (status) break;
            continue;
        }
        while (cur < k) SUBMIT_CUR();
        grom_batch_add(&batch, &rec, s0);
    }
    while (!S->fetch && cur < n_plan && bam_read_rec(&br, &rec) > 0) {
        /* cdp_lseq after the chromosome: the l_qseq of the record that ended
         * it (the R-side edge tests of its last bases read it, GROM.c:12047) */
        if (!batch_ended && batch.n_seen > 0 && rec.tid != order[cur]) {
            grom_batch_end_record(&batch, &rec);
            batch_ended = 1;
        }
        int k = grom_planner_feed(&pl, rec.tid);
        while (cur < n_plan && pl.k > cur) SUBMIT_CUR(); /* chromosome `cur` is complete */
        if (k >= 0 && k == cur) grom_batch_add(&batch, &rec, s0);
    }
    /* end of file: the chromosome being read and every later one */
    while (cur < n_plan) SUBMIT_CUR();
    #undef SUBMIT_CUR
    pool_finish(&pool, S, workers, tids, &next_write, vcf, &ctx_all, &status);
    bam_free_rec(&rec);
    bgzf_close_read(&br);
    fclose(vcf);
    finish_outputs(S, &ctx_all);
    free(ctx_all.p);
    free(plan);
    free(order);
    return status;
}

/* ---------------- streamed input: parallel decode -> pinned pieces -> HBM ---------------- */
typedef struct {
    cli_state *S;
    chrom_plan **plan;
    int n_plan;
    pthread_mutex_t mu;
    pthread_cond_t cv;
    int loaded, consumed, stop; /* refs loaded (a prefix of the plan) ahead of the consumer, at most `ahead` */
    int ahead;
    int next;         /* the next chromosome a loader thread takes */
    char *done;       /* per chromosome: its reference is loaded */
} fasta_feed;

#define FASTA_THREADS_MAX 8

/* A chromosome's reference buffer: 2 MB aligned and advised for huge pages,
 * so the first touch of a 250 MB chromosome is ~125 faults instead of ~61 k
 * (half of a single thread's load time went to page faults) */
static char *ref_alloc(long len) {
    const size_t huge = (size_t)2 << 20, n = ((size_t)len + 1 + huge - 1) / huge * huge;
    void *p = NULL;
    if (posix_memalign(&p, huge, n) != 0) return NULL;
#ifdef MADV_HUGEPAGE
    (void)madvise(p, n, MADV_HUGEPAGE);
#endif
    return (char *)p;
}

/* find_disc_svs loads each chromosome in order (GROM.c:21009-21045); here a
 * few threads do it ahead of the scans (one thread at ~0.9 GB/s of FASTA was
 * slower than the GPU decode: the whole run waited on it), each taking the
 * next chromosome of the plan; `loaded` counts the plan's loaded prefix */
static void *fasta_main(void *arg) {
    fasta_feed *F = (fasta_feed *)arg;
    for (;;) {
        pthread_mutex_lock(&F->mu);
        const int k = F->next;
        if (k < F->n_plan) F->next++;
        while (!F->stop && k < F->n_plan && k >= F->consumed + F->ahead) pthread_cond_wait(&F->cv, &F->mu);
        const int stop = F->stop || k >= F->n_plan;
        pthread_mutex_unlock(&F->mu);
        if (stop) break;
        chrom_plan *c = F->plan[k];
        c->ref = ref_alloc(c->len);
        if (c->ref && grom_fasta_load_at(&F->S->fa, c->fasta_idx, c->ref, c->len) < 0) {
            /* (the shared-stream loader: one thread at a time) */
            static pthread_mutex_t fmu = PTHREAD_MUTEX_INITIALIZER;
            pthread_mutex_lock(&fmu);
            grom_fasta_load(&F->S->fa, c->fasta_idx, c->ref, c->len);
            pthread_mutex_unlock(&fmu);
        }
        pthread_mutex_lock(&F->mu);
        F->done[k] = 1;
        while (F->loaded < F->n_plan && F->done[F->loaded]) F->loaded++;
        pthread_cond_broadcast(&F->cv);
        pthread_mutex_unlock(&F->mu);
    }
    return NULL;
}

/* the CPUs this process may use: the cgroup's CPU quota when it has one
 * (cpu.max "quota period"; a container's share of a large host), else the
 * online CPUs -- more decoder threads than that only contend */
static int host_cpus(void) {
    long ncpu = sysconf(_SC_NPROCESSORS_ONLN);
    FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r");
    if (f) {
        char q[64] = "";
        long period = 0;
        if (fscanf(f, "%63s %ld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
            const long c = (atol(q) + period - 1) / period;
            if (c >= 1 && c < ncpu) ncpu = c;
        }
        fclose(f);
    }
    return ncpu < 1 ? 1 : (int)ncpu;
}

/* GROM_CHROMS=name[,name...]: scan and write only these chromosomes (one
 * rank's share of a genome, bench.py --gpus N); the others keep their place
 * in the plan, so each scanned chromosome gets the records the serial stream
 * of a whole run would give it */
static int chrom_wanted(const char *name) {
    const char *w = getenv("GROM_CHROMS");
    if (!w || !*w) return 1;
    const size_t L = strlen(name);
    for (const char *p = w; *p;) {
        const char *e = strchr(p, ',');
        const size_t n = e ? (size_t)(e - p) : strlen(p);
        if (n == L && strncmp(p, name, n) == 0) return 1;
        if (!e) break;
        p = e + 1;
    }
    return 0;
}

/* GROM_CLI_PROCESS=1 (opt-in, for a `grom` process; never for in-process
 * callers such as the Python binding): the process ends once a streamed
 * run's outputs are written */
static int cli_process_exit(void) {
    const char *e = getenv("GROM_CLI_PROCESS");
    return e && atoi(e) == 1;
}

static void *stage_free_main(void *arg) {
    grom_stage_free((grom_stage *)arg);
    return NULL;
}

static int run_streamed(cli_state *S) {
    grom_params *P = &S->P;
    const double t_start = clock_gettime_s();
    /* the preliminary plan: every candidate (the length test needs the
     * insert size, which the same decode measures) */
    pd_chrom_in *cin = calloc(S->n_cand > 0 ? S->n_cand : 1, sizeof(pd_chrom_in));
    for (int c = 0; c < S->n_cand; c++) {
        cin[c].tid = S->plan[c].tid;
        cin[c].target_name = S->plan[c].target;
        cin[c].len = S->plan[c].len;
    }
    const char *dt = getenv("GROM_DECODE_THREADS");
    /* the host decoder's threads (GROM_DEVICE_DECODE=0 and plan-only runs):
     * the CPU share, at most 32 (its piece window grows with the count) */
    int n_thr = dt ? atoi(dt) : (host_cpus() < 32 ? host_cpus() : 32);
    if (n_thr < 1) n_thr = 1;
    char why[256] = "";
    pd_session *pd = pd_open(S->bam_name, &S->hdr, cin, S->n_cand, P->splitread, P->read_name_len, n_thr, why,
                             (int)sizeof(why));
    free(cin);
    if (!pd) {
        if (S->verbose) printf("streamed decode not used: %s\n", why);
        return CLI_FALLBACK;
    }
    /* GPUs: contexts need the insert statistics, stages do not */
    hip_ready(S);
    if (getenv("GROM_DEVICES")) S->n_dev = atoi(getenv("GROM_DEVICES"));
    if (S->n_dev < 1) S->n_dev = 1;
    if (!g_plan_only && S->n_dev > 1) {
        int avail = grom_device_count();
        if (avail < 1) { fprintf(stderr, "grom: no GPU\n"); pd_close(pd); return 1; }
        if (S->n_dev > avail - S->device) S->n_dev = avail - S->device;
        if (S->n_dev < 1) S->n_dev = 1;
    }
    int *dev_of = calloc(S->n_cand > 0 ? S->n_cand : 1, sizeof(int));
    {
        /* longest processing time first over the chromosome lengths */
        double load[64] = {0};
        int *idx = malloc(sizeof(int) * (S->n_cand > 0 ? S->n_cand : 1));
        for (int c = 0; c < S->n_cand; c++) idx[c] = c;
        for (int a = 1; a < S->n_cand; a++) /* insertion sort, longest first, stable */
            for (int b = a; b > 0 && S->plan[idx[b]].len > S->plan[idx[b - 1]].len; b--) {
                int t = idx[b]; idx[b] = idx[b - 1]; idx[b - 1] = t;
            }
        for (int a = 0; a < S->n_cand; a++) {
            int best = 0;
            for (int d = 1; d < S->n_dev; d++)
                if (load[d] < load[best]) best = d;
            dev_of[idx[a]] = S->device + best;
            load[best] += (double)S->plan[idx[a]].len;
        }
        free(idx);
    }
    const char *wd = getenv("GROM_WORKER_DEVICES");
    if (wd) { /* test hook: every stage on the first listed device */
        for (int c = 0; c < S->n_cand; c++) dev_of[c] = atoi(wd);
    }
    grom_stage *stages[256];
    int n_stages = 0;
    if (!g_plan_only) {
        int per_gpu = getenv("GROM_SCANS_PER_GPU") ? atoi(getenv("GROM_SCANS_PER_GPU")) : 2;
        if (per_gpu < 1) per_gpu = 1;
        /* one stage per scan: a scan gives its stage back before its CNV
         * path (grom_stage_on_consumed), so the next chromosome decodes into
         * it while the CNV path runs.  A third stage (GROM_STAGES=3, the
         * round-4/5 default) let the decode run one chromosome further ahead
         * for 15.5 GB more at 30x, and the whole run was no faster
         * (profiles/r05r: 4.03-4.04 s against 4.00-4.12 s) */
        int n_st = getenv("GROM_STAGES") ? atoi(getenv("GROM_STAGES")) : per_gpu;
        if (n_st < 1) n_st = 1;
        for (int d = 0; d < S->n_dev && !wd; d++)
            for (int k = 0; k < n_st && n_stages < 256; k++) {
                grom_stage *st = grom_stage_new(S->device + d);
                if (!st) break;
                stages[n_stages++] = st;
                pd_add_stage(pd, st, S->device + d);
            }
        for (int k = 0; wd && k < 4; k++) {
            grom_stage *st = grom_stage_new(atoi(wd));
            if (!st) break;
            stages[n_stages++] = st;
            pd_add_stage(pd, st, atoi(wd));
        }
    }
    /* a share of a multi-process run (GROM_CHROMS, bench.py --gpus N) reads
     * the insert statistics from <bam>.mean as the reference's -c children do
     * (load_insert_mean, GROM.c:1011-1026, 22253-22257) */
    int given = 0, g_mean = 0, g_lseq = 0, g_min = 0, g_max = 0;
    long g_mapped = 0;
    char mean_name[4096];
    snprintf(mean_name, sizeof(mean_name), "%s.mean", S->bam_name);
    if ((getenv("GROM_CHROMS") || S->one_chrom >= 0) && !g_plan_only) {
        FILE *mf = fopen(mean_name, "r");
        if (mf) {
            given = fscanf(mf, "%d %d %d %d %ld", &g_mean, &g_lseq, &g_min, &g_max, &g_mapped) == 5 && g_mean > 0;
            fclose(mf);
        }
        if (given) pd_stats_given(pd);
    }
    if (S->fetch) pd_set_fetch_mode(pd, 1);
    if (getenv("GROM_CHROMS")) {
        int *want = calloc(S->n_cand > 0 ? S->n_cand : 1, sizeof(int));
        for (int c = 0; c < S->n_cand; c++) want[c] = chrom_wanted(S->plan[c].name);
        pd_set_wanted(pd, want);
        free(want);
    }
    /* BAM decode on the GPUs (ddecode.hip) by default; the host decoder
     * threads with GROM_DEVICE_DECODE=0 (plan-only runs always use them) */
    {
        const char *dd = getenv("GROM_DEVICE_DECODE");
        pd_set_device_mode(pd, !g_plan_only && !(dd && atoi(dd) == 0));
    }
    if (pd_start(pd, P->min_mapq, S->n_dev, dev_of, g_plan_only)) {
        fprintf(stderr, "grom: %s\n", pd_error(pd));
        pd_close(pd);
        for (int i = 0; i < n_stages; i++) grom_stage_free(stages[i]);
        free(dev_of);
        return 1;
    }
    int status = 0;
    int lseq = 0, imin = 0, imax = 0;
    long mapped = 0;
    const double t_started = clock_gettime_s();
    /* the scan contexts while the head of the BAM is decoded (their insert
     * parameters are set once the statistics are known) */
    const int ws_fail = setup_workers(S);
    int imean;
    if (given) {
        imean = g_mean;
        lseq = g_lseq;
        imin = g_min;
        imax = g_max;
        mapped = g_mapped;
    } else {
        imean = pd_insert_stats(pd, grom_prob2(S->num_sd), P->min_mapq, &lseq, &imin, &imax, &mapped);
    }
    if (imean < 0) {
        const int fallback = imean == -2;
        if (!fallback) printf("ERROR: no reads to estimate the insert size from\n");
        else if (S->verbose) printf("streamed decode stopped: %s\n", pd_error(pd));
        pd_close(pd);
        for (int i = 0; i < n_stages; i++) grom_stage_free(stages[i]);
        free(dev_of);
        return fallback ? CLI_FALLBACK : 1;
    }
    if (given) {
        printf("Loading insert_mean et al from %s\n", mean_name);
        t_insert_printed = 1;
        grom_params_set_insert(&S->P, imean, imin, imax, lseq);
        printf("insert mean, insert minimum, insert maximum: %d %d %d\n", S->P.insert_mean, imin, imax);
        printf("median read length: %d\n", lseq);
    } else {
        print_insert(S, imean, lseq, imin, imax, mapped);
    }
    const double t_stats = clock_gettime_s();
    int *keep = calloc(S->n_cand > 0 ? S->n_cand : 1, sizeof(int));
    chrom_plan **plan = calloc(S->n_cand > 0 ? S->n_cand : 1, sizeof(chrom_plan *));
    int *pidx = calloc(S->n_cand > 0 ? S->n_cand : 1, sizeof(int));
    int n_plan = 0;
    for (int c = 0; c < S->n_cand; c++)
        if ((keep[c] = passes_length(S, &S->plan[c])) && chrom_wanted(S->plan[c].name)) {
            pidx[n_plan] = c;
            plan[n_plan++] = &S->plan[c];
        }
    pd_set_walk(pd, P->one_base_rd_len / 4 + 1, P->overlap_mult, P->insert_max_size, keep);
    FILE *vcf = NULL;
    grom_pool pool;
    grom_worker *workers = NULL;
    pthread_t *tids = NULL;
    textbuf ctx_all = {0};
    int next_write = 0, started = 0, fallback = 0;
    int *qord = NULL, *qpos = NULL;
    chrom_plan **qplan = NULL;
    fasta_feed F;
    memset(&F, 0, sizeof(F));
    pthread_t fthr[FASTA_THREADS_MAX];
    int fasta_started = 0, n_fthr = 0;
    double t_ctx = 0.0;
    if (ws_fail) { status = 1; goto done; }
    for (int d = 0; d < S->n_init; d++)
        if (grom_ctx_set_params(d, &S->P) != GROM_OK) { status = 1; goto done; }
    t_ctx = clock_gettime_s();
    vcf = fopen(S->out_name, "w");
    if (!vcf) { printf("Error opening file %s\n", S->out_name); status = 1; goto done; }
    if (S->one_chrom < 0) { /* (-c: rows only, the parent wrote the header) */
        if (P->vcf == 1) header(vcf, S->fasta_name, 0);
        else tab_header(vcf, P);
    }
    /* the order chromosomes are taken in: the device decoder's (longest
     * first), else BAM order; rows are written in BAM order either way */
    qord = malloc(sizeof(int) * (n_plan > 0 ? n_plan : 1));
    qpos = malloc(sizeof(int) * (n_plan > 0 ? n_plan : 1));
    qplan = malloc(sizeof(chrom_plan *) * (n_plan > 0 ? n_plan : 1));
    for (int k = 0; k < n_plan; k++) qord[k] = k;
    if (pd_device_mode(pd))
        for (int a = 1; a < n_plan; a++)
            for (int b = a; b > 0 && plan[qord[b]]->len > plan[qord[b - 1]]->len; b--) {
                const int t = qord[b];
                qord[b] = qord[b - 1];
                qord[b - 1] = t;
            }
    for (int q = 0; q < n_plan; q++) {
        qpos[qord[q]] = q;
        qplan[q] = plan[qord[q]];
    }
    F.S = S;
    F.plan = qplan;
    F.n_plan = g_plan_only ? 0 : n_plan;
    F.ahead = 4;
    F.done = calloc((size_t)(n_plan > 0 ? n_plan : 1), 1);
    pthread_mutex_init(&F.mu, NULL);
    pthread_cond_init(&F.cv, NULL);
    /* GROM_FASTA_THREADS (default 3) */
    n_fthr = getenv("GROM_FASTA_THREADS") ? atoi(getenv("GROM_FASTA_THREADS")) : 3;
    if (n_fthr < 1) n_fthr = 1;
    if (n_fthr > FASTA_THREADS_MAX) n_fthr = FASTA_THREADS_MAX;
    for (int t = 0; t < n_fthr; t++)
        if (pthread_create(&fthr[t], NULL, fasta_main, &F) != 0) {
            n_fthr = t;
            break;
        }
    if (n_fthr == 0) {
        fprintf(stderr, "grom: no FASTA loader thread\n");
        status = 1;
        goto done;
    }
    fasta_started = 1;
    /* (plan-only: the workers print each chromosome's plan line, so the host
     * tests run the pool beside the streamed decoder) */
    pool_start(&pool, S, n_plan, &workers, &tids);
    pool.pos = qpos;
    started = 1;
    for (int q = 0; q < n_plan; q++) {
        const int k = qord[q];
        grom_stage *st = NULL;
        pd_chrom_facts facts;
        const int rc = pd_wait_chrom(pd, pidx[k], &st, &facts);
        if (rc == 1) { fallback = 1; break; }
        if (rc != 0) {
            fprintf(stderr, "grom: streamed decode failed: %s\n", pd_error(pd));
            grom_set_last_error(pd_error(pd));
            status = 1;
            break;
        }
        if (!g_plan_only) {
            pthread_mutex_lock(&F.mu);
            while (F.loaded <= q) pthread_cond_wait(&F.cv, &F.mu);
            F.consumed = q + 1;
            pthread_cond_broadcast(&F.cv);
            pthread_mutex_unlock(&F.mu);
            if (!plan[k]->ref || grom_stage_set_ref(st, plan[k]->ref, plan[k]->len) != GROM_OK) {
                fprintf(stderr, "grom: staging the reference of %s failed: %s\n", plan[k]->name, grom_last_error());
                status = 1;
                pd_release_stage(pd, st);
                break;
            }
        }
        pthread_mutex_lock(&pool.mu);
        grom_job *j = &pool.jobs[q];
        j->cp = plan[k];
        j->stage = st;
        j->facts = facts;
        j->pd = pd;
        j->k = pidx[k];
        j->device = dev_of[pidx[k]];
        pd_trace(pd, PD_EV_HANDED, pidx[k], 0);
        j->ready = 1;
        pthread_cond_broadcast(&pool.cv);
        drain_rows(&pool, &next_write, n_plan, vcf, &ctx_all, &status);
        pthread_mutex_unlock(&pool.mu);
    }
done:
    if (fasta_started) {
        pthread_mutex_lock(&F.mu);
        F.stop = 1;
        pthread_cond_broadcast(&F.cv);
        pthread_mutex_unlock(&F.mu);
        for (int t = 0; t < n_fthr; t++) pthread_join(fthr[t], NULL);
        /* references loaded but never handed to a worker are freed with the
         * plan at the end of cli_run, after the workers are joined (a worker
         * frees its own job's reference when its scan ends) */
        pthread_mutex_destroy(&F.mu);
        pthread_cond_destroy(&F.cv);
    }
    free(F.done);
    const double t_loop = clock_gettime_s();
    if (started) pool_finish(&pool, S, workers, tids, &next_write, vcf, &ctx_all, &status);
    if (!fallback && status == 0 && S->verbose) {
        const double t_end = clock_gettime_s();
        printf("cli phases (s from start): candidates/FASTA lengths %.3f, decoder open %.3f, insert statistics %.3f, "
               "contexts %.3f, last chromosome handed %.3f, scans done %.3f; process start to CLI start %.3f\n",
               S->t_cand - S->t_cli0, t_started - S->t_cli0, t_stats - S->t_cli0, t_ctx - S->t_cli0, t_loop - S->t_cli0,
               t_end - S->t_cli0, S->t_load);
        pd_counters pc;
        pd_get_counters(pd, &pc);
        if (pc.device)
            printf("device decode: %lld records, %.2f GB compressed read and copied to HBM, %.2f GB inflated on the GPU; "
                   "file reads %.2f s (read ahead; waited for %.2f s), device work %.2f s (GPU inflate %.3f s, record walk %.3f s, "
                   "parse %.3f s; %lld of %lld walk sub-chunks re-walked), device buffer growth %.3f s, per-chromosome decode + "
                   "finalise %.2f s, idle stage blocks reclaimed %lld, %d decode workers, %lld statistics-only runs, wall %.2f s\n",
                   (long long)pc.records, pc.compressed_bytes / 1e9, pc.inflated_bytes / 1e9, pc.io_s, pc.wait_s,
                   pc.decode_thread_s,
                   pc.gpu_ms[0] / 1e3, pc.gpu_ms[1] / 1e3, pc.gpu_ms[2] / 1e3, (long long)pc.rewalked, (long long)pc.subchunks,
                   pc.gpu_ms[3] / 1e3, pc.upload_s, (long long)pc.reclaimed, pc.dd_workers, (long long)pc.stats_only_runs,
                   clock_gettime_s() - t_start);
        else
        printf("streamed decode: %lld records in %lld pieces, %d threads (%s), %.2f GB inflated, %.2f GB to HBM, "
               "decoder busy %.2f s (inflate %.2f s, file reads %.2f s), uploader %.2f s (waiting %.2f s), wall %.2f s\n",
               (long long)pc.records, (long long)pc.pieces, pc.threads, pc.libdeflate ? "libdeflate" : "zlib",
               pc.inflated_bytes / 1e9, pc.h2d_bytes / 1e9, pc.decode_thread_s, pc.inflate_s, pc.io_s, pc.upload_s, pc.wait_s,
               clock_gettime_s() - t_start);
    }
    S->t_scans = clock_gettime_s();
    /* the outputs first: freeing the stages and contexts is teardown */
    if (vcf) fclose(vcf);
    if (!fallback && status == 0) finish_outputs(S, &ctx_all);
    S->t_outputs = clock_gettime_s();
    if (!fallback && status == 0 && cli_process_exit()) {
        /* the `grom` executable ends here: every scan has finished and the
         * outputs are closed; the process's device memory, streams and pinned
         * buffers go with it (hipFree of ~150 GB of stages and scratch, and
         * the runtime's own teardown, are 0.1-0.6 s of a whole run) */
        if (S->verbose)
            printf("cli teardown (s from start): scans done %.3f, outputs %.3f, process exit without freeing\n",
                   S->t_scans - S->t_cli0, S->t_outputs - S->t_cli0);
        fflush(stdout);
        fflush(stderr);
        /* GROM_EXIT_HANDLERS=1: exit handlers still run (a profiler that
         * writes its records at exit, e.g. rocprofv3) */
        const char *eh = getenv("GROM_EXIT_HANDLERS");
        if (eh && atoi(eh) == 1) exit(0);
        _exit(0);
    }
    pd_close(pd);
    S->t_decclose = clock_gettime_s();
    if (getenv("GROM_PAR_FREE") && atoi(getenv("GROM_PAR_FREE")) == 1 && n_stages > 1) {
        /* (timing probe) the stages freed on threads of their own */
        pthread_t th[64];
        int started[64] = {0};
        for (int i = 0; i < n_stages && i < 64; i++)
            started[i] = pthread_create(&th[i], NULL, stage_free_main, stages[i]) == 0;
        for (int i = 0; i < n_stages; i++) {
            if (i < 64 && started[i]) pthread_join(th[i], NULL);
            else grom_stage_free(stages[i]);
        }
    } else {
        for (int i = 0; i < n_stages; i++) grom_stage_free(stages[i]);
    }
    S->t_pdclose = clock_gettime_s();
    free(ctx_all.p);
    free(plan);
    free(pidx);
    free(keep);
    free(dev_of);
    free(qord);
    free(qpos);
    free(qplan);
    if (fallback) {
        for (int d = 0; d < S->n_init; d++) grom_dev_fini(d);
        S->n_init = 0;
        return CLI_FALLBACK;
    }
    return status;
}

/* GROM_SEGV_TRACE=1 (diagnostics for in-process callers such as the Python
 * binding, which have no handler of the grom executable's): a fatal signal
 * prints the host stack before the process ends */
static void on_fatal_trace(int sig) {
    void *fr[64];
    const int n = backtrace(fr, 64);
    static const char msg[] = "grom: fatal signal, host stack:\n";
    if (write(2, msg, sizeof(msg) - 1) < 0) { /* nothing more to do */ }
    backtrace_symbols_fd(fr, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

static int cli_run(int argc, char **argv, int force_serial) {
    if (getenv("GROM_SEGV_TRACE")) {
        struct sigaction sa;
        memset(&sa, 0, sizeof(sa));
        sa.sa_handler = on_fatal_trace;
        sigaction(SIGSEGV, &sa, NULL);
        sigaction(SIGBUS, &sa, NULL);
    }
    optind = 0; /* GNU getopt: 0 fully re-initialises, so this is callable again */
    setlinebuf(stdout);
    cli_state *S = calloc(1, sizeof(cli_state));
    S->t_cli0 = clock_gettime_s();
    S->t_load = since_process_start();
    grom_params *P = &S->P;
    grom_default_params(P);
    S->max_chr_len = 300000000; /* g_max_chr_fasta_len, GROM.c:946 */
    S->num_sd = 3;
    S->verbose = getenv("GROM_VERBOSE") != NULL;
    S->n_dev = 1;
    S->one_chrom = -1;
    S->sub_end = 300000000; /* MAX_REGION, GROM.c:78 */
    if (getenv("GROM_DEVICE")) S->device = atoi(getenv("GROM_DEVICE"));
    int opt, ret = 1;
    /* getopt string of GROM.c:21908 */
    while ((opt = getopt(argc, argv,
                         "Z:W:X:Q:A:Y:B:D:E:K:N:V:U:L:F:SP:c:R:MG:i:r:o:p:q:s:v:g:l:d:b:n:a:y:z:e:fj:k:m:u:w:x:h")) != -1) {
        switch (opt) {
        case 'S': P->splitread = 0; break;
        case 'G': P->sv_list_len = atoi(optarg); break;
        case 'M': P->rmdup = 1; break;
        case 'i': S->bam_name = optarg; break;
        case 'r': S->fasta_name = optarg; break;
        case 'o': S->out_name = optarg; g_side_base = optarg; break;
        case 'B': S->max_chr_len = atol(optarg); break;
        case 'p': P->ploidy = atoi(optarg); break;
        case 'q': P->min_mapq = atoi(optarg); break;
        case 's': S->num_sd = atof(optarg); break;
        case 'g': P->gender = atoi(optarg); break;
        case 'l': P->overlap_mult = atoi(optarg); break;
        case 'b': P->min_base_qual = atoi(optarg); break;
        case 'n': P->min_snv = atoi(optarg); break;
        case 'a': P->min_snv_ratio = atof(optarg); break;
        case 'f': P->vcf = 0; break;
        case 'x': P->min_ave_bq = atof(optarg); break;
        case 'c':
            if (sscanf(optarg, "%d,%d,%d,%d", &S->one_chrom, &S->sub_child, &S->sub_start, &S->sub_end) < 1)
                S->one_chrom = -1;
            break;
        case 'P': { /* -P processes -> GPUs; 0 or beyond 256: serial, one GPU (GROM.c:21923-21927) */
            const int n = atoi(optarg);
            const char *ps = getenv("GROM_P_SERIAL");
            S->fetch = n >= 1 && n <= 256 && !(ps && atoi(ps) == 1);
            S->n_dev = n >= 1 && n <= 256 ? n : 1;
            break;
        }
        case 'Z': P->block_min = atol(optarg); break;
        case 'W': P->min_rd_window_len = atol(optarg); break;
        case 'X': P->max_rd_window_len = atol(optarg); break;
        case 'A': P->windows_sampling_factor = atol(optarg); break;
        case 'Y': P->min_blocks = atol(optarg); break;
        case 'D': P->min_repeat = atol(optarg); break;
        case 'E': P->min_repeat_stdev = atof(optarg); break;
        case 'K': P->ranks_stdev = atoi(optarg); break;
        case 'V': P->rd_pval_threshold = atof(optarg); break;
        case 'U': P->chr_rd_threshold_factor = atoi(optarg); break;
        case 'L': P->dup_threshold_factor = atol(optarg); break;
        case 'F': P->mapq_factor = atof(optarg); break;
        case 'v': P->pval_threshold = atof(optarg); break;
        case 'd': P->min_disc = atoi(optarg); break;
        case 'y': P->max_split_loss = atoi(optarg); break;
        case 'z': P->min_sr_len = atoi(optarg); break;
        case 'e': P->pval_insertion = atof(optarg); break;
        case 'j': P->min_sv_ratio = atof(optarg); break;
        case 'k': P->max_homopolymer = atoi(optarg); break;
        case 'm': P->min_indel_ratio = atof(optarg); break;
        case 'u': P->max_evidence_ratio = atof(optarg); break;
        case 'w': P->max_ins_range = atoi(optarg); break;
        case 'N': P->gen1000_window = atol(optarg); break;
        case 'h': print_help(); free(S); return 0;
        case '?': free(S); return 1;
        default: break; /* accepted; steers rows outside the implemented scan */
        }
    }
    P->rd_min_mapq = P->min_mapq;         /* GROM.c:22102 */
    P->pval_threshold1 = P->pval_threshold; /* GROM.c:22101 */
    P->sv_list2_len = P->sv_list_len / 10;  /* GROM.c:21925 */
    if (!force_serial) {
        printf("bam %s\n", S->bam_name ? S->bam_name : "(null)");
        printf("ref %s\n", S->fasta_name ? S->fasta_name : "(null)");
        printf("results %s\n", S->out_name ? S->out_name : "(null)");
    }
    if (!S->bam_name) { printf("ERROR: No bam file specified.\n"); free(S); return 1; }
    {
        bgzf_reader br;
        if (bgzf_open_read(&br, S->bam_name) != 0 || bam_read_header(&br, &S->hdr) != 0) {
            printf("\nCould not open %s\n", S->bam_name);
            bgzf_close_read(&br);
            free(S);
            return 1;
        }
        bgzf_close_read(&br);
    }
    if (!bai_loads(S->bam_name)) { printf("Could not open BAM indexing file\n"); goto out_hdr; }
    if (!S->out_name) { printf("ERROR: No output file specified.\n"); goto out_hdr; }
    if (S->one_chrom >= 0) {
        if (S->one_chrom >= S->hdr.n_ref) { printf("ERROR: -c %d: the BAM has %d targets\n", S->one_chrom, S->hdr.n_ref); goto out_hdr; }
        if (S->sub_start != 0) {
            printf("ERROR: -c with a sub-region (start %d): only whole-chromosome children are supported (-R is not)\n",
                   S->sub_start);
            goto out_hdr;
        }
        S->fetch = 1; /* g_parallel_mode = 1, GROM.c:22104 */
        snprintf(S->part_name, sizeof(S->part_name), "%s.%s-%d", S->out_name, S->hdr.ref_name[S->one_chrom], S->sub_child);
        S->out_name = S->part_name;
    } else {
        FILE *probe = fopen(S->out_name, "w");
        if (!probe) { printf("\nCould not open %s\n", S->out_name); goto out_hdr; }
        fclose(probe);
    }
    if (!S->fasta_name) { printf("ERROR: No reference file specified.\n"); goto out_hdr; }
    if (grom_fasta_open_cached(&S->fa, S->fasta_name) != 0) {
        printf("\nCould not open %s\n", S->fasta_name);
        goto out_hdr;
    }
    g_plan_only = getenv("GROM_PLAN_ONLY") != NULL;
    if (!g_plan_only) S->hip_started = pthread_create(&S->hip_thr, NULL, hip_init_main, &S->device) == 0;
    fp_sampler fps;
    memset(&fps, 0, sizeof(fps));
    if (!g_plan_only && S->verbose) fp_start(&fps, S->device);
    /* tables (read_binom_tables, GROM.c:22234) on a thread beside the decode */
    {
        size_t tn = (size_t)(GROM_MAX_TRIALS + 1) * (GROM_MAX_TRIALS + 1);
        S->hez = malloc(sizeof(double) * tn);
        S->mq = malloc(sizeof(double) * tn);
        S->tables_started = pthread_create(&S->tables_thr, NULL, tables_main, S) == 0;
        if (!S->tables_started) grom_build_tables(P->min_mapq, S->hez, S->mq);
    }
    /* candidate chromosomes in BAM header order (GROM.c:20826-21050); the
     * length test that needs the insert size comes later */
    S->plan = calloc(S->hdr.n_ref > 0 ? S->hdr.n_ref : 1, sizeof(chrom_plan));
    /* the loader's length of every matched FASTA entry (find_disc_svs loads
     * each chromosome, GROM.c:21009-21045), several entries at once */
    int *fi_of = malloc(sizeof(int) * (S->hdr.n_ref > 0 ? S->hdr.n_ref : 1));
    int *fi_list = malloc(sizeof(int) * (S->hdr.n_ref > 0 ? S->hdr.n_ref : 1));
    long *fi_len = calloc(S->fa.n > 0 ? S->fa.n : 1, sizeof(long));
    int n_fi = 0;
    for (int t = 0; t < S->hdr.n_ref; t++) {
        if (S->one_chrom >= 0 && t != S->one_chrom) { /* -c: loop_start = g_one_chromosome, GROM.c:20821 */
            fi_of[t] = -1;
            continue;
        }
        int fi = grom_match_target(&S->fa, S->hdr.ref_name[t]);
        char lc[GROM_MAX_CHR_NAMES];
        int bl = grom_target_name_lc(S->hdr.ref_name[t], lc, (int)sizeof(lc));
        if (P->gender == 0 && ((bl == 4 && strncmp(lc, "chry", 4) == 0) || (bl == 1 && lc[0] == 'y'))) fi = -1;
        fi_of[t] = fi;
        if (fi < 0) continue;
        int seen = 0;
        for (int a = 0; a < n_fi && !seen; a++) seen = fi_list[a] == fi;
        if (!seen) fi_list[n_fi++] = fi;
    }
    {
        long *lens = calloc(n_fi > 0 ? n_fi : 1, sizeof(long));
        const int thr = host_cpus() < 16 ? host_cpus() : 16;
        const int ok = getenv("GROM_FASTA_SERIAL") == NULL && grom_fasta_lengths(&S->fa, fi_list, n_fi, lens, thr) == 0;
        for (int a = 0; a < n_fi; a++) fi_len[fi_list[a]] = ok ? lens[a] : grom_fasta_load(&S->fa, fi_list[a], NULL, 0);
        free(lens);
    }
    for (int t = 0; t < S->hdr.n_ref; t++) {
        const int fi = fi_of[t];
        if (fi < 0) continue;
        long len = fi_len[fi];
        if (S->one_chrom >= 0 && len > S->sub_end) {
            printf("ERROR: -c region end %d is inside the chromosome (%ld bases): -R sub-regions are not supported\n",
                   S->sub_end, len);
            free(fi_of); free(fi_list); free(fi_len);
            goto out_hdr;
        }
        /* count_discordant_pairs re-derives the BAM target from the FASTA name
         * (GROM.c:1894-1961): the first target matching it */
        int32_t tid2 = -1;
        for (int a = 0; a < S->hdr.n_ref; a++)
            if (grom_match_target(&S->fa, S->hdr.ref_name[a]) == fi) { tid2 = a; break; }
        chrom_plan *c = &S->plan[S->n_cand++];
        c->fasta_idx = fi;
        c->tid = tid2;
        c->len = len;
        /* the name loop leaves the last target's name when nothing matches */
        c->target = strdup(S->hdr.n_ref > 0 ? S->hdr.ref_name[tid2 >= 0 ? tid2 : S->hdr.n_ref - 1] : "");
        snprintf(c->name, sizeof(c->name), "%.*s", S->fa.name_len[fi], S->fa.names[fi]);
    }
    free(fi_of);
    free(fi_list);
    free(fi_len);
    S->t_cand = clock_gettime_s();
    {
        size_t ol = strlen(S->out_name);
        if (S->one_chrom >= 0) /* the child's partial CTX file, GROM.c:20686 */
            snprintf(S->ctx_name, sizeof(S->ctx_name), "%s.ctx", S->out_name);
        else if (ol > 4 && strcmp(S->out_name + ol - 4, ".vcf") == 0)
            snprintf(S->ctx_name, sizeof(S->ctx_name), "%.*s.ctx.vcf", (int)(ol - 4), S->out_name);
        else
            snprintf(S->ctx_name, sizeof(S->ctx_name), "%s.ctx", S->out_name);
    }
    const char *ser = getenv("GROM_SERIAL_DECODE");
    if (force_serial || (ser && atoi(ser) > 0)) ret = run_serial(S);
    else ret = run_streamed(S);
    tables_join(S);
    for (int d = 0; d < S->n_init; d++) grom_dev_fini(d);
    if (S->verbose && S->t_outputs > 0)
        printf("cli teardown (s from start): scans done %.3f, outputs %.3f, decoder closed %.3f, stages freed %.3f, "
               "contexts freed %.3f\n", S->t_scans - S->t_cli0, S->t_outputs - S->t_cli0, S->t_decclose - S->t_cli0,
               S->t_pdclose - S->t_cli0, clock_gettime_s() - S->t_cli0);
    if (fps.started) fp_stop(&fps, clock_gettime_s() - S->t_cli0);
    for (int i = 0; i < S->n_cand; i++) {
        free(S->plan[i].target);
        free(S->plan[i].ref);
    }
    free(S->plan);
    free(S->hez);
    free(S->mq);
    grom_fasta_close(&S->fa);
out_hdr:
    tables_join(S);
    hip_ready(S);
    dd_ctx_drop_prepared();
    bam_free_header(&S->hdr);
    free(S);
    return ret;
}

int grom_cli_main(int argc, char **argv) {
    t_insert_printed = 0;
    int rc = cli_run(argc, argv, 0);
    if (rc == CLI_FALLBACK) {
        if (getenv("GROM_VERBOSE")) printf("reading the BAM serially\n");
        rc = cli_run(argc, argv, 1);
    }
    return rc;
}
