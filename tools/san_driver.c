/* tools/san_driver.c -- the host code under AddressSanitizer/UBSan or
 * ThreadSanitizer (make sanitize SAN=asan|tsan; tests/test_sanitize.py).
 *
 * No GPU is touched: every subcommand runs host-only paths of the library
 * built with the sanitizer (the device objects are linked uninstrumented and
 * never called).
 *   cli <grom args...>   the drop-in CLI with GROM_PLAN_ONLY set by the caller:
 *                        BAI planning, the threaded streamed decoder
 *                        (pdecode.c) or the serial reader, insert statistics,
 *                        the record plan and digests
 *   bai <bam> <n>        BAI rebuild (bamio.c) and n random region queries
 *                        checked against a linear scan
 *   fmt <n>              the SNV row formatter against snprintf (snvfmt.cpp)
 *   synth <len>          one synthetic chromosome batch (synth.c, hostapi.c)
 *   ctx                  the translocation post-pass (grom_main.c) on a few
 *                        raw CTX rows
 *   inflate <bam>        the device BGZF inflater's host twin against zlib on
 *                        every block (inflate_host.cpp)
 *   svrows <rec>...      svcall.cpp's candidate lists, SV assembly and rows on
 *                        recorded GPU-scan inputs (GROM_SV_HITS_DUMP), every
 *                        record on its own thread, four rounds, outputs
 *                        compared with the recorded rows
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/grom_amd.h"

static int cmd_bai(const char *bam, int64_t n) {
    if (grom_bai_build(bam) != 0) {
        fprintf(stderr, "bai build failed: %s\n", grom_last_error());
        return 1;
    }
    int64_t visited = 0;
    const int64_t bad = grom_bai_selftest(bam, n, 12345, &visited);
    printf("bai selftest: %lld mismatches over %lld records visited\n", (long long)bad, (long long)visited);
    return bad != 0;
}

static int cmd_fmt(int64_t n) {
    const int64_t bad = grom_fmt_selftest(n, 7);
    printf("fmt selftest: %lld mismatches\n", (long long)bad);
    return bad != 0;
}

static int cmd_synth(int64_t len) {
    grom_params P;
    grom_default_params(&P);
    const int64_t lens[2] = {len, len / 2};
    grom_synth_spec sp;
    memset(&sp, 0, sizeof(sp));
    sp.n_chr = 2;
    sp.chrom = 1;
    sp.chr_len = lens;
    sp.coverage = 10.0;
    sp.read_len = 100;
    sp.insert_mean = 400;
    sp.insert_sd = 50;
    sp.dup_frac = 0.05;
    sp.sv_per_mb = 20.0;
    sp.cnv_rate = 1e-5;
    sp.munmap_frac = 0.01;
    sp.seed = 3;
    grom_batch_handle *h = grom_synth_chrom(&sp, &P);
    if (!h) {
        fprintf(stderr, "synth failed: %s\n", grom_last_error());
        return 1;
    }
    grom_chrom c;
    grom_reads r;
    if (grom_batch_get(h, &c, &r) != 0) return 1;
    printf("synth: %lld reads on a %lld-base chromosome\n", (long long)r.n, (long long)c.len);
    grom_batch_release(h);
    return 0;
}

static int cmd_ctx(void) {
    /* raw CTX rows as the scans emit them: the post-pass pairs the two ends */
    /* raw row: type chr pos binom ev rd conc other mchr mpos rs re hez */
    static const char raw[] =
        "CTX_F\tchr1\t1000\t1e-10\t5.0\t30\t10\t0\t1\t-5000\t900\t990\t1e-5\n"
        "CTX_R\tchr2\t5000\t1e-10\t5.0\t30\t10\t0\t0\t1000\t5010\t5100\t1e-5\n";
    const char *names[2] = {"chr1", "chr2"};
    grom_out out;
    memset(&out, 0, sizeof(out));
    const int rc = grom_ctx_postpass(raw, sizeof(raw) - 1, names, 2, 600, 150, &out);
    printf("ctx post-pass: rc %d, %lld bytes\n", rc, (long long)out.ctx_len);
    grom_out_free(&out);
    return rc < 0;
}

int grom_sv_rows_replay(const char *path); /* svcall.cpp test hook (sv.h) */
int64_t grom_inflate_selftest(const char *bam_path, int64_t max_blocks, int64_t *n_blocks, int64_t *bytes);

static int cmd_inflate(const char *bam) {
    int64_t nb = 0, by = 0;
    const int64_t bad = grom_inflate_selftest(bam, 0, &nb, &by);
    printf("inflate selftest: %lld mismatches over %lld blocks (%lld bytes)\n", (long long)bad, (long long)nb,
           (long long)by);
    return bad != 0;
}

typedef struct {
    const char *path;
    int rc;
} replay_job;

static void *replay_main(void *arg) {
    replay_job *j = (replay_job *)arg;
    for (int r = 0; r < 4 && j->rc == 0; r++) j->rc = grom_sv_rows_replay(j->path);
    return NULL;
}

static int cmd_svrows(int n, char **paths) {
    replay_job *jobs = calloc((size_t)n, sizeof(replay_job));
    pthread_t *t = calloc((size_t)n, sizeof(pthread_t));
    for (int i = 0; i < n; i++) {
        jobs[i].path = paths[i];
        pthread_create(&t[i], NULL, replay_main, &jobs[i]);
    }
    int bad = 0;
    for (int i = 0; i < n; i++) {
        pthread_join(t[i], NULL);
        printf("svrows %s: rc %d\n", paths[i], jobs[i].rc);
        bad += jobs[i].rc != 0;
    }
    free(jobs);
    free(t);
    return bad != 0;
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: san_driver cli|bai|fmt|synth|ctx|svrows|inflate ...\n");
        return 2;
    }
    if (!strcmp(argv[1], "cli")) return grom_cli_main(argc - 1, argv + 1);
    if (!strcmp(argv[1], "bai") && argc >= 4) return cmd_bai(argv[2], atoll(argv[3]));
    if (!strcmp(argv[1], "fmt") && argc >= 3) return cmd_fmt(atoll(argv[2]));
    if (!strcmp(argv[1], "synth") && argc >= 3) return cmd_synth(atoll(argv[2]));
    if (!strcmp(argv[1], "ctx")) return cmd_ctx();
    if (!strcmp(argv[1], "svrows") && argc >= 3) return cmd_svrows(argc - 2, argv + 2);
    if (!strcmp(argv[1], "inflate") && argc >= 3) return cmd_inflate(argv[2]);
    fprintf(stderr, "bad arguments\n");
    return 2;
}
