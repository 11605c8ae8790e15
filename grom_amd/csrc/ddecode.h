/*
 * ddecode.h -- BAM decode on the device (ddecode.hip): BGZF block tables and
 * the GPU inflater (inflate.h, one block per lane).
 */
#ifndef GROM_AMD_DDECODE_H
#define GROM_AMD_DDECODE_H

#include <stdint.h>

#include "../../include/grom_amd.h"
#include "devmem.h"

#ifdef __cplusplus
extern "C" {
#endif

/* one BGZF block of a compressed range: its DEFLATE data in the range, and
 * where its ISIZE bytes go in the inflated stream */
typedef struct DdBlock {
    int64_t in_off;   /* its DEFLATE data in the range */
    int64_t out_off;  /* its first byte in the inflated stream */
    uint32_t in_len;
    uint32_t out_len; /* ISIZE */
    int64_t c_off;    /* the block's own start in the range */
} DdBlock;

/* the blocks of buf[0..len) (whole BGZF blocks): returns their number (and
 * fills out[0..cap) and *out_bytes), or -1 if the range is not whole blocks */
int64_t dd_block_table(const uint8_t *buf, int64_t len, DdBlock *out, int64_t cap, int64_t *out_bytes);
/* the whole blocks at the front of buf[0..len) (a block that does not end in
 * the buffer ends the table): their number, *consumed their bytes */
int64_t dd_block_table_prefix(const uint8_t *buf, int64_t len, DdBlock *out, int64_t cap, int64_t *out_bytes,
                              int64_t *consumed);

/* test hook: every whole block in the first max_bytes (<= 0: all) of a BAM
 * inflated on `device` and (check != 0) compared with zlib: the number of
 * blocks that differ or failed (0 = all equal), negative on error; the second
 * of two launches timed with HIP events */
int64_t grom_inflate_device_selftest(const char *bam_path, int device, int64_t max_bytes, int check, double *ms_kernel,
                                     int64_t *n_blocks, int64_t *bytes);

/* ---- one run (a chromosome's records in the file) on the device ---- */
typedef struct dd_ctx dd_ctx;
dd_ctx *dd_ctx_new(int device);
void dd_ctx_prepare(int device); /* one context made ahead (taken by the next dd_ctx_new on the device) */
void dd_ctx_drop_prepared(void); /* frees a prepared context nobody took */
void dd_ctx_free(dd_ctx *c);
/* summed HIP-event times of the parsed runs: inflate, record walk, parse;
 * ms[3]: wall time of decode buffer growth so far (every context) */
void dd_ctx_times(const dd_ctx *c, double ms[4]);
/* record-walk sub-chunks whose guessed start was wrong (re-walked) / all */
void dd_ctx_counts(const dd_ctx *c, int64_t *rewalked, int64_t *subchunks);
/* the device buffers sized for the largest run (`ubytes` inflated bytes, a
 * compressed span of `span`, `recs` records, `n_starts` index-named record
 * starts): the two piece slots and the chromosome-wide name arrays (growth
 * later frees buffers, which waits for the device) */
int dd_reserve(dd_ctx *c, int64_t span, int64_t ubytes, int64_t recs, int64_t n_starts, char *err, int errlen);
/* a run's compressed bytes (h_comp pinned, 64 readable bytes past comp_len)
 * copied into device slot 0/1 on the context's copy stream; returns at once,
 * h_comp must stay untouched until a dd_run_decode of the slot has returned */
int dd_comp_upload(dd_ctx *c, int slot, const uint8_t *h_comp, int64_t comp_len, char *err, int errlen);
/* the same in chunks from a ring of two pinned buffers: begin (device slot
 * sized), per chunk wait for its ring buffer, read into it, copy it to
 * dst_off; end (the slot complete, for dd_run_decode) */
int dd_comp_begin(dd_ctx *c, int slot, int64_t comp_len, char *err, int errlen);
int dd_comp_ring_wait(dd_ctx *c, int ring);
int dd_comp_chunk(dd_ctx *c, int slot, int ring, const uint8_t *h_buf, int64_t dst_off, int64_t n, char *err, int errlen);
int dd_comp_end(dd_ctx *c, int slot, int64_t comp_len, char *err, int errlen);
typedef struct dd_parse_out {
    int64_t n_rec, n_kept, n_drop, n_cig, n_bases, n_auxc;
    int32_t last_pos, last_lq, last_hclip, last_kept;
    /* the split-read candidates (host, valid until the next run): record
     * bytes (block_size first) at aux_bytes + aux_off[a], kept index aux_kidx[a] */
    const uint8_t *aux_bytes;
    const int64_t *aux_off, *aux_kidx;
} dd_parse_out;
/* one run on the device, piece by piece (~GROM_DD_PIECE_MB of inflated bytes,
 * whole record-start chunks): inflate, record walk, the insert statistics'
 * sample while stats_left > 0 (file order; stats_cb after each piece with
 * what it took), and with a stage the records j0.. parsed into it: every
 * array of the chromosome, untrimmed, aux_idx all -1 */
typedef struct dd_run_req {
    int slot;                 /* the compressed bytes' device slot (dd_comp_upload) */
    int64_t comp_len;
    const DdBlock *blk;       /* the run's BGZF blocks (host) */
    int64_t nblk;
    const int64_t *starts;    /* record starts in the inflated run: its first record, then the index's;
                                 starts[n_starts] = u_end */
    int64_t n_starts, u_end;  /* ... and the run's end */
    int32_t tid;              /* the run's target (record-start guesses, the record check) */
    int64_t j0;               /* the run's first record to take */
    int32_t read_name_len;
    int64_t ref_len;
    int64_t count;            /* the index's record count for the run (-1: unknown): sizes the stage */
    grom_stage *stage;        /* NULL: the insert statistics only */
    int64_t stats_left;       /* insert-size pairs still wanted (0: none) */
    int32_t min_mapq;
    int32_t *h_ins, *h_lq;    /* the sample continues here */
    void (*stats_cb)(void *arg, int64_t taken, int64_t m_contrib, int complete);
    void *stats_arg;
    /* the next run this context will decode, if its compressed bytes are on
     * the device already: fills *next (slot, comp_len, blk, nblk, starts,
     * n_starts, u_end, tid, count) and returns 1, its slot then held for
     * that run; its first piece is loaded while this run finishes */
    int (*next_cb)(void *arg, struct dd_run_req *next);
    void *next_arg;
} dd_run_req;
/* 0; -2 when the data contradicts the index plan (the CLI then reads
 * serially); -1.  *n_rec: the records walked (all of the run's with a stage) */
int dd_run_decode(dd_ctx *c, const dd_run_req *q, dd_parse_out *out, int64_t *n_rec, char *err, int errlen);
/* n <= 512 bytes of device memory to the host after the context's work */
int dd_copy_d2h(dd_ctx *c, void *dst, const void *src, size_t n);
/* kept reads and dropped records at positions below s0 (the walk's skip
 * prefix) in a staged chromosome (positions sorted) */
int dd_stage_prefix(dd_ctx *c, grom_stage *stage, int32_t s0, int64_t *sk, int64_t *sd);

/* the device's first allocation of the process (its memory set up), done
 * ahead on a start-up thread */
void dd_device_warm(int device);
/* wall time of a device allocation (stage growth), added to dd_ctx_times' ms[3] */
void grom_note_alloc_ns(int64_t ns, size_t bytes);
/* grom_scan_chrom_staged calls fn(arg, s) once its scan no longer reads the
 * stage (before the CNV path): the stage may take the next chromosome then */
void grom_stage_on_consumed(grom_stage *s, void (*fn)(void *, grom_stage *), void *arg);
/* free a stage's device block (an idle stage under memory pressure): the bytes
 * freed; the stage is empty and grows again when it is next filled */
int64_t grom_stage_drop(grom_stage *s);
/* device bytes a stage holds */
int64_t grom_stage_held(const grom_stage *s);


/* stage helpers for device-side fills (scan.hip) */
/* a stage holding exactly sz's counts (n_aux = capacity, the count starts at
 * 0), its device arrays in *dev (writable); waits for its earlier copies */
int grom_stage_fill_begin(grom_stage *s, const grom_stage_sizes *sz, grom_reads *dev);
/* the piece-wise decode: room for `need` in every array keeping the first
 * `have` entries (earlier pieces), the device arrays in *dev; then the final
 * counts (grom_stage_fill_set) */
int grom_stage_fill_ensure(grom_stage *s, const grom_stage_sizes *need, const grom_stage_sizes *have, grom_reads *dev);
int grom_stage_fill_set(grom_stage *s, const grom_stage_sizes *sz);
/* n split-read alignments: aux[k] for kept read kidx[k] (host arrays) */
int grom_stage_put_aux(grom_stage *s, const grom_aux *aux, const int64_t *kidx, int64_t n);
/* drop the first sd dropped records and count kept reads after the first sk */
int grom_stage_trim_drops(grom_stage *s, int64_t sd, int64_t sk);
/* the stage's device arrays, untrimmed (no reference check) */
int grom_stage_dev_reads(grom_stage *s, grom_reads *dev);
/* n bytes from device memory of `device` (synchronous); 0 or -1 */
int grom_copy_d2h(void *dst, const void *src, size_t n, int device);

#ifdef __cplusplus
}
#endif
#endif
