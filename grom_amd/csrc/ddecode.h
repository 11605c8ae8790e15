/*
 * ddecode.h -- BAM decode on the device (ddecode.hip): BGZF block tables and
 * the GPU inflater (inflate.h, one block per lane).
 */
#ifndef GROM_AMD_DDECODE_H
#define GROM_AMD_DDECODE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* one BGZF block of a compressed range: its DEFLATE data in the range, and
 * where its ISIZE bytes go in the inflated stream */
typedef struct DdBlock {
    int64_t in_off;
    int64_t out_off;
    uint32_t in_len;
    uint32_t out_len;
} DdBlock;

/* the blocks of buf[0..len) (whole BGZF blocks): returns their number (and
 * fills out[0..cap) and *out_bytes), or -1 if the range is not whole blocks */
int64_t dd_block_table(const uint8_t *buf, int64_t len, DdBlock *out, int64_t cap, int64_t *out_bytes);

/* test hook: every whole block in the first max_bytes (<= 0: all) of a BAM
 * inflated on `device` and (check != 0) compared with zlib: the number of
 * blocks that differ or failed (0 = all equal), negative on error; the second
 * of two launches timed with HIP events */
int64_t grom_inflate_device_selftest(const char *bam_path, int device, int64_t max_bytes, int check, double *ms_kernel,
                                     int64_t *n_blocks, int64_t *bytes);

#ifdef __cplusplus
}
#endif
#endif
