// ddecode.hip -- BAM decode on the device: BGZF blocks inflated on the GPU
// (inflate.h, one block per lane), for the streamed CLI path.
//
// The reference inflates every block on the host through htslib/zlib
// (my_samread, GROM.c:981-992).  A 30x genome is 180 GB of inflated BAM --
// 99 of the host decoder's 161 CPU-seconds per genome go to inflate alone
// (profiles/r04_genome_probe.txt) -- so here the compressed blocks go to HBM
// as they are (20 GB per genome) and the GPU inflates them.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>
#include <zlib.h>

#include "../../include/grom_amd.h"
#include "ddecode.h"
#include "inflate.h"

#define DD_LANES 64
#define DD_SLOTS 2   // compressed runs on the device (the prefetch thread's slots)
#define DD_RSLOTS 4  // piece slots (inflated bytes, record offsets): at most this many pieces in flight

// One BGZF block per lane: blk[j] = {offset of its DEFLATE data in `comp`,
// its length, offset of its output, ISIZE}; the output goes to out +
// (out_off - out_base) (a piece of a run: out holds the piece).  status[j] =
// GI_* code.  A block whose input is not inside comp[0, comp_cap) or whose
// output is not inside out[0, out_cap) is not touched: status GI_E_BOUNDS and
// bit 1 in *bounds (a block table that does not belong to the compressed
// slot or the piece is an error the host reports, never a wild access).
#define GI_E_BOUNDS 8
__device__ __forceinline__ bool dd_blk_inb(const DdBlock &b, int64_t o, int64_t comp_cap, int64_t out_cap) {
    return b.in_off >= 0 && b.in_off + (int64_t)b.in_len <= comp_cap && o >= 0 && b.out_len <= 65536u &&
           o + (int64_t)b.out_len <= out_cap;
}

// only_tokcap: the fallback launch of the two-phase inflate -- only the
// blocks phase 1 refused for their token count (status GI_E_TOKCAP)
__global__ void __launch_bounds__(DD_LANES, 2) k_inflate(const uint8_t *__restrict__ comp, int64_t comp_cap,
                                                      const DdBlock *__restrict__ blk, int64_t n_blk,
                                                      uint8_t *__restrict__ out, int64_t out_base, int64_t out_cap,
                                                      uint8_t *__restrict__ status, uint32_t *__restrict__ n_bad,
                                                      uint32_t *__restrict__ bounds, int only_tokcap) {
    extern __shared__ uint32_t dd_tab[];  // GI_LANE_DWORDS x DD_LANES: rows element-major across the lanes
    const int64_t j = (int64_t)blockIdx.x * DD_LANES + threadIdx.x;
    if (j >= n_blk) return;
    if (only_tokcap && status[j] != (uint8_t)GI_E_TOKCAP) return;
    const DdBlock b = blk[j];
    const int64_t o = b.out_off - out_base;
    if (!dd_blk_inb(b, o, comp_cap, out_cap)) {
        status[j] = (uint8_t)GI_E_BOUNDS;
        atomicAdd(n_bad, 1u);
        atomicOr(bounds, 1u);
        return;
    }
    const int rc = gi_inflate<DD_LANES>(comp + b.in_off, b.in_len, out + o, b.out_len, dd_tab, threadIdx.x);
    status[j] = (uint8_t)rc;
    if (rc) atomicAdd(n_bad, 1u);
}

// Phase 1 of the two-phase inflate (inflate.h, gi_tokens): one block per
// lane, its tokens to tok + j * tokcap, their count to ntok[j], its literals
// packed at the front of its output region.  A block over the token cap is
// left for the fallback launch (status GI_E_TOKCAP, not counted as bad).
__global__ void __launch_bounds__(DD_LANES, 2) k_huff(const uint8_t *__restrict__ comp, int64_t comp_cap,
                                                   const DdBlock *__restrict__ blk, int64_t n_blk,
                                                   uint8_t *__restrict__ out, int64_t out_base, int64_t out_cap,
                                                   uint32_t *__restrict__ tok, uint32_t *__restrict__ ntok,
                                                   uint32_t tokcap, uint8_t *__restrict__ status,
                                                   uint32_t *__restrict__ n_bad, uint32_t *__restrict__ bounds) {
    extern __shared__ uint32_t dd_tab[];
    const int64_t j = (int64_t)blockIdx.x * DD_LANES + threadIdx.x;
    if (j >= n_blk) return;
    const DdBlock b = blk[j];
    const int64_t o = b.out_off - out_base;
    if (!dd_blk_inb(b, o, comp_cap, out_cap)) {
        status[j] = (uint8_t)GI_E_BOUNDS;
        atomicAdd(n_bad, 1u);
        atomicOr(bounds, 1u);
        return;
    }
    const int rc = gi_tokens<DD_LANES>(comp + b.in_off, b.in_len, out + o, b.out_len, tok + (size_t)j * tokcap, tokcap,
                                       ntok + j, dd_tab, threadIdx.x);
    status[j] = (uint8_t)rc;
    if (rc && rc != GI_E_TOKCAP) atomicAdd(n_bad, 1u);
}

// Phase 2: one wave per block (GROM_LZ_LANE=1: one lane per block, gi_lz).
// One lane per block put ~10^5 blocks' recent output in flight at once and
// the match sources (half of them 256-1024 bytes back) fell out of L2
// (26 ms for 140 k blocks); a wave per block keeps a block's last few KB
// hot in its CU.  Tokens are taken 64 at a time: a prefix sum places each
// token's literals (already in place) and match, then the matches copy in
// rounds: a match copies once no unresolved match of the group writes into
// its source (the first round: sources below the group's lowest unresolved
// match; the lowest one always qualifies, its own overlap handled by
// gi_match's doubling).  Lanes of one wave share the CU's L1, so a round's
// stores are visible to the next round's loads after a workgroup-scope
// release/acquire (a wait for the stores).
__device__ __forceinline__ uint32_t lz_wave_incl(uint32_t v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t u = __shfl_up(v, d, 64);
        if (lane >= d) v += u;
    }
    return v;
}
__device__ __forceinline__ uint32_t lz_wave_min(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = min(v, (uint32_t)__shfl_xor(v, d, 64));
    return v;
}

__global__ void __launch_bounds__(64) k_lz77(const DdBlock *__restrict__ blk, int64_t n_blk, uint8_t *__restrict__ out,
                                             int64_t out_base, const uint32_t *__restrict__ tok,
                                             const uint32_t *__restrict__ ntok, uint32_t tokcap,
                                             uint8_t *__restrict__ status, uint32_t *__restrict__ n_bad) {
    const int64_t j = blockIdx.x;
    if (j >= n_blk || status[j] != 0) return;  // (uniform: one wave per block)
    const int lane = threadIdx.x;
    const DdBlock b = blk[j];
    uint8_t *dst = out + (b.out_off - out_base);
    const uint32_t n = ntok[j], olen = b.out_len;
    const uint32_t *tk = tok + (size_t)j * tokcap;
    uint32_t obase = 0;
    bool bad = false;
    for (uint32_t c0 = 0; c0 < n && !bad; c0 += 64) {
        const uint32_t k = c0 + (uint32_t)lane;
        const uint32_t t = k < n ? tk[k] : GI_TOK_LITONLY;
        const bool hm = !(t & GI_TOK_LITONLY);
        const uint32_t lc = t & 255u, len = hm ? ((t >> 8) & 255u) + 3u : 0u, d = ((t >> 16) & 0x7fffu) + 1u;
        const uint32_t span = lc + len;
        const uint32_t inc = lz_wave_incl(span, lane);
        const uint32_t m = obase + inc - len;  // the match's first byte
        obase += __shfl(inc, 63, 64);
        bool pend = hm;
        if (__any((hm && d > m) || obase > olen)) {  // (phase 1 checked these: a wrong table or token area)
            bad = true;
            break;
        }
        const uint32_t src = m - d, se = src + (len < d ? len : d);
        for (;;) {
            const uint64_t pm = __ballot(pend);
            if (pm == 0) break;
            const uint32_t P = lz_wave_min(pend ? m : 0xffffffffu);
            bool ready = pend && se <= P;
            if (__ballot(ready) != pm) {
                // the rest: blocked only by a pending match that writes into the source
                bool blocked = false;
                for (uint64_t q = pm; q; q &= q - 1) {
                    const int jl = __builtin_ctzll(q);
                    const uint32_t mj = __builtin_amdgcn_readlane(m, jl);
                    const uint32_t ej = mj + __builtin_amdgcn_readlane(len, jl);
                    blocked = blocked || (mj < se && ej > src);
                }
                ready = pend && !blocked;
            }
            if (ready) {
                gi_match(dst, m, len, d);
                pend = false;
            }
            // this round's stores before the next round's loads (one CU, one L1)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
    }
    if (lane == 0 && (bad || obase != olen)) {
        status[j] = (uint8_t)GI_E_SIZE;
        atomicAdd(n_bad, 1u);
    }
}

// the one-lane-per-block variant (GROM_LZ_LANE=1)
__global__ void __launch_bounds__(DD_LANES) k_lz77_lane(const DdBlock *__restrict__ blk, int64_t n_blk,
                                                        uint8_t *__restrict__ out, int64_t out_base,
                                                        const uint32_t *__restrict__ tok,
                                                        const uint32_t *__restrict__ ntok, uint32_t tokcap,
                                                        uint8_t *__restrict__ status, uint32_t *__restrict__ n_bad) {
    const int64_t j = (int64_t)blockIdx.x * DD_LANES + threadIdx.x;
    if (j >= n_blk || status[j] != 0) return;
    const DdBlock b = blk[j];
    const int rc = gi_lz(tok + (size_t)j * tokcap, ntok[j], out + (b.out_off - out_base), b.out_len);
    if (rc) {
        status[j] = (uint8_t)rc;
        atomicAdd(n_bad, 1u);
    }
}

// tokens per block of the two-phase inflate (GROM_INFLATE_TOKCAP, a multiple
// of 4; 0: the one-phase k_inflate alone)
static uint32_t dd_tokcap() {
    static const uint32_t cap = [] {
        const char *e = getenv("GROM_INFLATE_TOKCAP");
        long v = e ? atol(e) : 0;
        if (v < 0) v = 0;
        if (v > 65536) v = 65536;
        return (uint32_t)(v & ~3L);
    }();
    return cap;
}

// bytes of the token buffer the two-phase inflate of n_blk blocks needs (0: one-phase)
extern "C" size_t dd_inflate_tok_bytes(int64_t n_blk) {
    const uint32_t cap = dd_tokcap();
    return cap ? (size_t)n_blk * ((size_t)cap + 1) * 4 + 64 : 0;
}

extern "C" int dd_inflate_launch(hipStream_t st, const uint8_t *d_comp, int64_t comp_cap, const DdBlock *d_blk,
                                 int64_t n_blk, uint8_t *d_out, int64_t out_base, int64_t out_cap, uint8_t *d_status,
                                 uint32_t *d_bad, uint32_t *d_bounds, uint32_t *d_tok, size_t tok_bytes) {
    if (n_blk <= 0) return 0;
    const unsigned grid = (unsigned)((n_blk + DD_LANES - 1) / DD_LANES);
    // GROM_INFLATE_LDS_PAD (probe only): extra LDS bytes per wave, to measure
    // how the kernel's speed follows its occupancy
    static const int pad = getenv("GROM_INFLATE_LDS_PAD") ? atoi(getenv("GROM_INFLATE_LDS_PAD")) : 0;
    const uint32_t cap = dd_tokcap();
    if (cap == 0 || d_tok == nullptr || tok_bytes < dd_inflate_tok_bytes(n_blk)) {
        hipLaunchKernelGGL(k_inflate, dim3(grid), dim3(DD_LANES), GI_LANE_BYTES * DD_LANES + pad, st, d_comp, comp_cap,
                           d_blk, n_blk, d_out, out_base, out_cap, d_status, d_bad, d_bounds, 0);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    uint32_t *ntok = d_tok + (size_t)n_blk * cap;
    hipLaunchKernelGGL(k_huff, dim3(grid), dim3(DD_LANES), GI_LANE_BYTES * DD_LANES + pad, st, d_comp, comp_cap, d_blk,
                       n_blk, d_out, out_base, out_cap, d_tok, ntok, cap, d_status, d_bad, d_bounds);
    static const bool lane_lz = getenv("GROM_LZ_LANE") && atoi(getenv("GROM_LZ_LANE")) != 0;
    if (lane_lz)
        hipLaunchKernelGGL(k_lz77_lane, dim3(grid), dim3(DD_LANES), 0, st, d_blk, n_blk, d_out, out_base, d_tok, ntok,
                           cap, d_status, d_bad);
    else
        hipLaunchKernelGGL(k_lz77, dim3((unsigned)n_blk), dim3(64), 0, st, d_blk, n_blk, d_out, out_base, d_tok, ntok,
                           cap, d_status, d_bad);
    hipLaunchKernelGGL(k_inflate, dim3(grid), dim3(DD_LANES), GI_LANE_BYTES * DD_LANES + pad, st, d_comp, comp_cap,
                       d_blk, n_blk, d_out, out_base, out_cap, d_status, d_bad, d_bounds, 1);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---- BGZF block table of a byte range (host) ----
static uint16_t rd16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static uint32_t rd32(const uint8_t *p) {
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

extern "C" int64_t dd_block_table(const uint8_t *buf, int64_t len, DdBlock *out, int64_t cap, int64_t *out_bytes) {
    return dd_block_table_prefix(buf, len, out, cap, out_bytes, nullptr);
}

// the whole blocks at the front of buf[0..len): with `consumed` a block that
// does not end inside the buffer ends the table (*consumed: the bytes of the
// whole blocks), without it that is an error
extern "C" int64_t dd_block_table_prefix(const uint8_t *buf, int64_t len, DdBlock *out, int64_t cap, int64_t *out_bytes,
                                         int64_t *consumed) {
    int64_t off = 0, n = 0, ob = 0;
    while (off < len) {
        if (off + 18 > len) {
            if (consumed) break;
            return -1;
        }
        const uint8_t *h = buf + off;
        if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || !(h[3] & 4)) return -1;
        const int xlen = rd16(h + 10);
        int bsize = -1;
        for (int o = 0; o + 4 <= xlen;) {
            const int sl = rd16(h + 12 + o + 2);
            if (h[12 + o] == 'B' && h[12 + o + 1] == 'C' && sl == 2) bsize = rd16(h + 12 + o + 4);
            o += 4 + sl;
        }
        const int64_t blen = (int64_t)bsize + 1;
        if (bsize < 0 || blen < 12 + xlen + 8) return -1;
        if (off + blen > len) {
            if (consumed) break;
            return -1;
        }
        const uint32_t isize = rd32(h + blen - 4);
        if (isize > 65536) return -1;
        if (out && n < cap) {
            out[n].in_off = off + 12 + xlen;
            out[n].in_len = (uint32_t)(blen - 12 - xlen - 8);
            out[n].out_off = ob;
            out[n].out_len = isize;
            out[n].c_off = off;
        }
        n++;
        ob += isize;
        off += blen;
    }
    if (out_bytes) *out_bytes = ob;
    if (consumed) *consumed = off;
    return n;
}

// ---- test hook: every block of a BAM inflated on `device`, checked against zlib ----
extern "C" int64_t grom_inflate_device_selftest(const char *bam_path, int device, int64_t max_bytes, int check,
                                                double *ms_kernel, int64_t *n_blocks, int64_t *bytes) {
    FILE *f = fopen(bam_path, "rb");
    if (!f) return -1;
    fseek(f, 0, SEEK_END);
    int64_t size = ftell(f);
    fseek(f, 0, SEEK_SET);
    if (max_bytes > 0 && size > max_bytes) size = max_bytes;
    std::vector<uint8_t> file((size_t)size + 64, 0);
    if (fread(file.data(), 1, (size_t)size, f) != (size_t)size) { fclose(f); return -1; }
    fclose(f);
    // whole blocks only (a prefix of the file)
    int64_t used = 0, ob = 0;
    {
        int64_t off = 0;
        while (off + 18 <= size) {
            const uint8_t *h = file.data() + off;
            if (h[0] != 0x1f || h[1] != 0x8b) break;
            const int xlen = rd16(h + 10);
            int bsize = -1;
            for (int o = 0; o + 4 <= xlen;) {
                const int sl = rd16(h + 12 + o + 2);
                if (h[12 + o] == 'B' && h[12 + o + 1] == 'C' && sl == 2) bsize = rd16(h + 12 + o + 4);
                o += 4 + sl;
            }
            if (bsize < 0 || off + bsize + 1 > size) break;
            off += bsize + 1;
        }
        used = off;
    }
    const int64_t nb = dd_block_table(file.data(), used, nullptr, 0, &ob);
    if (nb < 0) return -2;
    std::vector<DdBlock> tab((size_t)nb);
    dd_block_table(file.data(), used, tab.data(), nb, &ob);
    if (hipSetDevice(device) != hipSuccess) return -3;
    uint8_t *d_comp = nullptr, *d_out = nullptr, *d_status = nullptr;
    DdBlock *d_blk = nullptr;
    uint32_t *d_bad = nullptr, *d_tok = nullptr;
    const size_t tok_bytes = dd_inflate_tok_bytes(nb);
    int64_t bad = -4;
    hipStream_t st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (hipMalloc(&d_comp, (size_t)used + 64) != hipSuccess || hipMalloc(&d_out, (size_t)ob + 64) != hipSuccess ||
        hipMalloc(&d_status, (size_t)nb + 1) != hipSuccess || hipMalloc(&d_blk, sizeof(DdBlock) * (size_t)(nb + 1)) != hipSuccess ||
        hipMalloc(&d_bad, 8) != hipSuccess || (tok_bytes && hipMalloc(&d_tok, tok_bytes) != hipSuccess) ||
        hipStreamCreate(&st) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
        hipEventCreate(&e1) != hipSuccess)
        goto done;
    {
        (void)hipMemcpyAsync(d_comp, file.data(), (size_t)used + 64, hipMemcpyHostToDevice, st);
        (void)hipMemcpyAsync(d_blk, tab.data(), sizeof(DdBlock) * (size_t)nb, hipMemcpyHostToDevice, st);
        (void)hipMemsetAsync(d_bad, 0, 8, st);
        // a warm launch, then the timed one
        for (int rep = 0; rep < 2; rep++) {
            (void)hipEventRecord(e0, st);
            if (dd_inflate_launch(st, d_comp, used + 64, d_blk, nb, d_out, 0, ob + 64, d_status, d_bad, d_bad + 1, d_tok,
                                  tok_bytes))
                goto done;
            (void)hipEventRecord(e1, st);
        }
        if (hipStreamSynchronize(st) != hipSuccess) goto done;
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms_kernel) *ms_kernel = ms;
        std::vector<uint8_t> got((size_t)ob + 64), status((size_t)nb);
        if (hipMemcpy(got.data(), d_out, (size_t)ob, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(status.data(), d_status, (size_t)nb, hipMemcpyDeviceToHost) != hipSuccess)
            goto done;
        bad = 0;
        std::vector<uint8_t> want(65536 + 64);
        for (int64_t j = 0; j < nb && !check; j++) bad += status[j] != 0;  // timing runs: statuses only
        for (int64_t j = 0; j < nb && check; j++) {
            z_stream zs;
            memset(&zs, 0, sizeof(zs));
            int zrc = inflateInit2(&zs, -15);
            zs.next_in = (Bytef *)(file.data() + tab[j].in_off);
            zs.avail_in = tab[j].in_len;
            zs.next_out = want.data();
            zs.avail_out = (uInt)want.size();
            if (zrc == Z_OK) zrc = inflate(&zs, Z_FINISH);
            const bool zok = zrc == Z_STREAM_END && zs.total_out == tab[j].out_len;
            inflateEnd(&zs);
            const bool same = zok ? (status[j] == 0 && memcmp(want.data(), got.data() + tab[j].out_off, tab[j].out_len) == 0)
                                  : status[j] != 0;
            if (!same) {
                if (bad < 5) fprintf(stderr, "device inflate: block %lld: zlib %d, device status %d\n", (long long)j, zrc,
                                     status[j]);
                bad++;
            }
        }
    }
done:
    if (n_blocks) *n_blocks = nb;
    if (bytes) *bytes = ob;
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (st) (void)hipStreamDestroy(st);
    (void)hipFree(d_comp);
    (void)hipFree(d_out);
    (void)hipFree(d_status);
    (void)hipFree(d_blk);
    (void)hipFree(d_bad);
    (void)hipFree(d_tok);
    return bad;
}

// ===========================================================================
// Records of one run (a chromosome's records in the file) on the device.
//
// The run's blocks are inflated into one contiguous stream U.  Record
// boundaries: the BAI's linear index names a record start every 16 kb of the
// reference (the first record overlapping each window), so the run is cut at
// those offsets into chunks, one lane walks each chunk's block_size chain
// (counting, then writing every record's offset), and a chunk must end
// exactly where the next one starts -- else the plan falls back to the host
// decoder.  Then one lane per record parses the fixed fields into the
// stage's structure-of-arrays, prefix sums place the CIGAR words, bases,
// qualities, dropped records and split-read candidates, one wave per read
// copies its packed bases and qualities, and read names become ids by a
// radix sort of 64-bit name hashes with every member of an equal-hash run
// compared byte for byte against the run's first (a collision falls back).
// This is the work pdecode.c's decode_piece + upload_piece do on the host,
// with the same results (tests/test_gpu_parity.py compares the digests).
// ===========================================================================
#include <hipcub/hipcub.hpp>

#include "bamio.h"
#include "copystats.h"  // (GROM_COPY_STATS, last: it wraps the runtime copy calls)

namespace {

struct DBuf {
    void *p = nullptr;
    size_t cap = 0;
};

std::atomic<int64_t> g_dgrow_ns{0};  // time in buffer growth (hipFree + hipMalloc), all contexts and stages

int dgrow(DBuf &b, size_t bytes, const char *what = nullptr) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return 0;
    const auto t0 = std::chrono::steady_clock::now();
    if (b.p) grom_dev_free(b.p, b.cap, GROM_DEVCAT_DECODE);
    b.p = nullptr;
    b.cap = 0;
    // growth slack: an eighth for small buffers, 1/64 for the run-sized ones
    // (reserved from estimates that carry their own margin)
    const size_t want = bytes + (bytes >= ((size_t)64 << 20) ? bytes / 64 : bytes / 8) + 256;
    const int e = grom_dev_malloc(&b.p, want, GROM_DEVCAT_DECODE);
    const int64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    g_dgrow_ns += ns;
    if (ns > 20000000 && getenv("GROM_VERBOSE"))
        fprintf(stderr, "grom: device buffer %s of %.3f GB took %.1f ms\n", what ? what : "", (double)want / 1e9, ns / 1e6);
    if (e != 0) return -1;
    b.cap = want;
    return 0;
}

template <class T> T *P(DBuf &b) { return (T *)b.p; }

// bad-state bits
enum : uint32_t { DB_INFLATE = 1, DB_CHAIN = 2, DB_RECORD = 4, DB_TID = 8, DB_UNSORTED = 16, DB_NAMES = 32,
                  DB_OFFCAP = 64, DB_BOUNDS = 128 };

__device__ __forceinline__ uint32_t ldu32(const uint8_t *U, int64_t o) {
    return (uint32_t)U[o] | (uint32_t)U[o + 1] << 8 | (uint32_t)U[o + 2] << 16 | (uint32_t)U[o + 3] << 24;
}

__device__ __forceinline__ uint32_t ldu32a(const uint8_t *U, int64_t p) {  // unaligned, from aligned words
    const uint32_t *a = (const uint32_t *)(U + (p & ~(int64_t)3));
    const uint32_t sh = (uint32_t)(p & 3) * 8;
    const uint32_t w0 = a[0], w1 = a[1];
    return sh ? (w0 >> sh) | (w1 << (32 - sh)) : w0;
}


// the 36-byte record header at o (block_size .. tlen) as 9 words, from 10
// aligned word loads
struct RecHdr {
    uint32_t w[9];
    __device__ int32_t bs() const { return (int32_t)w[0]; }
    __device__ int32_t tid() const { return (int32_t)w[1]; }
    __device__ int32_t pos() const { return (int32_t)w[2]; }
    __device__ int l_qname() const { return (int)(w[3] & 0xff); }
    __device__ int mapq() const { return (int)((w[3] >> 8) & 0xff); }
    __device__ int n_cigar() const { return (int)(w[4] & 0xffff); }
    __device__ int flag() const { return (int)(w[4] >> 16); }
    __device__ int32_t lq() const { return (int32_t)w[5]; }
    __device__ int32_t mtid() const { return (int32_t)w[6]; }
    __device__ int32_t mpos() const { return (int32_t)w[7]; }
    __device__ int32_t isz() const { return (int32_t)w[8]; }
};

__device__ __forceinline__ void load_hdr(const uint8_t *U, int64_t o, RecHdr &h) {
    const uint32_t *a = (const uint32_t *)(U + (o & ~(int64_t)3));
    const uint32_t sh = (uint32_t)(o & 3) * 8;
    uint32_t raw[10];
#pragma unroll
    for (int k = 0; k < 10; k++) raw[k] = a[k];
#pragma unroll
    for (int k = 0; k < 9; k++) h.w[k] = sh ? (raw[k] >> sh) | (raw[k + 1] << (32 - sh)) : raw[k];
}

__device__ __forceinline__ int32_t ld_bs(const uint8_t *U, int64_t o) {
    const uint32_t *a = (const uint32_t *)(U + (o & ~(int64_t)3));
    const uint32_t sh = (uint32_t)(o & 3) * 8;
    const uint32_t w0 = a[0], w1 = a[1];
    return (int32_t)(sh ? (w0 >> sh) | (w1 << (32 - sh)) : w0);
}

#define DD_MAX_REC (256 << 20)

// ---- record starts, many short chains per chunk (guess, then verify) ----
//
// A chunk between two index-named record starts holds ~3,000 records at 30x;
// walking its block_size chain on one lane is 3,000 dependent loads from HBM.
// Instead one workgroup takes the chunk, cut into sub-chunks of WS_G bytes:
// each lane guesses the first record start in its sub-chunk (a header whose
// fields fit the run -- block_size, target id, a NUL-terminated name, field
// sizes within block_size -- and whose successor's block_size and target id
// fit too) and walks the chain to the sub-chunk's end.  Then lane 0 follows
// the true chain across the sub-chunks: sub-chunk q's walk is taken when its
// guess equals the true chain's first start in it (the exit of sub-chunk
// q-1's accepted walk; sub-chunk 0 starts at the chunk's known start), by
// induction every accepted walk is the true chain's; any other sub-chunk is
// walked again from the true position.  A wrong guess costs one re-walk and
// never changes the result.
#define WS_G 4096
#define WS_T 256

__device__ __forceinline__ bool ws_plausible(const uint8_t *U, int64_t p, int64_t end, int32_t tid) {
    if (p + 40 > end) return false;
    const uint32_t *a = (const uint32_t *)(U + (p & ~(int64_t)3));
    const uint32_t sh = (uint32_t)(p & 3) * 8;
    uint32_t raw[7];
#pragma unroll
    for (int k = 0; k < 7; k++) raw[k] = a[k];
    uint32_t w[6];
#pragma unroll
    for (int k = 0; k < 6; k++) w[k] = sh ? (raw[k] >> sh) | (raw[k + 1] << (32 - sh)) : raw[k];
    const int32_t bs = (int32_t)w[0];
    if (bs < 34 || bs > (1 << 20) || (int32_t)w[1] != tid) return false;
    const int lqn = (int)(w[3] & 0xff), nc = (int)(w[4] & 0xffff);
    const int32_t lq = (int32_t)w[5];
    if (lqn < 1 || lq < 0 || 32 + (int64_t)lqn + 4 * (int64_t)nc + (lq + 1) / 2 + lq > (int64_t)bs) return false;
    if (p + 36 + lqn > end || U[p + 36 + lqn - 1] != 0) return false;
    const int64_t q = p + 4 + (int64_t)bs;
    if (q + 8 <= end) {
        const int32_t bs2 = ld_bs(U, q), tid2 = ld_bs(U, q + 4);
        if (bs2 < 34 || bs2 > (1 << 20) || tid2 != tid) return false;
    }
    return true;
}

// the first plausible record start in [lo, hi), -1 none: a sliding window of
// three aligned words gives each position's block_size and target id from
// registers (one new word per four positions); only positions whose two
// fields fit take the full test
__device__ __forceinline__ int64_t ws_guess(const uint8_t *U, int64_t lo, int64_t hi, int64_t end, int32_t tid) {
    int64_t a = lo & ~(int64_t)3;
    const uint32_t *wp = (const uint32_t *)(U + a);
    uint32_t w0 = wp[0], w1 = wp[1], w2 = wp[2];
    for (; a < hi; a += 4) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int64_t p = a + k;
            const uint32_t bs = k ? (w0 >> (8 * k)) | (w1 << (32 - 8 * k)) : w0;
            const uint32_t td = k ? (w1 >> (8 * k)) | (w2 << (32 - 8 * k)) : w1;
            if (p >= lo && p < hi && bs >= 34u && bs <= (1u << 20) && (int32_t)td == tid && ws_plausible(U, p, end, tid))
                return p;
        }
        w0 = w1;
        w1 = w2;
        w2 = wp[(a - (lo & ~(int64_t)3)) / 4 + 3];
    }
    return -1;
}

// walk from o while o < hi: records counted (and written from *w when off,
// below off_cap) and the exit; -1 exit for a block_size outside the record
// limits
__device__ __forceinline__ int64_t ws_walk(const uint8_t *U, int64_t o, int64_t hi, uint32_t &n, int64_t *off,
                                           int64_t w, int64_t off_cap = INT64_MAX) {
    n = 0;
    while (o < hi) {
        const int32_t bs = ld_bs(U, o);
        if (bs < 32 || bs > DD_MAX_REC) return -1;
        if (off && w + n < off_cap) off[w + n] = o;
        o += 4 + (int64_t)bs;
        n++;
    }
    return o;
}

// one workgroup per chunk [S[c], S[c+1]): counts per chunk (off == nullptr) or
// the record offsets from base[c] on
__global__ void __launch_bounds__(WS_T) k_walk_sub(const uint8_t *__restrict__ U, const int64_t *__restrict__ S,
                                                   int64_t sbase, int64_t n_chunks, int32_t tid, int guess,
                                                   uint32_t *__restrict__ q0_stats, uint32_t *__restrict__ cnt,
                                                   const uint32_t *__restrict__ base, int64_t *__restrict__ off,
                                                   uint32_t *__restrict__ bad, int64_t off_cap, int64_t ulen) {
    __shared__ int64_t s_start[WS_T], s_exit[WS_T];
    __shared__ uint32_t s_n[WS_T], s_pre[WS_T];
    __shared__ int64_t s_carry;
    __shared__ uint32_t s_total;
    __shared__ int s_fail;
    const int64_t c = blockIdx.x;
    if (c >= n_chunks) return;
    const int t = threadIdx.x;
    const int64_t c0 = S[c] - sbase, c1 = S[c + 1] - sbase;  // chunk bounds in U (a piece from sbase on)
    if (c0 < 0 || c1 < c0 || c1 > ulen) {  // record starts that are not this piece's: reported, never walked
        if (t == 0) atomicOr(bad, DB_BOUNDS);
        return;
    }
    const int64_t nsub = c1 > c0 ? (c1 - c0 + WS_G - 1) / WS_G : 0;
    if (t == 0) { s_carry = c0; s_total = 0; s_fail = 0; }
    __syncthreads();
    for (int64_t r0 = 0; r0 < nsub; r0 += WS_T) {
        const int64_t q = r0 + t;
        const int64_t lo = c0 + q * WS_G, hi = lo + WS_G < c1 ? lo + WS_G : c1;
        int64_t st = -1, ex = -1;
        uint32_t n = 0;
        if (q < nsub) {
            if (q == 0) st = c0;
            else if (guess == 2) st = lo;  // test hook: guesses that are mostly wrong
            else if (guess == 1)
                st = ws_guess(U, lo, hi, c1, tid);
            if (st >= 0) ex = ws_walk(U, st, hi, n, nullptr, 0);
        }
        s_start[t] = st;
        s_exit[t] = ex;
        s_n[t] = n;
        __syncthreads();
        if (t == 0) {  // the true chain across this round's sub-chunks
            int64_t carry = s_carry;
            const int m = (int)(nsub - r0 < WS_T ? nsub - r0 : WS_T);
            for (int k = 0; k < m && !s_fail; k++) {
                const int64_t khi = c0 + (r0 + k) * WS_G + WS_G < c1 ? c0 + (r0 + k) * WS_G + WS_G : c1;
                if (!(s_start[k] == carry && s_exit[k] >= 0)) {
                    if (!off && q0_stats) atomicAdd(q0_stats, 1u);  // GROM_VERBOSE: re-walked sub-chunks
                    uint32_t kn = 0;
                    const int64_t kex = ws_walk(U, carry, khi, kn, nullptr, 0);
                    if (kex < 0) { atomicOr(bad, DB_RECORD); s_fail = 1; break; }
                    s_start[k] = carry;
                    s_exit[k] = kex;
                    s_n[k] = kn;
                }
                carry = s_exit[k];
            }
            s_carry = carry;
        }
        __syncthreads();
        if (s_fail) return;
        // exclusive prefix of this round's counts (lane 0; 256 adds)
        if (t == 0) {
            const int m = (int)(nsub - r0 < WS_T ? nsub - r0 : WS_T);
            uint32_t acc = s_total;
            for (int k = 0; k < m; k++) { s_pre[k] = acc; acc += s_n[k]; }
            s_total = acc;
        }
        __syncthreads();
        if (off && q < nsub && s_n[t]) {
            uint32_t n2 = 0;
            const int64_t w0 = (int64_t)base[c] + s_pre[t];
            ws_walk(U, s_start[t], c0 + q * WS_G + WS_G < c1 ? c0 + q * WS_G + WS_G : c1, n2, off, w0, off_cap);
            if (w0 + n2 > off_cap) atomicOr(bad, DB_OFFCAP);
        }
        __syncthreads();
    }
    if (t == 0) {
        if (s_carry != c1) atomicOr(bad, DB_CHAIN);
        if (!off) cnt[c] = s_total;
    }
}

// which characters are 'Z'/'H' terminated, and the fixed sizes (bamio.c aux_type_size)
__device__ __forceinline__ int aux_sz(uint8_t t) {
    return (t == 'A' || t == 'c' || t == 'C') ? 1 : (t == 's' || t == 'S') ? 2 : (t == 'i' || t == 'I' || t == 'f') ? 4
         : (t == 'd') ? 8 : -1;
}

// bam_aux_find(b, "XP") || bam_aux_find(b, "SA") with bamio.c's skip rules
__device__ bool has_split_tag(const uint8_t *U, int64_t s, int64_t end) {
    while (s + 3 <= end) {
        const uint8_t t0 = U[s], t1 = U[s + 1], t = U[s + 2];
        if ((t0 == 'X' && t1 == 'P') || (t0 == 'S' && t1 == 'A')) return true;
        s += 3;
        if (t == 'Z' || t == 'H') {
            while (s < end && U[s]) s++;
            s++;
        } else if (t == 'B') {
            if (s + 5 > end) return false;
            const int sz = aux_sz(U[s]);
            const uint32_t n = ldu32(U, s + 1);
            if (sz < 0) return false;
            s += 5 + (int64_t)sz * n;
        } else {
            const int sz = aux_sz(t);
            if (sz < 0) return false;
            s += sz;
        }
    }
    return false;
}

// per record (file order, r >= j0 only): kept / dropped (GROM.c:6418),
// CIGAR words and bases of the kept, split-read candidates (0 < l_aux < 100
// and an XP/SA tag: grom_parse_aux's precondition, GROM.c:5763), positions
__global__ void k_rec_meta(const uint8_t *__restrict__ U, const int64_t *__restrict__ off, int64_t R, int64_t j0,
                           int32_t tid, uint32_t *__restrict__ keep, uint32_t *__restrict__ drop,
                           uint32_t *__restrict__ auxc, uint32_t *__restrict__ ncig, int64_t *__restrict__ nb,
                           uint32_t *__restrict__ nml, int32_t *__restrict__ rpos, uint32_t *__restrict__ bad) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < R; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t o = off[r];
        RecHdr h;
        load_hdr(U, o, h);
        const int32_t lq = h.lq();
        const int lqn = h.l_qname(), nc = h.n_cigar();
        if (lq < 0 || lqn < 1 || 32 + (int64_t)lqn + 4 * (int64_t)nc + (lq + 1) / 2 + lq > (int64_t)h.bs())
            atomicOr(bad, DB_RECORD);
        if (h.tid() != tid) atomicOr(bad, DB_TID);
        rpos[r] = h.pos();
        const bool in = r >= j0;
        const bool dropped = (h.flag() & GF_UNMAP) || (h.flag() & GF_DUP);
        const bool k = in && !dropped;
        keep[r] = k;
        drop[r] = in && dropped;
        ncig[r] = k ? (uint32_t)nc : 0u;
        nb[r] = k ? (((int64_t)lq + 1) & ~1LL) : 0;
        nml[r] = k ? (uint32_t)lqn : 0u;
        bool cand = false;
        if (k) {
            const int64_t data = o + 36, end = o + 4 + h.bs();
            const int64_t aux = data + lqn + 4 * (int64_t)nc + (lq + 1) / 2 + lq;
            const int64_t l_aux = end - aux;
            cand = l_aux > 0 && l_aux < 100 && has_split_tag(U, aux, end);
        }
        auxc[r] = cand;
    }
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

struct StageOut {
    int32_t *pos, *mtid, *mpos, *isize, *lq, *aidx;
    uint16_t *flag;
    uint8_t *mapq;
    uint32_t *coff, *cig, *nid;
    int64_t *boff;
    int32_t *dpos, *dlq;
    int64_t *dbef;
};

// FNV-1a of a read name (up to lqn bytes, stopping at its NUL) and its
// length; the bytes come 32 at a time from eight independent word loads
__device__ __forceinline__ int name_hash(const uint8_t *U, int64_t p, int lqn, uint64_t &hs) {
    hs = 0xcbf29ce484222325ULL;
    int L = 0;
    for (int base = 0; base < lqn; base += 32) {
        uint32_t w[8];
#pragma unroll
        for (int k = 0; k < 8; k++) w[k] = ldu32a(U, p + base + 4 * k);
#pragma unroll
        for (int k = 0; k < 32; k++) {
            const uint32_t c = (w[k >> 2] >> (8 * (k & 3))) & 0xffu;
            if (base + k >= lqn || c == 0) return L;
            hs = (hs ^ c) * 0x100000001b3ULL;
            L++;
        }
    }
    return L;
}

// What the pieces of a run before this one wrote: the offsets a piece's own
// exclusive scans start from in the chromosome's arrays, and the last
// record's position (the sort check across the piece boundary)
struct Carry {
    int64_t k, d, cig, b, nm;  // kept reads, dropped records, CIGAR words, bases, name bytes
    int32_t prev_pos;          // position of the record before the piece (unset: the piece starts the run)
    int32_t has_prev;
};

// the kept reads' fields, CIGAR words, names (into the chromosome's name
// bytes) and name hashes; the dropped records; the split-read candidates'
// record indices; the piece's last record.  r is a record of the piece (its
// offset off[r] in U), j0 the run's first record to take, relative to the
// piece (negative: the piece starts past it).
__global__ void k_rec_write(const uint8_t *__restrict__ U, const int64_t *__restrict__ off, int64_t R, int64_t j0,
                            const uint32_t *__restrict__ keep, const uint32_t *__restrict__ kidx,
                            const uint32_t *__restrict__ drop, const uint32_t *__restrict__ didx,
                            const uint32_t *__restrict__ auxc, const uint32_t *__restrict__ aidx,
                            const uint32_t *__restrict__ coff_s, const int64_t *__restrict__ boff_s,
                            const uint32_t *__restrict__ nmo_s, const int32_t *__restrict__ rpos, StageOut so, Carry car,
                            int64_t *__restrict__ srcs, uint8_t *__restrict__ nm, int64_t *__restrict__ nmoff,
                            uint64_t *__restrict__ keys, uint32_t *__restrict__ vals, int64_t *__restrict__ acand,
                            int32_t read_name_len, int32_t *__restrict__ last, uint32_t *__restrict__ bad) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < R; r += (int64_t)gridDim.x * blockDim.x) {
        if (r > j0 && (r > 0 ? rpos[r] < rpos[r - 1] : (car.has_prev && rpos[0] < car.prev_pos)))
            atomicOr(bad, DB_UNSORTED);
        const int64_t o = off[r];
        RecHdr h;
        load_hdr(U, o, h);
        int32_t hc = 0;
        const int lqn = h.l_qname(), nc = h.n_cigar();
        if (keep[r]) {
            const int64_t i = car.k + kidx[r];
            const int64_t cg0 = car.cig + coff_s[r];
            so.pos[i] = h.pos();
            so.flag[i] = (uint16_t)h.flag();
            so.mapq[i] = (uint8_t)h.mapq();
            so.mtid[i] = h.mtid();
            so.mpos[i] = h.mpos();
            so.isize[i] = h.isz();
            so.lq[i] = h.lq();
            so.coff[i] = (uint32_t)cg0;
            so.boff[i] = car.b + boff_s[r];
            so.aidx[i] = -1;
            srcs[kidx[r]] = o + 36 + lqn + 4 * (int64_t)nc;  // the packed bases in U (the qualities follow)
            const int64_t cg = o + 36 + lqn;
            for (int c = 0; c < nc; c++) {
                const uint32_t op = ldu32(U, cg + 4 * c);
                so.cig[cg0 + c] = op;
                if ((op & 15u) == GC_HARD_CLIP) hc += (int32_t)(op >> 4);
            }
            // the name's bytes (l_qname, its NUL included) for the id check
            // after the last piece (k_name_ids)
            const int64_t nb0 = car.nm + nmo_s[r];
            nmoff[i] = nb0;
            for (int c = 0; c < lqn; c++) nm[nb0 + c] = U[o + 36 + c];
            // name: up to its NUL (pdecode.c buf_intern); empty or >= read_name_len: id 0 (GROM.c:6813)
            uint64_t hs = 0;
            const int L = name_hash(U, o + 36, lqn, hs);
            keys[i] = (L == 0 || L >= read_name_len) ? 0ull : (mix64(hs ^ (uint64_t)L * 0x9e3779b97f4a7c15ULL) | 1ull);
            vals[i] = (uint32_t)i;
            if (auxc[r]) acand[aidx[r]] = r;
        } else if (drop[r]) {
            const int64_t d = car.d + didx[r];
            so.dpos[d] = h.pos();
            so.dlq[d] = h.lq();
            so.dbef[d] = car.k + (int64_t)kidx[r];  // kept reads before it (exclusive scan)
        }
        if (r == R - 1) {  // the piece's last record: position, length, hard clips, kept
            if (!keep[r]) {
                const int64_t cg = o + 36 + lqn;
                for (int c = 0; c < nc; c++) {
                    const uint32_t op = ldu32(U, cg + 4 * c);
                    if ((op & 15u) == GC_HARD_CLIP) hc += (int32_t)(op >> 4);
                }
            }
            last[0] = h.pos();
            last[1] = h.lq();
            last[2] = hc;
            last[3] = keep[r] ? 1 : 0;
        }
    }
}

// Packed bases and qualities of the kept reads.  A read's regions tile the
// stage arrays with no gaps (quality bytes [b, b + nb), bases [b/2, b/2 +
// nb/2), nb = l_qseq rounded up to even, the pad quality byte 0), so the copy
// is driven by the destination: fixed tiles of it, each with the reads that
// touch it.
#define CP_T 8192  // destination bytes per tile: one workgroup, 8 dwords per thread
#define CP_J (CP_T / 1024)
#define CP_G 4  // dwords whose loads are in flight together
#define CP_R 1024   // reads a tile may touch, staged in LDS (more: the tile reads them from global memory)

// the read holding each tile's first destination byte, for the tiles of one
// piece: its reads are kept reads k0.. (n of them) whose regions fill the
// destination [lo, hi) of the qualities and [lo/2, hi/2) of the packed bases
// (read i's qualities [b, b + nb), bases [b/2, b/2 + nb/2), b = boff[i], nb =
// l_qseq rounded up to even); tile t (every CP_T bytes) is entry t - lo /
// CP_T, read indices relative to k0; entry 0 (a tile that starts before the
// piece) is the piece's first read
__global__ void k_tile_first(const int64_t *__restrict__ boff, const int32_t *__restrict__ lq, int64_t k0, int64_t n,
                             int64_t lo, int64_t *__restrict__ tfq, int64_t *__restrict__ tfs) {
    const int64_t tq0 = lo / CP_T, ts0 = (lo / 2) / CP_T;
    if (blockIdx.x == 0 && threadIdx.x == 0) tfq[0] = tfs[0] = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = boff[k0 + i], nb = ((int64_t)lq[k0 + i] + 1) & ~1LL;
        if (nb <= 0) continue;
        for (int64_t t = (b + CP_T - 1) / CP_T; t * CP_T < b + nb; t++) tfq[t - tq0] = i;
        for (int64_t t = (b / 2 + CP_T - 1) / CP_T; t * CP_T < b / 2 + nb / 2; t++) tfs[t - ts0] = i;
    }
}

// One workgroup per CP_T destination bytes of the qualities (QUAL) or the
// packed bases: every dword of the tile stored whole and coalesced.  The
// tile's reads are staged in LDS; each thread finds the read of each of its
// dwords, issues all of their source loads (two aligned words and a shift
// when the four bytes come from one read), then stores; a dword across a read
// boundary (or an odd-length read's pad quality byte, 0) is built byte by
// byte.  The tile is large so the per-tile chain of dependent loads (its
// first read, the staged fields) is paid once per 16 KB.  A piece writes only
// its destination bytes [dlo, dhi): the dwords it shares with the pieces
// either side take byte stores.
template <bool QUAL>
__global__ void __launch_bounds__(256) k_copy_tiles(const uint8_t *__restrict__ U, const int64_t *__restrict__ srcs,
                                                    const int64_t *__restrict__ boff, const int32_t *__restrict__ lq,
                                                    int64_t k0, int64_t n, const int64_t *__restrict__ tf,
                                                    int64_t n_tiles, int64_t dlo, int64_t dhi, int stage_cap,
                                                    uint8_t *__restrict__ dst) {
    __shared__ int64_t s_beg[CP_R], s_src[CP_R];
    __shared__ int32_t s_len[CP_R];
    __shared__ uint8_t s_odd[CP_R];
    const int64_t t_first = dlo / CP_T;
    // byte y of the destination (dlo <= y < dhi): read q (local) holds it
    auto byte_at = [&](int64_t y, int64_t q) -> uint32_t {
        const int64_t i = k0 + q, nb = ((int64_t)lq[i] + 1) & ~1LL;
        const int64_t b0 = QUAL ? boff[i] : boff[i] / 2, L = QUAL ? nb : nb / 2;
        if (QUAL && (lq[i] & 1) && y == b0 + L - 1) return 0u;
        return U[(QUAL ? srcs[q] + nb / 2 : srcs[q]) + (y - b0)];
    };
    for (int64_t tt = blockIdx.x; tt < n_tiles; tt += gridDim.x) {
        const int64_t t = t_first + tt;
        const int64_t r0 = tf[tt], r1 = tt + 1 < n_tiles ? tf[tt + 1] : n - 1;
        const int64_t nr = r1 - r0 + 1;
        const bool staged = nr <= stage_cap;
        __syncthreads();
        if (staged)
            for (int64_t k = threadIdx.x; k < nr; k += blockDim.x) {
                const int64_t q = r0 + k, i = k0 + q, nb = ((int64_t)lq[i] + 1) & ~1LL;
                s_beg[k] = QUAL ? boff[i] : boff[i] / 2;
                s_len[k] = (int32_t)(QUAL ? nb : nb / 2);
                s_src[k] = QUAL ? srcs[q] + nb / 2 : srcs[q];
                s_odd[k] = (uint8_t)(lq[i] & 1);
            }
        __syncthreads();
        if (!staged) {  // more reads than LDS holds (tiny reads): each dword searched in global memory
            for (int j = 0; j < CP_J; j++) {
                const int64_t x = t * CP_T + 4 * (int64_t)(threadIdx.x + 256 * j);
                if (x + 4 <= dlo || x >= dhi) continue;
                int64_t lo = r0, hi = r1;
                const int64_t x0 = x < dlo ? dlo : x;
                while (lo < hi) {
                    const int64_t mid = (lo + hi + 1) / 2;
                    if ((QUAL ? boff[k0 + mid] : boff[k0 + mid] / 2) <= x0) lo = mid;
                    else hi = mid - 1;
                }
                int64_t q = lo;
                const bool whole = x >= dlo && x + 4 <= dhi;
                uint32_t v = 0;
                for (int jj = 0; jj < 4; jj++) {
                    const int64_t y = x + jj;
                    if (y < dlo || y >= dhi) continue;
                    int64_t nb = ((int64_t)lq[k0 + q] + 1) & ~1LL;
                    while (y >= (QUAL ? boff[k0 + q] + nb : boff[k0 + q] / 2 + nb / 2) && q < r1) {
                        q++;
                        nb = ((int64_t)lq[k0 + q] + 1) & ~1LL;
                    }
                    const uint32_t byte = byte_at(y, q);
                    if (whole) v |= byte << (8 * jj);
                    else dst[y] = (uint8_t)byte;
                }
                if (whole) *(uint32_t *)(dst + x) = v;
            }
            continue;
        }
        // Each dword takes its bytes from at most two reads: A, the read that
        // holds its first byte (nA bytes, the last of them possibly an odd
        // read's pad byte, 0), and B, the next read (the other 4 - nA).  The
        // loads of both (two aligned words each) are issued for all of the
        // thread's dwords before any is stored.  A dword at a piece edge, or
        // one that touches a third read or B's pad byte, goes byte by byte.
        // (in groups of CP_G dwords: all of a thread's eight at once took ~200
        // registers, two waves per SIMD)
        int k = 0;  // reads are in destination order: each search starts from the previous dword's read
        const int64_t t0 = t * CP_T;
        for (int g = 0; g < CP_J; g += CP_G) {
        uint32_t wa0[CP_G], wa1[CP_G], wb0[CP_G], wb1[CP_G];
        uint32_t gen = 0, sha = 0, shb = 0, nam = 0, padm = 0;
#pragma unroll
        for (int jg = 0; jg < CP_G; jg++) {
            const int j = g + jg;
            const int32_t xr = 4 * (threadIdx.x + 256 * j);  // offset in the tile
            const int64_t x = t0 + xr;
            const int64_t x0 = x < dlo ? dlo : x;
            int lo = k, hi = (int)nr - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) / 2;
                if (s_beg[mid] <= x0) lo = mid;
                else hi = mid - 1;
            }
            k = lo;
            const int64_t e = s_beg[k] + s_len[k];  // the end of read A's bytes
            const int64_t nA = e - x < 4 ? e - x : 4;
            const bool padA = QUAL && s_odd[k] && e - 1 <= x + 3;
            bool ok = x >= dlo && x + 4 <= dhi && nA > 0;
            int64_t pb = 0;
            if (ok && nA < 4) {
                const int k2 = k + 1;
                ok = k2 < (int)nr && s_beg[k2] == e && x + 4 <= e + s_len[k2] &&
                     !(QUAL && s_odd[k2] && e + s_len[k2] - 1 <= x + 3);
                if (ok) pb = s_src[k2] + (x - e);
            }
            const int64_t pa = s_src[k] + (x - s_beg[k]);
            const uint32_t *a = (const uint32_t *)(U + (pa & ~(int64_t)3));
            const uint32_t *bb = (const uint32_t *)(U + (pb & ~(int64_t)3));
            const bool two = ok && nA < 4;
            gen |= (uint32_t)ok << jg;
            sha |= (uint32_t)(pa & 3) << (2 * jg);
            shb |= (uint32_t)(pb & 3) << (2 * jg);
            nam |= (uint32_t)(nA & 7) << (3 * jg);
            padm |= (uint32_t)padA << jg;
            wa0[jg] = ok ? a[0] : 0u;
            wa1[jg] = ok && (pa & 3) ? a[1] : 0u;
            wb0[jg] = two ? bb[0] : 0u;
            wb1[jg] = two && (pb & 3) ? bb[1] : 0u;
        }
#pragma unroll
        for (int jg = 0; jg < CP_G; jg++) {
            const int j = g + jg;
            const int64_t x = t0 + 4 * (threadIdx.x + 256 * j);
            if (x + 4 <= dlo || x >= dhi) continue;
            if ((gen >> jg) & 1u) {
                const uint32_t s1 = ((sha >> (2 * jg)) & 3u) * 8, s2 = ((shb >> (2 * jg)) & 3u) * 8;
                const uint32_t va = s1 ? (wa0[jg] >> s1) | (wa1[jg] << (32 - s1)) : wa0[jg];
                const uint32_t vb = s2 ? (wb0[jg] >> s2) | (wb1[jg] << (32 - s2)) : wb0[jg];
                const uint32_t nA = (nam >> (3 * jg)) & 7u;
                const uint32_t ma = nA >= 4 ? 0xffffffffu : (1u << (8 * nA)) - 1u;
                uint32_t v = (va & ma) | (vb & ~ma);
                if ((padm >> jg) & 1u) v &= ~(0xffu << (8 * (nA - 1)));  // A's pad byte
                *(uint32_t *)(dst + x) = v;
                continue;
            }
            // a piece edge, a third read or B's pad byte in this dword: the
            // read again, then byte by byte
            const int64_t x0 = x < dlo ? dlo : x;
            int lo = 0, hi = (int)nr - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) / 2;
                if (s_beg[mid] <= x0) lo = mid;
                else hi = mid - 1;
            }
            const bool whole = x >= dlo && x + 4 <= dhi;
            uint32_t v = 0;
            int q = lo;
            for (int jj = 0; jj < 4; jj++) {
                const int64_t y = x + jj;
                if (y < dlo || y >= dhi) continue;
                while (y >= s_beg[q] + s_len[q] && q + 1 < (int)nr) q++;
                uint32_t byte = 0;
                if (!(QUAL && s_odd[q] && y == s_beg[q] + s_len[q] - 1)) byte = U[s_src[q] + (y - s_beg[q])];
                if (whole) v |= byte << (8 * jj);
                else dst[y] = (uint8_t)byte;
            }
            if (whole) *(uint32_t *)(dst + x) = v;
        }
        }
    }
}

// The same copy driven by the reads: 16 lanes per kept read, lane l moving
// bytes [16 l, 16 l + 16) of its quality (QUAL) or packed-base region with
// one unaligned 16-byte load and store; the region's last partial piece is
// loaded whole too (U has slack past every record) and stored exactly, as
// 8/4/2/1-byte stores (a 16-byte store past a read's end would write the
// next read's bytes, another lane's; round 5 moved those bytes one by one);
// an odd-length read's pad quality byte is 0.  A wave's loads and stores
// cover four reads' regions, contiguous in both arrays.
template <bool QUAL>
__global__ void __launch_bounds__(256) k_copy_reads(const uint8_t *__restrict__ U, const int64_t *__restrict__ srcs,
                                                    const int64_t *__restrict__ boff, const int32_t *__restrict__ lq,
                                                    int64_t k0, int64_t n, uint8_t *__restrict__ dst) {
    typedef uint32_t u32x4 __attribute__((vector_size(16)));
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t q = gid >> 4;
    if (q >= n) return;
    const int32_t l = lq[k0 + q];
    const int64_t nb = ((int64_t)l + 1) & ~1LL;
    const int64_t L = QUAL ? nb : nb / 2;
    const int64_t off = 16 * (gid & 15);
    for (int64_t o = off; o < L; o += 256) {
        const uint8_t *src = U + (QUAL ? srcs[q] + nb / 2 : srcs[q]) + o;
        uint8_t *d = dst + (QUAL ? boff[k0 + q] : boff[k0 + q] / 2) + o;
        const int64_t m = L - o < 16 ? L - o : 16;
        const bool pad = QUAL && (l & 1) && o + m == L;  // the region's last byte is the pad
        u32x4 v;
        __builtin_memcpy(&v, src, 16);
        if (pad) {  // byte m - 1 of the piece: 0
            const int pb = (int)m - 1;
            const uint32_t keep = ~(0xffu << (8 * (pb & 3)));
            v[0] &= (pb >> 2) == 0 ? keep : 0xffffffffu;
            v[1] &= (pb >> 2) == 1 ? keep : 0xffffffffu;
            v[2] &= (pb >> 2) == 2 ? keep : 0xffffffffu;
            v[3] &= (pb >> 2) == 3 ? keep : 0xffffffffu;
        }
        if (m == 16) {
            __builtin_memcpy(d, &v, 16);
        } else {
            uint32_t w[4] = {v[0], v[1], v[2], v[3]};
            gi_put_part(d, w, (uint32_t)m);
        }
    }
}

// equal-hash runs: every member's name equal to the run head's (the names'
// bytes, nmoff[i]..nmoff[i + 1], up to the NUL); ids = head + 1
__global__ void k_name_ids(const uint8_t *__restrict__ nm, const int64_t *__restrict__ nmoff,
                           const uint64_t *__restrict__ keys, const uint32_t *__restrict__ vals,
                           const uint32_t *__restrict__ head, int64_t n, uint32_t *__restrict__ nid,
                           uint32_t *__restrict__ bad) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t i = vals[p];
        if (keys[p] == 0) { nid[i] = 0; continue; }
        const uint32_t hp = head[p];
        nid[i] = hp + 1;
        if (hp == (uint32_t)p) continue;
        const uint32_t h = vals[hp];
        const int64_t a0 = nmoff[i], la = nmoff[i + 1] - a0, b0 = nmoff[h], lb = nmoff[h + 1] - b0;
        // Names of equal length: 32 bytes at a time, the nine aligned words
        // that cover each side's 32 loaded at once (a name's bytes are
        // scattered over the chromosome's name array; a byte loop touched
        // each of its lines ~25 times).  A mismatch -- or names of different
        // lengths -- is settled by the byte loop (a NUL ends a name).
        bool eq = true, slow = la != lb;
        for (int64_t c = 0; !slow && c < la; c += 32) {
            const uint8_t *pa = nm + a0 + c, *pb = nm + b0 + c;
            const uint32_t *wa = (const uint32_t *)((uintptr_t)pa & ~(uintptr_t)3);
            const uint32_t *wb = (const uint32_t *)((uintptr_t)pb & ~(uintptr_t)3);
            const uint32_t sa = (uint32_t)((uintptr_t)pa & 3) * 8, sb = (uint32_t)((uintptr_t)pb & 3) * 8;
            uint32_t A[9], B[9];
#pragma unroll
            for (int w = 0; w < 9; w++) {
                A[w] = wa[w];
                B[w] = wb[w];
            }
            const int64_t m = la - c < 32 ? la - c : 32;
#pragma unroll
            for (int w = 0; w < 8; w++) {
                const uint32_t x = (uint32_t)((((uint64_t)A[w + 1] << 32) | A[w]) >> sa);
                const uint32_t y = (uint32_t)((((uint64_t)B[w + 1] << 32) | B[w]) >> sb);
                const int64_t left = m - 4 * w;
                const uint32_t mk = left >= 4 ? 0xffffffffu : left <= 0 ? 0u : (1u << (8 * left)) - 1u;
                slow |= ((x ^ y) & mk) != 0;
            }
        }
        if (slow) {
            for (int64_t c = 0; eq; c++) {
                const uint8_t x = c < la ? nm[a0 + c] : 0, y = c < lb ? nm[b0 + c] : 0;
                if (x != y) eq = false;
                else if (x == 0 || c + 1 >= la) break;
            }
        }
        if (!eq) atomicOr(bad, DB_NAMES);
    }
}

__global__ void k_seg_head(const uint64_t *__restrict__ keys, int64_t n, uint32_t *__restrict__ head) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x)
        head[p] = (p == 0 || keys[p] != keys[p - 1]) ? (uint32_t)p : 0u;
}

// find_insert_mean's per-record test (GROM.c:1226-1317), every record of the run
__global__ void k_stats(const uint8_t *__restrict__ U, const int64_t *__restrict__ off, int64_t R, int32_t min_mapq,
                        uint32_t *__restrict__ q, int32_t *__restrict__ v, int32_t *__restrict__ lqo,
                        int64_t *__restrict__ m) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < R; r += (int64_t)gridDim.x * blockDim.x) {
        RecHdr h;
        load_hdr(U, off[r], h);
        const int fl = h.flag();
        const bool dropped = (fl & GF_UNMAP) || (fl & GF_DUP);
        bool take = false;
        int32_t val = 0;
        if (!dropped) {
            if (!(fl & GF_PAIRED)) { take = true; val = h.lq(); }
            else if (!(fl & GF_MUNMAP) && h.tid() == h.mtid() && h.pos() < h.mpos() && (fl & GF_PROPER) && h.isz() > 0) {
                take = true;
                val = h.isz();
            }
        }
        q[r] = take;
        v[r] = val;
        lqo[r] = h.lq();
        m[r] = (!dropped && h.mapq() >= min_mapq) ? (int64_t)h.lq() : 0;
    }
}

__global__ void k_stats_take(const uint32_t *__restrict__ q, const uint32_t *__restrict__ qi,
                             const int32_t *__restrict__ v, const int32_t *__restrict__ lq,
                             const int64_t *__restrict__ m_incl, int64_t R, int64_t cap, int32_t *__restrict__ ins_out,
                             int32_t *__restrict__ lq_out, int64_t *__restrict__ m_at_cap) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < R; r += (int64_t)gridDim.x * blockDim.x) {
        if (!q[r] || qi[r] >= cap) continue;
        ins_out[qi[r]] = v[r];
        lq_out[qi[r]] = lq[r];
        if (qi[r] == cap - 1) *m_at_cap = m_incl[r];
    }
}

// pack the split-read candidates' records (their full bytes) for the host parse
__global__ void k_aux_pack(const uint8_t *__restrict__ U, const int64_t *__restrict__ off,
                           const int64_t *__restrict__ acand, const int64_t *__restrict__ pk_off, int64_t n,
                           uint8_t *__restrict__ out) {
    for (int64_t a = blockIdx.x; a < n; a += gridDim.x) {
        const int64_t o = off[acand[a]];
        const int64_t len = pk_off[a + 1] - pk_off[a];
        for (int64_t k = threadIdx.x; k < len; k += blockDim.x) out[pk_off[a] + k] = U[o + k];
    }
}

__global__ void k_aux_len(const uint8_t *__restrict__ U, const int64_t *__restrict__ off,
                          const int64_t *__restrict__ acand, int64_t n, int64_t *__restrict__ len,
                          const uint32_t *__restrict__ kidx, int64_t *__restrict__ akidx, int64_t *__restrict__ aoff0) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *aoff0 = 0;  // (the offsets' inclusive scan starts at aoff0 + 1)
    for (int64_t a = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; a < n; a += (int64_t)gridDim.x * blockDim.x) {
        len[a] = 4 + (int64_t)ld_bs(U, off[acand[a]]);
        akidx[a] = kidx[acand[a]];
    }
}

inline unsigned grid_for(int64_t n, int per = 256, unsigned cap = 65536) {
    int64_t g = (n + per - 1) / per;
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

}  // namespace

// totals of the exclusive scans (last element + its input), and the CIGAR
// offsets' closing entry
__global__ void k_totals(const uint32_t *keep, const uint32_t *kidx, const uint32_t *drop, const uint32_t *didx,
                         const uint32_t *auxc, const uint32_t *aidx, const uint32_t *ncig, const uint32_t *coff,
                         const int64_t *nb, const int64_t *boff, const uint32_t *nml, const uint32_t *nmo, int64_t R,
                         int64_t *tot) {
    if (blockIdx.x || threadIdx.x) return;
    if (R == 0) {
        for (int k = 0; k < 6; k++) tot[k] = 0;
        return;
    }
    const int64_t r = R - 1;
    tot[0] = (int64_t)kidx[r] + keep[r];
    tot[1] = (int64_t)didx[r] + drop[r];
    tot[2] = (int64_t)aidx[r] + auxc[r];
    tot[3] = (int64_t)coff[r] + ncig[r];
    tot[4] = boff[r] + nb[r];
    tot[5] = (int64_t)nmo[r] + nml[r];
}

__global__ void k_set_u32(uint32_t *p, uint32_t v) {
    if (!blockIdx.x && !threadIdx.x) *p = v;
}

// first index with a[i] >= x in a sorted array (one lane)
__global__ void k_lower_bound(const int32_t *a, int64_t n, int32_t x, int64_t *out) {
    if (blockIdx.x || threadIdx.x) return;
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) / 2;
        if (a[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    *out = lo;
}

// one loaded run: its inflated bytes and record offsets, loaded on the slot's
// own stream (the prefetch thread inflates and walks run k+1 while the worker
// parses run k on the context's stream)
struct RunSlot {
    DBuf U, blk, status, misc, S, ccnt, cbase, off, tmp;  // (blk, S: unused by the piece decode)
    DBuf tok;  // the two-phase inflate's tokens and per-block counts (dd_inflate_tok_bytes)
    hipStream_t st = nullptr;
    hipEvent_t ev[3] = {};
    int64_t *h_small = nullptr;  // pinned, mapped: k_piece_summary writes it
    int64_t *d_small = nullptr;  // its device address
    bool misc_clean = false;     // misc's flag words are zero (k_piece_summary clears them)
    int64_t R = 0, nblk = 0, ubytes = 0;
};

struct dd_ctx {
    int device = -1;
    RunSlot rs[DD_RSLOTS];
    int depth = 2;  // pieces in flight (GROM_DD_DEPTH, 1..DD_RSLOTS)
    // the next run's first piece, issued while this run's last pieces parse
    // (dd_run_decode's next_cb): its compressed slot, length, first record
    // start and the piece slot it went to
    struct {
        int valid, comp_slot, rslot;
        int64_t comp_len, u_lo;
    } pre = {};
    hipStream_t st = nullptr;
    hipStream_t cst = nullptr;  // compressed runs' host->device copies (dd_comp_upload, the prefetch thread)
    // Compressed-slot ownership between the prefetch thread (which fills a
    // slot) and the worker (which decodes from it).  comp_gen[k] counts the
    // fills of slot k (dd_comp_begin); tab_gen[k] is the fill whose block table
    // and record starts rblk[k]/rS[k] hold (upload_run_tables); a piece is
    // issued only when they agree.  slot_busy[k]: a run's pieces may still
    // read slot k (set by dd_run_decode and the next-run issue, cleared once
    // its streams are drained); a refill waits for it.
    std::atomic<uint64_t> comp_gen[DD_SLOTS] = {};
    uint64_t tab_gen[DD_SLOTS] = {};
    std::mutex slot_mu;
    std::condition_variable slot_cv;
    int slot_busy[DD_SLOTS] = {};
    hipEvent_t tev = nullptr;  // the next run's tables uploaded on its piece slot's stream (issue_next)
    int trace = 0;             // GROM_DD_TRACE: one stderr line per fill and piece
    DBuf dcomp[DD_SLOTS];
    hipEvent_t cev[DD_SLOTS] = {};
    int64_t dcomp_len[DD_SLOTS] = {};
    hipEvent_t ev[4] = {};
    hipEvent_t pev[DD_RSLOTS] = {};  // the piece in slot k is parsed (its U and record offsets are free)
    hipEvent_t rev[2] = {};         // the copy out of pinned ring buffer k is done (dd_comp_chunk)
    DBuf misc;  // the parse's and the statistics' flags and scalars
    DBuf keep, kidx, drop, didx, auxc, aidx, ncig, coff, nb, boff, rpos, krec, keys, vals, keys2, vals2, head, tmp;
    DBuf srcs, tfq, tfs;  // per kept read: its bases' offset in U; per copy tile: its first read
    DBuf sq, sqi, sv, slq, sm, s_ins, s_lq, acand, alen, aoff, akidx, apack;
    DBuf rblk[DD_SLOTS], rS[DD_SLOTS];  // per compressed slot: the run's BGZF block table and record starts
    DBuf nml, nmo, nm, nmoff;  // per piece record: name length, its offset; per chromosome: name bytes, offsets
    // inflated bytes per piece (GROM_DD_PIECE_MB): a launch of k_inflate takes
    // at least the time one lane needs for one block, so a piece must hold a
    // good part of a chip's worth of blocks (two pieces are in flight): 3 GB
    // is ~48 k blocks, ~750 waves.  Round 5 measured 2 GB as fast as 3 GB
    // (profiles/r05r) while the one FASTA loader thread set the run's pace;
    // with that fixed, 3 GB pieces cut the inflate's event time 1.88 ->
    // 1.49 s and the run 3.8 -> 3.55 s for 3 GB more HBM (profiles/r06g, r06i)
    int64_t piece_bytes = (int64_t)3 << 30;
    std::vector<uint8_t> aux_bytes;  // the last run's split-read candidates (dd_parse_out)
    std::vector<int64_t> aux_off, aux_kidx;
    int64_t *h_small = nullptr;  // pinned: totals and scalars
    uint8_t *h_aux = nullptr;    // pinned: packed split-read candidate records
    size_t h_aux_cap = 0;
    float ms_inflate = 0, ms_walk = 0, ms_parse = 0;
    int64_t n_rewalk = 0, n_sub = 0;  // record-walk sub-chunks re-walked by the verifying lane / all
    int cp_cap = CP_R;  // copy tiles staged in LDS up to this many reads (GROM_TEST_CP_UNSTAGED: 0, tests)
    int ws_guess = 1;  // record-start guesses: 1 plausible headers, 0 none, 2 sub-chunk starts (GROM_WS_GUESS, tests)
};

#define DCK(x)                                                                                       \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) {                                                                      \
            if (err) snprintf(err, (size_t)errlen, "HIP error %s at %s:%d", hipGetErrorString(e_), __FILE__, \
                              __LINE__);                                                             \
            return -1;                                                                               \
        }                                                                                            \
    } while (0)
#define DGROW(b, bytes)                                                                              \
    do {                                                                                             \
        if (dgrow((b), (bytes), #b)) {                                                               \
            if (err) snprintf(err, (size_t)errlen, "device decode: hipMalloc(%zu) failed", (size_t)(bytes)); \
            return -1;                                                                               \
        }                                                                                            \
    } while (0)

// The device's first allocation of a process pays for setting up its memory
// (~0.3 s on an MI355X): done by the CLI's start-up thread while the index
// and the FASTA lengths are read, instead of by the decode's first buffer
extern "C" void dd_device_warm(int device) {
    if (hipSetDevice(device) != hipSuccess) return;
    void *p = nullptr;
    if (hipMalloc(&p, (size_t)1 << 20) == hipSuccess) (void)hipFree(p);
}

extern "C" void dd_ctx_free(dd_ctx *c);

// The decode is the whole run's critical path while the scans of earlier
// chromosomes share the GPU: GROM_DD_PRIORITY=1 gives its streams the
// device's highest queue priority.  Off by default: on the configs[2] whole
// run the last chromosome was handed ~0.15 s earlier but the scans it held
// back finished ~0.6 s later
static hipError_t dd_stream_new(hipStream_t *st) {
    const char *e = getenv("GROM_DD_PRIORITY");
    int least = 0, greatest = 0;
    if (e != nullptr && atoi(e) != 0 && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess &&
        greatest != least)
        return hipStreamCreateWithPriority(st, hipStreamNonBlocking, greatest);
    return hipStreamCreateWithFlags(st, hipStreamNonBlocking);
}

// A context made ahead (dd_ctx_prepare, the CLI's HIP start-up thread, while
// the host reads the FASTA lengths and the BAI): making one takes ~0.1 s
// (streams, events, pinned words) that otherwise sat on the run's critical
// path before the first chromosome's read.  The first dd_ctx_new on its
// device takes it; dd_ctx_drop_prepared frees one nobody took.
static std::mutex g_prep_mu;
static dd_ctx *g_prep = nullptr;
static dd_ctx *dd_ctx_make(int device);

extern "C" void dd_ctx_prepare(int device) {
    dd_ctx *c = dd_ctx_make(device);
    std::lock_guard<std::mutex> lk(g_prep_mu);
    if (g_prep) dd_ctx_free(c);
    else g_prep = c;
}

extern "C" void dd_ctx_drop_prepared(void) {
    dd_ctx *c;
    {
        std::lock_guard<std::mutex> lk(g_prep_mu);
        c = g_prep;
        g_prep = nullptr;
    }
    dd_ctx_free(c);
}

extern "C" dd_ctx *dd_ctx_new(int device) {
    {
        std::lock_guard<std::mutex> lk(g_prep_mu);
        if (g_prep && g_prep->device == device) {
            dd_ctx *c = g_prep;
            g_prep = nullptr;
            if (hipSetDevice(device) != hipSuccess) { dd_ctx_free(c); return nullptr; }
            return c;
        }
    }
    return dd_ctx_make(device);
}

static dd_ctx *dd_ctx_make(int device) {
    if (hipSetDevice(device) != hipSuccess) return nullptr;
    dd_ctx *c = new dd_ctx();
    c->device = device;
    if (getenv("GROM_WS_GUESS")) c->ws_guess = atoi(getenv("GROM_WS_GUESS"));
    if (getenv("GROM_TEST_CP_UNSTAGED")) c->cp_cap = 0;
    if (getenv("GROM_DD_PIECE_MB") && atof(getenv("GROM_DD_PIECE_MB")) > 0)
        c->piece_bytes = std::max<int64_t>((int64_t)(atof(getenv("GROM_DD_PIECE_MB")) * 1048576.0), 4096);
    if (getenv("GROM_DD_DEPTH")) c->depth = std::min(std::max(atoi(getenv("GROM_DD_DEPTH")), 1), DD_RSLOTS);
    c->trace = getenv("GROM_DD_TRACE") != nullptr;
    if (dd_stream_new(&c->st) != hipSuccess) { delete c; return nullptr; }
    (void)hipEventCreateWithFlags(&c->tev, hipEventDisableTiming);
    if (dd_stream_new(&c->cst) != hipSuccess) c->cst = nullptr;
    for (int k = 0; k < 4; k++) (void)hipEventCreate(&c->ev[k]);
    for (int k = 0; k < DD_SLOTS; k++) (void)hipEventCreateWithFlags(&c->cev[k], hipEventDisableTiming);
    for (int k = 0; k < DD_RSLOTS; k++) (void)hipEventCreateWithFlags(&c->pev[k], hipEventDisableTiming);
    for (int k = 0; k < 2; k++) (void)hipEventCreateWithFlags(&c->rev[k], hipEventDisableTiming);
    if (hipHostMalloc((void **)&c->h_small, 64 * sizeof(int64_t), 0) != hipSuccess) c->h_small = nullptr;
    for (int k = 0; k < DD_RSLOTS; k++) {
        RunSlot &r = c->rs[k];
        if (dd_stream_new(&r.st) != hipSuccess) r.st = nullptr;
        for (int e = 0; e < 3; e++) (void)hipEventCreate(&r.ev[e]);
        if (hipHostMalloc((void **)&r.h_small, 16 * sizeof(int64_t), hipHostMallocMapped) != hipSuccess ||
            hipHostGetDevicePointer((void **)&r.d_small, r.h_small, 0) != hipSuccess)
            r.h_small = nullptr;
        if (!r.st || !r.h_small) { dd_ctx_free(c); return nullptr; }
    }
    return c;
}

extern "C" void dd_ctx_free(dd_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    // every stream drained before any buffer is freed: a next-run piece issued
    // ahead (issue_next) may still be reading a compressed slot
    if (c->st) (void)hipStreamSynchronize(c->st);
    if (c->cst) (void)hipStreamSynchronize(c->cst);
    for (int k = 0; k < DD_RSLOTS; k++)
        if (c->rs[k].st) (void)hipStreamSynchronize(c->rs[k].st);
    if (c->tev) (void)hipEventDestroy(c->tev);
    for (int k = 0; k < DD_SLOTS; k++) {
        if (c->dcomp[k].p) grom_dev_free(c->dcomp[k].p, c->dcomp[k].cap, GROM_DEVCAT_DECODE);
        if (c->cev[k]) (void)hipEventDestroy(c->cev[k]);
        if (k < 2 && c->rev[k]) (void)hipEventDestroy(c->rev[k]);
    }
    for (int k = 0; k < DD_RSLOTS; k++) {
        if (c->pev[k]) (void)hipEventDestroy(c->pev[k]);
        RunSlot &r = c->rs[k];
        if (r.st) (void)hipStreamSynchronize(r.st);
        DBuf *rb[] = {&r.U, &r.blk, &r.status, &r.misc, &r.S, &r.ccnt, &r.cbase, &r.off, &r.tmp, &r.tok};
        for (DBuf *b : rb)
            if (b->p) grom_dev_free(b->p, b->cap, GROM_DEVCAT_DECODE);
        for (int e = 0; e < 3; e++)
            if (r.ev[e]) (void)hipEventDestroy(r.ev[e]);
        if (r.h_small) (void)hipHostFree(r.h_small);
        if (r.st) (void)hipStreamDestroy(r.st);
    }
    DBuf *all[] = {&c->misc, &c->keep,
                   &c->kidx, &c->drop, &c->didx, &c->auxc, &c->aidx, &c->ncig, &c->coff, &c->nb, &c->boff, &c->rpos,
                   &c->krec, &c->keys, &c->vals, &c->keys2, &c->vals2, &c->head, &c->tmp, &c->sq, &c->sqi, &c->sv,
                   &c->srcs, &c->tfq, &c->tfs,
                   &c->slq, &c->sm, &c->s_ins, &c->s_lq, &c->acand, &c->alen, &c->aoff, &c->akidx, &c->apack,
                   &c->rblk[0], &c->rS[0], &c->rblk[1], &c->rS[1], &c->nml, &c->nmo, &c->nm, &c->nmoff};
    for (DBuf *b : all)
        if (b->p) grom_dev_free(b->p, b->cap, GROM_DEVCAT_DECODE);
    for (int k = 0; k < 4; k++)
        if (c->ev[k]) (void)hipEventDestroy(c->ev[k]);
    if (c->h_small) (void)hipHostFree(c->h_small);
    if (c->h_aux) (void)hipHostFree(c->h_aux);
    if (c->st) (void)hipStreamDestroy(c->st);
    if (c->cst) (void)hipStreamDestroy(c->cst);
    delete c;
}

extern "C" void grom_note_alloc_ns(int64_t ns, size_t bytes) {
    g_dgrow_ns += ns;
    if (ns > 20000000 && getenv("GROM_VERBOSE"))
        fprintf(stderr, "grom: stage buffer of %.2f GB took %.1f ms\n", (double)bytes / 1e9, ns / 1e6);
}

extern "C" void dd_ctx_times(const dd_ctx *c, double *ms) {
    ms[0] = c->ms_inflate;
    ms[1] = c->ms_walk;
    ms[2] = c->ms_parse;
    ms[3] = (double)g_dgrow_ns.load() / 1e6;
}

extern "C" void dd_ctx_counts(const dd_ctx *c, int64_t *rewalked, int64_t *subchunks) {
    *rewalked = c->n_rewalk;
    *subchunks = c->n_sub;
}

// The buffers of one piece (the piece slots, ~GROM_DD_PIECE_MB of inflated
// bytes each) and the chromosome-wide ones, sized once for the largest run
// (recs records, n_starts record starts, its compressed span): a later run
// beyond the estimate still grows them.  Growing a buffer frees the old one,
// which waits for the whole device.
extern "C" int dd_reserve(dd_ctx *c, int64_t span, int64_t ubytes, int64_t recs, int64_t n_starts, char *err,
                          int errlen) {
    DCK(hipSetDevice(c->device));
    // a piece ends past its target (at a chunk boundary, on whole blocks)
    const int64_t pb = std::min<int64_t>(c->piece_bytes, ubytes) * 11 / 10 + (4 << 20);
    // records in a piece at the run's mean record size (+25%); a piece with
    // more grows its offsets (dd_run_decode)
    const int64_t pr = (int64_t)((double)pb * (double)recs / (double)std::max<int64_t>(ubytes, 1) * 1.3) + 4096;
    const int64_t nblk = ubytes / 32768 + 4096;  // BGZF blocks hold at most 64 KiB
    (void)span;  // (the compressed slots grow on the prefetch thread, dd_comp_upload)
    for (int k = 0; k < DD_SLOTS; k++) {
        DGROW(c->rblk[k], sizeof(DdBlock) * (size_t)(nblk + 1));
        DGROW(c->rS[k], sizeof(int64_t) * (size_t)(n_starts + 2));
    }
    for (int k = 0; k < c->depth; k++) {
        RunSlot &r = c->rs[k];
        DGROW(r.U, (size_t)pb + 64);
        DGROW(r.status, (size_t)(pb / 16384 + 1024));
        // (a piece's blocks: at most ~pb / 32 KiB, BGZF writers fill blocks to
        // ~64 KiB; a piece beyond the estimate grows it in issue_piece)
        if (dd_inflate_tok_bytes(1)) DGROW(r.tok, dd_inflate_tok_bytes(pb / 60000 + 64));
        DGROW(r.misc, 256);
        DGROW(r.ccnt, sizeof(uint32_t) * (size_t)(n_starts + 1));
        DGROW(r.cbase, sizeof(uint32_t) * (size_t)(n_starts + 1));
        DGROW(r.off, 8 * (size_t)(pr + 1));
        size_t tb = 0;
        DCK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (uint32_t *)nullptr, (uint32_t *)nullptr, (int)(n_starts + 1),
                                             r.st));
        DGROW(r.tmp, tb);
    }
    DGROW(c->misc, 256);
    {
        size_t tb = 0, t2 = 0, t3 = 0, t4 = 0;
        const int rp = (int)std::min<int64_t>(pr + 1, INT32_MAX), rn = (int)std::min<int64_t>(recs + 1, INT32_MAX);
        DCK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (uint32_t *)nullptr, (uint32_t *)nullptr, rp, c->st));
        DCK(hipcub::DeviceScan::ExclusiveSum(nullptr, t2, (int64_t *)nullptr, (int64_t *)nullptr, rp, c->st));
        DCK(hipcub::DeviceRadixSort::SortPairs(nullptr, t3, (uint64_t *)nullptr, (uint64_t *)nullptr, (uint32_t *)nullptr,
                                               (uint32_t *)nullptr, rn, 0, 64, c->st));
        DCK(hipcub::DeviceScan::InclusiveScan(nullptr, t4, (uint32_t *)nullptr, (uint32_t *)nullptr, hipcub::Max(), rn,
                                              c->st));
        DGROW(c->tmp, std::max(std::max(tb, t2), std::max(t3, t4)));
    }
    // per piece record
    const size_t p4 = 4 * (size_t)(pr + 1), p8 = 8 * (size_t)(pr + 1);
    DGROW(c->keep, p4); DGROW(c->kidx, p4); DGROW(c->drop, p4); DGROW(c->didx, p4); DGROW(c->auxc, p4);
    DGROW(c->aidx, p4); DGROW(c->ncig, p4); DGROW(c->coff, p4); DGROW(c->nml, p4); DGROW(c->nmo, p4);
    DGROW(c->nb, p8); DGROW(c->boff, p8); DGROW(c->rpos, p4); DGROW(c->srcs, p8);
    DGROW(c->tfq, 8 * (size_t)(pb / CP_T + 4));
    DGROW(c->tfs, 8 * (size_t)(pb / 2 / CP_T + 4));
    const size_t na = (size_t)(pr / 8 + 2);
    DGROW(c->acand, 8 * na); DGROW(c->alen, 8 * na); DGROW(c->aoff, 16 * na);  // (aoff also holds the kept indices)
    DGROW(c->apack, (size_t)(pr / 64 + 1) * 512);
    // per chromosome: name hashes and their sort, the names' bytes
    const size_t r4 = 4 * (size_t)(recs + 1), r8 = 8 * (size_t)(recs + 1);
    DGROW(c->keys, r8); DGROW(c->vals, r4); DGROW(c->keys2, r8); DGROW(c->vals2, r4); DGROW(c->head, r4);
    DGROW(c->nmoff, r8);
    DGROW(c->nm, (size_t)recs * 24 + 4096);
    // the insert statistics' sample (the cap's worth)
    const size_t take = 4 * (size_t)std::min<int64_t>(recs + 1, (int64_t)1 << 24);
    DGROW(c->s_ins, take); DGROW(c->s_lq, take);
    return 0;
}

// a run's compressed bytes (pinned, readable 64 bytes past comp_len) into the
// device slot, on the copy stream: returns at once; the host buffer must stay
// untouched until a dd_run_decode of the slot has returned
extern "C" int dd_comp_upload(dd_ctx *c, int slot, const uint8_t *h_comp, int64_t comp_len, char *err, int errlen) {
    if (slot < 0 || slot >= DD_SLOTS) return -1;
    DCK(hipSetDevice(c->device));
    hipStream_t cs = c->cst ? c->cst : c->st;
    {
        std::lock_guard<std::mutex> lk(c->slot_mu);
        if (c->slot_busy[slot]) {
            if (err) snprintf(err, (size_t)errlen, "device decode: compressed slot %d refilled while its run decodes", slot);
            return -1;
        }
        c->comp_gen[slot]++;
    }
    DGROW(c->dcomp[slot], (size_t)comp_len + 64);
    DCK(hipMemcpyAsync(c->dcomp[slot].p, h_comp, (size_t)comp_len + 64, hipMemcpyHostToDevice, cs));
    DCK(hipEventRecord(c->cev[slot], cs));
    c->dcomp_len[slot] = comp_len;
    return 0;
}

// A run's compressed bytes in chunks (the prefetch thread reads them into a
// ring of two pinned buffers): dd_comp_begin sizes the device slot, each
// dd_comp_chunk copies one buffer to its place on the copy stream (the ring
// buffer is free again once dd_comp_ring_wait returns), dd_comp_end marks the
// slot complete for dd_run_decode
extern "C" int dd_comp_begin(dd_ctx *c, int slot, int64_t comp_len, char *err, int errlen) {
    if (slot < 0 || slot >= DD_SLOTS) return -1;
    DCK(hipSetDevice(c->device));
    {
        // the slot's last run must be drained before it is refilled (the
        // prefetch protocol guarantees it; a wait here is reported)
        std::unique_lock<std::mutex> lk(c->slot_mu);
        if (c->slot_busy[slot]) {
            fprintf(stderr, "grom: device decode: compressed slot %d asked for while its run decodes (waiting)\n", slot);
            if (!c->slot_cv.wait_for(lk, std::chrono::seconds(60), [&] { return !c->slot_busy[slot]; })) {
                if (err) snprintf(err, (size_t)errlen, "device decode: compressed slot %d never drained", slot);
                return -1;
            }
        }
        c->comp_gen[slot]++;
    }
    hipStream_t cs = c->cst ? c->cst : c->st;
    c->dcomp_len[slot] = -1;
    if (c->trace) fprintf(stderr, "ddtrace ctx=%p fill slot=%d gen=%llu len=%lld\n", (void *)c, slot,
                          (unsigned long long)c->comp_gen[slot].load(), (long long)comp_len);
    DGROW(c->dcomp[slot], (size_t)comp_len + 64);
    DCK(hipMemsetAsync(P<uint8_t>(c->dcomp[slot]) + comp_len, 0, 64, cs));
    return 0;
}

extern "C" int dd_comp_ring_wait(dd_ctx *c, int ring) {
    if (ring < 0 || ring > 1 || !c->rev[ring]) return 0;
    return hipEventSynchronize(c->rev[ring]) == hipSuccess ? 0 : -1;
}

extern "C" int dd_comp_chunk(dd_ctx *c, int slot, int ring, const uint8_t *h_buf, int64_t dst_off, int64_t n, char *err,
                             int errlen) {
    if (slot < 0 || slot >= DD_SLOTS || ring < 0 || ring > 1) return -1;
    DCK(hipSetDevice(c->device));
    hipStream_t cs = c->cst ? c->cst : c->st;
    DCK(hipMemcpyAsync(P<uint8_t>(c->dcomp[slot]) + dst_off, h_buf, (size_t)n, hipMemcpyHostToDevice, cs));
    DCK(hipEventRecord(c->rev[ring], cs));
    return 0;
}

extern "C" int dd_comp_end(dd_ctx *c, int slot, int64_t comp_len, char *err, int errlen) {
    if (slot < 0 || slot >= DD_SLOTS) return -1;
    DCK(hipSetDevice(c->device));
    hipStream_t cs = c->cst ? c->cst : c->st;
    DCK(hipEventRecord(c->cev[slot], cs));
    c->dcomp_len[slot] = comp_len;
    return 0;
}

// A DBuf grown to `bytes` keeping its first `keep` bytes (a copy on `st`)
static int dgrow_keep(DBuf &b, size_t bytes, size_t keep, hipStream_t st) {
    if (b.cap >= bytes) return 0;
    DBuf nb;
    if (dgrow(nb, bytes + bytes / 8)) return -1;
    if (keep && b.p) {
        if (hipMemcpyAsync(nb.p, b.p, keep, hipMemcpyDeviceToDevice, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return -1;
    }
    if (b.p) grom_dev_free(b.p, b.cap, GROM_DEVCAT_DECODE);
    b = nb;
    return 0;
}

// ---- a run decoded piece by piece ----
//
// A chromosome's run inflates to ~15 GB at 30x (chr1).  It is decoded in
// pieces of whole record-start chunks (the index's 16 kb windows: a chunk
// boundary is a record start, so no record crosses a piece), each ~piece_bytes
// of inflated data: the piece's BGZF blocks are inflated into a piece slot,
// its records walked, the insert statistics taken from it while they are
// wanted, and its records parsed straight into the stage at the offsets the
// earlier pieces reached (the carries).  The read names go to a chromosome-wide
// byte array, so the read-name ids (a sort of the name hashes and a byte
// check of every equal-hash run) come after the last piece.
struct Piece {
    int64_t ca, cb, u_lo, u_hi, bf, bl, base, pbytes;
};

// a run's pieces: consecutive record-start chunks [ca, cb) of about
// piece_bytes of inflated data each, on whole BGZF blocks
static void plan_pieces(const dd_run_req *q, int64_t piece_bytes, std::vector<Piece> &pcs) {
    const int64_t nblk = q->nblk, ns = q->n_starts;
    auto block_of = [&](int64_t u) {  // the block whose output holds inflated offset u
        int64_t lo = 0, hi = nblk - 1;
        while (lo < hi) {
            const int64_t mid = (lo + hi + 1) / 2;
            if (q->blk[mid].out_off <= u) lo = mid;
            else hi = mid - 1;
        }
        return lo;
    };
    pcs.clear();
    for (int64_t ca = 0; ca < ns;) {
        int64_t cb = ca + 1;
        while (cb < ns && q->starts[cb] - q->starts[ca] < piece_bytes) cb++;
        Piece pc;
        pc.ca = ca;
        pc.cb = cb;
        pc.u_lo = q->starts[ca];
        pc.u_hi = cb < ns ? q->starts[cb] : q->u_end;
        if (pc.u_hi > pc.u_lo) {
            pc.bf = block_of(pc.u_lo);
            pc.bl = block_of(pc.u_hi - 1);
            pc.base = q->blk[pc.bf].out_off;
            pc.pbytes = q->blk[pc.bl].out_off + q->blk[pc.bl].out_len - pc.base;
            pcs.push_back(pc);
        }
        ca = cb;
    }
}

// records per inflated byte of the run (the index's count)
static double run_rpb(const dd_run_req *q) {
    return q->count > 0 && q->u_end > q->starts[0] ? (double)q->count / (double)(q->u_end - q->starts[0]) : 1.0 / 34.0;
}

// the run's block table and record starts (+ its end) into its compressed
// slot's device buffers (host copies from pageable memory: done on return)
static int upload_run_tables(dd_ctx *c, const dd_run_req *q, hipStream_t st, char *err, int errlen) {
    const int64_t nblk = q->nblk, ns = q->n_starts;
    DBuf &rblk = c->rblk[q->slot], &rS = c->rS[q->slot];
    c->tab_gen[q->slot] = c->comp_gen[q->slot].load();
    DGROW(rblk, sizeof(DdBlock) * (size_t)(nblk + 1));
    DGROW(rS, sizeof(int64_t) * (size_t)(ns + 2));
    DCK(hipMemcpyAsync(rblk.p, q->blk, sizeof(DdBlock) * (size_t)nblk, hipMemcpyHostToDevice, st));
    // (starts[ns] holds the run's end, dd_run_req)
    DCK(hipMemcpyAsync(rS.p, q->starts, sizeof(int64_t) * (size_t)(ns + 1), hipMemcpyHostToDevice, st));
    return 0;
}

// A piece slot sized once for the run's largest piece: a buffer that grows
// inside the piece loop frees its old block, and a free waits for the whole
// device (the loads in flight, the scans), which serialised the pipeline
static int size_slot(RunSlot &r, const std::vector<Piece> &pcs, double rpb, char *err, int errlen) {
    int64_t mx_pb = 0, mx_blk = 0, mx_ch = 0, mx_oc = 0;
    for (const Piece &pc : pcs) {
        mx_pb = std::max(mx_pb, pc.pbytes);
        mx_blk = std::max(mx_blk, pc.bl - pc.bf + 2);
        mx_ch = std::max(mx_ch, pc.cb - pc.ca + 1);
        mx_oc = std::max(mx_oc, (int64_t)((double)pc.pbytes * rpb * 1.3) + 4096);
    }
    DGROW(r.U, (size_t)mx_pb + 64);
    DGROW(r.status, (size_t)mx_blk);
    DGROW(r.ccnt, sizeof(uint32_t) * (size_t)mx_ch);
    DGROW(r.cbase, sizeof(uint32_t) * (size_t)mx_ch);
    DGROW(r.misc, 256);
    DGROW(r.off, 8 * (size_t)(mx_oc + 1));
    size_t tb = 0;
    DCK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (uint32_t *)nullptr, (uint32_t *)nullptr, (int)mx_ch, r.st));
    DGROW(r.tmp, tb);
    return 0;
}

// a piece's load results for the host, written straight to the slot's mapped
// pinned words (four runtime copies per piece before): the records walked
// (the last chunk's base and count), the flag words and the re-walk count;
// the flag words are cleared for the slot's next piece
__global__ void k_piece_summary(const uint32_t *__restrict__ cbase, const uint32_t *__restrict__ ccnt, int64_t nch,
                                uint32_t *__restrict__ rb, uint32_t *__restrict__ out) {
    if (threadIdx.x == 0) {
        out[0] = cbase[nch - 1];
        out[1] = ccnt[nch - 1];
        out[2] = rb[0];
        out[3] = rb[1];
        out[4] = rb[4];
        out[5] = rb[5];
    }
    __syncthreads();
    if (threadIdx.x < 16) rb[threadIdx.x] = 0;
}

// The load of one piece (inflate, record walk) on piece slot k's own stream.
// The slot is reused once the parse of the piece before in it is done (pev);
// the offsets walk writes up to the slot's record capacity (a piece with more
// records is walked again by the caller after its buffer grows).
static int issue_piece(dd_ctx *c, const dd_run_req *q, const Piece &pc, int k, double rpb, char *err, int errlen) {
    RunSlot &r = c->rs[k];
    hipStream_t ls = r.st;
    // the compressed slot still holds this run, and its tables are this fill's
    if (c->dcomp_len[q->slot] != q->comp_len || c->tab_gen[q->slot] != c->comp_gen[q->slot].load() ||
        pc.bf < 0 || pc.bl >= q->nblk || pc.bl < pc.bf || pc.cb > q->n_starts) {
        if (err) snprintf(err, (size_t)errlen, "device decode: piece of target %d issued against compressed slot %d "
                          "(length %lld, run %lld; table fill %llu, slot fill %llu)", q->tid, q->slot,
                          (long long)c->dcomp_len[q->slot], (long long)q->comp_len, (unsigned long long)c->tab_gen[q->slot],
                          (unsigned long long)c->comp_gen[q->slot].load());
        return -1;
    }
    if (c->trace)
        fprintf(stderr, "ddtrace ctx=%p piece tid=%d slot=%d gen=%llu rslot=%d chunks=%lld-%lld blocks=%lld-%lld u=%lld-%lld\n",
                (void *)c, q->tid, q->slot, (unsigned long long)c->tab_gen[q->slot], k, (long long)pc.ca, (long long)pc.cb,
                (long long)pc.bf, (long long)pc.bl, (long long)pc.u_lo, (long long)pc.u_hi);
    DCK(hipStreamWaitEvent(ls, c->pev[k], 0));
    DCK(hipStreamWaitEvent(ls, c->cev[q->slot], 0));
    DGROW(r.U, (size_t)pc.pbytes + 64);
    DGROW(r.status, (size_t)(pc.bl - pc.bf + 2));
    if (dd_inflate_tok_bytes(1)) DGROW(r.tok, dd_inflate_tok_bytes(pc.bl - pc.bf + 1));
    DGROW(r.ccnt, sizeof(uint32_t) * (size_t)(pc.cb - pc.ca + 1));
    DGROW(r.cbase, sizeof(uint32_t) * (size_t)(pc.cb - pc.ca + 1));
    DGROW(r.misc, 256);
    // record offsets: the run's mean record size (+30%)
    const int64_t ocap = std::max<int64_t>((int64_t)(r.off.cap / 8) - 1, (int64_t)((double)pc.pbytes * rpb * 1.3) + 4096);
    DGROW(r.off, 8 * (size_t)(ocap + 1));
    uint32_t *rb = P<uint32_t>(r.misc);
    if (!r.misc_clean) DCK(hipMemsetAsync(r.misc.p, 0, 64, ls));
    r.misc_clean = true;
    DCK(hipEventRecord(r.ev[0], ls));
    if (dd_inflate_launch(ls, P<uint8_t>(c->dcomp[q->slot]), q->comp_len, P<DdBlock>(c->rblk[q->slot]) + pc.bf,
                          pc.bl - pc.bf + 1, P<uint8_t>(r.U), pc.base, pc.pbytes, P<uint8_t>(r.status), rb + 1, rb + 5,
                          P<uint32_t>(r.tok), r.tok.cap)) {
        if (err) snprintf(err, (size_t)errlen, "inflate launch failed");
        return -1;
    }
    DCK(hipEventRecord(r.ev[1], ls));
    const int64_t nch = pc.cb - pc.ca;
    const int64_t *Sp = P<int64_t>(c->rS[q->slot]) + pc.ca;
    hipLaunchKernelGGL(k_walk_sub, dim3((unsigned)nch), dim3(WS_T), 0, ls, P<uint8_t>(r.U), Sp, pc.base, nch, q->tid,
                       c->ws_guess, rb + 4, P<uint32_t>(r.ccnt), (const uint32_t *)nullptr, (int64_t *)nullptr, rb,
                       (int64_t)INT64_MAX, pc.pbytes);
    size_t tb = 0;
    DCK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, P<uint32_t>(r.ccnt), P<uint32_t>(r.cbase), (int)nch, ls));
    DGROW(r.tmp, tb);
    DCK(hipcub::DeviceScan::ExclusiveSum(r.tmp.p, tb, P<uint32_t>(r.ccnt), P<uint32_t>(r.cbase), (int)nch, ls));
    hipLaunchKernelGGL(k_walk_sub, dim3((unsigned)nch), dim3(WS_T), 0, ls, P<uint8_t>(r.U), Sp, pc.base, nch, q->tid,
                       c->ws_guess, (uint32_t *)nullptr, (uint32_t *)nullptr, P<uint32_t>(r.cbase), P<int64_t>(r.off), rb,
                       ocap, pc.pbytes);
    DCK(hipGetLastError());
    hipLaunchKernelGGL(k_piece_summary, dim3(1), dim3(64), 0, ls, P<uint32_t>(r.cbase), P<uint32_t>(r.ccnt), nch, rb,
                       (uint32_t *)r.d_small);
    DCK(hipGetLastError());
    DCK(hipEventRecord(r.ev[2], ls));
    return 0;
}

static void slot_busy_set(dd_ctx *c, int slot, int busy) {
    std::lock_guard<std::mutex> lk(c->slot_mu);
    c->slot_busy[slot] = busy;
    if (!busy) c->slot_cv.notify_all();
}

static int run_decode(dd_ctx *c, const dd_run_req *q, dd_parse_out *po, int64_t *n_rec, char *err, int errlen);

// One run, its compressed slot held busy until every stream that may read it
// is drained -- on an error too (pieces issued ahead are then still in flight)
extern "C" int dd_run_decode(dd_ctx *c, const dd_run_req *q, dd_parse_out *po, int64_t *n_rec, char *err, int errlen) {
    if (q->slot < 0 || q->slot >= DD_SLOTS) {
        if (err) snprintf(err, (size_t)errlen, "device decode: no compressed slot %d", q->slot);
        return -1;
    }
    slot_busy_set(c, q->slot, 1);
    const int rc = run_decode(c, q, po, n_rec, err, errlen);
    if (rc != 0) {
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->st);
        for (int k = 0; k < DD_RSLOTS; k++) (void)hipStreamSynchronize(c->rs[k].st);
        if (c->pre.valid) {  // (a next-run piece issued before the error: drained above)
            c->pre.valid = 0;
            slot_busy_set(c, c->pre.comp_slot, 0);
        }
    }
    if (!(c->pre.valid && c->pre.comp_slot == q->slot)) slot_busy_set(c, q->slot, 0);
    return rc;
}

static int run_decode(dd_ctx *c, const dd_run_req *q, dd_parse_out *po, int64_t *n_rec, char *err, int errlen) {
    DCK(hipSetDevice(c->device));
    memset(po, 0, sizeof(*po));
    *n_rec = 0;
    if (q->slot < 0 || q->slot >= DD_SLOTS || c->dcomp_len[q->slot] != q->comp_len) {
        if (err) snprintf(err, (size_t)errlen, "device decode: slot %d does not hold the run", q->slot);
        return -1;
    }
    hipStream_t st = c->st;
    std::vector<Piece> pcs;
    plan_pieces(q, c->piece_bytes, pcs);
    const double rpb = run_rpb(q);
    const int D = c->depth;
    // This run's first piece already loading (issued by the run before, while
    // its last pieces parsed)?  Its piece slot is then the base of this run's
    // slot order; a piece issued for a run that is not this one is drained.
    int base = 0;
    bool pre = false;
    if (c->pre.valid) {
        if (c->pre.comp_slot == q->slot && c->pre.comp_len == q->comp_len && !pcs.empty() && pcs[0].u_lo == c->pre.u_lo &&
            c->tab_gen[q->slot] == c->comp_gen[q->slot].load()) {
            base = c->pre.rslot;
            pre = true;
            // this run's later pieces (other slots' streams, ordered after the
            // context stream's events below) read the tables the next-run issue
            // uploaded on the first piece's stream
            DCK(hipStreamWaitEvent(st, c->tev, 0));
        } else {
            DCK(hipStreamSynchronize(c->rs[c->pre.rslot].st));
            if (c->pre.comp_slot != q->slot) slot_busy_set(c, c->pre.comp_slot, 0);
        }
        c->pre.valid = 0;
    }
    if (!pre && upload_run_tables(c, q, st, err, errlen)) return -1;
    DCK(hipStreamWaitEvent(st, c->cev[q->slot], 0));
    for (int k = 0; k < D && k < (int)pcs.size(); k++)
        if (!(pre && k == 0) && size_slot(c->rs[(base + k) % D], pcs, rpb, err, errlen)) return -1;
    const bool parse = q->stage != nullptr;
    Carry car{};
    int64_t R_tot = 0, n_aux = 0, apack_tot = 0;
    int64_t stats_left = q->stats_left;
    int32_t *h_ins = q->h_ins, *h_lq = q->h_lq;
    grom_stage_sizes have{}, cap{};
    grom_reads dv{};
    std::vector<uint8_t> aux_bytes;
    std::vector<int64_t> aux_off(1, 0), aux_kidx;
    int32_t last[4] = {0, 0, 0, 0};
    if (parse && grom_stage_begin(q->stage, nullptr) != GROM_OK) {
        if (err) snprintf(err, (size_t)errlen, "%s", grom_last_error());
        return -1;
    }
    DGROW(c->misc, 256);
    uint32_t *bad = P<uint32_t>(c->misc);
    int64_t *tot = (int64_t *)((char *)c->misc.p + 128);
    int32_t *d_last = (int32_t *)((char *)c->misc.p + 192);
    DCK(hipMemsetAsync(c->misc.p, 0, 256, st));
    for (int k = 0; k < D; k++) DCK(hipEventRecord(c->pev[k], st));
    // The load of piece p (inflate, record walk) runs on piece slot
    // (base + p) % D's own stream, issued D - 1 pieces ahead: it overlaps the
    // statistics and the parse of the pieces before on the context's stream,
    // and the loads in flight together fill the chip (a launch of k_inflate
    // takes at least one lane's time for one block, whatever its size).  When
    // this run issues no more pieces, the next run's first piece (next_cb: its
    // compressed bytes already on the device) goes to the slot that frees
    // next, so its inflate overlaps this run's last parses and name ids
    // instead of waiting for them (24 such drains per genome).
    auto issue = [&](size_t p) -> int { return issue_piece(c, q, pcs[p], (int)((base + p) % D), rpb, err, errlen); };
    auto issue_next = [&](int k) -> int {
        dd_run_req nq;
        memset(&nq, 0, sizeof(nq));
        if (!q->next_cb || !q->next_cb(q->next_arg, &nq)) return 0;
        if (nq.slot < 0 || nq.slot >= DD_SLOTS || nq.slot == q->slot || c->dcomp_len[nq.slot] != nq.comp_len) return 0;
        std::vector<Piece> np;
        plan_pieces(&nq, c->piece_bytes, np);
        if (np.empty()) return 0;
        const double nrpb = run_rpb(&nq);
        slot_busy_set(c, nq.slot, 1);
        c->pre.valid = 1;  // (set first: an error below drains and releases it)
        c->pre.comp_slot = nq.slot;
        c->pre.rslot = k;
        if (upload_run_tables(c, &nq, c->rs[k].st, err, errlen)) return -1;
        DCK(hipEventRecord(c->tev, c->rs[k].st));
        if (size_slot(c->rs[k], np, nrpb, err, errlen) || issue_piece(c, &nq, np[0], k, nrpb, err, errlen)) return -1;
        c->pre.valid = 1;
        c->pre.comp_slot = nq.slot;
        c->pre.comp_len = nq.comp_len;
        c->pre.u_lo = np[0].u_lo;
        c->pre.rslot = k;
        return 0;
    };
    for (size_t p = pre ? 1 : 0; p + 1 < (size_t)D && p < pcs.size(); p++)
        if (issue(p)) return -1;
    for (size_t p = 0; p < pcs.size(); p++) {
        const Piece &pc = pcs[p];
        RunSlot &r = c->rs[(base + p) % D];
        const bool ahead = parse || stats_left > 0;  // (statistics only: stop at the cap)
        if (p + D - 1 < pcs.size() && ahead && issue(p + D - 1)) return -1;
        if (p + D - 1 == pcs.size() && ahead && D > 1 && issue_next((int)((base + pcs.size()) % D))) return -1;
        DCK(hipEventSynchronize(r.ev[2]));
        const uint32_t *hs = (const uint32_t *)r.h_small;
        const int64_t R = (int64_t)hs[0] + hs[1];
        c->n_rewalk += hs[4];
        c->n_sub += (pc.u_hi - pc.u_lo + WS_G - 1) / WS_G;
        if (hs[5] || (hs[2] & DB_BOUNDS)) {  // a block table or record starts outside the piece: a bug, reported
            if (err) snprintf(err, (size_t)errlen, "device decode: piece %zu of target %d reads outside its buffers "
                              "(inflate %u, walk %#x; compressed slot %d fill %llu)", p, q->tid, hs[5], hs[2], q->slot,
                              (unsigned long long)c->tab_gen[q->slot]);
            fprintf(stderr, "grom: %s\n", err ? err : "device decode: bounds");
            return -1;
        }
        if (hs[3]) {
            if (err) snprintf(err, (size_t)errlen, "device inflate: %u blocks failed", hs[3]);
            return -2;
        }
        if (hs[2] & ~DB_OFFCAP) {
            if (err) snprintf(err, (size_t)errlen, "device decode: record chain (%#x) does not follow the index", hs[2]);
            return -2;
        }
        if (hs[2] & DB_OFFCAP) {  // more records than the slot's capacity: the offsets again
            DGROW(r.off, 8 * (size_t)(R + 1));
            DCK(hipMemsetAsync(r.misc.p, 0, 4, r.st));
            hipLaunchKernelGGL(k_walk_sub, dim3((unsigned)(pc.cb - pc.ca)), dim3(WS_T), 0, r.st, P<uint8_t>(r.U),
                               P<int64_t>(c->rS[q->slot]) + pc.ca, pc.base, pc.cb - pc.ca, q->tid, c->ws_guess, (uint32_t *)nullptr,
                               (uint32_t *)nullptr, P<uint32_t>(r.cbase), P<int64_t>(r.off), P<uint32_t>(r.misc),
                               (int64_t)INT64_MAX, pc.pbytes);
            r.misc_clean = false;  // (the re-walk's flag words stay)
            DCK(hipEventRecord(r.ev[2], r.st));
            DCK(hipEventSynchronize(r.ev[2]));
        }
        {
            float a = 0, b = 0;
            (void)hipEventElapsedTime(&a, r.ev[0], r.ev[1]);
            (void)hipEventElapsedTime(&b, r.ev[1], r.ev[2]);
            c->ms_inflate += a;
            c->ms_walk += b;
        }
        DCK(hipStreamWaitEvent(st, r.ev[2], 0));
        // ---- insert statistics (find_insert_mean's sample, file order) ----
        if (stats_left > 0 && R > 0) {
            DGROW(c->keep, 4 * (size_t)(R + 1));
            DGROW(c->kidx, 4 * (size_t)(R + 1));
            DGROW(c->drop, 4 * (size_t)(R + 1));
            DGROW(c->didx, 4 * (size_t)(R + 1));
            DGROW(c->nb, 8 * (size_t)(R + 1));
            DBuf &sq = c->keep, &sqi = c->kidx, &sv = c->drop, &slq = c->didx, &sm = c->nb;
            const int64_t take_cap = std::min<int64_t>(stats_left, R);
            DGROW(c->s_ins, 4 * (size_t)take_cap);
            DGROW(c->s_lq, 4 * (size_t)take_cap);
            hipLaunchKernelGGL(k_stats, dim3(grid_for(R)), dim3(256), 0, st, P<uint8_t>(r.U), P<int64_t>(r.off), R,
                               q->min_mapq, P<uint32_t>(sq), P<int32_t>(sv), P<int32_t>(slq), P<int64_t>(sm));
            size_t t1 = 0, t2 = 0;
            DCK(hipcub::DeviceScan::ExclusiveSum(nullptr, t1, P<uint32_t>(sq), P<uint32_t>(sqi), (int)R, st));
            DCK(hipcub::DeviceScan::InclusiveSum(nullptr, t2, P<int64_t>(sm), P<int64_t>(sm), (int)R, st));
            DGROW(c->tmp, std::max(t1, t2));
            DCK(hipcub::DeviceScan::ExclusiveSum(c->tmp.p, t1, P<uint32_t>(sq), P<uint32_t>(sqi), (int)R, st));
            DCK(hipcub::DeviceScan::InclusiveSum(c->tmp.p, t2, P<int64_t>(sm), P<int64_t>(sm), (int)R, st));
            int64_t *mcap = (int64_t *)((char *)c->misc.p + 64);
            DCK(hipMemsetAsync(mcap, 0xff, 8, st));
            hipLaunchKernelGGL(k_stats_take, dim3(grid_for(R)), dim3(256), 0, st, P<uint32_t>(sq), P<uint32_t>(sqi),
                               P<int32_t>(sv), P<int32_t>(slq), P<int64_t>(sm), R, take_cap, P<int32_t>(c->s_ins),
                               P<int32_t>(c->s_lq), mcap);
            DCK(hipMemcpyAsync(c->h_small, P<uint32_t>(sqi) + R - 1, 4, hipMemcpyDeviceToHost, st));
            DCK(hipMemcpyAsync((char *)c->h_small + 4, P<uint32_t>(sq) + R - 1, 4, hipMemcpyDeviceToHost, st));
            DCK(hipMemcpyAsync(c->h_small + 1, P<int64_t>(sm) + R - 1, 8, hipMemcpyDeviceToHost, st));
            DCK(hipMemcpyAsync(c->h_small + 2, mcap, 8, hipMemcpyDeviceToHost, st));
            DCK(hipStreamSynchronize(st));
            const uint32_t *hs = (const uint32_t *)c->h_small;
            const int64_t nq = (int64_t)hs[0] + hs[1];
            const int64_t n = std::min<int64_t>(nq, stats_left);
            if (n > 0) {
                DCK(hipMemcpyAsync(h_ins, c->s_ins.p, 4 * (size_t)n, hipMemcpyDeviceToHost, st));
                DCK(hipMemcpyAsync(h_lq, c->s_lq.p, 4 * (size_t)n, hipMemcpyDeviceToHost, st));
                DCK(hipStreamSynchronize(st));
            }
            const int complete = nq >= stats_left;
            const int64_t m = complete ? c->h_small[2] : c->h_small[1];
            stats_left -= n;
            h_ins += n;
            h_lq += n;
            if (q->stats_cb) q->stats_cb(q->stats_arg, n, m, complete);
        }
        // ---- parse into the stage ----
        if (parse && R > 0) {
            const int64_t j0l = q->j0 - R_tot;  // the run's first record to take, in this piece
            const size_t p4 = 4 * (size_t)(R + 1), p8 = 8 * (size_t)(R + 1);
            DGROW(c->keep, p4); DGROW(c->kidx, p4); DGROW(c->drop, p4); DGROW(c->didx, p4); DGROW(c->auxc, p4);
            DGROW(c->aidx, p4); DGROW(c->ncig, p4); DGROW(c->coff, p4); DGROW(c->nml, p4); DGROW(c->nmo, p4);
            DGROW(c->nb, p8); DGROW(c->boff, p8); DGROW(c->rpos, p4);
            hipLaunchKernelGGL(k_rec_meta, dim3(grid_for(R)), dim3(256), 0, st, P<uint8_t>(r.U), P<int64_t>(r.off), R,
                               std::max<int64_t>(j0l, 0), q->tid, P<uint32_t>(c->keep), P<uint32_t>(c->drop),
                               P<uint32_t>(c->auxc), P<uint32_t>(c->ncig), P<int64_t>(c->nb), P<uint32_t>(c->nml),
                               P<int32_t>(c->rpos), bad);
            size_t t1 = 0, t2 = 0;
            DCK(hipcub::DeviceScan::ExclusiveSum(nullptr, t1, P<uint32_t>(c->keep), P<uint32_t>(c->kidx), (int)R, st));
            DCK(hipcub::DeviceScan::ExclusiveSum(nullptr, t2, P<int64_t>(c->nb), P<int64_t>(c->boff), (int)R, st));
            DGROW(c->tmp, std::max(t1, t2));
            DCK(hipcub::DeviceScan::ExclusiveSum(c->tmp.p, t1, P<uint32_t>(c->keep), P<uint32_t>(c->kidx), (int)R, st));
            DCK(hipcub::DeviceScan::ExclusiveSum(c->tmp.p, t1, P<uint32_t>(c->drop), P<uint32_t>(c->didx), (int)R, st));
            DCK(hipcub::DeviceScan::ExclusiveSum(c->tmp.p, t1, P<uint32_t>(c->auxc), P<uint32_t>(c->aidx), (int)R, st));
            DCK(hipcub::DeviceScan::ExclusiveSum(c->tmp.p, t1, P<uint32_t>(c->ncig), P<uint32_t>(c->coff), (int)R, st));
            DCK(hipcub::DeviceScan::ExclusiveSum(c->tmp.p, t1, P<uint32_t>(c->nml), P<uint32_t>(c->nmo), (int)R, st));
            DCK(hipcub::DeviceScan::ExclusiveSum(c->tmp.p, t2, P<int64_t>(c->nb), P<int64_t>(c->boff), (int)R, st));
            hipLaunchKernelGGL(k_totals, dim3(1), dim3(1), 0, st, P<uint32_t>(c->keep), P<uint32_t>(c->kidx),
                               P<uint32_t>(c->drop), P<uint32_t>(c->didx), P<uint32_t>(c->auxc), P<uint32_t>(c->aidx),
                               P<uint32_t>(c->ncig), P<uint32_t>(c->coff), P<int64_t>(c->nb), P<int64_t>(c->boff),
                               P<uint32_t>(c->nml), P<uint32_t>(c->nmo), R, tot);
            // the flag words (misc + 0) and the totals (misc + 128) in one copy
            int64_t *hm = c->h_small + 16;
            DCK(hipMemcpyAsync(hm, c->misc.p, 176, hipMemcpyDeviceToHost, st));
            DCK(hipStreamSynchronize(st));
            const int64_t n = hm[16], nd = hm[17], na = hm[18], ncg = hm[19];
            const int64_t nbs = hm[20], nmb = hm[21];
            if (((const uint32_t *)hm)[0]) {
                if (err) snprintf(err, (size_t)errlen, "device decode: records do not parse as the run's (%#x)",
                                  ((const uint32_t *)hm)[0]);
                return -2;
            }
            // the stage: the first piece sizes it for the whole run from its
            // own shares (+6%), later pieces grow it when the run outgrows that
            grom_stage_sizes need{};
            need.n = have.n + n;
            need.n_drop = have.n_drop + nd;
            need.n_cigar_ops = have.n_cigar_ops + ncg;
            need.n_bases = have.n_bases + nbs;
            need.n_aux = 1;
            need.ref_len = q->ref_len;
            if (p == 0 && q->count > R) {
                const double f = (double)q->count / (double)R * 1.02;
                cap.n = (int64_t)(f * (double)n) + 1024;
                cap.n_drop = (int64_t)(f * (double)nd) + 1024;
                cap.n_cigar_ops = (int64_t)(f * (double)ncg) + 1024;
                cap.n_bases = ((int64_t)(f * (double)nbs) + 1024) & ~(int64_t)1;
                // the split-read records the host appends after the run
                // (at most one per candidate)
                cap.n_aux = (int64_t)(f * 1.5 * (double)na) + 1024;
                cap.ref_len = q->ref_len;
            }
            if (need.n > cap.n || need.n_drop > cap.n_drop || need.n_cigar_ops > cap.n_cigar_ops ||
                need.n_bases > cap.n_bases || p == 0) {
                cap.n = std::max(cap.n, need.n);
                cap.n_drop = std::max(cap.n_drop, need.n_drop);
                cap.n_cigar_ops = std::max(cap.n_cigar_ops, need.n_cigar_ops);
                cap.n_bases = std::max(cap.n_bases, need.n_bases);
                cap.n_aux = std::max<int64_t>(cap.n_aux, n_aux + na + 1024);
                cap.ref_len = q->ref_len;
                if (grom_stage_fill_ensure(q->stage, &cap, &have, &dv) != GROM_OK) {
                    if (err) snprintf(err, (size_t)errlen, "%s", grom_last_error());
                    return -1;
                }
            }
            // the chromosome's name bytes and hash arrays
            const int64_t nm_cap = p == 0 && q->count > R ? (int64_t)((double)nmb * (double)q->count / (double)R * 1.02)
                                                          : car.nm + nmb;
            if (dgrow_keep(c->nm, (size_t)std::max<int64_t>(nm_cap, car.nm + nmb) + 64, (size_t)car.nm, st) ||
                dgrow_keep(c->nmoff, 8 * (size_t)(cap.n + 2), 8 * (size_t)car.k, st) ||
                dgrow_keep(c->keys, 8 * (size_t)(cap.n + 1), 8 * (size_t)car.k, st) ||
                dgrow_keep(c->vals, 4 * (size_t)(cap.n + 1), 4 * (size_t)car.k, st)) {
                if (err) snprintf(err, (size_t)errlen, "device decode: hipMalloc failed (name arrays)");
                return -1;
            }
            DGROW(c->srcs, 8 * (size_t)(n + 1));
            // aoff: the candidates' offsets [0, na] and right after them their
            // kept indices (akidx), so one copy brings both back
            DGROW(c->acand, 8 * (size_t)(na + 2)); DGROW(c->alen, 8 * (size_t)(na + 2)); DGROW(c->aoff, 16 * (size_t)(na + 2));
            int64_t *akidx = P<int64_t>(c->aoff) + na + 1;
            StageOut so;
            so.pos = (int32_t *)dv.pos; so.mtid = (int32_t *)dv.mtid; so.mpos = (int32_t *)dv.mpos;
            so.isize = (int32_t *)dv.isize; so.lq = (int32_t *)dv.l_qseq; so.aidx = (int32_t *)dv.aux_idx;
            so.flag = (uint16_t *)dv.flag; so.mapq = (uint8_t *)dv.mapq; so.coff = (uint32_t *)dv.cigar_off;
            so.cig = (uint32_t *)dv.cigar; so.nid = (uint32_t *)dv.name_id; so.boff = (int64_t *)dv.base_off;
            so.dpos = (int32_t *)dv.drop_pos; so.dlq = (int32_t *)dv.drop_lq; so.dbef = (int64_t *)dv.drop_before;
            hipLaunchKernelGGL(k_rec_write, dim3(grid_for(R)), dim3(256), 0, st, P<uint8_t>(r.U), P<int64_t>(r.off), R,
                               j0l, P<uint32_t>(c->keep), P<uint32_t>(c->kidx), P<uint32_t>(c->drop), P<uint32_t>(c->didx),
                               P<uint32_t>(c->auxc), P<uint32_t>(c->aidx), P<uint32_t>(c->coff), P<int64_t>(c->boff),
                               P<uint32_t>(c->nmo), P<int32_t>(c->rpos), so, car, P<int64_t>(c->srcs),
                               P<uint8_t>(c->nm), P<int64_t>(c->nmoff), P<uint64_t>(c->keys), P<uint32_t>(c->vals),
                               P<int64_t>(c->acand), q->read_name_len, d_last, bad);
            const bool tiles = getenv("GROM_COPY_TILES") != nullptr;  // (A/B of the two copies)
            if (n > 0 && !tiles) {  // the bases and qualities of the piece's kept reads
                const unsigned g = (unsigned)((16 * n + 255) / 256);
                hipLaunchKernelGGL(k_copy_reads<true>, dim3(g), dim3(256), 0, st, P<uint8_t>(r.U), P<int64_t>(c->srcs),
                                   (const int64_t *)so.boff, (const int32_t *)so.lq, car.k, n, (uint8_t *)dv.qual);
                hipLaunchKernelGGL(k_copy_reads<false>, dim3(g), dim3(256), 0, st, P<uint8_t>(r.U), P<int64_t>(c->srcs),
                                   (const int64_t *)so.boff, (const int32_t *)so.lq, car.k, n, (uint8_t *)dv.seq);
            } else if (n > 0) {
                const int64_t lo = car.b, hi = car.b + nbs;
                const int64_t nt_q = (hi + CP_T - 1) / CP_T - lo / CP_T, nt_s = (hi / 2 + CP_T - 1) / CP_T - (lo / 2) / CP_T;
                DGROW(c->tfq, 8 * (size_t)(nt_q + 1));
                DGROW(c->tfs, 8 * (size_t)(nt_s + 1));
                hipLaunchKernelGGL(k_tile_first, dim3(grid_for(n)), dim3(256), 0, st, (const int64_t *)so.boff,
                                   (const int32_t *)so.lq, car.k, n, lo, P<int64_t>(c->tfq), P<int64_t>(c->tfs));
                if (nt_q > 0)
                    hipLaunchKernelGGL(k_copy_tiles<true>, dim3((unsigned)std::min<int64_t>(nt_q, 1 << 16)), dim3(256), 0, st,
                                       P<uint8_t>(r.U), P<int64_t>(c->srcs), (const int64_t *)so.boff, (const int32_t *)so.lq,
                                       car.k, n, P<int64_t>(c->tfq), nt_q, lo, hi, c->cp_cap, (uint8_t *)dv.qual);
                if (nt_s > 0)
                    hipLaunchKernelGGL(k_copy_tiles<false>, dim3((unsigned)std::min<int64_t>(nt_s, 1 << 16)), dim3(256), 0,
                                       st, P<uint8_t>(r.U), P<int64_t>(c->srcs), (const int64_t *)so.boff,
                                       (const int32_t *)so.lq, car.k, n, P<int64_t>(c->tfs), nt_s, lo / 2, hi / 2,
                                       c->cp_cap, (uint8_t *)dv.seq);
            }
            // split-read candidates: lengths, offsets, kept indices, packed bytes -> host
            if (na > 0) {
                hipLaunchKernelGGL(k_aux_len, dim3(grid_for(na)), dim3(256), 0, st, P<uint8_t>(r.U), P<int64_t>(r.off),
                                   P<int64_t>(c->acand), na, P<int64_t>(c->alen), P<uint32_t>(c->kidx), akidx,
                                   P<int64_t>(c->aoff));
                size_t t3 = 0;
                DCK(hipcub::DeviceScan::InclusiveSum(nullptr, t3, P<int64_t>(c->alen), P<int64_t>(c->aoff) + 1, (int)na, st));
                DGROW(c->tmp, t3);
                DCK(hipcub::DeviceScan::InclusiveSum(c->tmp.p, t3, P<int64_t>(c->alen), P<int64_t>(c->aoff) + 1, (int)na, st));
                DCK(hipMemcpyAsync(c->h_small + 8, P<int64_t>(c->aoff) + na, 8, hipMemcpyDeviceToHost, st));
            }
            // the flag words and the piece's last record (misc + 192) in one copy
            DCK(hipMemcpyAsync(hm, c->misc.p, 208, hipMemcpyDeviceToHost, st));
            DCK(hipStreamSynchronize(st));
            memcpy(last, hm + 24, 16);
            if (((const uint32_t *)hm)[0]) {
                const uint32_t b1 = ((const uint32_t *)hm)[0];
                if (err) snprintf(err, (size_t)errlen, "device decode: %s (%#x)",
                                  (b1 & DB_UNSORTED) ? "records are not sorted by position" : "record check failed", b1);
                return -2;
            }
            if (na > 0) {
                const int64_t apack = c->h_small[8];
                DGROW(c->apack, (size_t)apack + 16);
                hipLaunchKernelGGL(k_aux_pack, dim3(grid_for(na, 1, 65536)), dim3(64), 0, st, P<uint8_t>(r.U),
                                   P<int64_t>(r.off), P<int64_t>(c->acand), P<int64_t>(c->aoff), na, P<uint8_t>(c->apack));
                const size_t ab0 = aux_bytes.size(), ao0 = aux_off.size(), ak0 = aux_kidx.size();
                aux_bytes.resize(ab0 + (size_t)apack);
                aux_off.resize(ao0 + (size_t)na);
                aux_kidx.resize(ak0 + (size_t)na);
                DCK(hipMemcpyAsync(aux_bytes.data() + ab0, c->apack.p, (size_t)apack, hipMemcpyDeviceToHost, st));
                std::vector<int64_t> ok2(2 * (size_t)na);  // offsets [1, na], then the kept indices
                DCK(hipMemcpyAsync(ok2.data(), P<int64_t>(c->aoff) + 1, 16 * (size_t)na, hipMemcpyDeviceToHost, st));
                DCK(hipStreamSynchronize(st));
                memcpy(aux_off.data() + ao0, ok2.data(), 8 * (size_t)na);
                memcpy(aux_kidx.data() + ak0, ok2.data() + na, 8 * (size_t)na);
                for (size_t k = ao0; k < ao0 + (size_t)na; k++) aux_off[k] += apack_tot;  // run-wide offsets
                for (size_t k = ak0; k < ak0 + (size_t)na; k++) aux_kidx[k] += car.k;    // kept index in the chromosome
                apack_tot += apack;
                n_aux += na;
            }
            // the carries for the next piece
            car.k += n;
            car.d += nd;
            car.cig += ncg;
            car.b += nbs;
            car.nm += nmb;
            car.prev_pos = last[0];
            car.has_prev = 1;
            have.n = car.k;
            have.n_drop = car.d;
            have.n_cigar_ops = car.cig;
            have.n_bases = car.b;
        }
        DCK(hipEventRecord(c->pev[(base + p) % D], st));  // the slot's piece is done with
        R_tot += R;
        if (!parse && stats_left <= 0) break;  // statistics only: the cap is reached
    }
    for (int k = 0; k < D; k++)  // (loads issued ahead; the next run's first piece goes on)
        if (!(c->pre.valid && k == c->pre.rslot)) DCK(hipStreamSynchronize(c->rs[k].st));
    *n_rec = R_tot;
    po->n_rec = R_tot;
    if (!parse) return 0;
    // ---- after the last piece: the stage's final counts, the name ids ----
    const int64_t n = car.k;
    DCK(hipEventRecord(c->ev[2], st));
    grom_stage_sizes fin{};
    fin.n = n;
    fin.n_drop = car.d;
    fin.n_cigar_ops = car.cig;
    fin.n_bases = car.b;
    fin.ref_len = q->ref_len;
    if (grom_stage_fill_ensure(q->stage, &fin, &have, &dv) != GROM_OK || grom_stage_fill_set(q->stage, &fin) != GROM_OK) {
        if (err) snprintf(err, (size_t)errlen, "%s", grom_last_error());
        return -1;
    }
    hipLaunchKernelGGL(k_set_u32, dim3(1), dim3(1), 0, st, (uint32_t *)dv.cigar_off + n, (uint32_t)car.cig);
    if (n > 0) {
        DCK(hipMemcpyAsync(P<int64_t>(c->nmoff) + n, &car.nm, 8, hipMemcpyHostToDevice, st));
        DGROW(c->keys2, 8 * (size_t)(n + 1));
        DGROW(c->vals2, 4 * (size_t)(n + 1));
        DGROW(c->head, 4 * (size_t)(n + 1));
        size_t tb = 0, t2 = 0;
        DCK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, P<uint64_t>(c->keys), P<uint64_t>(c->keys2),
                                               P<uint32_t>(c->vals), P<uint32_t>(c->vals2), (int)n, 0, 64, st));
        DCK(hipcub::DeviceScan::InclusiveScan(nullptr, t2, P<uint32_t>(c->head), P<uint32_t>(c->head), hipcub::Max(),
                                              (int)n, st));
        DGROW(c->tmp, std::max(tb, t2));
        DCK(hipcub::DeviceRadixSort::SortPairs(c->tmp.p, tb, P<uint64_t>(c->keys), P<uint64_t>(c->keys2),
                                               P<uint32_t>(c->vals), P<uint32_t>(c->vals2), (int)n, 0, 64, st));
        hipLaunchKernelGGL(k_seg_head, dim3(grid_for(n)), dim3(256), 0, st, P<uint64_t>(c->keys2), n,
                           P<uint32_t>(c->head));
        DCK(hipcub::DeviceScan::InclusiveScan(c->tmp.p, t2, P<uint32_t>(c->head), P<uint32_t>(c->head), hipcub::Max(),
                                              (int)n, st));
        hipLaunchKernelGGL(k_name_ids, dim3(grid_for(n)), dim3(256), 0, st, P<uint8_t>(c->nm), P<int64_t>(c->nmoff),
                           P<uint64_t>(c->keys2), P<uint32_t>(c->vals2), P<uint32_t>(c->head), n,
                           (uint32_t *)dv.name_id, bad);
    }
    DCK(hipMemcpyAsync(c->h_small, bad, 8, hipMemcpyDeviceToHost, st));
    DCK(hipEventRecord(c->ev[3], st));
    DCK(hipStreamSynchronize(st));
    if (((const uint32_t *)c->h_small)[0] & DB_NAMES) {
        if (err) snprintf(err, (size_t)errlen, "device decode: read-name hash collision (%#x)", ((const uint32_t *)c->h_small)[0]);
        return -2;
    }
    float d = 0;
    (void)hipEventElapsedTime(&d, c->ev[2], c->ev[3]);
    c->ms_parse += d;
    po->n_kept = n;
    po->n_drop = car.d;
    po->n_cig = car.cig;
    po->n_bases = car.b;
    po->n_auxc = n_aux;
    po->last_pos = last[0];
    po->last_lq = last[1];
    po->last_hclip = last[2];
    po->last_kept = last[3];
    // the split-read candidates (host): the context keeps them until the next run
    c->aux_bytes.swap(aux_bytes);
    c->aux_off.swap(aux_off);
    c->aux_kidx.swap(aux_kidx);
    po->aux_bytes = c->aux_bytes.data();
    po->aux_off = c->aux_off.data();
    po->aux_kidx = c->aux_kidx.data();
    return 0;
}

// n bytes of device memory to the host, ordered after this context's work
extern "C" int dd_copy_d2h(dd_ctx *c, void *dst, const void *src, size_t n) {
    if (hipSetDevice(c->device) != hipSuccess || n > 64 * sizeof(int64_t) ||
        hipMemcpyAsync(c->h_small, src, n, hipMemcpyDeviceToHost, c->st) != hipSuccess ||
        hipStreamSynchronize(c->st) != hipSuccess)
        return -1;
    memcpy(dst, c->h_small, n);
    return 0;
}

extern "C" int dd_stage_prefix(dd_ctx *c, grom_stage *stage, int32_t s0, int64_t *sk, int64_t *sd) {
    if (hipSetDevice(c->device) != hipSuccess) return -1;
    grom_reads dv;
    if (grom_stage_dev_reads(stage, &dv) != GROM_OK) return -1;
    int64_t *o = (int64_t *)((char *)c->misc.p + 224);
    hipLaunchKernelGGL(k_lower_bound, dim3(1), dim3(1), 0, c->st, dv.pos, dv.n, s0, o);
    hipLaunchKernelGGL(k_lower_bound, dim3(1), dim3(1), 0, c->st, dv.drop_pos, dv.n_drop, s0, o + 1);
    if (hipMemcpyAsync(c->h_small, o, 16, hipMemcpyDeviceToHost, c->st) != hipSuccess ||
        hipStreamSynchronize(c->st) != hipSuccess)
        return -1;
    *sk = c->h_small[0];
    *sd = c->h_small[1];
    return 0;
}
