"""grom_amd -- Python view of the MI355X-native GROM scan library.

The product is the C ABI in ``include/grom_amd.h`` (``grom_amd/lib/libgrom_amd.so``)
and the drop-in CLI ``grom_amd/bin/grom``.  This module only binds them with
ctypes for tests and ``bench.py``; it has no compute of its own and raises if the
HIP library is missing (there is no CPU fallback).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(ROOT)
# GROM_AMD_LIB selects another build of the same library (kernel tuning variants)
LIB_PATH = os.environ.get("GROM_AMD_LIB") or os.path.join(ROOT, "lib", "libgrom_amd.so")
GROM_BIN = os.path.join(ROOT, "bin", "grom")
SYNTH_BIN = os.path.join(ROOT, "bin", "grom_synth")
MAX_TRIALS = 1000
NCOUNT = 40


class Params(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "min_mapq", "rd_min_mapq", "min_base_qual", "min_snv", "ploidy", "gender", "splitread", "rmdup", "vcf",
        "overlap_mult", "sv_list_len", "rmdup_list_len", "read_name_len", "sc_min")] + \
        [(n, C.c_double) for n in ("min_snv_ratio", "min_ave_bq", "snv_rd_min_factor", "high_cov_min_snv_ratio")] + \
        [(n, C.c_int32) for n in ("insert_mean", "insert_min_size", "insert_max_size", "lseq", "one_base_rd_len",
                                  "half_one_base_rd_len", "r14_one_base_rd_len", "r34_one_base_rd_len",
                                  "ranks_stdev", "chr_rd_threshold_factor")] + \
        [(n, C.c_int64) for n in ("min_repeat", "min_blocks", "block_min", "min_rd_window_len", "max_rd_window_len",
                                  "windows_sampling_factor", "dup_threshold_factor")] + \
        [(n, C.c_double) for n in ("min_repeat_stdev", "rd_pval_threshold", "mapq_factor")] + \
        [(n, C.c_int32) for n in ("min_disc", "sc_range", "max_split_loss", "min_sr_len", "max_homopolymer",
                                  "max_ins_range", "sv_list2_len", "pad_sv")] + \
        [(n, C.c_double) for n in ("pval_threshold", "pval_threshold1", "pval_insertion1", "pval_insertion",
                                   "min_sv_ratio", "min_indel_ratio", "max_evidence_ratio", "range_mult",
                                   "max_inv_rd_diff", "min_overlap_ratio")] + \
        [("gen1000_window", C.c_int64)]


class Chrom(C.Structure):
    _fields_ = [("ref", C.c_void_p), ("len", C.c_int64), ("name", C.c_char_p), ("tid", C.c_int32),
                ("n_skip", C.c_int32), ("p_last", C.c_int32), ("cnv", C.c_int32), ("seed", C.c_uint32),
                ("lseq_tail", C.c_int32), ("pad", C.c_int32)]


class Reads(C.Structure):
    _fields_ = [("n", C.c_int64), ("n_cigar_ops", C.c_int64), ("n_bases", C.c_int64)] + \
        [(n, C.c_void_p) for n in ("pos", "flag", "mapq", "mtid", "mpos", "isize", "l_qseq", "cigar_off", "cigar",
                                   "base_off", "seq", "qual", "name_id")] + \
        [("n_aux", C.c_int64), ("aux_idx", C.c_void_p), ("aux", C.c_void_p),
         ("n_drop", C.c_int64), ("drop_pos", C.c_void_p), ("drop_lq", C.c_void_p), ("drop_before", C.c_void_p)]


class Aux(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("pos", "start_adj", "end_adj", "end_adj_indel")] + \
        [("mq", C.c_int16), ("strand", C.c_uint8), ("same_chr", C.c_uint8), ("pad", C.c_int32)]


class SynthSpec(C.Structure):
    """grom_synth_spec: one chromosome of a multi-chromosome synthetic genome."""
    _fields_ = [("n_chr", C.c_int32), ("chrom", C.c_int32), ("chr_len", C.POINTER(C.c_int64)),
                ("names", C.c_char_p), ("coverage", C.c_double), ("read_len", C.c_int32), ("ploidy", C.c_int32),
                ("insert_mean", C.c_double), ("insert_sd", C.c_double), ("dup_frac", C.c_double),
                ("sv_per_mb", C.c_double), ("cnv_rate", C.c_double), ("cnv_min", C.c_int64),
                ("cnv_max", C.c_int64), ("chr_cov", C.POINTER(C.c_double)), ("munmap_frac", C.c_double),
                ("seed", C.c_uint64)]


class Out(C.Structure):
    _fields_ = [("vcf", C.c_void_p), ("vcf_len", C.c_size_t), ("vcf_cap", C.c_size_t),
                ("ctx", C.c_void_p), ("ctx_len", C.c_size_t), ("ctx_cap", C.c_size_t),
                ("side", C.c_void_p), ("side_len", C.c_size_t), ("side_cap", C.c_size_t),
                ("side_written", C.c_int32), ("side_pad", C.c_int32)]


class Stats(C.Structure):
    _fields_ = [("ms_total", C.c_double), ("ms_pileup", C.c_double), ("ms_cnv", C.c_double),
                ("cnv_rows", C.c_int64), ("bases_evaluated", C.c_int64),
                ("snv_candidates", C.c_int64), ("mismatch_events", C.c_int64)]


class IndelRec(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("pos", "ins", "ins_len", "del_f", "del_f_len", "del_f_rd", "del_r",
                                         "del_r_len", "del_r_rd", "other_len")] + \
        [("ins_seq", C.c_char * 52), ("pad", C.c_int32)]


class SvRec(C.Structure):
    _fields_ = [("pos", C.c_int32), ("other_len", C.c_int32), ("cnt", C.c_int32 * 10), ("rs", C.c_int32 * 10),
                ("re", C.c_int32 * 10), ("dist", C.c_double * 10), ("ctx_mchr", C.c_int32 * 2)] + \
        [(n, C.c_int32) for n in ("rd_add", "conc", "ins", "mun_f", "mun_r", "pad")]


# numpy view of the breakpoint test-hook records (grom_sv_rec)
SV_DTYPE = np.dtype([("pos", "<i4"), ("other_len", "<i4"), ("cnt", "<i4", 10), ("rs", "<i4", 10), ("re", "<i4", 10),
                     ("dist", "<f8", 10), ("ctx_mchr", "<i4", 2), ("rd_add", "<i4"), ("conc", "<i4"), ("ins", "<i4"),
                     ("mun_f", "<i4"), ("mun_r", "<i4"), ("pad", "<i4")])


# every function declared in include/grom_amd.h, with its ctypes signature
_SIGS = {
    "grom_abi_version": (C.c_int, []),
    "grom_abi_struct_size": (C.c_size_t, [C.c_int]),
    "grom_device_count": (C.c_int, []),
    "grom_last_error": (C.c_char_p, []),
    "grom_set_last_error": (None, [C.c_char_p]),
    "grom_device_mem_free": (C.c_int64, [C.c_int]),
    "grom_dev_init": (C.c_int, [C.c_int, C.POINTER(Params), C.c_void_p, C.c_void_p]),
    "grom_dev_fini": (None, [C.c_int]),
    "grom_ctx_init": (C.c_int, [C.c_int, C.c_int, C.POINTER(Params), C.c_void_p, C.c_void_p]),
    "grom_ctx_set_params": (C.c_int, [C.c_int, C.POINTER(Params)]),
    "grom_scan_chrom": (C.c_int, [C.c_int, C.POINTER(Chrom), C.POINTER(Reads), C.POINTER(Out), C.POINTER(Stats)]),
    "grom_scan_chrom_device": (C.c_int, [C.c_int, C.POINTER(Chrom), C.POINTER(Reads), C.POINTER(Out),
                                         C.POINTER(Stats)]),
    "grom_debug_counts": (C.c_int, [C.c_int, C.POINTER(Chrom), C.POINTER(Reads), C.POINTER(C.c_int32), C.c_void_p,
                                    C.c_int64, C.c_void_p]),
    "grom_debug_indels": (C.c_int64, [C.c_int, C.c_void_p, C.c_int64]),
    "grom_debug_sv": (C.c_int64, [C.c_int, C.c_void_p, C.c_int64]),
    "grom_build_tables": (None, [C.c_int32, C.c_void_p, C.c_void_p]),
    "grom_default_params": (None, [C.POINTER(Params)]),
    "grom_params_set_insert": (None, [C.POINTER(Params), C.c_int32, C.c_int32, C.c_int32, C.c_int32]),
    "grom_out_free": (None, [C.POINTER(Out)]),
    "grom_fmt_selftest": (C.c_int64, [C.c_int64, C.c_uint64]),
    "grom_bai_build": (C.c_int, [C.c_char_p]),
    "grom_bai_summary": (C.c_int, [C.c_char_p, C.POINTER(C.c_int64)]),
    "grom_bai_selftest": (C.c_int64, [C.c_char_p, C.c_int64, C.c_uint64, C.POINTER(C.c_int64)]),
    "grom_upload": (C.c_int, [C.c_int, C.POINTER(Chrom), C.POINTER(Reads), C.POINTER(Chrom), C.POINTER(Reads)]),
    "grom_synth_batch": (C.c_void_p, [C.c_int64, C.c_double, C.c_int32, C.c_double, C.c_double, C.c_uint64,
                                      C.POINTER(Params)]),
    "grom_synth_chrom": (C.c_void_p, [C.POINTER(SynthSpec), C.POINTER(Params)]),
    "grom_synth_chrom_stream": (C.c_void_p, [C.POINTER(SynthSpec), C.POINTER(Params)]),  # ABI 7
    "grom_reads_digest": (C.c_uint64, [C.POINTER(Reads)]),
    "grom_resident_new": (C.c_void_p, [C.c_int, C.POINTER(Chrom), C.POINTER(Reads), C.POINTER(Chrom),
                                       C.POINTER(Reads)]),
    "grom_resident_bytes": (C.c_int64, [C.c_void_p]),
    "grom_resident_free": (None, [C.c_void_p]),
    "grom_batch_get": (C.c_int, [C.c_void_p, C.POINTER(Chrom), C.POINTER(Reads)]),
    "grom_batch_release": (None, [C.c_void_p]),
    "grom_cli_main": (C.c_int, [C.c_int, C.POINTER(C.c_char_p)]),
    "grom_ctx_postpass": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(C.c_char_p), C.c_int32, C.c_int32, C.c_int32,
                                    C.POINTER(Out)]),
    # streamed input (ABI 5)
    "grom_pinned_alloc": (C.c_void_p, [C.c_size_t]),
    "grom_pinned_free": (None, [C.c_void_p]),
    "grom_stage_new": (C.c_void_p, [C.c_int]),
    "grom_stage_free": (None, [C.c_void_p]),
    "grom_stage_begin": (C.c_int, [C.c_void_p, C.c_void_p]),
    "grom_stage_set_ref": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64]),
    "grom_stage_append": (C.c_int64, [C.c_void_p, C.POINTER(Reads)]),
    "grom_stage_ticket_done": (C.c_int, [C.c_void_p, C.c_int64]),
    "grom_stage_ticket_wait": (C.c_int, [C.c_void_p, C.c_int64]),
    "grom_stage_trim": (C.c_int, [C.c_void_p, C.c_int64]),
    "grom_stage_patch_aux": (C.c_int, [C.c_void_p, C.c_int64, C.POINTER(Aux)]),
    "grom_stage_bytes": (C.c_int64, [C.c_void_p]),
    "grom_stage_view": (C.c_int, [C.c_void_p, C.POINTER(Chrom), C.POINTER(Chrom), C.POINTER(Reads)]),
    "grom_scan_chrom_staged": (C.c_int, [C.c_int, C.c_void_p, C.POINTER(Chrom), C.POINTER(Out), C.POINTER(Stats)]),
    "grom_debug_counts_staged": (C.c_int, [C.c_int, C.c_void_p, C.POINTER(Chrom), C.POINTER(C.c_int32), C.c_void_p,
                                           C.c_int64, C.c_void_p]),
}

_lib = None


def lib() -> C.CDLL:
    """The loaded HIP library; raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"grom_amd: {LIB_PATH} missing -- run `make` (or __graft_entry__.build()); "
                               "there is no CPU fallback")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    return lib().grom_last_error().decode()


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc}): {last_error()}")


def default_params() -> Params:
    p = Params()
    lib().grom_default_params(C.byref(p))
    return p


def build_tables(min_mapq: int = 20):
    """(hez, mq) binomial tables exactly as a `-q min_mapq` run uses them."""
    hez = np.zeros((MAX_TRIALS + 1, MAX_TRIALS + 1), np.float64)
    mq = np.zeros_like(hez)
    lib().grom_build_tables(min_mapq, hez.ctypes.data, mq.ctypes.data)
    return hez, mq


class Device:
    """One initialised GPU (grom_dev_init / grom_dev_fini)."""

    def __init__(self, device: int, params: Params, slot: "int | None" = None):
        """slot: the library context to use (default: the device number); a
        second slot on the same device scans concurrently with the first."""
        self.device = device if slot is None else slot  # the slot every call names
        self.gpu = device
        self.params = params
        self.hez, self.mq = build_tables(params.min_mapq)
        check(lib().grom_ctx_init(self.device, device, C.byref(params), self.hez.ctypes.data, self.mq.ctypes.data),
              "grom_ctx_init")

    def close(self):
        lib().grom_dev_fini(self.device)

    def scan(self, chrom: Chrom, reads: Reads, device_resident: bool = False, out: "Out | None" = None):
        """Scan one chromosome; returns (VCF text, Stats).  With a caller-owned
        `out` (reused across calls, freed with grom_out_free) the text stays
        in out.vcf and the first element is its length instead."""
        own = out is None
        if own:
            out = Out()
        else:
            out.vcf_len = 0
            out.ctx_len = 0
        st = Stats()
        fn = lib().grom_scan_chrom_device if device_resident else lib().grom_scan_chrom
        check(fn(self.device, C.byref(chrom), C.byref(reads), C.byref(out), C.byref(st)), "scan")
        if not own:
            return out.vcf_len, st
        text = C.string_at(out.vcf, out.vcf_len).decode() if out.vcf_len else ""
        lib().grom_out_free(C.byref(out))
        return text, st

    def scan_rows(self, chrom: Chrom, reads: Reads, device_resident: bool = False):
        """Scan one chromosome; returns (VCF text, raw CTX rows, Stats).  The raw
        CTX rows of every chromosome feed ctx_postpass."""
        out, st = Out(), Stats()
        fn = lib().grom_scan_chrom_device if device_resident else lib().grom_scan_chrom
        check(fn(self.device, C.byref(chrom), C.byref(reads), C.byref(out), C.byref(st)), "scan")
        vcf = C.string_at(out.vcf, out.vcf_len).decode() if out.vcf_len else ""
        ctx = C.string_at(out.ctx, out.ctx_len).decode() if out.ctx_len else ""
        lib().grom_out_free(C.byref(out))
        return vcf, ctx, st

    def upload(self, chrom: Chrom, reads: Reads):
        dc, dr = Chrom(), Reads()
        check(lib().grom_upload(self.device, C.byref(chrom), C.byref(reads), C.byref(dc), C.byref(dr)), "upload")
        return dc, dr

    def debug_counts(self, chrom: Chrom, reads: Reads):
        lo = max(self.params.one_base_rd_len // 4 + 1, 2 * self.params.insert_max_size + 1)
        n_eval = max(chrom.p_last - lo + 1, 0)
        cnt = np.zeros((max(n_eval, 1), NCOUNT), np.int32)
        caf = np.zeros((3, chrom.len), np.int32)
        first = C.c_int32(0)
        check(lib().grom_debug_counts(self.device, C.byref(chrom), C.byref(reads), C.byref(first), cnt.ctypes.data,
                                      cnt.size, caf.ctypes.data), "grom_debug_counts")
        return cnt[:n_eval], caf


class Resident:
    """A chromosome's inputs kept in HBM (grom_resident_new); scan them from any
    context on the same device with Device.scan(..., device_resident=True)."""

    def __init__(self, device: int, chrom: Chrom, reads: Reads):
        self.chrom, self.reads = Chrom(), Reads()
        self.h = lib().grom_resident_new(device, C.byref(chrom), C.byref(reads), C.byref(self.chrom),
                                         C.byref(self.reads))
        if not self.h:
            raise RuntimeError(f"grom_resident_new failed: {last_error()}")
        self.bytes = lib().grom_resident_bytes(self.h)
        # the name is host text owned by the source batch: keep a copy here
        self.chrom.name = bytes(chrom.name or b"")

    def close(self):
        if self.h:
            lib().grom_resident_free(self.h)
            self.h = None


class SynthBatch:
    """A synthetic chromosome and the read batch its scan ingests (host memory)."""

    def __init__(self, length: int, coverage: float = 30.0, read_len: int = 150, insert_mean: float = 500.0,
                 insert_sd: float = 50.0, seed: int = 2, params: Params | None = None, _handle=None):
        self.params = params if params is not None else default_params()
        self.h = _handle if _handle is not None else lib().grom_synth_batch(
            length, coverage, read_len, insert_mean, insert_sd, seed, C.byref(self.params))
        if not self.h:
            raise RuntimeError("grom_synth_batch failed")
        self.chrom, self.reads = Chrom(), Reads()
        check(lib().grom_batch_get(self.h, C.byref(self.chrom), C.byref(self.reads)), "grom_batch_get")

    @classmethod
    def genome_chrom(cls, lengths, chrom: int, params: Params, names=None, coverage: float = 30.0,
                     read_len: int = 150, ploidy: int = 2, insert_mean: float = 500.0, insert_sd: float = 50.0,
                     dup_frac: float = 0.0, sv_per_mb: float = 0.0, cnv_rate: float = 0.0,
                     cnv_range=(0, 0), chr_cov=None, munmap_frac: float = 0.002, seed: int = 2,
                     stream: bool = False) -> "SynthBatch":
        """Chromosome `chrom` of a multi-chromosome synthetic genome (grom_synth_chrom).
        `params` keeps genome-wide insert statistics once set (see include/grom_amd.h).
        stream=True: as the chromosome's scan sees it inside the genome's BAM
        (grom_synth_chrom_stream: the serial stream's Q1 drops and pending-record length)."""
        arr = (C.c_int64 * len(lengths))(*lengths)
        cov = (C.c_double * len(lengths))(*chr_cov) if chr_cov is not None else None
        sp = SynthSpec(len(lengths), chrom, arr, ",".join(names).encode() if names else None, coverage, read_len,
                       ploidy, insert_mean, insert_sd, dup_frac, sv_per_mb, cnv_rate, cnv_range[0], cnv_range[1],
                       cov, munmap_frac, seed)
        fn = lib().grom_synth_chrom_stream if stream else lib().grom_synth_chrom
        h = fn(C.byref(sp), C.byref(params))
        if not h:
            raise RuntimeError(f"grom_synth_chrom failed for chromosome {chrom}: {last_error()}")
        return cls(lengths[chrom], params=params, _handle=h)

    def close(self):
        if self.h:
            lib().grom_batch_release(self.h)
            self.h = None

    @property
    def n_reads(self) -> int:
        return self.reads.n

    @property
    def n_bases(self) -> int:
        return self.reads.n_bases


def ctx_postpass(raw: str, target_names, insert_max: int, lseq: int) -> str:
    """main's translocation post-pass (grom_ctx_postpass) over the raw CTX rows
    of every chromosome in chromosome order: the BND rows of .ctx.vcf."""
    names = (C.c_char_p * max(len(target_names), 1))(*[n.encode() for n in target_names])
    out = Out()
    data = raw.encode()
    check(lib().grom_ctx_postpass(data, len(data), names, len(target_names), insert_max, lseq, C.byref(out)),
          "grom_ctx_postpass")
    text = C.string_at(out.ctx, out.ctx_len).decode() if out.ctx_len else ""
    lib().grom_out_free(C.byref(out))
    return text


def cli_main(args, env=None, cwd=None) -> int:
    """Run the drop-in CLI in this process (loads the HIP library here)."""
    saved_env, saved_cwd = dict(os.environ), os.getcwd()
    try:
        if env:
            os.environ.update(env)
        if cwd:
            os.chdir(cwd)
        argv = [b"grom"] + [str(a).encode() for a in args]
        arr = (C.c_char_p * (len(argv) + 1))(*argv, None)
        return lib().grom_cli_main(len(argv), arr)
    finally:
        os.chdir(saved_cwd)
        os.environ.clear()
        os.environ.update(saved_env)


def run_grom(args, env=None, check_rc=True, timeout=600):
    """Run the drop-in CLI as a subprocess (GPU)."""
    e = dict(os.environ)
    if env:
        e.update(env)
    r = subprocess.run([GROM_BIN] + list(args), env=e, capture_output=True, text=True, timeout=timeout)
    if check_rc and r.returncode != 0:
        raise RuntimeError(f"grom failed ({r.returncode}): {r.stdout[-2000:]} {r.stderr[-2000:]}")
    return r


def run_synth(prefix, *args, timeout=600):
    r = subprocess.run([SYNTH_BIN, "-o", prefix] + [str(a) for a in args], capture_output=True, text=True,
                       timeout=timeout)
    if r.returncode != 0:
        raise RuntimeError(f"grom_synth failed: {r.stderr}")
    return prefix + ".bam", prefix + ".fa"
