"""GPU parity: the HIP scan against the oracle on the same synthetic inputs.

Everything here is integer/byte work or a fixed sequence of IEEE operations,
so the bar is bit-exact: per-base counters (GROM_NCOUNT int32 per evaluated
base), the three whole-chromosome read-depth arrays, and the VCF bytes (with
##fileDate pinned; ##reference is the same path for both)."""
import filecmp
import os
import re
import subprocess
import sys

import numpy as np
import pytest

import grom_amd
from _util import CASES, load_counts, load_indels, run_grom, run_oracle, synth

pytestmark = pytest.mark.gpu

RUNS = [
    ("one_chr", []),
    ("three_chr", []),
    ("lowmapq_clip", []),
    ("lowmapq_clip", ["-q", "10", "-b", "25", "-n", "2", "-a", "0.3"]),
    ("dups", ["-M"]),
    ("dups", []),
    ("empty_middle", []),
    ("one_chr", ["-p", "4", "-x", "28"]),
    ("one_chr", ["-G", "40"]),  # forces mid-scan SNV list flushes (GROM.c:11201)
    ("dups", ["-n", "6", "-a", "0.1"]),  # -n above 4: the 8-slot build of the gather kernel
    ("dups", ["-n", "12", "-a", "0.05"]),  # the 16-slot build
    ("c5_tetra_male", ["-n", "20", "-a", "0.05", "-p", "4"]),  # the 32-slot build at 60x
    # -n above 32: slot columns in global memory (k_scan_tile_mem); at 60x the
    # homozygous sites fill all 40 slots
    ("c5_tetra_male", ["-n", "40", "-a", "0.05", "-p", "4"]),
    ("dups", ["-n", "100", "-a", "0.01"]),
    ("indels", []),
    ("indels", ["-M"]),
    ("indels", ["-q", "10"]),
    # breakpoint path (rows A8-A10, A13): split reads, pair classes, the
    # per-base tests, the candidate lists, SV rows and the CTX post-pass
    ("sv", []),
    ("sv", ["-S"]),
    ("sv", ["-d", "2", "-u", "0.5", "-j", "0.02"]),
    ("sv", ["-l", "2"]),
    # BASELINE configs[4] and configs[2] shapes
    ("c5_tetra_male", ["-p", "4", "-g", "1"]),
    ("c5_tetra_male", ["-p", "4", "-g", "1", "-M", "-V", "1"]),
    ("c3_genome", ["-M"]),
    ("c3_genome", ["-M", "-V", "1"]),
    # dense breakpoint SVs (>= 50 rows of each class) and SURVEY 8(d)'s C1s
    ("sv_many", []),
    ("c1s", []),
    ("c1s", ["-V", "1", "-n", "2"]),
    # -f tab-separated rows (g_vcf == 0): SNV rows with their reference
    # context, every breakpoint class, CNV rows under their column headers,
    # the CTX post-pass table; -G 40 adds mid-scan SNV flushes (cdp_lseq of
    # the pending record)
    ("sv", ["-f"]),
    ("c3_genome", ["-M", "-V", "1", "-f"]),
    ("one_chr", ["-G", "40", "-f"]),
    # any -p >= 1 (GROM.c:22003; the reference's 100-byte GT text overflows
    # above 50, both sides print the whole 119-character genotype)
    ("one_chr", ["-p", "60"]),
    # a negative -q: every read is high quality on every path (signed compares)
    ("lowmapq_clip", ["-q", "-1"]),
]

# read-depth CNV path (detect_del_dup, GROM.c:18228): -V 1 keeps every call
# (the default 1e-9 p-value cut removes most)
CNV_RUNS = [
    ("cnv", []),
    ("cnv", ["-V", "1"]),
    ("cnv", ["-V", "1", "-K", "0"]),
    ("cnv", ["-V", "1", "-A", "3", "-X", "4000", "-W", "60", "-L", "3", "-F", "0.3"]),
    ("cnv_multi", ["-V", "1", "-p", "3"]),
    ("cnv_multi", ["-V", "1", "-M", "-U", "1", "-Y", "2", "-Z", "20000"]),
    ("cnv_long", ["-V", "1", "-M"]),
    ("cnv_long", []),
    ("wide_insert", []),
    ("wide_insert", ["-V", "1"]),
    # -X past the chromosome lengths and beyond 1e6 with -A 20: every sampled
    # window straddles up to six sampling passes of its block (GROM.c:18967-19018)
    ("cnv_multi", ["-V", "1", "-X", "2500000", "-A", "20", "-W", "100"]),
    ("cnv", ["-V", "1", "-X", "40000", "-A", "9"]),
    ("cnv", ["-V", "1", "-p", "60"]),
]


def _names(datadir, tag):
    return sorted(f.split(".")[-2] for f in os.listdir(datadir) if f.startswith(tag + ".") and f.endswith(".cnt"))




def _check_sv_records(datadir, o_dump, g_dump, ch):
    """Per-base breakpoint cluster state (rows A8/A9: every evaluated base with
    a DEL/DUP/INV/CTX cluster count or an occupied "other" slot -- counts,
    running-mean distances bit for bit, first/last read positions, CTX mate
    chromosomes, the pair binning's depth adds, concordant, short-insert and
    unmapped-mate sums) against the oracle's ring at the same base."""
    o = np.fromfile(datadir / f"{o_dump}.{ch}.sv", dtype=grom_amd.SV_DTYPE)
    g = np.fromfile(datadir / f"{g_dump}.{ch}.sv", dtype=grom_amd.SV_DTYPE)
    assert o.shape == g.shape, (ch, o.shape, g.shape, o["pos"][:5], g["pos"][:5])
    if o.tobytes() != g.tobytes():
        ob, gb = o.view(np.uint8).reshape(len(o), -1), g.view(np.uint8).reshape(len(g), -1)
        i = int(np.nonzero((ob != gb).any(axis=1))[0][0])
        raise AssertionError((ch, "first differing breakpoint record", o[i], g[i]))
    return len(o)


def _check_counters(datadir, case, extra, tag, env_extra=None):
    bam, fa = synth(datadir, case, CASES[case])
    o_dump, g_dump = f"o_{tag}", f"g_{tag}"
    run_oracle(datadir, bam, fa, f"o_{tag}.vcf", extra, dump=str(datadir / o_dump))
    run_grom(datadir, bam, fa, f"g_{tag}.vcf", extra, dump=str(datadir / g_dump),
             env_extra=dict(env_extra or {}, GROM_SV_DEBUG="1"))
    chroms = _names(datadir, o_dump)
    assert chroms
    for ch in chroms:
        oc = load_counts(datadir / f"{o_dump}.{ch}.cnt")
        gp = datadir / f"{g_dump}.{ch}.cnt"
        gc = load_counts(gp) if os.path.getsize(gp) else np.zeros((0, oc.shape[1]), np.int32)
        assert oc.shape == gc.shape, (ch, oc.shape, gc.shape)
        if oc.size:
            diff = np.nonzero((oc != gc).any(axis=1))[0]
            assert diff.size == 0, (ch, "first differing base", oc[diff[0]].tolist(), gc[diff[0]].tolist())
        ocaf = np.fromfile(datadir / f"{o_dump}.{ch}.caf", np.int32)
        gcaf = np.fromfile(datadir / f"{g_dump}.{ch}.caf", np.int32)
        assert np.array_equal(ocaf, gcaf), ch
        # CIGAR indel evidence (row A7): one record per evaluated base an I/D op reached
        oi = load_indels(datadir / f"{o_dump}.{ch}.ind")
        gi = load_indels(datadir / f"{g_dump}.{ch}.ind")
        assert oi.shape == gi.shape, (ch, oi.shape, gi.shape)
        bad = np.nonzero(oi != gi)[0]
        assert bad.size == 0, (ch, "first differing indel record", oi[bad[0]], gi[bad[0]])
        if case == "indels":
            assert (oi["other_len"] > 0).sum() > 10 and (oi["ins"] > 0).sum() > 10
        n_sv = _check_sv_records(datadir, o_dump, g_dump, ch)
        if case in ("sv", "sv_many", "c3_genome"):
            assert n_sv > 1000, (ch, n_sv)
    ov, gv = open(datadir / f"o_{tag}.vcf").read(), open(datadir / f"g_{tag}.vcf").read()
    assert ov.count("\n") > 46
    assert ov == gv
    assert filecmp.cmp(datadir / f"o_{tag}.ctx.vcf", datadir / f"g_{tag}.ctx.vcf", shallow=False)
    if "-f" in extra:
        # tab rows: every class named in its first column
        kinds = {l.split("\t")[0] for l in gv.splitlines()[2:]}
        assert "SNV" in kinds, kinds
        if case == "sv":
            assert {"DEL", "DUP", "INV_F", "INDEL_INS", "INDEL_DEL"} <= kinds, kinds
        if "-V" in extra:
            assert {"SV Type", "DEL RD", "DUP RD"} <= kinds, kinds
        return
    if case in ("sv", "sv_many"):
        # the comparison covered every breakpoint row class
        alts = [l.split("\t")[4] for l in gv.splitlines() if not l.startswith("#")]
        assert {"<DEL>", "<DUP>", "<INV>"} <= set(alts), set(alts)
        if case == "sv_many":
            for cls in ("<DEL>", "<DUP>", "<INV>", "<INS>"):
                assert alts.count(cls) >= 50, (cls, alts.count(cls))
        assert any(l.startswith("SPR:SEV:SRD:SCO:ECO") or "SPR:SEV:SRD:SCO:ECO" in l for l in gv.splitlines())
        bnd = [l for l in open(datadir / f"g_{tag}.ctx.vcf") if not l.startswith("#")]
        assert bnd and all("SVTYPE=BND" in l for l in bnd)
        if case == "sv_many":
            assert len(bnd) >= 50, len(bnd)
    if case == "c1s":
        # the tilapia contig, its soft-masked (lower-case) REF bases printed as loaded
        rows = [l for l in gv.splitlines() if not l.startswith("#")]
        assert rows and all(l.startswith("gl831235-1\t") for l in rows)
        assert any(l.split("\t")[3].islower() for l in rows)


@pytest.mark.parametrize("case,extra", RUNS, ids=[f"{c}{''.join(e)}" for c, e in RUNS])
def test_counters_and_vcf_bit_exact(datadir, case, extra):
    _check_counters(datadir, case, extra, f"{case}{''.join(extra).replace('-', '_')}")


@pytest.mark.parametrize("case,extra", [("dups", ["-n", "3"]), ("c5_tetra_male", ["-n", "20", "-a", "0.05", "-p", "4"])],
                         ids=["dups-n3", "tetra-n20"])
def test_global_name_slots_forced(datadir, case, extra):
    """The global-slot kernel (built for -n above 32) forced at small -n, where
    the register builds also run: both must equal the oracle."""
    _check_counters(datadir, case, extra, "memslots" + "".join(extra), env_extra={"GROM_MEM_SLOTS": "1"})


@pytest.mark.parametrize("case,extra", [("cnv", ["-V", "1"]), ("wide_insert", ["-V", "1"]), ("huge_insert", [])],
                         ids=["cnv", "wide_insert", "huge_insert"])
def test_gc_windows_prefix_form(datadir, case, extra):
    """k_cnv_gc_global, the GC/ACGT window form for insert means above the
    tile kernel's 16,384 halo: forced at insert means 500 and 2,200 (where
    CNV calls exist to compare), and on its own at a 20 kb insert library."""
    bam, fa, tag = _oracle_once(datadir, case, extra)
    run_grom(datadir, bam, fa, f"g_gcglobal_{tag}.vcf", extra,
             env_extra={"GROM_GC_GLOBAL": "1"} if case != "huge_insert" else None)
    ov, gv = open(datadir / f"o_{tag}.vcf").read(), open(datadir / f"g_gcglobal_{tag}.vcf").read()
    if "-V" in extra:
        assert ov.count("<DEL>") + ov.count("<DUP>") > 0
    assert ov == gv


@pytest.mark.parametrize("case,extra", [("dups", ["-M"]), ("c5_tetra_male", ["-p", "4", "-g", "1"])],
                         ids=["dups-M", "tetra"])
def test_heavy_tile_route(datadir, case, extra):
    """Tiles with more reads than the register kernels' 16-bit counters hold
    go to k_scan_tile_mem (32-bit counters): forced for every tile."""
    _check_counters(datadir, case, extra, "heavy" + "".join(extra), env_extra={"GROM_HEAVY_TILES": "1"})


def test_tab_output_names(datadir):
    """-f with an output name without .vcf: rows in OUT, the translocation
    table in OUT.ctx (GROM.c:20494-20505, 22446-22460)."""
    bam, fa = synth(datadir, "sv", CASES["sv"])
    run_oracle(datadir, bam, fa, "o_tabnames.txt", ["-f"])
    run_grom(datadir, bam, fa, "g_tabnames.txt", ["-f"])
    for suffix in ("", ".ctx"):
        o = open(datadir / f"o_tabnames.txt{suffix}").read()
        g = open(datadir / f"g_tabnames.txt{suffix}").read()
        assert o == g, suffix
        assert o.count("\n") > 1
    rows = open(datadir / "g_tabnames.txt").read().splitlines()
    assert rows[1].startswith("SV\tChromosome\t")
    kinds = {l.split("\t")[0] for l in rows[2:]}
    assert {"SNV", "DEL", "DUP", "INDEL_INS", "INDEL_DEL"} <= kinds, kinds


def test_breakpoint_context_buffer_retry(datadir):
    """The pileup's breakpoint context records (one per clipped or marked base)
    go to a buffer sized by a guess; a scan that wants more runs again with
    room (scan.hip).  GROM_SV_CTX_CAP=2000 makes the first pass overflow on the
    sv case: counters, breakpoint records and rows must still be the oracle's."""
    _check_counters(datadir, "sv", [], "svctxcap", env_extra={"GROM_SV_CTX_CAP": "2000"})


def _oracle_once(datadir, case, extra):
    """The oracle's VCF for (case, flags), run once per session (the long-region
    cases take the oracle about a minute)."""
    bam, fa = synth(datadir, case, CASES[case])
    tag = f"{case}{''.join(extra).replace('-', '_').replace('.', 'p')}"
    if not os.path.exists(datadir / f"o_{tag}.vcf"):
        run_oracle(datadir, bam, fa, f"o_{tag}.vcf", extra)
    return bam, fa, tag


@pytest.mark.parametrize("case,extra", CNV_RUNS, ids=[f"{c}{''.join(e)}" for c, e in CNV_RUNS])
def test_cnv_rows_bit_exact(datadir, case, extra):
    bam, fa, tag = _oracle_once(datadir, case, extra)
    run_grom(datadir, bam, fa, f"g_{tag}.vcf", extra)
    ov, gv = open(datadir / f"o_{tag}.vcf").read(), open(datadir / f"g_{tag}.vcf").read()
    if "-V" in extra:
        assert ov.count("<DEL>") + ov.count("<DUP>") > 0
    assert ov == gv


@pytest.mark.parametrize("case,extra", [("cnv", ["-V", "1"]), ("cnv_long", ["-V", "1", "-M"]),
                                        ("cnv_multi", ["-V", "1", "-p", "3"])],
                         ids=["cnv_V1", "cnv_long_V1_M", "cnv_multi_V1_p3"])
def test_cnv_wave_window_search(datadir, case, extra):
    """GROM_CNV_BUDGET=1 leaves every DEL/DUP window search past its first
    ML+256 bases (phase B) and every call's slide and trim (phases C/D) to
    the walk's wave-cooperative routines (phase_ab_wave, phase_cd_wave): the
    rows must still be the oracle's."""
    bam, fa, tag = _oracle_once(datadir, case, extra)
    run_grom(datadir, bam, fa, f"gw_{tag}.vcf", extra, env_extra={"GROM_CNV_BUDGET": "1"})
    ov, gv = open(datadir / f"o_{tag}.vcf").read(), open(datadir / f"gw_{tag}.vcf").read()
    assert ov.count("<DEL>") + ov.count("<DUP>") > 0
    assert ov == gv


@pytest.mark.parametrize("case,extra", [("cnv", ["-V", "1"]), ("cnv_long", ["-V", "1", "-M"]),
                                        ("cnv_multi", ["-V", "1", "-p", "3"])],
                         ids=["cnv_V1", "cnv_long_V1_M", "cnv_multi_V1_p3"])
def test_cnv_classify_queue(datadir, case, extra):
    """The candidate classification as a per-wave work queue (k_cnv_classify,
    GROM_CNV_CLS=1: lanes refill from the wave's queue share when their
    candidate is decided) instead of one lane per candidate (the default,
    faster on the 150 Mb timing case): the same rows as the oracle's."""
    bam, fa, tag = _oracle_once(datadir, case, extra)
    run_grom(datadir, bam, fa, f"gq_{tag}.vcf", extra, env_extra={"GROM_CNV_CLS": "1"})
    ov, gv = open(datadir / f"o_{tag}.vcf").read(), open(datadir / f"gq_{tag}.vcf").read()
    assert ov.count("<DEL>") + ov.count("<DUP>") > 0
    assert ov == gv


@pytest.mark.parametrize("case,extra", [("cnv", ["-V", "1"]), ("cnv_multi", ["-V", "1", "-p", "3"])],
                         ids=["cnv_V1", "cnv_multi_V1_p3"])
def test_cnv_serial_stdev_path(datadir, case, extra):
    """The chromosome depth stdev (GROM.c:16664-16685) decided from the
    histogram bound and redone in base order on the host (GROM_CNV_SERIAL_SD
    forces the host path; it also runs whenever the bound cannot decide or the
    depth exceeds the histogram) give the oracle's rows."""
    bam, fa = synth(datadir, case, CASES[case])
    tag = f"serialsd_{case}"
    run_oracle(datadir, bam, fa, f"o_{tag}.vcf", extra)
    run_grom(datadir, bam, fa, f"g_{tag}.vcf", extra, env_extra={"GROM_CNV_SERIAL_SD": "1"})
    ov, gv = open(datadir / f"o_{tag}.vcf").read(), open(datadir / f"g_{tag}.vcf").read()
    assert ov.count("<DEL>") + ov.count("<DUP>") > 0
    assert ov == gv


def _stats(path):
    out = {}
    if os.path.exists(path):
        for line in open(path):
            name, over, repl = line.split()
            out[name] = (int(over.split("=")[1]), int(repl.split("=")[1]))
    return out


@pytest.mark.parametrize("case,extra,cap", [("cnv", ["-V", "1"], "100"), ("cnv_multi", ["-V", "1", "-p", "3"], "150"),
                                            ("c3_genome", ["-M", "-V", "1"], "60")],
                         ids=["cnv_cap100", "cnv_multi_cap150", "c3_genome_cap60"])
def test_cnv_reservoir_draws_forced(datadir, case, extra, cap):
    """once a GC bin holds g_sample_lists_len depth samples, each
    new one draws grom_rand (glibc random()) to replace a kept sample
    (GROM.c:18385-18451).  GROM_SAMPLE_LISTS_LEN lowers the cap in the oracle
    and in the product alike, so the draws run thousands of times on a small
    input: the number of draws past the cap and of replacements, and the rows,
    must be the oracle's."""
    bam, fa = synth(datadir, case, CASES[case])
    tag = f"res{cap}_{case}"
    env = {"GROM_SAMPLE_LISTS_LEN": cap}
    so, sg = str(datadir / f"o_{tag}.stats"), str(datadir / f"g_{tag}.stats")
    run_oracle_env = dict(env, GROM_CNV_STATS=so)
    from _util import run, ORACLE_BIN
    run(ORACLE_BIN, ["-i", bam, "-r", fa, "-o", f"o_{tag}.vcf"] + extra, str(datadir), run_oracle_env)
    run_grom(datadir, bam, fa, f"g_{tag}.vcf", extra, env_extra=dict(env, GROM_CNV_STATS=sg))
    o, g = _stats(so), _stats(sg)
    assert o == g, (o, g)
    assert sum(v[0] for v in o.values()) > 1000 and sum(v[1] for v in o.values()) > 0, o
    assert open(datadir / f"o_{tag}.vcf").read() == open(datadir / f"g_{tag}.vcf").read()


def test_cnv_reservoir_draws_at_the_reference_cap(datadir):
    """The same draws at the reference's own cap of 100,000 samples: a 30 Mb
    contig whose windows all have one GC content (grom_synth -R) puts every
    depth sample in one bin, as the longest configs[2] chromosomes do with
    their dominant bins.  Draw counts and rows equal the oracle's."""
    case = "cnv_reservoir"
    bam, fa = synth(datadir, case, CASES[case])
    so, sg = str(datadir / "o_resfull.stats"), str(datadir / "g_resfull.stats")
    from _util import run, ORACLE_BIN
    run(ORACLE_BIN, ["-i", bam, "-r", fa, "-o", "o_resfull.vcf", "-V", "1"], str(datadir), {"GROM_CNV_STATS": so})
    run_grom(datadir, bam, fa, "g_resfull.vcf", ["-V", "1"], env_extra={"GROM_CNV_STATS": sg})
    o, g = _stats(so), _stats(sg)
    assert o == g, (o, g)
    assert o["chr1"][0] > 10000, o
    ov, gv = open(datadir / "o_resfull.vcf").read(), open(datadir / "g_resfull.vcf").read()
    assert ov.count("<DEL>") + ov.count("<DUP>") > 0
    assert ov == gv


@pytest.mark.parametrize("case,extra", [("three_chr", []), ("sv", ["-S"]), ("c3_genome", ["-M", "-V", "1"]),
                                        ("empty_middle", [])],
                         ids=["three_chr", "sv_S", "c3_genome_M_V1", "empty_middle"])
def test_serial_reader_path(datadir, case, extra):
    """The serial reader (GROM_SERIAL_DECODE=1: one pass over the record
    stream, host batches uploaded per chromosome) -- the CLI's fallback when an
    index lacks what the streamed decoder needs -- gives the oracle's VCF."""
    bam, fa = synth(datadir, case, CASES[case])
    tag = f"ser_{case}{''.join(extra).replace('-', '_')}"
    run_oracle(datadir, bam, fa, f"o_{tag}.vcf", extra)
    run_grom(datadir, bam, fa, f"g_{tag}.vcf", extra, env_extra={"GROM_SERIAL_DECODE": "1"})
    for ext in (".vcf", ".ctx.vcf"):
        assert open(datadir / f"o_{tag}{ext}").read() == open(datadir / f"g_{tag}{ext}").read(), ext


def test_amplicon_depth_tiles(datadir):
    """Tiles on both sides of the 16-bit packed-counter bound: the register
    build takes the tiles of at most PACK_MAX_READS reads, k_scan_tile_mem
    the heavier ones (with 32-bit counters), and every per-base counter, caf
    value and VCF byte is the oracle's."""
    bam, fa = synth(datadir, "amplicon", CASES["amplicon"])
    hits = _tile_read_counts(bam)
    pack_max = 65535  # PACK_MAX_READS, grom_amd/csrc/scan_common.h
    assert (hits <= pack_max).any() and (hits > pack_max).any(), (hits.min(), hits.max())
    _check_counters(datadir, "amplicon", [], "amplicon")


def _tile_read_counts(bam, halo=151, tile=256):
    """Reads whose start lies in [t0 - halo, t0 + tile) for every 256-base
    tile (k_tile_ranges' read range; 2x150 bp reads without clips), from the
    BAM's records (BGZF members are gzip members)."""
    import gzip
    import struct
    raw = gzip.decompress(open(bam, "rb").read())
    o = 4
    (l_text,) = struct.unpack_from("<i", raw, o)
    o += 4 + l_text
    (n_ref,) = struct.unpack_from("<i", raw, o)
    o += 4
    for _ in range(n_ref):
        (l_name,) = struct.unpack_from("<i", raw, o)
        o += 8 + l_name
    keys = []
    while o + 12 <= len(raw):
        bs, tid, pos = struct.unpack_from("<iii", raw, o)
        keys.append(tid * (1 << 32) + pos)
        o += 4 + bs
    k = np.array(keys, dtype=np.int64)
    out = []
    for tid in np.unique(k >> 32):
        p = np.sort(k[(k >> 32) == tid] & 0xffffffff)
        t0 = np.arange(0, int(p[-1]) + 1, tile)
        out.append(np.searchsorted(p, t0 + tile) - np.searchsorted(p, t0 - halo))
    return np.concatenate(out)


@pytest.mark.parametrize("case,extra", [("sv", ["-d", "2", "-k", "8", "-v", "0.01", "-j", "0.02"]),
                                        ("c3_genome", ["-M", "-V", "1", "-N", "5000"]),
                                        ("cnv_multi", ["-V", "1", "-p", "3", "-q", "10", "-S"])],
                         ids=["sv_opts", "c3_genome", "cnv_multi"])
def test_integration_stub(datadir, case, extra):
    """INTEGRATION.md section 2's GROM.c binding, compiled as written
    (tools/gromc_binding.c), scanning every chromosome through grom_scan_chrom
    with the globals it copies: the same VCF rows and BND rows as the CLI."""
    import subprocess
    from _util import FILEDATE, GROM_BIN, SEED
    bam, fa = synth(datadir, case, CASES[case])
    tag = f"stub_{case}"
    env = dict(os.environ, GROM_FILEDATE=FILEDATE, GROM_SEED=SEED)
    exe = os.path.join(os.path.dirname(GROM_BIN), "gromc_binding")
    r = subprocess.run([exe, "-i", bam, "-r", fa, "-o", f"b_{tag}.vcf"] + extra, cwd=str(datadir), env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    run_grom(datadir, bam, fa, f"g_{tag}.vcf", extra)

    def rows(path):
        return [ln for ln in open(path) if not ln.startswith("#")]
    g = rows(datadir / f"g_{tag}.vcf")
    assert len(g) > 40 and rows(datadir / f"b_{tag}.vcf") == g
    assert rows(datadir / f"b_{tag}.vcf.ctx.vcf") == rows(datadir / f"g_{tag}.ctx.vcf")


def test_rank_shares_merge_to_one_run(datadir):
    """bench.py --gpus N's whole run: each rank's CLI scans its share of the
    chromosomes (GROM_CHROMS, raw CTX rows kept with GROM_CTX_RAW); rank 0's
    merge (grom_amd.shard.merge_rank_outputs: rows in chromosome order, one
    translocation post-pass) is byte-identical to a one-process run."""
    from grom_amd.shard import assign_chromosomes, merge_rank_outputs
    names = ["chr1", "chr2", "chrX", "chrY"]
    lengths = [700_000, 600_000, 500_000, 400_000]
    bam, fa = synth(datadir, "shares", ["-L", ",".join(map(str, lengths)), "-n", ",".join(names), "-s", "6", "-X", "6",
                                        "-D", "0.05", "-V", "2e-6", "-W", "20000,80000"])
    flags = ["-M", "-g", "1"]
    run_grom(datadir, bam, fa, "one.vcf", flags)
    shares = assign_chromosomes(lengths, 3)
    for r, share in enumerate(shares):
        run_grom(datadir, bam, fa, f"r{r}.vcf", flags,
                 env_extra={"GROM_CHROMS": ",".join(names[i].lower() for i in share),
                            "GROM_CTX_RAW": str(datadir / f"r{r}.raw"),
                            "GROM_VCF_SEGS": str(datadir / f"r{r}.segs")})
    m = open(bam + ".mean").read().split()
    vcf, bnd = merge_rank_outputs([str(datadir / f"r{r}.vcf") for r in range(3)],
                                  [str(datadir / f"r{r}.raw") for r in range(3)], [n.lower() for n in names], names,
                                  int(m[3]), int(m[1]))
    one = open(datadir / "one.vcf").read()
    assert one.count("\n") > 100 and vcf == one
    one_ctx = "".join(l for l in open(datadir / "one.ctx.vcf") if not l.startswith("#"))
    assert bnd == one_ctx and bnd.count("SVTYPE=BND") >= 2
    # bench.py's merge: every rank copies its rows to their offsets from the
    # CLI's segment index (three threads stand in for the ranks)
    import threading
    from grom_amd.shard import merge_rank_outputs_parallel
    bar, got = threading.Barrier(3), [None] * 3

    def gather_of(r):
        def g(obj):
            # (the merge gathers several times: the second wait keeps a fast
            # rank's next entry out of got until every rank has its copy)
            got[r] = obj
            bar.wait()
            res = list(got)
            bar.wait()
            return res
        return g
    errs = []

    def rank_main(r):
        try:
            merge_rank_outputs_parallel(r, str(datadir / f"r{r}.vcf"), [names[i].lower() for i in shares[r]],
                                        [n.lower() for n in names], str(datadir / "par.vcf"), gather_of(r), bar.wait,
                                        [str(datadir / f"r{k}.raw") for k in range(3)], names, int(m[3]), int(m[1]),
                                        str(datadir / "par.ctx.vcf"), segs_path=str(datadir / f"r{r}.segs"))
        except BaseException as e:  # noqa: BLE001 -- re-raised below
            errs.append(e)
            bar.abort()
    ths = [threading.Thread(target=rank_main, args=(r,)) for r in range(3)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errs, errs
    assert open(datadir / "par.vcf").read() == one
    assert open(datadir / "par.ctx.vcf").read() == bnd


@pytest.mark.parametrize("mode", ["host", "device"])
def test_late_fallback_to_serial_reader(datadir, capfd, mode):
    """The streamed decoder's plan contradicted partway through the file
    (host decoder: GROM_TEST_SOFT_ABORT at a later piece; device decoder:
    GROM_TEST_DD_ABORT at the second chromosome it decodes -- both after
    chromosomes were handed to the scans): the CLI reruns through the serial
    reader, the outputs are the oracle's, and stdout carries the insert-size
    lines once."""
    bam, fa = synth(datadir, "three_chr", CASES["three_chr"])
    run_oracle(datadir, bam, fa, "o_late.vcf")
    capfd.readouterr()
    env = ({"GROM_DEVICE_DECODE": "0", "GROM_PIECE_RECS": "2000", "GROM_TEST_SOFT_ABORT": "20"} if mode == "host"
           else {"GROM_DEVICE_DECODE": "1", "GROM_TEST_DD_ABORT": "1"})
    run_grom(datadir, bam, fa, "g_late.vcf", env_extra=dict(env, GROM_VERBOSE="1"))
    out = capfd.readouterr().out
    assert "reading the BAM serially" in out, out[-2000:]
    assert out.count("insert_min_size, insert_max_size") == 1, out[-2000:]
    assert out.count("median read length") == 1
    for ext in (".vcf", ".ctx.vcf"):
        assert open(datadir / f"o_late{ext}").read() == open(datadir / f"g_late{ext}").read(), ext


@pytest.mark.gpu
@pytest.mark.parametrize("case,extra", [("cnv", ["-N", "1000"]), ("cnv_multi", ["-V", "1", "-N", "777"]),
                                        ("three_chr", ["-N", "5000"])])
def test_gen1000_side_file(datadir, case, extra):
    """-N: the per-chromosome <results>.1000gen.<chr> side file (GROM.c:20234-
    20345) -- per window of -N bases the copy number of its qualifying bases
    and their deviation, in the reference's summation order -- is the
    oracle's, byte for byte, for every chromosome; the VCF is unchanged."""
    import glob
    bam, fa = synth(datadir, case, CASES[case])
    tag = f"g1k_{case}{''.join(extra).replace('-', '_')}"
    run_oracle(datadir, bam, fa, f"o_{tag}.vcf", extra)
    run_grom(datadir, bam, fa, f"g_{tag}.vcf", extra)
    of = sorted(glob.glob(str(datadir / f"o_{tag}.vcf.1000gen.*")))
    gf = sorted(glob.glob(str(datadir / f"g_{tag}.vcf.1000gen.*")))
    assert of and [os.path.basename(f)[2:] for f in of] == [os.path.basename(f)[2:] for f in gf], (of, gf)
    for a, b in zip(of, gf):
        ta, tb = open(a).read(), open(b).read()
        assert ta == tb, a
    assert any(open(f).read() for f in of)  # at least one chromosome has complete windows
    assert open(datadir / f"o_{tag}.vcf").read() == open(datadir / f"g_{tag}.vcf").read()


def test_device_resident_path_matches_host_path():
    import grom_amd
    b = grom_amd.SynthBatch(300_000, seed=21)
    dev = grom_amd.Device(0, b.params)
    try:
        t1, s1 = dev.scan(b.chrom, b.reads)
        dc, dr = dev.upload(b.chrom, b.reads)
        t2, s2 = dev.scan(dc, dr, device_resident=True)
        assert t1 == t2 and t1.count("\n") > 50
        assert s2.bases_evaluated == s1.bases_evaluated > 0
    finally:
        dev.close()
        b.close()


@pytest.mark.parametrize("workers,extra", [("0,0,0", []), ("0,0", ["-V", "1"])], ids=["w3", "w2_cnv"])
def test_sharded_cli_matches_one_gpu(datadir, workers, extra):
    """Chromosomes scanned by several device workers (GROM_WORKER_DEVICES maps
    workers onto this box's one GPU; on an 8-GPU node -P 8 gives one per GPU)
    give the byte-identical VCF, rows in chromosome order -- the oracle's
    under the same -P 8 (each chromosome its own records, as the reference's
    -c children read them)."""
    import grom_amd
    from _util import FILEDATE, SEED
    case = "three_chr" if not extra else "cnv_multi"
    bam, fa = synth(datadir, case, CASES[case])
    tag = f"shard_{workers.replace(',', '')}"
    run_oracle(datadir, bam, fa, f"o_{tag}.vcf", extra + ["-P", "8"])
    env = {"GROM_FILEDATE": FILEDATE, "GROM_SEED": SEED, "GROM_WORKER_DEVICES": workers}
    rc = grom_amd.cli_main(["-i", bam, "-r", fa, "-o", f"g_{tag}.vcf", "-P", "8"] + extra, env=env, cwd=str(datadir))
    assert rc == 0, grom_amd.last_error()
    assert open(datadir / f"o_{tag}.vcf").read() == open(datadir / f"g_{tag}.vcf").read()


@pytest.mark.parametrize("case,extra", [("three_chr", ["-P", "2"]), ("empty_middle", ["-P", "2"]),
                                        ("sv", ["-P", "1", "-S"]), ("c3_genome", ["-P", "3", "-M", "-V", "1"])],
                         ids=["three_chr_P2", "empty_middle_P2", "sv_P1_S", "c3_genome_P3"])
def test_p_reference_semantics(datadir, case, extra):
    """GROM -P n: the reference reads every chromosome through bam_fetch
    (GROM.c:21051-21064; -P n > 1 forks -c children that do the same,
    549-599), so no chromosome loses the two records at its start that the
    serial stream consumes (Q1) and an empty chromosome starves nothing (Q21):
    its rows differ from a serial run's.  The CLI's -P n gives the oracle's -P
    rows byte for byte (device decode, the host decoder threads and the serial
    reader); GROM_P_SERIAL=1 keeps the serial stream's rows on n GPUs."""
    bam, fa = synth(datadir, case, CASES[case])
    tag = f"pref_{case}{''.join(extra).replace('-', '_')}"
    run_oracle(datadir, bam, fa, f"o_{tag}.vcf", extra)
    i = extra.index("-P")
    flags = extra[:i] + extra[i + 2:]  # (the serial run: the same flags without "-P n")
    run_oracle(datadir, bam, fa, f"os_{tag}.vcf", flags)
    outs = {}
    for mode, env in (("dev", {}), ("host", {"GROM_DEVICE_DECODE": "0"}), ("serial_reader", {"GROM_SERIAL_DECODE": "1"}),
                      ("p_serial", {"GROM_P_SERIAL": "1"})):
        run_grom(datadir, bam, fa, f"g{mode}_{tag}.vcf", extra, env_extra=env)
        outs[mode] = open(datadir / f"g{mode}_{tag}.vcf").read() + open(datadir / f"g{mode}_{tag}.ctx.vcf").read()
    want = open(datadir / f"o_{tag}.vcf").read() + open(datadir / f"o_{tag}.ctx.vcf").read()
    serial = open(datadir / f"os_{tag}.vcf").read() + open(datadir / f"os_{tag}.ctx.vcf").read()
    for mode in ("dev", "host", "serial_reader"):
        assert outs[mode] == want, mode
    assert outs["p_serial"] == serial
    if case == "empty_middle":  # chr3's rows exist only without Q21's starvation
        assert "\nchr3\t" in want and "\nchr3\t" not in serial
    if case == "three_chr":
        # the -c children -P n forks (GROM.c:549-599): target t alone, rows to
        # OUT.<target>-0 and raw CTX rows to OUT.<target>-0.ctx; the parent's
        # header followed by the children's rows in target order is -P's VCF
        import grom_amd
        base = f"c_{tag}.vcf"
        parts = []
        for t, name in enumerate(["chr1", "chr2", "chr3"]):
            run_grom(datadir, bam, fa, base, ["-c", f"{t},0,0,300000000"])
            parts.append(open(datadir / f"{base}.{name}-0").read())
            assert os.path.exists(datadir / f"{base}.{name}-0.ctx")
        got = open(datadir / f"gdev_{tag}.vcf").read()
        hdr = "".join(l for l in got.splitlines(keepends=True) if l.startswith("#"))
        assert hdr + "".join(parts) == got
        assert not os.path.exists(datadir / base)  # a child writes no full results file


def test_two_contexts_scan_concurrently():
    """Two library contexts on one GPU (grom_ctx_init; bench's --inflight 2)
    scanning the same device-resident chromosome from two host threads give
    the text of a lone scan."""
    import threading

    import grom_amd
    b = grom_amd.SynthBatch(400_000, seed=23)
    d0 = grom_amd.Device(0, b.params)
    d1 = grom_amd.Device(0, b.params, slot=8)
    try:
        dc, dr = d0.upload(b.chrom, b.reads)
        want, _ = d0.scan(dc, dr, device_resident=True)
        assert want.count("\n") > 50
        got = {0: [], 1: []}

        def run(k, dev):
            for _ in range(3):
                got[k].append(dev.scan(dc, dr, device_resident=True)[0])

        ts = [threading.Thread(target=run, args=(k, d)) for k, d in ((0, d0), (1, d1))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert got[0] == [want] * 3 and got[1] == [want] * 3
    finally:
        d1.close()
        d0.close()
        b.close()


def test_configs1_full_chromosome_vcf(datadir):
    """BASELINE configs[1] at full size: one 100 Mb chromosome at 30x through
    the GPU CLI and through the oracle; VCF and .ctx.vcf byte-identical."""
    bam, fa = synth(datadir, "c2_100mb", ["-L", "100000000", "-s", "2"])
    run_oracle(datadir, bam, fa, "o_c2.vcf")
    run_grom(datadir, bam, fa, "g_c2.vcf")
    for ext in (".vcf", ".ctx.vcf"):
        assert filecmp.cmp(datadir / f"o_c2{ext}", datadir / f"g_c2{ext}", shallow=False), ext
    rows = sum(1 for ln in open(datadir / "g_c2.vcf") if not ln.startswith("#"))
    assert rows > 50000


# ---- multi-GPU path: chromosomes sharded over two ranks (both on this GPU) ----
GENOME_LENGTHS = [700_000, 600_000, 500_000, 400_000]
GENOME_NAMES = ["chr1", "chr2", "chrX", "chrY"]


def _gpu_scan_factory(slot):
    import grom_amd
    p = grom_amd.default_params()
    p.rmdup = 1
    probe = grom_amd.SynthBatch.genome_chrom([2_000_000], 0, p, seed=6)
    probe.close()
    dev = grom_amd.Device(0, p, slot=slot)

    def scan(i):
        b = grom_amd.SynthBatch.genome_chrom(GENOME_LENGTHS, i, p, names=GENOME_NAMES, sv_per_mb=4.0,
                                             dup_frac=0.05, cnv_rate=2e-6, cnv_range=(20_000, 80_000), seed=6)
        try:
            vcf, ctx, _ = dev.scan_rows(b.chrom, b.reads)
            return vcf, ctx
        finally:
            b.close()

    def post(raw):
        return grom_amd.ctx_postpass(raw, GENOME_NAMES, p.insert_max_size, p.lseq)
    return dev, scan, post


def _gpu_shard_worker(rank, world, port, q):
    import torch.distributed as dist
    from grom_amd.shard import gather_to_rank0, sharded_genome_text
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev, scan, post = _gpu_scan_factory(rank)
        q.put((rank, sharded_genome_text(scan, GENOME_LENGTHS, world, rank, gather_to_rank0, ctx_post=post)))
        dev.close()
    finally:
        dist.destroy_process_group()


def test_two_ranks_sharded_genome_matches_one_rank():
    """configs[3]'s sharding on one GPU: two processes (gloo for the gather),
    each scanning its longest-processing-time share of a 4-contig genome; the
    merged VCF rows equal a one-process scan of every chromosome."""
    import socket
    import torch.multiprocessing as mp
    from grom_amd.shard import sharded_genome_text
    dev, scan, post = _gpu_scan_factory(40)
    one = sharded_genome_text(scan, GENOME_LENGTHS, 1, 0, ctx_post=post)
    dev.close()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gpu_shard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == one
    vcf, bnd = one
    assert vcf.count("\n") > 100 and "chrx" in vcf
    # the translocation rows of the whole genome, paired across the ranks' chromosomes
    assert bnd.count("SVTYPE=BND") >= 2, bnd


def _inflate_inputs(tmp_path):
    """synthetic BAMs compressed by libdeflate (levels 1, 6, 9) and by zlib,
    and BGZF files of stored, fixed-Huffman, Huffman-only, run-length and
    overlapping-match blocks (the CPU test's chunks)"""
    import zlib
    from test_host import _bgzf_blocks
    paths = []
    for lv, nolib in (("1", False), ("6", False), ("9", False), ("6", True)):
        env = dict(os.environ, GROM_SYNTH_LEVEL=lv)
        if nolib:
            env["GROM_NO_LIBDEFLATE"] = "1"
        prefix = str(tmp_path / f"inf{lv}{int(nolib)}")
        import subprocess
        from _util import SYNTH_BIN
        r = subprocess.run([SYNTH_BIN, "-o", prefix, "-L", "1500000", "-s", "9", "-X", "20", "-D", "0.1"], env=env,
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        paths.append(prefix + ".bam")
    import random
    rng = random.Random(5)
    chunks = [b"", b"A", bytes(rng.getrandbits(8) for _ in range(65280))]
    for period in (1, 2, 3, 5, 8, 9, 31, 300):
        unit = bytes(rng.getrandbits(8) for _ in range(period))
        chunks.append((unit * (60000 // period + 1))[:60000])
    for level, strategy in ((0, zlib.Z_DEFAULT_STRATEGY), (6, zlib.Z_FIXED), (6, zlib.Z_HUFFMAN_ONLY),
                            (6, zlib.Z_RLE), (9, zlib.Z_DEFAULT_STRATEGY)):
        p = tmp_path / f"chunks{level}_{strategy}.bgzf"
        p.write_bytes(_bgzf_blocks(chunks, level, strategy) * 3)
        paths.append(str(p))
    return paths


_INFLATE_SELFTEST = """
import ctypes, sys
sys.path.insert(0, sys.argv[1])
import grom_amd
f = grom_amd.lib().grom_inflate_device_selftest
f.restype = ctypes.c_int64
f.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
              ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
for path in sys.argv[2:]:
    ms, nb, by = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64()
    bad = f(path.encode(), 0, 0, 1, ctypes.byref(ms), ctypes.byref(nb), ctypes.byref(by))
    print(path, bad, nb.value, flush=True)
"""


def test_device_inflate_matches_zlib(datadir, tmp_path):
    """The GPU BGZF inflater (ddecode.hip, one block per lane) against zlib
    on every block of _inflate_inputs."""
    import ctypes
    lib = grom_amd.lib()
    f = lib.grom_inflate_device_selftest
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                  ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
    paths = _inflate_inputs(tmp_path)
    for path in paths:
        ms, nb, by = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64()
        bad = f(path.encode(), 0, 0, 1, ctypes.byref(ms), ctypes.byref(nb), ctypes.byref(by))
        assert bad == 0 and nb.value > 10, (path, bad, nb.value)


@pytest.mark.parametrize("tokcap", ["4096", "64"])
def test_two_phase_inflate_matches_zlib(tmp_path, tokcap):
    """The two-phase inflate variant (GROM_INFLATE_TOKCAP, DESIGN.md 4.5:
    Huffman tokens, then the wave-per-block LZ77 replay) against zlib on the
    same inputs; a cap of 64 tokens sends nearly every block of the BAMs to
    the one-phase fallback launch (status GI_E_TOKCAP).  A child process: the
    cap is read once per process."""
    paths = _inflate_inputs(tmp_path)
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _INFLATE_SELFTEST, repo] + paths, capture_output=True, text=True,
                       env=dict(os.environ, GROM_INFLATE_TOKCAP=tokcap), timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.split("\n")
    got = [l.rsplit(" ", 2) for l in lines if l.strip()]
    assert len(got) == len(paths), r.stdout
    for path, bad, nb in got:
        assert int(bad) == 0 and int(nb) > 10, (path, bad, nb)


@pytest.mark.parametrize("case,extra", [("three_chr", []), ("sv", ["-S"]), ("sv", []), ("dups", ["-M"]),
                                        ("empty_middle", []), ("c3_genome", ["-M", "-V", "1"]), ("indels", []),
                                        ("c5_tetra_male", ["-p", "4", "-g", "1"]), ("lowmapq_clip", [])],
                         ids=["three_chr", "sv_S", "sv", "dups_M", "empty_middle", "c3_genome", "indels", "c5",
                              "lowmapq_clip"])
def test_device_decode_matches_host_decode(datadir, capfd, case, extra):
    """BAM decode on the GPU (ddecode.hip: the runs inflated, walked and
    parsed on the device; GROM_DEVICE_DECODE=1) stages, for every chromosome,
    exactly the input the host decoder threads (pdecode.c) stage: same stream
    facts and the same digest of every array, CIGAR/base/quality/SA-XP
    content, dropped record and name-id relation; and the outputs are the
    oracle's.  Mode "3w" runs three device decode workers on the GPU
    (GROM_DD_WORKERS), each with its own decode context, prefetch thread and
    chromosomes, sharing the stages (the in-process shape of the reference's
    concurrent -P children, GROM.c:549-599).  Modes "g0"/"g2" run
    the record walk's guess-then-verify (k_walk_sub) with no guesses and with
    guesses at raw sub-chunk offsets (almost all wrong): every sub-chunk is
    then walked again from the true chain, with the same result.  Mode "cu"
    copies every base/quality tile through its global-memory path (the one
    tiles with more reads than LDS holds take).  Modes "pc"/"pcu" decode each
    run in pieces of 64 kB of inflated records (GROM_DD_PIECE_MB; the default
    is 1 GB, one piece per run at these sizes): many piece boundaries, the
    carries of every stage array across them, copy tiles shared by two
    pieces (their shared dwords stored byte by byte), "pcu" with the
    global-memory tile path as well."""
    bam, fa = synth(datadir, case, CASES[case])
    tag = f"dd_{case}{''.join(extra).replace('-', '_')}"
    run_oracle(datadir, bam, fa, f"o_{tag}.vcf", extra)
    lines = {}
    modes = {"0": {"GROM_DEVICE_DECODE": "0"}, "1": {"GROM_DEVICE_DECODE": "1"},
             "3w": {"GROM_DEVICE_DECODE": "1", "GROM_DD_WORKERS": "3"},
             "g0": {"GROM_DEVICE_DECODE": "1", "GROM_WS_GUESS": "0"},
             "g2": {"GROM_DEVICE_DECODE": "1", "GROM_WS_GUESS": "2"},
             "cu": {"GROM_DEVICE_DECODE": "1", "GROM_COPY_TILES": "1", "GROM_TEST_CP_UNSTAGED": "1"},
             "pc": {"GROM_DEVICE_DECODE": "1", "GROM_DD_PIECE_MB": "0.0625"},
             "pcu": {"GROM_DEVICE_DECODE": "1", "GROM_DD_PIECE_MB": "0.0625", "GROM_COPY_TILES": "1"}}
    for mode, env in modes.items():
        capfd.readouterr()
        run_grom(datadir, bam, fa, f"g{mode}_{tag}.vcf", extra,
                 env_extra=dict(env, GROM_STAGE_DIGEST="1", GROM_VERBOSE="1"))
        out = capfd.readouterr().out
        assert ("device decode:" in out) == (mode != "0"), out[-1500:]
        if mode == "3w":
            assert " 3 decode workers," in out, out[-1500:]
        lines[mode] = sorted(l for l in out.splitlines() if l.startswith("stage "))
    assert lines["1"] and all(lines[m] == lines["0"] for m in modes), {m: lines[m][:3] for m in modes}
    for mode in modes:
        for ext in (".vcf", ".ctx.vcf"):
            assert open(datadir / f"o_{tag}{ext}").read() == open(datadir / f"g{mode}_{tag}{ext}").read(), (mode, ext)


def _sha_rows(path, rows_only=False):
    import hashlib
    h = hashlib.sha256()
    rows = 0
    with open(path, "rb") as f:
        for line in f:
            row = not line.startswith(b"#")
            if row or not rows_only:
                h.update(line)
            rows += row
    return h.hexdigest(), rows


@pytest.mark.parametrize("case", ["c4_20mb_60x", "genome_s010", "genome_s100", "c4_share_400mb_60x"])
def test_oracle_digest_cases(datadir, case):
    """Inputs too large for the oracle inside a GPU test, checked against the
    oracle's digests (tests/golden/oracle_<case>.json, written on the CPU by
    tools/make_golden_genome.py): BASELINE configs[4]'s shape at 20 Mb (60x
    tetraploid male donor, -p 4 -g 1 -M -V 1), a 24-contig genome at 0.1 of
    GRCh38's lengths (configs[2]'s shape, -M -g 1), and the bench's own
    full-scale configs[2] genome (3.09 Gb, a 20 GB BAM; the oracle took 2.6 h
    on one core, 3,178,516 rows), and the largest 8-GPU share's chromosomes
    (chr2, chr14, chr22: 400 Mb) in configs[4]'s shape (60x tetraploid,
    -p 4 -g 1 -M; 393,804 rows, the oracle took 38 min).  The BAM is written here
    by the same deterministic grom_synth call; VCF and .ctx.vcf must hash to
    the oracle's."""
    import json
    from _util import REPO
    rec = json.load(open(os.path.join(REPO, "tests", "golden", f"oracle_{case}.json")))
    d = datadir / case
    d.mkdir(exist_ok=True)
    synth(d, "genome", rec["synth_args"])
    run_grom(d, "genome.bam", "genome.fa", "o.vcf", rec["cli_flags"])
    ro = rec.get("sha_of") == "rows"
    assert _sha_rows(d / "o.vcf", ro) == (rec["vcf_sha256"], rec["vcf_rows"])
    assert _sha_rows(d / "o.ctx.vcf", ro) == (rec["ctx_sha256"], rec["ctx_rows"])


@pytest.mark.parametrize("case,cap", [("c3_genome", "20000"), ("c3_genome", "150000"), ("cnv_multi", "20000")],
                         ids=["cap_in_first_run", "cap_past_first_run", "first_run_not_longest"])
def test_device_decode_stats_prefix(datadir, capfd, case, cap):
    """The device decoder takes the insert statistics (find_insert_mean,
    GROM.c:1205-1318: the first 10^7 qualifying records in file order) from
    the pieces of the first run as they are decoded for its chromosome, and
    goes on into the runs after it (the statistics alone) when the first run
    holds too few.  With the cap lowered for the test (GROM_TEST_INSERT_CAP,
    read by both decoders): a cap the first run holds (reached in its first
    pieces with 64 kB pieces) and one past it.  cnv_multi's first contig is
    not its longest: one worker decodes it first anyway (the sample is in file
    order), and of two workers the one that gathers the statistics does not
    parse it (a statistics-only pass over it).  The "workers" mode runs two
    workers on the GPU with 0.25 MB pieces: the mode that faulted the device
    in round 5 (the next run's block table read before its upload landed,
    DESIGN.md 4.5)."""
    bam, fa = synth(datadir, case, CASES[case])
    extra = ["-M", "-V", "1"]
    common = {"GROM_TEST_INSERT_CAP": cap, "GROM_STAGE_DIGEST": "1", "GROM_VERBOSE": "1"}
    modes = {"host": {"GROM_DEVICE_DECODE": "0"},
             "device": {"GROM_DEVICE_DECODE": "1"},
             "pieces": {"GROM_DEVICE_DECODE": "1", "GROM_DD_PIECE_MB": "0.0625"},
             "workers": {"GROM_DEVICE_DECODE": "1", "GROM_DD_PIECE_MB": "0.25", "GROM_DD_WORKERS": "2"}}
    got = {}
    for mode, env in modes.items():
        capfd.readouterr()
        run_grom(datadir, bam, fa, f"pfx_{case}_{cap}_{mode}.vcf", extra, env_extra=dict(common, **env))
        out = capfd.readouterr().out
        if mode == "workers":
            assert " 2 decode workers," in out, out[-1500:]
            if case == "cnv_multi":  # the gatherer (worker 0) does not own the first run: a statistics-only pass
                assert int(re.search(r"(\d+) statistics-only runs", out).group(1)) >= 1, out[-1500:]
        ins = [l for l in out.splitlines() if l.startswith(("insert mean", "insert_min_size", "median read"))]
        stages = sorted(l for l in out.splitlines() if l.startswith("stage "))
        vcf = open(datadir / f"pfx_{case}_{cap}_{mode}.vcf").read() + open(datadir / f"pfx_{case}_{cap}_{mode}.ctx.vcf").read()
        got[mode] = (ins, stages, vcf)
    assert got["host"][0] and got["host"][1]
    for mode in modes:
        assert got[mode] == got["host"], mode


@pytest.mark.parametrize("case,extra,env", [
    ("cnv_multi", ["-V", "1", "-M"], {"GROM_DD_WORKERS": "2"}),
    ("cnv_multi", ["-V", "1", "-M"], {"GROM_DD_WORKERS": "2", "GROM_DD_PIECE_MB": "0.125"}),
    ("c3_genome", ["-M", "-V", "1"], {"GROM_DD_WORKERS": "3", "GROM_DD_PIECE_MB": "0.25"})],
    ids=["cnv_multi_2w", "cnv_multi_2w_pieces", "c3_genome_3w_pieces"])
def test_decode_workers_share_session(datadir, capfd, case, extra, env):
    """Several device decode workers in one session on one GPU: the shape
    `grom -P n` runs across n GPUs (one decode worker per GPU, pdecode.c
    dw_main), mapped onto the one GPU of the test box.  Worker 0 gathers the
    insert statistics (find_insert_mean, GROM.c:1205-1318) but, with
    cnv_multi's longer second contig dealt to it first, does not own the
    first run in file order: it reads the statistics from that run (and the
    next) alone, while worker 1 parses it.  Each worker issues its next run's
    first piece ahead; the workers share the stages.  Full statistics cap,
    default and small pieces; every staged chromosome's digest equals the host
    decoder's and the VCF/.ctx.vcf the oracle's, at the full insert-sample
    cap."""
    bam, fa = synth(datadir, case, CASES[case])
    tag = f"dw_{case}_{'_'.join(f'{k}{v}' for k, v in env.items())}".replace(".", "")
    run_oracle(datadir, bam, fa, f"o_{tag}.vcf", extra)
    stages = {}
    for mode, e in {"host": {"GROM_DEVICE_DECODE": "0"}, "dev": dict(env, GROM_DEVICE_DECODE="1")}.items():
        capfd.readouterr()
        run_grom(datadir, bam, fa, f"{mode}_{tag}.vcf", extra, env_extra=dict(e, GROM_STAGE_DIGEST="1", GROM_VERBOSE="1"))
        out = capfd.readouterr().out
        stages[mode] = sorted(l for l in out.splitlines() if l.startswith("stage "))
        if mode == "dev":
            assert f" {env['GROM_DD_WORKERS']} decode workers," in out, out[-1500:]
            if case == "cnv_multi":
                assert int(re.search(r"(\d+) statistics-only runs", out).group(1)) >= 1, out[-1500:]
        for ext in (".vcf", ".ctx.vcf"):
            assert open(datadir / f"o_{tag}{ext}").read() == open(datadir / f"{mode}_{tag}{ext}").read(), (mode, ext)
    assert stages["host"] and stages["dev"] == stages["host"]


_FOOT = re.compile(r"buffers: peak ([\d.]+) GB together, per kind scan ([\d.]+), breakpoint ([\d.]+), CNV ([\d.]+), "
                   r"stages ([\d.]+), decode ([\d.]+), phase arenas ([\d.]+) GB; (\d+) allocations waited")


def test_hbm_cap_waits_for_memory(datadir):
    """Running short of device memory does not fail the run (devmem.h): with a
    test-only cap on this process's device memory (GROM_TEST_HBM_CAP) below
    what the run holds uncapped -- room for the scan contexts, the decoder and
    about one and a half input stages -- allocations first free idle stages'
    blocks and then wait for a scan to give its stage back.  The rows must
    still be the oracle's.  Three stages (the CLI's default is one per scan
    context, two): the cap leaves room for one and a half of them, so a scan
    can always go on while another waits."""
    from _util import FILEDATE, GROM_BIN, SEED
    case, extra = "c3_genome", ["-M", "-V", "1"]
    bam, fa, tag = _oracle_once(datadir, case, extra)
    env = dict(os.environ, GROM_FILEDATE=FILEDATE, GROM_SEED=SEED, GROM_VERBOSE="1", GROM_STAGES="3")

    def run(out, more):
        r = subprocess.run([GROM_BIN, "-i", bam, "-r", fa, "-o", out] + extra, env=dict(env, **more),
                           cwd=str(datadir), capture_output=True, text=True, timeout=150)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        m = _FOOT.search(r.stdout)
        assert m, r.stdout[-2000:]
        return [float(x) for x in m.groups()[:7]], int(m.group(8)), r.stdout

    (tot, _, _, _, stages, _, _), _, _ = run("g_cap_free.vcf", {})
    cap = (tot - stages + 0.5 * stages) * 1e9
    (tot2, *_), waits, out = run("g_cap.vcf", {"GROM_TEST_HBM_CAP": str(int(cap)), "GROM_ALLOC_WAIT_S": "40"})
    reclaimed = int(re.search(r"idle stage blocks reclaimed (\d+)", out).group(1))
    assert waits + reclaimed > 0, out[-1500:]
    assert tot2 * 1e9 <= cap * 1.0001
    for ext in (".vcf", ".ctx.vcf"):
        assert open(datadir / f"o_{tag}{ext}").read() == open(datadir / f"g_cap{ext}").read()
