"""CPU tests of the host side: the C ABI library, the serial-stream planner and
the generator.  No GPU calls."""
import ctypes
import os
import re

import pytest

from _util import CASES, REPO, synth, run, run_oracle, GROM_BIN

HEADER = os.path.join(REPO, "include", "grom_amd.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w \*]*?\b(grom_\w+)\s*\(", text, flags=re.M)
    return sorted(set(names))


def test_library_exports_every_declared_symbol():
    import grom_amd
    lib = grom_amd.lib()
    names = declared_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n
    assert lib.grom_abi_version() == 6
    # the ctypes mirror has the C layout of every ABI struct
    for i, st in enumerate((grom_amd.Params, grom_amd.Chrom, grom_amd.Reads, grom_amd.Out, grom_amd.Stats,
                              grom_amd.IndelRec, grom_amd.Aux, grom_amd.SvRec)):
        assert lib.grom_abi_struct_size(i) == ctypes.sizeof(st), st.__name__
    assert grom_amd.SV_DTYPE.itemsize == ctypes.sizeof(grom_amd.SvRec)
    # and the python binding declares a signature for each
    assert set(names) <= set(grom_amd._SIGS), set(names) - set(grom_amd._SIGS)


def test_device_calls_fail_loudly_without_device():
    import grom_amd
    p = grom_amd.default_params()
    lib = grom_amd.lib()
    rc = lib.grom_scan_chrom(0, None, None, None, None)
    assert rc != 0  # device 0 never initialised in this process


def test_generator_is_deterministic(datadir, tmp_path):
    a, _ = synth(datadir, "one_chr", CASES["one_chr"])
    b, _ = synth(tmp_path, "one_chr", CASES["one_chr"])
    assert open(a, "rb").read() == open(b, "rb").read()


def parse_plan(stdout):
    out = {}
    for line in stdout.splitlines():
        if line.startswith("plan "):
            f = line.split()
            kv = dict(x.split("=") for x in f[2:])
            out[f[1]] = {k: int(v, 16 if k == "digest" else 10) for k, v in kv.items()}
    return out


def parse_meta(path):
    d = {}
    for line in open(path):
        k, v = line.split()
        d[k] = int(v)
    return d


@pytest.mark.parametrize("case", ["one_chr", "three_chr", "empty_middle", "lowmapq_clip"])
def test_stream_plan_matches_oracle_walk(datadir, case):
    """The per-chromosome record plan (skip prefix, last base reached) equals what
    the oracle's serial walk did, including the two records lost at every
    chromosome boundary (Q1) and the empty chromosome swallowing the file (Q21)."""
    bam, fa = synth(datadir, case, CASES[case])
    dump = str(datadir / f"plan_{case}")
    run_oracle(datadir, bam, fa, f"plan_{case}.vcf", dump=dump)
    r = run(GROM_BIN, ["-i", bam, "-r", fa, "-o", f"plan_{case}_g.vcf"], str(datadir), {"GROM_PLAN_ONLY": "1"})
    plan = parse_plan(r.stdout)
    assert plan, r.stdout
    for name, p in plan.items():
        meta = parse_meta(f"{dump}.{name}.meta")
        assert p["n_skip"] == meta["n_skip"], (name, p, meta)
        if p["p_last"] >= 0:
            assert p["p_last"] + 1 == meta["p_end"], (name, p, meta)
        else:
            assert meta["n_ingested"] == 0


@pytest.mark.parametrize("case,extra", [(c, []) for c in CASES] + [("sv", ["-S"]), ("dups", ["-M"]),
                                                                    ("sv", ["-l", "2"])],
                         ids=[c for c in CASES] + ["sv_S", "dups_M", "sv_l2"])
def test_streamed_decode_matches_serial_reader(datadir, case, extra):
    """The parallel, index-driven decoder (pdecode.c: pieces cut at BAI
    offsets, decoded by several threads, fixed up in file order) hands every
    chromosome's scan exactly the input of the serial reader (stream.c, the
    restated my_samread loop): same stream facts (skip prefix, last base,
    pending record length, Q1/Q21) and the same digest of every array, CIGAR,
    base, quality and SA/XP record, dropped record, and of which overlapping
    reads share a read name.  Small pieces (GROM_PIECE_RECS) force many piece
    borders inside each chromosome."""
    bam, fa = synth(datadir, case, CASES[case])
    base = ["-i", bam, "-r", fa, "-o", f"pd_{case}.vcf"] + extra
    ser = run(GROM_BIN, base, str(datadir), {"GROM_PLAN_ONLY": "1", "GROM_SERIAL_DECODE": "1"})
    out = {}
    for thr, recs in (("1", "1000"), ("4", "777"), ("3", "65536")):
        r = run(GROM_BIN, base, str(datadir), {"GROM_PLAN_ONLY": "1", "GROM_DECODE_THREADS": thr,
                                               "GROM_PIECE_RECS": recs, "GROM_VERBOSE": "1"})
        assert "streamed decode:" in r.stdout, r.stdout[-2000:]
        out[thr] = sorted(l for l in r.stdout.splitlines() if l.startswith("plan "))
    want = sorted(l for l in ser.stdout.splitlines() if l.startswith("plan "))
    assert want
    for thr, got in out.items():
        assert got == want, (thr, got, want)


def test_q21_empty_chromosome_starves_later_ones(datadir):
    bam, fa = synth(datadir, "empty_middle", CASES["empty_middle"])
    r = run(GROM_BIN, ["-i", bam, "-r", fa, "-o", "q21.vcf"], str(datadir), {"GROM_PLAN_ONLY": "1"})
    plan = parse_plan(r.stdout)
    assert plan["chr1"]["reads"] > 0
    assert plan["chr2"]["reads"] == 0 and plan["chr3"]["reads"] == 0


def test_fmt_2f_matches_printf():
    """The VCF writer's exact %.2f (snvfmt.cpp) against glibc printf on 400k
    integer ratios, exact binary ties and edge cases (inf, nan, -0.0)."""
    import grom_amd
    assert grom_amd.lib().grom_fmt_selftest(200000, 12345) == 0


def _find_genome_length(fa):
    """find_genome_length (GROM.c:1321-1428) in Python: fgets(1000) lines,
    names cut at the first non-graph byte, lower-cased, file offsets after the
    header line."""
    recs, mappable, cur = [], 0, 0
    with open(fa, "rb") as f:
        while True:
            line = f.readline(999)
            if not line:
                break
            if line[:1] != b">":
                for c in line:
                    if chr(c).isalpha():
                        mappable += c not in b"Nn"
                        cur += 1
                continue
            if recs:
                recs[-1][3] = cur
            cur = 0
            end = len(line)
            for w in range(len(line) - 1, 0, -1):
                if not (0x21 <= line[w] <= 0x7e):
                    end = w
            end = min(end, 50)
            recs.append([len(recs), end - 1, f.tell(), 0, line[1:end].decode().lower()])
    if recs:
        recs[-1][3] = cur
    return mappable, recs


def test_fasta_info_cache_written_and_trusted(datadir, tmp_path):
    """The CLI writes <fasta>.info in save_genome_info's format (GROM.c:1028-1045)
    and, like GROM.c:22308, trusts it when it loads: a renamed chromosome in the
    cache makes that BAM target unmatched."""
    import shutil
    bam0, fa0 = synth(datadir, "three_chr", CASES["three_chr"])
    bam, fa = str(tmp_path / "g.bam"), str(tmp_path / "g.fa")
    shutil.copy(bam0, bam)
    shutil.copy(fa0, fa)
    shutil.copy(bam0 + ".bai", bam + ".bai")
    r = run(GROM_BIN, ["-i", bam, "-r", fa, "-o", "a.vcf"], str(tmp_path), {"GROM_PLAN_ONLY": "1"})
    assert {"chr1", "chr2", "chr3"} <= set(parse_plan(r.stdout)), r.stdout
    mappable, recs = _find_genome_length(fa)
    want = f"{len(recs)} {mappable}\n" + "".join(f"{i} {nl} {pos} {ln} {nm}\n" for i, nl, pos, ln, nm in recs)
    assert open(fa + ".info").read() == want
    lines = want.splitlines(True)
    lines[2] = lines[2].replace("chr2", "chrz")
    open(fa + ".info", "w").writelines(lines)
    r = run(GROM_BIN, ["-i", bam, "-r", fa, "-o", "b.vcf"], str(tmp_path), {"GROM_PLAN_ONLY": "1"})
    plan = parse_plan(r.stdout)
    assert "chr1" in plan and "chr3" in plan and "chr2" not in plan, r.stdout
    # a cache that does not parse is rebuilt from the FASTA
    open(fa + ".info", "w").write("3 1\n0 x\n")
    run(GROM_BIN, ["-i", bam, "-r", fa, "-o", "c.vcf"], str(tmp_path), {"GROM_PLAN_ONLY": "1"})
    assert open(fa + ".info").read().splitlines()[1:] == want.splitlines()[1:]
