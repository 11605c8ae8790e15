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
    assert lib.grom_abi_version() == 7
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


@pytest.mark.parametrize("case,extra", [("one_chr", []), ("three_chr", []), ("empty_middle", []), ("lowmapq_clip", []),
                                        ("three_chr", ["-P", "2"]), ("empty_middle", ["-P", "2"]),
                                        ("lowmapq_clip", ["-P", "1"])],
                         ids=["one_chr", "three_chr", "empty_middle", "lowmapq_clip", "three_chr_P2", "empty_middle_P2",
                              "lowmapq_clip_P1"])
def test_stream_plan_matches_oracle_walk(datadir, case, extra):
    """The per-chromosome record plan (skip prefix, last base reached) equals what
    the oracle's serial walk did, including the two records lost at every
    chromosome boundary (Q1) and the empty chromosome swallowing the file (Q21).
    With -P n each chromosome reads its own records (bam_fetch, GROM.c:21051-
    21064 / the -c children, 549-599): no Q1 drops, no Q21 starvation, in the
    CLI and in the oracle alike."""
    bam, fa = synth(datadir, case, CASES[case])
    tag = case + "".join(extra).replace("-", "_")
    dump = str(datadir / f"plan_{tag}")
    run_oracle(datadir, bam, fa, f"plan_{tag}.vcf", extra, dump=dump)
    r = run(GROM_BIN, ["-i", bam, "-r", fa, "-o", f"plan_{tag}_g.vcf"] + extra, str(datadir), {"GROM_PLAN_ONLY": "1"})
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


@pytest.mark.parametrize("case,subsets", [("three_chr", ["chr2", "chr1,chr3"]), ("empty_middle", ["chr3", "chr1"]),
                                          ("sv", ["chr2"])])
def test_chromosome_subset_keeps_serial_facts(datadir, case, subsets):
    """GROM_CHROMS (one rank's share in bench.py --gpus N): the chosen
    chromosomes get exactly the input a whole run gives them (Q1/Q21 follow the
    full plan), through the streamed decoder and the serial reader; the
    others are not decoded."""
    bam, fa = synth(datadir, case, CASES[case])
    base = ["-i", bam, "-r", fa, "-o", f"sub_{case}.vcf"]
    full = {l.split()[1]: l for l in run(GROM_BIN, base, str(datadir), {"GROM_PLAN_ONLY": "1"}).stdout.splitlines()
            if l.startswith("plan ")}
    assert full
    for sub in subsets:
        names = sub.split(",")
        for extra in ({"GROM_PIECE_RECS": "1500"}, {"GROM_SERIAL_DECODE": "1"}):
            r = run(GROM_BIN, base, str(datadir), dict(extra, GROM_PLAN_ONLY="1", GROM_CHROMS=sub))
            got = {l.split()[1]: l for l in r.stdout.splitlines() if l.startswith("plan ")}
            if "GROM_SERIAL_DECODE" not in extra:
                assert sorted(got) == sorted(n for n in names if n in full), (sub, got)
            for n, line in got.items():
                if n in names:
                    assert line == full[n], (sub, extra, line, full[n])


def test_q21_empty_chromosome_starves_later_ones(datadir):
    bam, fa = synth(datadir, "empty_middle", CASES["empty_middle"])
    r = run(GROM_BIN, ["-i", bam, "-r", fa, "-o", "q21.vcf"], str(datadir), {"GROM_PLAN_ONLY": "1"})
    plan = parse_plan(r.stdout)
    assert plan["chr1"]["reads"] > 0
    assert plan["chr2"]["reads"] == 0 and plan["chr3"]["reads"] == 0


@pytest.mark.parametrize("case", ["three_chr", "empty_middle", "sv", "dups"])
def test_p_fetch_streamed_matches_serial_reader(datadir, case):
    """-P n (the reference's per-chromosome bam_fetch input): the streamed
    decoder and the serial reader hand every chromosome the same input (facts
    and digests); it differs from the serial stream's exactly at the
    chromosome boundaries -- no chromosome after the first loses records (Q1)
    and an empty chromosome starves nothing (Q21); GROM_P_SERIAL=1 restores
    the serial stream's input."""
    bam, fa = synth(datadir, case, CASES[case])
    base = ["-i", bam, "-r", fa, "-o", f"pf_{case}.vcf"]
    plans = {}
    for mode, args, env in (("serial", [], {}), ("fetch", ["-P", "2"], {}), ("fetch_reader", ["-P", "2"], {"GROM_SERIAL_DECODE": "1"}),
                            ("fetch_pieces", ["-P", "2"], {"GROM_PIECE_RECS": "777", "GROM_DECODE_THREADS": "3"}),
                            ("p_serial", ["-P", "2"], {"GROM_P_SERIAL": "1"})):
        r = run(GROM_BIN, base + args, str(datadir), dict(env, GROM_PLAN_ONLY="1"))
        plans[mode] = parse_plan(r.stdout)
    assert plans["fetch"] and plans["fetch"] == plans["fetch_reader"] == plans["fetch_pieces"]
    assert plans["p_serial"] == plans["serial"]
    first = min(plans["serial"], key=lambda n: plans["serial"][n]["tid"])
    for n, p in plans["fetch"].items():
        q = plans["serial"][n]
        if n == first or (case == "empty_middle" and n == "chr2"):
            assert p == q, (n, p, q)
        elif case == "empty_middle":
            assert q["reads"] == 0 and p["reads"] > 0, (n, p, q)  # Q21 in the serial stream only
        else:
            assert p["reads"] >= q["reads"] and p != q, (n, p, q)  # the two records Q1 drops


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


def test_integration_stub_is_the_compiled_text():
    """INTEGRATION.md section 2 shows exactly the stub that
    tools/gromc_binding.c compiles (between its BEGIN/END markers), and the
    built program links against the library and starts (usage exit)."""
    import re
    import subprocess
    src = open(os.path.join(REPO, "tools", "gromc_binding.c")).read()
    a = src.index("/* ---- BEGIN INTEGRATION.md §2 stub ---- */\n")
    a = src.index("\n", a) + 1
    b = src.index("/* ---- END INTEGRATION.md §2 stub ---- */")
    md = open(os.path.join(REPO, "INTEGRATION.md")).read()
    blocks = re.findall(r"```c\n(.*?)```", md, flags=re.S)
    assert src[a:b] in blocks
    stub = src[a:b]
    # every option-set global of the scan reaches grom_params (GROM.c:21908-22103)
    for g in ("g_min_disc", "g_max_split_loss", "g_min_sr_len", "g_max_homopolymer", "g_max_ins_range",
              "g_pval_threshold", "g_pval_insertion", "g_min_sv_ratio", "g_min_indel_ratio", "g_max_evidence_ratio",
              "g_1000gen_window", "g_sv_list2_len", "lseq_tail"):
        assert g in stub, g
    exe = os.path.join(REPO, "grom_amd", "bin", "gromc_binding")
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr


def test_synth_stream_batches_match_the_cli_plan(datadir):
    """grom_synth_chrom_stream (what bench.py keeps resident) gives each
    chromosome exactly the input the CLI's streamed decoder stages from the
    genome's BAM (-g 1: every contig processed): same stream facts and digest,
    so the resident pass and the whole CLI run can be compared row for row."""
    import ctypes
    import grom_amd
    lengths, names = [700_000, 500_000, 400_000, 300_000], ["chr1", "chr2", "chrX", "chrY"]
    args = ["-L", ",".join(map(str, lengths)), "-n", ",".join(names), "-s", "3", "-X", "5", "-D", "0.05",
            "-V", "2e-06", "-W", "20000,80000"]
    bam, fa = synth(datadir, "gstream", args)
    r = run(GROM_BIN, ["-i", bam, "-r", fa, "-o", "gs.vcf", "-M", "-g", "1"], str(datadir), {"GROM_PLAN_ONLY": "1"})
    plan = parse_plan(r.stdout)
    assert sorted(plan) == sorted(n.lower() for n in names), plan
    imean, lseq, imin, imax = (int(x) for x in open(bam + ".mean").read().split()[:4])
    p = grom_amd.default_params()
    p.rmdup = 1
    grom_amd.lib().grom_params_set_insert(ctypes.byref(p), imean, imin, imax, lseq)
    for i, name in enumerate(names):
        b = grom_amd.SynthBatch.genome_chrom(lengths, i, p, names=names, sv_per_mb=5.0, dup_frac=0.05, cnv_rate=2e-6,
                                             cnv_range=(20_000, 80_000), seed=3, stream=True)
        try:
            got = {"reads": b.reads.n, "n_skip": b.chrom.n_skip, "p_last": b.chrom.p_last,
                   "lseq_tail": b.chrom.lseq_tail,
                   "digest": grom_amd.lib().grom_reads_digest(ctypes.byref(b.reads))}
        finally:
            b.close()
        want = plan[name.lower()]
        assert got == {k: want[k] for k in got}, (name, got, want)


def _bgzf_blocks(chunks, level, strategy):
    """BGZF blocks (gzip members with the BC extra field) of each chunk, raw
    DEFLATE at the given zlib level/strategy."""
    import struct
    import zlib
    out = bytearray()
    for data in chunks:
        c = zlib.compressobj(level, zlib.DEFLATED, -15, 8, strategy)
        body = c.compress(data) + c.flush()
        bsize = 18 + len(body) + 8 - 1
        out += bytes([0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, ord("B"), ord("C"), 2, 0]) + struct.pack("<H", bsize)
        out += body + struct.pack("<II", zlib.crc32(data) & 0xffffffff, len(data))
    return bytes(out)


def test_inflate_twin_matches_zlib(tmp_path):
    """The device BGZF inflater's decoder (inflate.h), compiled for the host,
    against zlib on every kind of DEFLATE block: stored (level 0 and
    incompressible data), fixed Huffman, dynamic Huffman at levels 1-9, the
    Huffman-only and run-length strategies, matches overlapping their source
    at periods 1-300 (the pattern and chunked copy paths), empty and 64 KiB
    blocks, and corrupted streams (both must fail)."""
    import ctypes
    import random
    import zlib
    import grom_amd
    rng = random.Random(5)
    chunks = [b"", b"A", bytes(rng.getrandbits(8) for _ in range(65280)), b"ACGT" * 16320]
    for period in (1, 2, 3, 5, 8, 9, 31, 300):
        unit = bytes(rng.getrandbits(8) for _ in range(period))
        chunks.append((unit * (60000 // period + 1))[:60000])
    chunks.append(bytes(rng.choice(b"ACGTN") for _ in range(50000)))
    chunks.append(b"".join(b"read%07d\t" % i + bytes(rng.choice(b"#+5?AEI") for _ in range(150)) for i in range(300)))
    lib = grom_amd.lib()
    f = lib.grom_inflate_selftest
    f.restype, f.argtypes = ctypes.c_int64, [ctypes.c_char_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64),
                                             ctypes.POINTER(ctypes.c_int64)]
    cases = [(0, zlib.Z_DEFAULT_STRATEGY)] + [(lv, zlib.Z_DEFAULT_STRATEGY) for lv in (1, 6, 9)] + \
            [(6, zlib.Z_FIXED), (6, zlib.Z_HUFFMAN_ONLY), (6, zlib.Z_RLE), (9, zlib.Z_FILTERED)]
    for level, strategy in cases:
        path = tmp_path / f"b{level}_{strategy}.bgzf"
        path.write_bytes(_bgzf_blocks(chunks, level, strategy))
        nb, by = ctypes.c_int64(), ctypes.c_int64()
        assert f(str(path).encode(), 0, ctypes.byref(nb), ctypes.byref(by)) == 0, (level, strategy)
        assert nb.value == len(chunks) and by.value == sum(map(len, chunks))
    # corrupted blocks: flipped bytes inside the DEFLATE data; both decoders
    # must agree that each block fails or succeeds (and on its bytes)
    good = bytearray(_bgzf_blocks(chunks[2:8], 6, zlib.Z_DEFAULT_STRATEGY))
    for k in range(40):
        bad = bytearray(good)
        i = 18 + rng.randrange(200)
        bad[i] ^= 1 << rng.randrange(8)
        path = tmp_path / f"bad{k}.bgzf"
        path.write_bytes(bytes(bad))
        nb, by = ctypes.c_int64(), ctypes.c_int64()
        assert f(str(path).encode(), 1, ctypes.byref(nb), ctypes.byref(by)) == 0, k


def test_fasta_pread_loader_matches_fgets_loader(tmp_path):
    """grom_fasta_load_at (pread + memchr chunks, several chromosomes at once)
    gives grom_fasta_load's bytes and lengths (fgets(line, 1000) per chunk,
    the alpha cut re-measured only when a chunk's length changes;
    GROM.c:21009-21045) on awkward files: lines over 999 bytes (split into
    fgets chunks, one starting with '>'), changing widths, trailing spaces and
    digits, CRLF, no final newline, empty entries; a NUL byte returns -2."""
    import random
    import grom_amd
    lib = grom_amd.lib()
    lib.grom_fasta_open.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    lib.grom_fasta_load.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_long]
    lib.grom_fasta_load.restype = ctypes.c_long
    lib.grom_fasta_load_at.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_long]
    lib.grom_fasta_load_at.restype = ctypes.c_long
    lib.grom_fasta_lengths.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_long), ctypes.c_int]
    lib.grom_fasta_close.argtypes = [ctypes.c_void_p]
    rng = random.Random(11)

    def seq(n):
        return "".join(rng.choice("ACGTNacgtn") for _ in range(n))

    entries = [
        ">c1 desc\n" + "".join(seq(60) + "\n" for _ in range(300)) + seq(17) + "\n",
        ">c2\n" + seq(2500) + "\n" + seq(80) + "  \n" + seq(80) + "12\n" + seq(3) + "\n",
        ">c3\r\n" + "".join(seq(70) + "\r\n" for _ in range(50)),
        ">c4\n" + seq(998) + ">" + seq(500) + "\n" + seq(60) + "\n",  # a chunk starting with '>'
        ">empty\n",
        ">c5\n" + seq(999) + "\n" + seq(1000) + "\n" + seq(1998) + "\n" + "".join(seq(rng.randint(1, 120)) + "\n" for _ in range(400)),
        ">c6\n" + "".join(seq(50) + "\n" for _ in range(100000)),
        ">last\n" + seq(61) + "\n" + seq(61),  # no final newline
    ]
    path = tmp_path / "odd.fa"
    path.write_text("".join(entries))
    f = ctypes.create_string_buffer(256)
    assert lib.grom_fasta_open(f, str(path).encode()) == 0
    n = ctypes.c_int.from_buffer(f, 8).value
    assert n == len(entries)
    lens_want = []
    for i in range(n):
        L = lib.grom_fasta_load(f, i, None, 0)
        buf_a = ctypes.create_string_buffer(L + 1)
        buf_b = ctypes.create_string_buffer(L + 1)
        assert lib.grom_fasta_load(f, i, buf_a, L) == L
        assert lib.grom_fasta_load_at(f, i, buf_b, L) == L, i
        assert buf_a.raw == buf_b.raw, i
        lens_want.append(L)
    idx = (ctypes.c_int * n)(*range(n))
    out = (ctypes.c_long * n)()
    assert lib.grom_fasta_lengths(f, idx, n, out, 4) == 0
    assert list(out) == lens_want
    lib.grom_fasta_close(f)
    nul = tmp_path / "nul.fa"
    nul.write_bytes(b">a\nACGT\x00ACGT\n")
    assert lib.grom_fasta_open(f, str(nul).encode()) == 0
    assert lib.grom_fasta_load_at(f, 0, None, 0) == -2
    lib.grom_fasta_close(f)


def test_block_table_in_chunks(tmp_path):
    """The prefetch thread builds a run's BGZF block table chunk by chunk
    (pdecode.c pf_read: a ring of pinned buffers, each holding the whole
    blocks that fit): the tables of every chunk, shifted by the chunk's
    offsets, must equal the table of the whole range, for chunk sizes that cut
    blocks anywhere, down to one block per chunk."""
    import zlib
    import grom_amd
    rng = __import__("random").Random(9)
    chunks = [bytes(rng.choice(b"ACGT#+5?") for _ in range(rng.randrange(1, 65280))) for _ in range(60)]
    data = _bgzf_blocks(chunks, 6, zlib.Z_DEFAULT_STRATEGY)

    class Blk(ctypes.Structure):
        _fields_ = [("in_off", ctypes.c_int64), ("out_off", ctypes.c_int64), ("in_len", ctypes.c_uint32),
                    ("out_len", ctypes.c_uint32), ("c_off", ctypes.c_int64)]
    lib = grom_amd.lib()
    tab, pre = lib.dd_block_table, lib.dd_block_table_prefix
    tab.restype = pre.restype = ctypes.c_int64
    tab.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.POINTER(Blk), ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
    pre.argtypes = tab.argtypes + [ctypes.POINTER(ctypes.c_int64)]
    whole = (Blk * 100)()
    ub = ctypes.c_int64()
    n = tab(data, len(data), whole, 100, ctypes.byref(ub))
    assert n == len(chunks) and ub.value == sum(map(len, chunks))
    ref = [(b.in_off, b.out_off, b.in_len, b.out_len, b.c_off) for b in whole[:n]]
    for size in (70000, 100000, 250000, 1 << 20):
        got, off, ob = [], 0, 0
        while off < len(data):
            buf = data[off:off + size]
            part = (Blk * 100)()
            cb, used = ctypes.c_int64(), ctypes.c_int64()
            k = pre(buf, len(buf), part, 100, ctypes.byref(cb), ctypes.byref(used))
            assert k > 0 and used.value > 0
            got += [(b.in_off + off, b.out_off + ob, b.in_len, b.out_len, b.c_off + off) for b in part[:k]]
            off += used.value
            ob += cb.value
        assert got == ref, size


def test_c_child_plans_match_p(datadir):
    """-c t,0,0,end (the child -P n forks per chromosome, GROM.c:549-599,
    21928-21930): target t alone, with the same bam_fetch input -P gives it;
    partial outputs OUT.<target>-0 (+ .ctx) and no full results file; a
    sub-region (-R) child is refused."""
    case = "three_chr"
    bam, fa = synth(datadir, case, CASES[case])
    p = parse_plan(run(GROM_BIN, ["-i", bam, "-r", fa, "-o", "cp.vcf", "-P", "2"], str(datadir),
                       {"GROM_PLAN_ONLY": "1"}).stdout)
    for t, name in enumerate(["chr1", "chr2", "chr3"]):
        r = run(GROM_BIN, ["-i", bam, "-r", fa, "-o", "cc.vcf", "-c", f"{t},0,0,300000000"], str(datadir),
                {"GROM_PLAN_ONLY": "1"})
        got = parse_plan(r.stdout)
        assert got == {name: p[name]}, (t, got)
        assert os.path.exists(os.path.join(str(datadir), f"cc.vcf.{name}-0.ctx"))
    assert not os.path.exists(os.path.join(str(datadir), "cc.vcf"))
    import subprocess
    r = subprocess.run([GROM_BIN, "-i", bam, "-r", fa, "-o", "cr.vcf", "-c", "1,1,100000,200000"], cwd=str(datadir),
                       capture_output=True, text=True, env=dict(os.environ, GROM_PLAN_ONLY="1"))
    assert r.returncode != 0 and "sub-region" in r.stdout
