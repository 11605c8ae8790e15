"""Pin the oracle (and the product's host tables) to the reference's only golden
vectors: test_data/test_outuput_tilapia_*.vcf (v1.0.0 output; its input BAM is a
missing blob, so these fix header text, record layout and the binomial-table
values printed in every SNV row -- SURVEY.md §4, §8c)."""
import ctypes
import re

import numpy as np
import pytest

from _util import GOLDEN_CTX, GOLDEN_VCF, ORACLE_LIB, FILEDATE, synth, run_oracle, CASES


def oracle_tables(min_mapq=20):
    lib = ctypes.CDLL(ORACLE_LIB)
    mq = np.zeros((1001, 1001))
    hez = np.zeros((1001, 1001))
    lib.grom_oracle_tables(min_mapq, mq.ctypes.data_as(ctypes.c_void_p), hez.ctypes.data_as(ctypes.c_void_p))
    return mq, hez


def golden_snv_rows():
    rows = []
    for line in open(GOLDEN_VCF):
        if line.startswith("#"):
            continue
        f = line.rstrip("\n").split("\t")
        if f[8].startswith("GT:PR:AF"):
            rows.append(f)
    return rows


def test_golden_has_expected_content():
    rows = golden_snv_rows()
    assert len(rows) == 18099


def test_oracle_mq_table_matches_every_golden_snv_pr():
    """PR = g_mq_prob_binom_cdf_table[n][k] (GROM.c:11141-11147) and AF = (float)k/n
    (GROM.c:11135) for all 18,099 SNV rows of the golden VCF."""
    mq, _ = oracle_tables(20)
    bad = []
    for f in golden_snv_rows():
        v = f[9].split(":")
        cnt = list(map(int, v[3:7]))
        alt = "ACGT".index(f[4])
        n, k = sum(cnt), cnt[alt]
        pr = mq[1000][k * 1000 // n] if n > 1000 else mq[n][k]
        af = np.float32(k) / np.float32(n)
        if "%e" % pr != v[1] or "%e" % float(af) != v[2]:
            bad.append((f[1], n, k, v[1], "%e" % pr))
    assert not bad, bad[:10]


def test_golden_genotype_rule():
    """GT = round(AF * ploidy) ones, at least one (GROM.c:15081-15103)."""
    for f in golden_snv_rows():
        v = f[9].split(":")
        ratio = float(v[2])
        cn = max(int(np.round(ratio * 2)) if ratio * 2 % 1 != 0.5 else int(ratio * 2 + 0.5), 1)
        gt = "/".join("1" if i < cn else "0" for i in range(2))
        assert v[0] == gt, (f[1], v[0], gt)


def test_product_tables_equal_oracle_tables():
    import grom_amd
    for q in (20, 5, 35):
        mq_o, hez_o = oracle_tables(q)
        hez_p, mq_p = grom_amd.build_tables(q)
        assert np.array_equal(mq_o.view(np.uint64), mq_p.view(np.uint64)), q
        assert np.array_equal(hez_o.view(np.uint64), hez_p.view(np.uint64)), q


def test_oracle_header_matches_golden(datadir):
    bam, fa = synth(datadir, "one_chr", CASES["one_chr"])
    run_oracle(datadir, bam, fa, "hdr.vcf")
    mine = [l for l in open(datadir / "hdr.vcf") if l.startswith("#")]
    gold = [l for l in open(GOLDEN_VCF) if l.startswith("#")]
    assert len(mine) == len(gold)
    for a, b in zip(mine, gold):
        if a.startswith("##fileDate") or a.startswith("##reference"):
            continue
        assert a == b
    mine_ctx = [l for l in open(datadir / "hdr.ctx.vcf")]
    gold_ctx = [l for l in open(GOLDEN_CTX)]
    assert len(mine_ctx) == len(gold_ctx)
    for a, b in zip(mine_ctx, gold_ctx):
        if not (a.startswith("##fileDate") or a.startswith("##reference")):
            assert a == b


def test_oracle_snv_row_layout_matches_golden(datadir):
    bam, fa = synth(datadir, "one_chr", CASES["one_chr"])
    run_oracle(datadir, bam, fa, "lay.vcf")
    pat = re.compile(r"^[^\t]+\t\d+\t\t[A-Za-z]\t[ACGT]\t\.\t\.\t\.\tGT:PR:AF:A:C:G:T:AL:CL:GL:TL:BQ:MQ:PIR:FS\t"
                     r"[01](/[01])*:\d\.\d{6}e[+-]\d\d:\d\.\d{6}e[+-]\d\d(:\d+){8}(:-?\d+\.\d\d){4}$")
    rows = [l.rstrip("\n") for l in open(datadir / "lay.vcf")
            if not l.startswith("#") and l.split("\t")[8].startswith("GT:PR:AF")]
    assert rows, "no SNV rows on the synthetic case"
    for r in rows:
        assert pat.match(r), r
    for f in golden_snv_rows()[:2000]:
        assert pat.match("\t".join(f)), f


def test_oracle_snv_acceptance_on_every_golden_row():
    """The oracle's SNV acceptance test (grom_oracle_snv_pick, the function its
    walk calls; GROM.c:11126-11156) accepts every one of the 18,099 golden SNV
    rows with the defaults (-n 3, -a 0.2, -x 15) and picks the printed ALT from
    the printed A:C:G:T counts.  BQ is printed as %.2f of bq_all/rc_all, so the
    test feeds bq_all = 100*BQ over rc_all = 100; a row printed at exactly the
    -x bound would be ambiguous (none is)."""
    lib = ctypes.CDLL(ORACLE_LIB)
    fn = lib.grom_oracle_snv_pick
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_long, ctypes.c_long, ctypes.c_int,
                   ctypes.c_double, ctypes.c_double]
    bad, ambiguous, multi = [], 0, 0
    for f in golden_snv_rows():
        v = f[9].split(":")
        cnt = (ctypes.c_int * 4)(*map(int, v[3:7]))
        bq = float(v[11])
        if abs(bq - 15.0) < 0.006:
            ambiguous += 1
            continue
        alts = [a for a in range(4) if "ACGT"[a] != f[3].upper() and cnt[a] >= 3]
        multi += len(alts) > 1
        got = fn(cnt, ord(f[3]), int(round(bq * 100)), 100, 3, 0.2, 15.0)
        if got < 0 or "ACGT"[got] != f[4]:
            bad.append((f[1], f[3], f[4], list(cnt), bq, got))
    assert ambiguous == 0
    assert not bad, bad[:10]
    # and the predicate rejects what it must: a reference-base "alt", too few
    # reads, too low a ratio, too low an average base quality
    c = (ctypes.c_int * 4)(0, 0, 10, 0)
    assert fn(c, ord("g"), 3000, 100, 3, 0.2, 15.0) == -1
    assert fn((ctypes.c_int * 4)(20, 0, 2, 0), ord("A"), 3000, 100, 3, 0.05, 15.0) == -1
    assert fn((ctypes.c_int * 4)(90, 0, 10, 0), ord("A"), 3000, 100, 3, 0.2, 15.0) == -1
    assert fn((ctypes.c_int * 4)(0, 0, 10, 0), ord("A"), 1400, 100, 3, 0.2, 15.0) == -1
    assert fn((ctypes.c_int * 4)(0, 5, 5, 0), ord("A"), 3000, 100, 3, 0.2, 15.0) == 1  # tie: the first
