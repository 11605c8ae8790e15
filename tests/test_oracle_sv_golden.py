"""Pin the breakpoint path (rows A10/A13) to the reference's golden VCF.

test_data/test_outuput_tilapia_*.vcf (GROM v1.0.0; its input BAM is a missing
blob) holds 1,222 INDEL_INS rows, 1,355 INDEL_DEL rows (a few printed as
<DEL> when longer than 98 bp), 19 <INS>, 5 <INV> and 127 <DEL> breakpoint
calls.  The counts behind them cannot be regenerated, but every row carries
the values the reference's tests computed from them, so the parts of the
restatement that turn counts into rows are pinned here:

- SPR / EPR are g_mq_prob_binom_cdf_table[n][k] at the printed depth n and
  evidence k (GROM.c:11357, 11470, 11640, 12478-12500, 12559-12580);
- the row filters of GROM.c:15320-16580 (p-value, evidence ratio,
  homopolymer) hold on every row;
- row layout, field order (including the INDEL_DEL fields printed under
  shifted FORMAT keys, GROM.c:16449) and the row-type order SNV, DUP, INV,
  INS, INDEL_INS, INDEL_DEL, DEL.

The same layouts are then checked on the oracle's own output for a synthetic
genome with deletions, duplications, inversions, insertions, translocations
and split reads."""
import re

import numpy as np
import pytest

from _util import CASES, GOLDEN_VCF, synth, run_oracle
from test_oracle_golden import oracle_tables

AF = 6  # cdp_add_factor
PVAL = 0.001  # g_pval_threshold (also g_pval_threshold1, GROM.c:22101)

# SV parity case: one 600 kb chromosome + a 300 kb partner for translocations
SV_CASE = CASES["sv"]


def _rows():
    out = []
    for line in open(GOLDEN_VCF):
        if line.startswith("#"):
            continue
        out.append(line.rstrip("\n").split("\t"))
    return out


def row_kind(f):
    fmt = f[8]
    if fmt.startswith("GT:PR:AF"):
        return "SNV"
    if fmt.startswith("SPR:SEV:SRD"):
        return "INDEL_INS"
    if fmt.endswith("SSC:ESC:HP"):
        return "INDEL_DEL"
    return {"<DUP>": "DUP", "<INV>": "INV", "<INS>": "INS", "<DEL>": "DEL"}[f[4]]


ORDER = ["SNV", "DUP", "INV", "INS", "INDEL_INS", "INDEL_DEL", "DEL"]


def _mq_at(mq, n, ev):
    """MQ[n][k] with k = count / 6 for a printed count / 6.0 (%.1f)."""
    cnt = int(round(float(ev) * AF))
    if n > 1000:
        return mq[1000][cnt * 1000 // (AF * n)]
    return mq[n][cnt // AF]


def test_golden_row_type_order():
    kinds = [row_kind(f) for f in _rows()]
    ranks = [ORDER.index(k) for k in kinds]
    assert ranks == sorted(ranks)
    counts = {k: kinds.count(k) for k in ORDER}
    assert counts["INDEL_INS"] == 1222 and counts["INS"] == 19 and counts["INV"] == 5
    assert counts["INDEL_DEL"] + counts["DEL"] == 1355 + 127


def test_golden_indel_ins_rows():
    """SPR = MQ[SRD][SEV] (GROM.c:11357), SPR <= g_pval_threshold and
    SEV/SRD > g_min_indel_ratio (GROM.c:16254), HP <= 10, END and the end
    fields of an insertion list entry are never set (END=0, ECO=EOT=0)."""
    mq, _ = oracle_tables(20)
    n = 0
    for f in _rows():
        if row_kind(f) != "INDEL_INS":
            continue
        n += 1
        v = f[9].split(":")
        spr, sev, srd, sco, eco, sot, eot, ssc, hp = float(v[0]), v[1], int(v[2]), int(v[3]), int(v[4]), int(v[5]), \
            int(v[6]), int(v[7]), int(v[8])
        assert "%e" % _mq_at(mq, srd, sev) == v[0], f
        assert spr <= PVAL
        assert float(sev) * AF / srd > 0.125 * AF
        assert hp <= 10 and f[7] == "END=0" and eco == 0 and eot == 0
        assert f[3] == "." and re.fullmatch(r"[ACGTNacgtn]+|<INS>", f[4])
    assert n == 1222


def test_golden_indel_del_rows():
    """INDEL_DEL: the printf fills SPR:EPR:SEV:EEV with binom/binom/f/r and the
    next eight keys with conc, conc, other, other, rd, rd, sc, sc
    (GROM.c:16449).  So SPR = MQ[field 9][SEV] and EPR = MQ[field 10][EEV];
    REF spans POS..END."""
    mq, _ = oracle_tables(20)
    n = 0
    for f in _rows():
        if row_kind(f) != "INDEL_DEL":
            continue
        n += 1
        v = f[9].split(":")
        rd_s, rd_e = int(v[8]), int(v[9])
        assert "%e" % _mq_at(mq, rd_s, v[2]) == v[0], f
        assert "%e" % _mq_at(mq, rd_e, v[3]) == v[1], f
        assert float(v[0]) <= PVAL and float(v[1]) <= PVAL
        assert float(v[2]) / rd_s > 0.125 and float(v[3]) / rd_e > 0.125
        assert int(v[12]) <= 10
        end = int(f[7][4:])
        if f[4] == "<DEL>":
            assert end - int(f[1]) + 1 >= 99
        else:
            assert len(f[3]) == end - int(f[1]) + 1 and f[4] == "."
    assert n > 1300


def test_golden_breakpoint_rows():
    """<DEL>/<INV> breakpoint calls: SPR = MQ[SRD][SEV], EPR = MQ[ERD][EEV]
    (GROM.c:12478-12500 and the nine sibling tests), the evidence ratio
    filter SEV/SRD >= g_min_sv_ratio (GROM.c:15322) and, for INV, both
    p-values <= g_pval_threshold (GROM.c:15795).  <INS>: END=POS and both
    p-values <= g_pval_insertion (GROM.c:15946)."""
    mq, _ = oracle_tables(20)
    seen = {"DEL": 0, "INV": 0, "INS": 0}
    for f in _rows():
        k = row_kind(f)
        if k not in seen:
            continue
        seen[k] += 1
        v = f[9].split(":")
        if k == "INS":
            assert f[7] == "END=" + f[1] and float(v[0]) <= 1e-10 and float(v[1]) <= 1e-10
            continue
        srd, erd = int(v[4]), int(v[5])
        assert "%e" % _mq_at(mq, srd, v[2]) == v[0], f
        assert "%e" % _mq_at(mq, erd, v[3]) == v[1], f
        assert float(v[2]) / srd >= 0.05 and float(v[3]) / erd >= 0.05
        if k == "INV":
            assert float(v[0]) <= PVAL and float(v[1]) <= PVAL
    assert seen["INV"] == 5 and seen["INS"] == 19 and seen["DEL"] > 100


ROW_PATTERNS = {
    "INDEL_INS": r"^[^\t]+\t\d+\t\.\t\.\t([ACGTNacgtn]+|<INS>)\t\.\t\.\tEND=0\tSPR:SEV:SRD:SCO:ECO:SOT:EOT:SSC:HP\t"
                 r"\d\.\d{6}e[+-]\d\d:\d+\.\d(:\d+){7}$",
    "INDEL_DEL": r"^[^\t]+\t\d+\t\.\t([ACGTNacgtn]+\t\.|\.\t<DEL>)\t\.\t\.\tEND=\d+\t"
                 r"SPR:EPR:SEV:EEV:SRD:ERD:SCO:ECO:SOT:EOT:SSC:ESC:HP\t(\d\.\d{6}e[+-]\d\d:){2}\d+\.\d:\d+\.\d(:\d+){9}$",
    "PAIR": r"^[^\t]+\t\d+\t\.\t\.\t<(DEL|DUP|INV)>\t\.\t\.\tEND=\d+\tSPR:EPR:SEV:EEV:SRD:ERD:SCO:ECO:SOT:EOT:SFR:SLR:EFR:ELR\t"
            r"(\d\.\d{6}e[+-]\d\d:){2}\d+\.\d:\d+\.\d(:-?\d+){10}$",
    "INS": r"^[^\t]+\t\d+\t\.\t\.\t<INS>\t\.\t\.\tEND=\d+\tSPR:EPR:SEV:EEV:SRD:ERD:SCO:ECO:SOT:EOT\t"
           r"(\d\.\d{6}e[+-]\d\d:){2}\d+\.\d:\d+\.\d(:\d+){6}$",
}


def _pattern_for(f):
    k = row_kind(f)
    return {"INDEL_INS": "INDEL_INS", "INDEL_DEL": "INDEL_DEL", "INS": "INS"}.get(k, "PAIR")


def test_golden_rows_match_layouts():
    for f in _rows():
        if row_kind(f) == "SNV":
            continue
        assert re.match(ROW_PATTERNS[_pattern_for(f)], "\t".join(f)), f


def test_oracle_sv_rows_layout_and_order(datadir):
    """The oracle's rows on the synthetic SV genome follow the golden layouts
    and row-type order, and every breakpoint class is exercised."""
    bam, fa = synth(datadir, "sv", SV_CASE)
    run_oracle(datadir, bam, fa, "sv.vcf")
    rows = [l.rstrip("\n").split("\t") for l in open(datadir / "sv.vcf") if not l.startswith("#")]
    mq, _ = oracle_tables(20)
    by_chr = {}
    for f in rows:
        by_chr.setdefault(f[0], []).append(row_kind(f))
        if row_kind(f) == "SNV":
            continue
        assert re.match(ROW_PATTERNS[_pattern_for(f)], "\t".join(f)), f
        v = f[9].split(":")
        if row_kind(f) == "INDEL_INS":
            assert "%e" % _mq_at(mq, int(v[2]), v[1]) == v[0], f
        elif row_kind(f) == "INDEL_DEL":
            assert "%e" % _mq_at(mq, int(v[8]), v[2]) == v[0], f
    for kinds in by_chr.values():
        ranks = [ORDER.index(k) for k in kinds]
        assert ranks == sorted(ranks)
    kinds = [row_kind(f) for f in rows]
    for k in ("INDEL_INS", "INDEL_DEL", "DEL", "DUP", "INV"):
        assert k in kinds, (k, sorted(set(kinds)))
    ctx = [l for l in open(datadir / "sv.ctx.vcf") if not l.startswith("#")]
    assert ctx, "no translocation rows"
    for l in ctx:
        assert re.match(r"^[^\t]+\t\d+\t\d+\tN\t(N\[|N\]|\[|\])[^\t]+\t\.\t\.\tSVTYPE=BND;MATEID=\d+\t"
                        r"SPR:SEV:SRD:SCO:SOT:SFR:SLR:SHPR\t\d\.\d{6}e[+-]\d\d:\d+\.\d(:\d+){5}:\d\.\d{6}e[+-]\d\d$", l), l
