"""CPU check of the oracle's CIGAR indel evidence (row A7, GROM.c:7187-7423)
against an independent pure-Python restatement over the BAM records.

No reference output covers these per-base values (the golden VCF of the
tilapia test has no INDEL rows and its BAM is missing), so they are "parity
unpinned" against the reference itself; this test pins the C oracle to a
second, separately written reading of the same lines, and the GPU parity tests
pin the HIP pass to the oracle."""
import gzip
import os
import re
import struct

import numpy as np

from _util import CASES, load_indels, run_oracle, synth

NT16 = "=ACMGRSVTWYHKDBN"
OTHER_LEN, ISEQ_LEN = 50, 50                       # GROM.c:837, 904
T_I, T_DF, T_DR = 11, 12, 13                       # OTHER_INDEL_*, GROM.c:679-681


def bam_records(path):
    """(pos, flag, mapq, cigar [(op, len)], seq str) for every record (BGZF is gzip)."""
    data = gzip.open(path).read()
    assert data[:4] == b"BAM\x01"
    l_text = struct.unpack_from("<i", data, 4)[0]
    o = 8 + l_text
    n_ref = struct.unpack_from("<i", data, o)[0]
    o += 4
    for _ in range(n_ref):
        l_name = struct.unpack_from("<i", data, o)[0]
        o += 4 + l_name + 4
    while o < len(data):
        bs = struct.unpack_from("<i", data, o)[0]
        rec = data[o + 4:o + 4 + bs]
        o += 4 + bs
        _tid, pos, l_rn, mapq, _bin, n_cig, flag, l_seq = struct.unpack_from("<iiBBHHHi", rec, 0)
        p = 32 + l_rn
        cig = [(w & 15, w >> 4) for w in struct.unpack_from(f"<{n_cig}I", rec, p)]
        p += 4 * n_cig
        sq = rec[p:p + (l_seq + 1) // 2]
        seq = "".join(NT16[(sq[k >> 1] >> (4 * (1 - (k & 1)))) & 15] for k in range(l_seq))
        yield pos, flag, mapq, cig, seq


def fold(state, x, typ, add, ln, iseq):
    """GROM.c:7209-7283 (I), 7289-7352 (D forward end), 7356-7420 (D reverse end)."""
    s = state.setdefault(x, {"c": {T_I: 0, T_DF: 0, T_DR: 0}, "d": {T_I: 0, T_DF: 0, T_DR: 0},
                             "rd": {T_DF: 0, T_DR: 0}, "seq": bytearray(52), "ot": []})
    if typ != T_I:
        s["rd"][typ] += 1
    if s["c"][typ] == 0:
        s["c"][typ], s["d"][typ] = add, ln
        if typ == T_I and ln <= ISEQ_LEN:
            s["seq"][:ln] = iseq.encode()
        return
    if ln == s["d"][typ]:
        s["c"][typ] += add
        return
    ot = s["ot"]                                    # [type, count, length] in slot order
    for slot in ot:
        if slot[0] == typ and slot[2] == ln:
            slot[1] += add
            if slot[1] > s["c"][typ]:
                slot[1], s["c"][typ] = s["c"][typ], slot[1]
                slot[2], s["d"][typ] = s["d"][typ], slot[2]
            return
    if len(ot) < OTHER_LEN:
        ot.append([typ, add, ln])
        return
    for slot in ot:
        if slot[1] <= add:
            slot[:] = [typ, add, ln]
            return


def test_oracle_indel_evidence_matches_python_restatement(datadir):
    args = list(CASES["indels"])
    args[args.index("-L") + 1] = "60000"
    bam, fa = synth(datadir, "indels_small", args)
    r = run_oracle(datadir, bam, fa, "o_ind_small.vcf", dump=str(datadir / "o_ind_small"))
    mean, _imin, imax = map(int, re.search(r"insert maximum: (\d+) (\d+) (\d+)", r.stdout).groups())
    rd_len = 2 * 8 * max(2 * mean - 1, imax + 1)      # GROM.c:22282-22290
    idx_start = rd_len // 4 + 1                       # GROM.c:2918
    meta = dict(l.split() for l in open(datadir / "o_ind_small.chr1.meta"))
    lo, hi = max(idx_start, 2 * imax + 1), int(meta["p_end"]) - 1

    state, n_in = {}, 0
    for pos, flag, mapq, cig, seq in bam_records(bam):
        if pos < idx_start:                           # Q2: skipped before the walk
            continue
        n_in += 1
        if flag & 0x4 or flag & 0x400:                # GROM.c:6418
            continue
        add = 6 if mapq >= 20 else 0                  # GROM.c:5829-5836
        tp, sb = pos, 0
        for op, ln in cig[:1000]:
            if op == 4:
                sb += ln
            elif op in (0, 3, 7, 8):
                tp += ln
                sb += 0 if op == 3 else ln
            elif op == 1:
                fold(state, tp, T_I, add, ln, seq[sb:sb + ln] if ln <= ISEQ_LEN else "")
                sb += ln
            elif op == 2:
                fold(state, tp, T_DF, add, ln, "")
                fold(state, tp + ln - 1, T_DR, add, ln, "")
                tp += ln
    assert n_in == int(meta["n_ingested"])

    got = load_indels(datadir / "o_ind_small.chr1.ind")
    want = sorted(x for x in state if lo <= x <= hi)
    assert len(want) > 20 and got["pos"].tolist() == want
    for g in got:
        s = state[int(g["pos"])]
        exp = (s["c"][T_I], s["d"][T_I], s["c"][T_DF], s["d"][T_DF], s["rd"][T_DF],
               s["c"][T_DR], s["d"][T_DR], s["rd"][T_DR], len(s["ot"]))
        have = tuple(int(g[k]) for k in ("ins", "ins_len", "del_f", "del_f_len", "del_f_rd", "del_r", "del_r_len",
                                         "del_r_rd", "other_len"))
        assert have == exp, (int(g["pos"]), have, exp)
        assert g["ins_seq"] == bytes(s["seq"]).rstrip(b"\0")
    assert (got["other_len"] > 0).sum() > 0
