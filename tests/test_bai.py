"""BAM index (row 8f-1): the builder, the loader and region fetches.

The reference only checks that an index loads (GROM.c:22128-22138) and its
`-P` children fetch regions through it (bam_fetch, GROM.c:216-261).  The
builder's index is checked by fetching seeded random regions through it and
comparing with a full scan; the loader is pinned to the one index the
reference ships (test_data/tilapia_SAMD00023995_GL831235-1.bam.bai, written
by samtools 1.3.1, copied to tests/golden/) by an independent Python parse of
the SAM v1 section 5.2 layout."""
import ctypes as C
import os
import struct

import pytest

from _util import CASES, synth

GOLDEN_BAI = os.path.join(os.path.dirname(__file__), "golden", "tilapia_GL831235-1.bam.bai")


def _py_bai_summary(path):
    d = open(path, "rb").read()
    assert d[:4] == b"BAI\x01"
    n_ref, = struct.unpack_from("<i", d, 4)
    o, bins, chunks, intv = 8, 0, 0, 0
    for _ in range(n_ref):
        n_bin, = struct.unpack_from("<i", d, o)
        o += 4
        for _ in range(n_bin):
            b, n_chunk = struct.unpack_from("<Ii", d, o)
            assert b <= 37450
            o += 8
            for k in range(n_chunk):
                beg, end = struct.unpack_from("<QQ", d, o + 16 * k)
                assert b == 37450 or beg < end
            o += 16 * n_chunk
            chunks += n_chunk
        bins += n_bin
        n_intv, = struct.unpack_from("<i", d, o)
        o += 4 + 8 * n_intv
        intv += n_intv
    no_coor = struct.unpack_from("<Q", d, o)[0] if o + 8 <= len(d) else -1
    return [n_ref, bins, chunks, intv, no_coor], o + (8 if no_coor != -1 else 0) == len(d)


def _summary(path):
    import grom_amd
    out = (C.c_int64 * 5)()
    assert grom_amd.lib().grom_bai_summary(path.encode(), out) == 0
    return list(out)


def test_loader_reads_the_reference_index():
    want, whole = _py_bai_summary(GOLDEN_BAI)
    assert whole
    assert want[0] >= 1 and want[2] > 0
    assert _summary(GOLDEN_BAI) == want


@pytest.mark.parametrize("case", ["three_chr", "sv", "dups"])
def test_built_index_fetches_what_a_full_scan_finds(datadir, case):
    import grom_amd
    bam, _ = synth(datadir, case, CASES[case])
    bai = bam + ".bai"
    s, whole = _py_bai_summary(bai)
    assert whole and s == _summary(bai)
    assert s[1] > s[0]  # real bins, not the minimal empty index
    seen = C.c_int64(0)
    bad = grom_amd.lib().grom_bai_selftest(bam.encode(), 400, 7, C.byref(seen))
    assert bad == 0 and seen.value > 0


def test_rebuilt_index_is_byte_identical(datadir, tmp_path):
    import shutil
    import grom_amd
    bam0, _ = synth(datadir, "three_chr", CASES["three_chr"])
    bam = str(tmp_path / "x.bam")
    shutil.copy(bam0, bam)
    assert grom_amd.lib().grom_bai_build(bam.encode()) == 0
    assert open(bam + ".bai", "rb").read() == open(bam0 + ".bai", "rb").read()


def test_cli_rejects_an_index_that_does_not_load(datadir, tmp_path):
    import shutil
    import subprocess
    from _util import GROM_BIN
    bam0, fa0 = synth(datadir, "one_chr", CASES["one_chr"])
    bam, fa = str(tmp_path / "y.bam"), str(tmp_path / "y.fa")
    shutil.copy(bam0, bam)
    shutil.copy(fa0, fa)
    open(bam + ".bai", "wb").write(b"BAI\x01\xff")
    env = dict(os.environ, GROM_PLAN_ONLY="1")
    r = subprocess.run([GROM_BIN, "-i", bam, "-r", fa, "-o", "y.vcf"], cwd=str(tmp_path), env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "Could not open BAM indexing file" in r.stdout


def test_fetch_over_long_regions(datadir):
    """Region queries far longer than a leaf-bin list holds (a whole 80 Mb
    chromosome, 100 Mb spans): every bin is tested by its level's range, so
    the records past 64 Mb are fetched too."""
    import grom_amd
    bam, _ = synth(datadir, "sparse80", ["-L", "80000000", "-c", "0.05", "-s", "44"])
    seen = C.c_int64(0)
    bad = grom_amd.lib().grom_bai_selftest(bam.encode(), 60, 11, C.byref(seen))
    assert bad == 0 and seen.value > 0
