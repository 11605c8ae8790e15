"""CPU checks of the CNV oracle's restatements of the C library behaviour the
reference's static binary links, pinned against this
host's glibc: rand() after srand() (TYPE_3 additive feedback, unchanged since
glibc 2.0, so also glibc 2.12's) and qsort (merge sort in glibc < 2.37), and a
seed-determinism check of the oracle's CNV rows."""
import ctypes
import os

import numpy as np
import pytest

from _util import CASES, ORACLE_LIB, run_oracle, synth

libc = ctypes.CDLL("libc.so.6")
libc.rand.restype = ctypes.c_int
libc.srand.argtypes = [ctypes.c_uint]


def oracle():
    lib = ctypes.CDLL(ORACLE_LIB)
    lib.grom_oracle_rand_seq.argtypes = [ctypes.c_uint, ctypes.c_int, ctypes.c_void_p]
    lib.grom_oracle_msort_lo.argtypes = [ctypes.c_void_p, ctypes.c_long]
    lib.grom_oracle_grom_rand.argtypes = [ctypes.c_uint, ctypes.c_long, ctypes.c_int, ctypes.c_void_p]
    return lib


@pytest.mark.parametrize("seed", [0, 1, 7, 1792129490, 4294967295])
def test_rand_matches_glibc(seed):
    n = 5000
    out = np.zeros(n, np.int32)
    oracle().grom_oracle_rand_seq(seed, n, out.ctypes.data)
    libc.srand(seed)
    ref = np.array([libc.rand() for _ in range(n)], np.int32)
    assert np.array_equal(out, ref)


def test_grom_rand_digitwise_bounds():
    """grom_rand(max) (GROM.c:1185-1201) draws decimal digits below max."""
    out = np.zeros(2000, np.int64)
    oracle().grom_oracle_grom_rand(11, 123457, 2000, out.ctypes.data)
    assert out.min() >= 0 and out.max() < 123457
    assert len(np.unique(out)) > 1500


CMP = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p)


@CMP
def _cmp_lo(a, b):
    """cmpfunc (GROM.c:1105) applied to doubles: int subtraction of the low words."""
    x = ctypes.c_uint32.from_address(a).value
    y = ctypes.c_uint32.from_address(b).value
    return ctypes.c_int32((x - y) & 0xffffffff).value


@pytest.mark.skipif(tuple(int(v) for v in os.confstr("CS_GNU_LIBC_VERSION").split()[1].split(".")[:2]) >= (2, 37),
                    reason="glibc >= 2.37 replaced the merge sort")
@pytest.mark.parametrize("n", [1, 2, 17, 1000, 40000])
def test_msort_matches_glibc_qsort(n):
    rng = np.random.default_rng(n)
    a = (rng.integers(0, 60, n) / rng.uniform(10, 40)).astype(np.float64)  # ratios like rd / ave
    b = a.copy()
    oracle().grom_oracle_msort_lo(a.ctypes.data, n)
    libc.qsort(b.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(n), ctypes.c_size_t(8), _cmp_lo)
    assert np.array_equal(a.view(np.uint64), b.view(np.uint64))


def test_oracle_cnv_rows_deterministic_for_a_seed(tmp_path):
    bam, fa = synth(tmp_path, "cnv_small", ["-L", "400000", "-s", "21", "-V", "0.00001", "-W", "15000,60000",
                                             "-Q", "0.05"])
    run_oracle(tmp_path, bam, fa, "a.vcf", ["-V", "1"])
    run_oracle(tmp_path, bam, fa, "b.vcf", ["-V", "1"])
    a = open(tmp_path / "a.vcf").read()
    assert a == open(tmp_path / "b.vcf").read()
    assert a.count("SD:Z:CN:CS") > 0
