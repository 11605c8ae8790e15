"""Host code under sanitizers (CPU only): AddressSanitizer + UBSan, and
ThreadSanitizer for the threaded paths.

`make sanitize SAN=asan|tsan` builds tools/san_driver.c against the library's
host sources compiled with the sanitizer (the device objects are linked
uninstrumented and never called) and grom_synth.  The runs cover:
  - the parallel BAM writer (synth.c: generator threads + compression queue,
    libdeflate per-thread compressors) and the BAI it writes (bamio.c);
  - the drop-in CLI with GROM_PLAN_ONLY: BAI planning, the streamed decoder
    (pdecode.c: decoder threads, the in-order uploader, tail sets, insert
    statistics) with small pieces so many borders are crossed, and the serial
    reader (GROM_SERIAL_DECODE);
  - BAI region queries against a linear scan, the SNV row formatter, the
    synthetic-batch builder and the translocation post-pass.
  - the scan worker pool: in plan-only mode the streamed decoder hands every
    chromosome to the pool's threads, which print its plan line;
  - svcall.cpp's candidate lists, SV assembly and rows (sv_rows) on inputs
    recorded from real GPU scans of the "sv" parity case (tests/golden/
    svh_*.svh.gz, written by tools/record_sv_hits.sh with GROM_SV_HITS_DUMP:
    parameters, reference, the per-base hits, every INV depth query with its
    answer, and the rows the GPU run wrote), replayed on concurrent threads,
    four rounds each, and compared with the recorded rows;
  - the device BGZF inflater's host twin (inflate.h) on the synthetic BAM.
Any sanitizer report fails the test (UBSan is built with
-fno-sanitize-recover, ASan/TSan exit non-zero).
"""
import glob
import gzip
import os
import shutil
import subprocess

import pytest

from _util import REPO

SYNTH_ARGS = ["-L", "300000,200000,150000", "-s", "3", "-c", "12", "-l", "100", "-X", "5", "-V", "1e-5",
              "-W", "2000,20000"]


def _build(san):
    if not shutil.which("g++"):
        pytest.skip("no host compiler")
    r = subprocess.run(["make", "-s", "sanitize", f"SAN={san}", "-j8"], cwd=REPO, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    d = os.path.join(REPO, "build", f"san-{san}")
    return os.path.join(d, "san_driver"), os.path.join(d, "grom_synth")


def _run(cmd, cwd, env=None, timeout=300):
    e = dict(os.environ)
    e.update(env or {})
    e.setdefault("ASAN_OPTIONS", "abort_on_error=0:detect_leaks=1")
    e.setdefault("TSAN_OPTIONS", "halt_on_error=1")
    r = subprocess.run(cmd, cwd=cwd, env=e, capture_output=True, text=True, timeout=timeout)
    out = r.stdout + r.stderr
    assert "Sanitizer" not in out and "runtime error" not in out, out[-6000:]
    assert r.returncode == 0, out[-6000:]
    return out


@pytest.mark.parametrize("san", ["asan", "tsan"])
def test_host_code_under_sanitizer(san, tmp_path):
    driver, synth = _build(san)
    d = str(tmp_path)
    _run([synth, "-o", "s"] + SYNTH_ARGS, d)
    plans = []
    for env in ({}, {"GROM_PIECE_RECS": "1500"}, {"GROM_SERIAL_DECODE": "1"}):
        out = _run([driver, "cli", "-i", "s.bam", "-r", "s.fa", "-o", "o.vcf"], d,
                   dict(env, GROM_PLAN_ONLY="1"))
        plans.append(sorted(line for line in out.splitlines() if line.startswith("plan ")))
    assert len(plans[0]) == 3 and plans[0] == plans[1] == plans[2], plans
    # svcall.cpp on recorded GPU-scan inputs, every record on its own thread
    recs = []
    for gz in sorted(glob.glob(os.path.join(REPO, "tests", "golden", "svh_*.svh.gz"))):
        path = os.path.join(d, os.path.basename(gz)[:-3])
        with gzip.open(gz, "rb") as fi, open(path, "wb") as fo:
            fo.write(fi.read())
        recs.append(path)
    assert len(recs) >= 2
    out = _run([driver, "svrows"] + recs, d)
    assert out.count(": rc 0") == len(recs), out
    if san == "asan":  # single-threaded helpers: once is enough
        assert "0 mismatches" in _run([driver, "inflate", "s.bam"], d)
        assert "0 mismatches" in _run([driver, "bai", "s.bam", "3000"], d)
        assert "0 mismatches" in _run([driver, "fmt", "20000"], d)
        assert "reads on a" in _run([driver, "synth", "200000"], d)
        assert "rc 0" in _run([driver, "ctx"], d)
