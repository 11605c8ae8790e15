"""Several device decode workers on one GPU (GROM_DD_WORKERS):
runs the CLI in this process (as the GPU tests do) on a synthetic case, first
with the host decoder, then repeatedly with the worker modes, and compares the
staged chromosome digests and the output with the host decoder's.  With
GROM_DD_TRACE=1 every compressed-slot fill and piece issue is logged to
stderr (kept under the output directory).

  python tools/dd_workers_probe.py OUTDIR [REPEATS]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from _util import CASES, FILEDATE, SEED, synth  # noqa: E402

import grom_amd  # noqa: E402


def run(d, bam, fa, out, env):
    e = {"GROM_FILEDATE": FILEDATE, "GROM_SEED": SEED, "GROM_STAGE_DIGEST": "1", "GROM_VERBOSE": "1"}
    e.update(env)
    # stdout/stderr of the library go to files (fd level)
    so, se = os.path.join(d, out + ".stdout"), os.path.join(d, out + ".stderr")
    sys.stdout.flush()
    sys.stderr.flush()
    o1, o2 = os.dup(1), os.dup(2)
    f1, f2 = os.open(so, os.O_WRONLY | os.O_CREAT | os.O_TRUNC), os.open(se, os.O_WRONLY | os.O_CREAT | os.O_TRUNC)
    os.dup2(f1, 1)
    os.dup2(f2, 2)
    try:
        rc = grom_amd.cli_main(["-i", bam, "-r", fa, "-o", out, "-M", "-V", "1"], env=e, cwd=d)
    finally:
        os.dup2(o1, 1)
        os.dup2(o2, 2)
        os.close(f1)
        os.close(f2)
        os.close(o1)
        os.close(o2)
    txt = open(so).read()
    stages = sorted(l for l in txt.splitlines() if l.startswith("stage "))
    ins = [l for l in txt.splitlines() if l.startswith(("insert mean", "insert_min_size", "median read"))]
    vcf = open(os.path.join(d, out)).read() if rc == 0 else ""
    return rc, ins, stages, vcf, open(se).read()


def main():
    d = os.path.abspath(sys.argv[1])
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    os.makedirs(d, exist_ok=True)
    case = os.environ.get("PROBE_CASE", "c3_genome")
    cap = os.environ.get("PROBE_CAP", "20000")
    bam, fa = synth(d, case, CASES[case])
    common = {"GROM_TEST_INSERT_CAP": cap}
    host = run(d, bam, fa, "host.vcf", dict(common, GROM_DEVICE_DECODE="0"))
    assert host[0] == 0 and host[2], host[4][-2000:]
    modes = {
        "device": {},
        "pieces": {"GROM_DD_PIECE_MB": "0.0625"},
        "w2_025": {"GROM_DD_PIECE_MB": "0.25", "GROM_DD_WORKERS": "2"},
        "w2": {"GROM_DD_WORKERS": "2"},
        "w3_0625": {"GROM_DD_PIECE_MB": "0.0625", "GROM_DD_WORKERS": "3"},
    }
    only = os.environ.get("PROBE_MODES")
    bad = 0
    for rep in range(reps):
        for m, env in modes.items():
            if only and m not in only.split(","):
                continue
            e = dict(common, GROM_DEVICE_DECODE="1", GROM_DD_WORKERS_UNSAFE="1", **env)
            if os.environ.get("PROBE_TRACE", "1") == "1":
                e["GROM_DD_TRACE"] = "1"
            tag = f"{m}_r{rep}"
            rc, ins, stages, vcf, err = run(d, bam, fa, tag + ".vcf", e)
            same = rc == 0 and ins == host[1] and stages == host[2] and vcf == host[3]
            fb = "fall" in err.lower() or "serial" in err.lower()
            print(f"{tag}: rc={rc} same={same} stages={len(stages)}/{len(host[2])} fallback_note={fb}", flush=True)
            if not same:
                bad += 1
                for a, b in zip(stages, host[2]):
                    if a != b:
                        print("   got ", a, "\n   want", b, flush=True)
                        break
                for l in err.splitlines():
                    if "ddtrace" not in l:
                        print("   stderr:", l[:300], flush=True)
    print("mismatching runs:", bad, flush=True)


if __name__ == "__main__":
    main()
