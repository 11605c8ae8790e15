"""tools/r04_parent.py BAM FA MODE -- the whole-run CLI as a child of a Python
process that has (MODE=cuda) or has not (MODE=plain) initialised a GPU context
through torch: the child's device allocation time and wall time."""
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
bam, fa, mode = sys.argv[1:4]
if mode != "plain":
    import torch
    if mode == "cuda":
        torch.cuda.synchronize()
from grom_amd import GROM_BIN  # noqa: E402

env = dict(os.environ, GROM_FILEDATE="20260101", GROM_SEED="7", GROM_VERBOSE="1")
for k in range(2):
    t0 = time.perf_counter()
    r = subprocess.run([GROM_BIN, "-i", bam, "-r", fa, "-o", os.path.join(os.path.dirname(bam), "p.vcf"), "-M", "-g", "1"],
                       env=env, capture_output=True, text=True)
    dt = time.perf_counter() - t0
    dec = [l for l in r.stdout.splitlines() if l.startswith(("device decode", "cli phases"))]
    print(f"{mode} run {k}: rc {r.returncode}, {dt:.2f} s")
    for l in dec:
        print("   ", l[:400])
