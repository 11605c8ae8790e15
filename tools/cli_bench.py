"""tools/cli_bench.py -- the whole-run CLI leg of bench.py on its own: write the
scaled 24-contig 30x BAM, time the drop-in CLI as a fresh process, compare its
VCF with the oracle's.  usage: python tools/cli_bench.py [scale] [--no-oracle]"""
import json
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

scale = float(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else 0.04
keep = os.environ.get("CLI_BENCH_DIR")
d = keep or tempfile.mkdtemp()
print(json.dumps({"cpus": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}), flush=True)
st = bench.cli_whole_run_start(d, bench.C3, ["-M"], scale)
print(json.dumps(st["info"]), flush=True)
if "--no-oracle" in sys.argv:
    st["proc"].kill()
else:
    print(json.dumps(bench.cli_whole_run_finish(st)), flush=True)
