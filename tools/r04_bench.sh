#!/bin/bash
# round-4: the GPU parity tests named on the command line, then the driver's
# bench command (N=1) with its stderr kept
set -o pipefail
mkdir -p gpurun_out/bench
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 250 --timeout-method thread "$@" > gpurun_out/bench/pytest.log 2>&1 \
    || { tail -40 gpurun_out/bench/pytest.log; exit 1; }
  tail -3 gpurun_out/bench/pytest.log
fi
timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench/bench.json 2> gpurun_out/bench/bench_stderr.log || { tail -30 gpurun_out/bench/bench_stderr.log; exit 1; }
cat gpurun_out/bench/bench.json
tail -20 gpurun_out/bench/bench_stderr.log
