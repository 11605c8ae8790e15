#!/bin/bash
# round-4: the whole GPU suite (one pytest process), then whole-run timings
set -o pipefail
mkdir -p gpurun_out/full
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/full/gputest.log 2>&1 \
  || { tail -40 gpurun_out/full/gputest.log; exit 1; }
tail -3 gpurun_out/full/gputest.log
bash tools/r04_whole.sh ${WHOLE_OUT:-full_whole} ${WHOLE_SCALE:-1.0} ${WHOLE_RUNS:-3}
