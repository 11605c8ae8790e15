#!/bin/bash
# the whole GPU suite, then the stage-free A/B on the configs[2] genome
set -o pipefail
mkdir -p gpurun_out/full3
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/full3/gputest.log 2>&1 || { tail -30 gpurun_out/full3/gputest.log; exit 1; }
tail -3 gpurun_out/full3/gputest.log
bash tools/r04_ab.sh s35ab GROM_PAR_FREE 6
