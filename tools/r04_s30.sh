#!/bin/bash
# CNV parity cases, then the CNV timing counters on one 150 Mb chromosome
set -o pipefail
mkdir -p gpurun_out/s30
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_parity.py -k "cnv or c3_genome" > gpurun_out/s30/pytest.log 2>&1 || { tail -40 gpurun_out/s30/pytest.log; exit 1; }
tail -3 gpurun_out/s30/pytest.log
bash tools/r04_cnvtiming.sh
