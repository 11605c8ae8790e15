#!/bin/bash
# CNV parity cases + the digest cases, the inflater probe, whole-run timings
set -o pipefail
mkdir -p gpurun_out/s27
T=tests/test_gpu_parity.py
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $T -k "cnv or digest or c3_genome or device_decode" > gpurun_out/s27/pytest.log 2>&1 || { tail -40 gpurun_out/s27/pytest.log; exit 1; }
tail -3 gpurun_out/s27/pytest.log
bash tools/r04_inflate2.sh && ALT_ENV=GROM_DD_PRELOAD=0 bash tools/r04_whole.sh s27w 1.0 3
