#!/bin/bash
# device-decode parity (+ digests), then whole-run timings
set -o pipefail
mkdir -p gpurun_out/s34
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_parity.py -k "device_decode or late_fallback or c3_genome_cap" > gpurun_out/s34/pytest.log 2>&1 || { tail -40 gpurun_out/s34/pytest.log; exit 1; }
tail -3 gpurun_out/s34/pytest.log
bash tools/r04_whole.sh s34w 1.0 3
