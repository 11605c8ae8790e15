#!/bin/bash
# the GPU inflater on a 5%-scale configs[2] BAM: throughput and a zlib check
set -o pipefail
mkdir -p gpurun_out /tmp/infl
L=$(python3 -c "import bench; print(','.join(str(max(int(l*0.05),1000000)) for _,l in bench.GRCH38))")
N=$(python3 -c "import bench; print(','.join(n for n,_ in bench.GRCH38))")
timeout -k 10 200 grom_amd/bin/grom_synth -o /tmp/infl/g -L $L -n $N -s 3 -c 30.0 -l 150 -D 0.05 -X 0.71 -V 1.6e-07 -W 10000,1000000 || exit 1
timeout -k 10 300 python tools/inflate_probe.py /tmp/infl/g.bam 0 0 > gpurun_out/inflate2.json || exit 1
timeout -k 10 300 python tools/inflate_probe.py /tmp/infl/g.bam 3e8 1 >> gpurun_out/inflate2.json || exit 1
cat gpurun_out/inflate2.json
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 tests/test_gpu_parity.py::test_device_inflate_matches_zlib 2>&1 | tail -3
