#!/bin/bash
# round-4: the inflater alone on a 5%-scale configs[2] BAM (one launch over
# every block, HIP events) with and without the zlib check, then the device
# inflate / decode parity tests
set -o pipefail
mkdir -p gpurun_out/infl2 /tmp/infl
L=$(python3 -c "import bench; print(','.join(str(max(int(l*0.05),1000000)) for _,l in bench.GRCH38))")
N=$(python3 -c "import bench; print(','.join(n for n,_ in bench.GRCH38))")
timeout -k 10 200 grom_amd/bin/grom_synth -o /tmp/infl/g -L $L -n $N -s 3 -c 30.0 -l 150 -D 0.05 -X 0.71 -V 1.6e-07 -W 10000,1000000 > /dev/null || exit 1
timeout -k 10 120 python tools/inflate_probe.py /tmp/infl/g.bam 0 0 > gpurun_out/infl2/probe.json || exit 1
timeout -k 10 200 python tools/inflate_probe.py /tmp/infl/g.bam 3e8 1 >> gpurun_out/infl2/probe.json || exit 1
cat gpurun_out/infl2/probe.json
T="tests/test_gpu_parity.py"
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread "$T::test_device_inflate_matches_zlib" \
  "$T::test_device_decode_matches_host_decode" "$T::test_device_decode_stats_prefix" > gpurun_out/infl2/pytest.log 2>&1 || { tail -30 gpurun_out/infl2/pytest.log; exit 1; }
tail -3 gpurun_out/infl2/pytest.log
