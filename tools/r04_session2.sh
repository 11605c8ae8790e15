#!/bin/bash
# round-4 GPU session 2: the GPU inflater's throughput, then the device
# decoder against the host decoder
set -o pipefail
mkdir -p gpurun_out /tmp/infl
L=$(python3 -c "import bench; print(','.join(str(max(int(l*0.05),1000000)) for _,l in bench.GRCH38))")
N=$(python3 -c "import bench; print(','.join(n for n,_ in bench.GRCH38))")
timeout -k 10 200 grom_amd/bin/grom_synth -o /tmp/infl/g -L $L -n $N -s 3 -c 30.0 -l 150 -D 0.05 -X 0.71 -V 1.6e-07 -W 10000,1000000 || exit 1
timeout -k 10 300 python tools/inflate_probe.py /tmp/infl/g.bam 0 0 > gpurun_out/s2_inflate.json || exit 1
cat gpurun_out/s2_inflate.json
T="tests/test_gpu_parity.py"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "$T::test_device_inflate_matches_zlib" "$T::test_device_decode_matches_host_decode" \
  > gpurun_out/s2_pytest.log 2>&1; rc=$?
tail -30 gpurun_out/s2_pytest.log
[ $rc -ne 0 ] && exit $rc
cd /tmp/infl && export GROM_FILEDATE=20260101 GROM_SEED=7
for m in 0 1; do
  ( time GROM_VERBOSE=1 GROM_DEVICE_DECODE=$m timeout -k 10 120 $GRAFT_REPO_ROOT/grom_amd/bin/grom -i g.bam -r g.fa -o w$m.vcf -M -g 1 > w$m.out ) 2> w$m.time || exit 1
  grep -h "decode:\|cli phases" w$m.out; cat w$m.time
done
cmp w0.vcf w1.vcf && cmp w0.ctx.vcf w1.ctx.vcf && echo "whole-run outputs identical"
