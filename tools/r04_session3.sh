#!/bin/bash
# round-4 GPU session 3: the step-wise inflater's throughput and zlib check,
# device decode parity (1 and 3 workers), configs[4]-shape digest case, and
# whole-run timings at 5% scale (host decode, device decode 1 and 2 workers)
set -o pipefail
mkdir -p gpurun_out /tmp/infl
L=$(python3 -c "import bench; print(','.join(str(max(int(l*0.05),1000000)) for _,l in bench.GRCH38))")
N=$(python3 -c "import bench; print(','.join(n for n,_ in bench.GRCH38))")
timeout -k 10 200 grom_amd/bin/grom_synth -o /tmp/infl/g -L $L -n $N -s 3 -c 30.0 -l 150 -D 0.05 -X 0.71 -V 1.6e-07 -W 10000,1000000 || exit 1
timeout -k 10 120 python tools/inflate_probe.py /tmp/infl/g.bam 0 0 > gpurun_out/s3_inflate.json || exit 1
timeout -k 10 200 python tools/inflate_probe.py /tmp/infl/g.bam 3e8 1 >> gpurun_out/s3_inflate.json || exit 1
cat gpurun_out/s3_inflate.json
T="tests/test_gpu_parity.py"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "$T::test_device_inflate_matches_zlib" "$T::test_device_decode_matches_host_decode" "$T::test_oracle_digest_cases[c4_20mb_60x]" \
  > gpurun_out/s3_pytest.log 2>&1; rc=$?
tail -20 gpurun_out/s3_pytest.log
[ $rc -ne 0 ] && exit $rc
cd /tmp/infl && export GROM_FILEDATE=20260101 GROM_SEED=7
for m in 0 1 2; do
  w=1; d=1; [ $m = 0 ] && d=0; [ $m = 2 ] && w=2
  ( time GROM_VERBOSE=1 GROM_DEVICE_DECODE=$d GROM_DD_WORKERS=$w timeout -k 10 120 $GRAFT_REPO_ROOT/grom_amd/bin/grom -i g.bam -r g.fa -o w$m.vcf -M -g 1 > w$m.out ) 2> w$m.time || exit 1
  echo "== mode $m"; grep -h "decode:\|cli phases" w$m.out; cat w$m.time
done
cmp w0.vcf w1.vcf && cmp w0.ctx.vcf w1.ctx.vcf && cmp w0.vcf w2.vcf && echo "whole-run outputs identical"
