#!/bin/bash
# round-4 GPU session 5: kernel stats of a whole CLI run with the device
# decoder (0.2-scale genome under rocprofv3), then the full configs[2] BAM
# through the whole-run CLI (device decode by default) twice
set -o pipefail
out=gpurun_out/s5
mkdir -p $out
repo=$(pwd)
T="tests/test_gpu_parity.py"
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread \
  "$T::test_device_decode_matches_host_decode" "$T::test_oracle_digest_cases" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
work=/tmp/g5
mkdir -p $work
export GROM_FILEDATE=20260101 GROM_SEED=7
TIMEFORMAT='%R s wall, %U s user, %S s sys'
Ls=$(python3 -c "import bench; print(','.join(str(max(int(l*0.2),1000000)) for _,l in bench.GRCH38))")
L=$(python3 -c "import bench; print(','.join(str(l) for _,l in bench.GRCH38))")
N=$(python3 -c "import bench; print(','.join(n for n,_ in bench.GRCH38))")
SY="-s 3 -c 30.0 -l 150 -D 0.05 -X 0.7123660266165851 -V 1.6190136968558754e-07 -W 10000,1000000"
timeout -k 10 200 $repo/grom_amd/bin/grom_synth -o $work/s -L $Ls -n $N $SY > /dev/null || exit 1
cd $work
GROM_VERBOSE=1 timeout -k 10 120 $repo/grom_amd/bin/grom -i s.bam -r s.fa -o warm.vcf -M -g 1 > /dev/null || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $repo/$out/prof -o run -- \
    $repo/grom_amd/bin/grom -i $work/s.bam -r $work/s.fa -o $work/p.vcf -M -g 1 > $repo/$out/prof_run.log 2>&1 || { tail $repo/$out/prof_run.log; exit 1; }
cd $repo
find $out/prof -name "*stats*" | head
cd $work
timeout -k 10 400 $repo/grom_amd/bin/grom_synth -o $work/g -L $L -n $N $SY > /dev/null || exit 1
for r in 1 2; do
  { time GROM_VERBOSE=1 GROM_TRACE=$repo/$out/trace_$r.csv timeout -k 10 120 $repo/grom_amd/bin/grom \
      -i g.bam -r g.fa -o w_$r.vcf -M -g 1 > $repo/$out/whole_$r.log 2>&1 ; } 2> $repo/$out/whole_$r.time || { tail $repo/$out/whole_$r.log; exit 1; }
  echo "== run $r: $(cat $repo/$out/whole_$r.time)"
  grep -h "decode\|cli " $repo/$out/whole_$r.log
done
cmp w_1.vcf w_2.vcf && cmp w_1.ctx.vcf w_2.ctx.vcf && echo "runs identical"
sha256sum w_1.vcf w_1.ctx.vcf | tee $repo/$out/full_sha.txt
grep -vc '^#' w_1.vcf
rm -rf $work
