#!/bin/bash
# round-4 GPU session 4: the full configs[2] BAM (3.09 Gb, 30x) through the
# whole-run CLI with the host decoder and with the device decoder (1, 2, 3
# workers); outputs compared; the configs[4]-shape digest case
set -o pipefail
out=gpurun_out/s4
mkdir -p $out
repo=$(pwd)
T="tests/test_gpu_parity.py"
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread \
  "$T::test_oracle_digest_cases[c4_20mb_60x]" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
work=/tmp/g4
mkdir -p $work
L=$(python3 -c "import bench; print(','.join(str(l) for _,l in bench.GRCH38))")
N=$(python3 -c "import bench; print(','.join(n for n,_ in bench.GRCH38))")
t0=$(date +%s.%N)
timeout -k 10 400 $repo/grom_amd/bin/grom_synth -o $work/g -L $L -n $N -s 3 -c 30.0 -l 150 -D 0.05 \
    -X 0.7123660266165851 -V 1.6190136968558754e-07 -W 10000,1000000 > /dev/null || exit 1
t1=$(date +%s.%N)
echo "synth $(python3 -c "print(round($t1 - $t0, 1))") s, $(stat -c %s $work/g.bam) bytes" | tee $out/synth.txt
cd $work
export GROM_FILEDATE=20260101 GROM_SEED=7
TIMEFORMAT='%R s wall, %U s user, %S s sys'
for m in ${MODES:-h d1 d2 d3}; do
  case $m in h) e="GROM_DEVICE_DECODE=0";; d1) e="GROM_DEVICE_DECODE=1 GROM_DD_WORKERS=1";;
             d2) e="GROM_DEVICE_DECODE=1 GROM_DD_WORKERS=2";; d3) e="GROM_DEVICE_DECODE=1 GROM_DD_WORKERS=3";; esac
  { time env $e GROM_VERBOSE=1 GROM_TRACE=$repo/$out/trace_$m.csv timeout -k 10 120 $repo/grom_amd/bin/grom \
      -i g.bam -r g.fa -o w_$m.vcf -M -g 1 > $repo/$out/whole_$m.log 2>&1 ; } 2> $repo/$out/whole_$m.time || { tail $repo/$out/whole_$m.log; exit 1; }
  echo "== $m: $(cat $repo/$out/whole_$m.time)"
  grep -h "decode\|cli " $repo/$out/whole_$m.log
  if [ $m != h ]; then cmp w_h.vcf w_$m.vcf && cmp w_h.ctx.vcf w_$m.ctx.vcf && echo "$m outputs identical to h" || exit 1; fi
done
rm -rf $work
