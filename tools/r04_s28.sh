#!/bin/bash
# tools/r04_s28.sh OUT -- configs[2] genome once; RUNS whole-run CLI calls
# alternating the decode stream priority (GROM_DD_PRIORITY 1/0, outputs
# compared), then one run under rocprofv3 --kernel-trace --stats
set -o pipefail
out=gpurun_out/$1
mkdir -p $out
repo=$(pwd)
work=/tmp/g28
mkdir -p $work
export GROM_FILEDATE=20260101 GROM_SEED=7
TIMEFORMAT='%R s wall, %U s user, %S s sys'
L=$(python3 -c "import bench; print(','.join(str(l) for _,l in bench.GRCH38))")
N=$(python3 -c "import bench; print(','.join(n for n,_ in bench.GRCH38))")
SY="-s 3 -c 30.0 -l 150 -D 0.05 -X 0.7123660266165851 -V 1.6190136968558754e-07 -W 10000,1000000"
timeout -k 10 400 $repo/grom_amd/bin/grom_synth -o $work/g -L $L -n $N $SY > /dev/null || exit 1
echo "synth done"
cd $work
for r in 1 2 3 4 5; do
  p=$(( r % 2 ))
  { time GROM_DD_PRIORITY=$p GROM_VERBOSE=1 timeout -k 10 120 $repo/grom_amd/bin/grom \
      -i g.bam -r g.fa -o w_$r.vcf -M -g 1 > $repo/$out/whole_$r.log 2>&1 ; } 2> $repo/$out/whole_$r.time \
      || { tail $repo/$out/whole_$r.log; exit 1; }
  echo "== run $r priority $p: $(cat $repo/$out/whole_$r.time)"
  grep -h "decode\|cli " $repo/$out/whole_$r.log
  [ $r -gt 1 ] && { cmp w_1.vcf w_$r.vcf && cmp w_1.ctx.vcf w_$r.ctx.vcf || exit 1; }
done
cd /tmp && export TMPDIR=/tmp
GROM_EXIT_HANDLERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $repo/$out/prof -o run -- \
    $repo/grom_amd/bin/grom -i $work/g.bam -r $work/g.fa -o $work/p.vcf -M -g 1 > $repo/$out/prof_run.log 2>&1 || { tail $repo/$out/prof_run.log; exit 1; }
cd $repo
db=$(find $out/prof -name "*.db" | head -1)
timeout -k 10 200 python3 tools/kstats.py $db $out/kernel_stats.csv | head -40
rm -rf $work $out/prof
