#!/bin/bash
# tools/r04_ab.sh OUT VAR RUNS -- configs[2] genome once; RUNS whole-run CLI
# calls alternating VAR=1 / VAR=0 (odd runs 1), outputs compared; the cli
# phase and teardown lines of each run
set -o pipefail
out=gpurun_out/$1
var=$2
runs=${3:-6}
mkdir -p $out
repo=$(pwd)
work=/tmp/gab
mkdir -p $work
export GROM_FILEDATE=20260101 GROM_SEED=7
TIMEFORMAT='%R s wall'
L=$(python3 -c "import bench; print(','.join(str(l) for _,l in bench.GRCH38))")
N=$(python3 -c "import bench; print(','.join(n for n,_ in bench.GRCH38))")
SY="-s 3 -c 30.0 -l 150 -D 0.05 -X 0.7123660266165851 -V 1.6190136968558754e-07 -W 10000,1000000"
timeout -k 10 400 $repo/grom_amd/bin/grom_synth -o $work/g -L $L -n $N $SY > /dev/null || exit 1
echo "synth done"
cd $work
GROM_VERBOSE=1 timeout -k 10 120 $repo/grom_amd/bin/grom -i g.bam -r g.fa -o w_0.vcf -M -g 1 > $repo/$out/warm.log 2>&1 || exit 1
for r in $(seq 1 $runs); do
  v=$(( r % 2 ))
  { time env $var=$v GROM_VERBOSE=1 timeout -k 10 120 $repo/grom_amd/bin/grom \
      -i g.bam -r g.fa -o w_$r.vcf -M -g 1 > $repo/$out/whole_$r.log 2>&1 ; } 2> $repo/$out/whole_$r.time \
      || { tail $repo/$out/whole_$r.log; exit 1; }
  echo "== run $r $var=$v: $(cat $repo/$out/whole_$r.time)"
  grep -h "cli " $repo/$out/whole_$r.log
  cmp <(grep -v '^##' w_0.vcf) <(grep -v '^##' w_$r.vcf) || exit 1
done
rm -rf $work
