#!/bin/bash
# tools/r04_prof.sh OUT SCALE -- a configs[2]-shape genome at SCALE through the
# whole-run CLI under rocprofv3 --kernel-trace --memory-copy-trace --stats
# (one warm run first, which writes <fasta>.info); kernel summary in OUT
set -o pipefail
out=gpurun_out/$1
scale=$2
mkdir -p $out
repo=$(pwd)
work=/tmp/gp
mkdir -p $work
export GROM_FILEDATE=20260101 GROM_SEED=7
L=$(python3 -c "import bench; print(','.join(str(max(int(l*$scale),1000000)) for _,l in bench.GRCH38))")
N=$(python3 -c "import bench; print(','.join(n for n,_ in bench.GRCH38))")
SY="-s 3 -c 30.0 -l 150 -D 0.05 -X 0.7123660266165851 -V 1.6190136968558754e-07 -W 10000,1000000"
timeout -k 10 400 $repo/grom_amd/bin/grom_synth -o $work/g -L $L -n $N $SY > /dev/null || exit 1
cd $work
GROM_VERBOSE=1 timeout -k 10 120 $repo/grom_amd/bin/grom -i g.bam -r g.fa -o warm.vcf -M -g 1 > $repo/$out/warm.log 2>&1 || exit 1
grep -h "decode\|cli " $repo/$out/warm.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $repo/$out/prof -o run -- \
    $repo/grom_amd/bin/grom -i $work/g.bam -r $work/g.fa -o $work/p.vcf -M -g 1 > $repo/$out/prof_run.log 2>&1 || { tail $repo/$out/prof_run.log; exit 1; }
cd $repo
db=$(find $out/prof -name "*.db" | head -1)
python3 tools/kstats.py $db $out/kernel_stats.csv | head -40
rm -rf $work
