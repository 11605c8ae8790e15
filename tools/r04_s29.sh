#!/bin/bash
# tools/r04_s29.sh OUT -- configs[2] genome; one warm whole run, then one
# under rocprofv3 --kernel-trace --stats (kernel summary in OUT)
set -o pipefail
out=gpurun_out/$1
mkdir -p $out
repo=$(pwd)
work=/tmp/g29
mkdir -p $work
export GROM_FILEDATE=20260101 GROM_SEED=7
L=$(python3 -c "import bench; print(','.join(str(l) for _,l in bench.GRCH38))")
N=$(python3 -c "import bench; print(','.join(n for n,_ in bench.GRCH38))")
SY="-s 3 -c 30.0 -l 150 -D 0.05 -X 0.7123660266165851 -V 1.6190136968558754e-07 -W 10000,1000000"
timeout -k 10 400 $repo/grom_amd/bin/grom_synth -o $work/g -L $L -n $N $SY > /dev/null || exit 1
echo "synth done"
cd $work
GROM_VERBOSE=1 timeout -k 10 120 $repo/grom_amd/bin/grom -i g.bam -r g.fa -o warm.vcf -M -g 1 > $repo/$out/warm.log 2>&1 || exit 1
grep -h "decode\|cli " $repo/$out/warm.log
cd /tmp && export TMPDIR=/tmp
GROM_EXIT_HANDLERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $repo/$out/prof -o run -- \
    $repo/grom_amd/bin/grom -i $work/g.bam -r $work/g.fa -o $work/p.vcf -M -g 1 > $repo/$out/prof_run.log 2>&1 || { tail $repo/$out/prof_run.log; exit 1; }
cd $repo
cmp $work/warm.vcf $work/p.vcf || exit 1
find $out/prof -name "*.csv" | head
db=$(find $out/prof -name "*.db" | head -1)
[ -n "$db" ] && timeout -k 10 200 python3 tools/kstats.py $db $out/kernel_stats.csv | head -45
find $out/prof -name "*kernel_stats.csv" -exec cp {} $out/rocprof_kernel_stats.csv \;
rm -rf $work $out/prof
