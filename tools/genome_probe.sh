#!/bin/bash
# tools/genome_probe.sh -- on the gpurun box: the host's CPU share, the
# full configs[2] BAM (24 GRCh38 contigs, 3.09 Gb, 30x) written by grom_synth,
# the host decode alone at several thread counts (GROM_PLAN_ONLY +
# GROM_DECODE_ONLY: no GPU) and the whole-run CLI.  Outputs under
# gpurun_out/genome_probe/.
#   usage: tools/genome_probe.sh [decode thread counts, default "16 32 64"]
set -o pipefail
out=gpurun_out/genome_probe
mkdir -p $out
repo=$(pwd)
threads=${1:-"16 32 64"}
{
    echo "nproc $(nproc)"
    cat /sys/fs/cgroup/cpu.max 2>/dev/null | sed 's/^/cpu.max /'
    grep -c ^processor /proc/cpuinfo | sed 's/^/cpuinfo /'
    taskset -p $$ 2>/dev/null
    free -g
    df -h /tmp /dev/shm . 2>/dev/null
} > $out/env.txt 2>&1
cat $out/env.txt
work=${GENOME_DIR:-/tmp/genome_probe}
mkdir -p $work
L=248956422,242193529,198295559,190214555,181538259,170805979,159345973,145138636,138394717,133797422,135086622,133275309,114364328,107043718,101991189,90338345,83257441,80373285,58617616,64444167,46709983,50818468,156040895,57227415
N=chr1,chr2,chr3,chr4,chr5,chr6,chr7,chr8,chr9,chr10,chr11,chr12,chr13,chr14,chr15,chr16,chr17,chr18,chr19,chr20,chr21,chr22,chrX,chrY
TIMEFORMAT='%R s wall, %U s user, %S s sys'
t0=$(date +%s.%N)
timeout -k 10 400 $repo/grom_amd/bin/grom_synth -o $work/g -L $L -n $N -s 3 -c 30.0 -l 150 -D 0.05 \
    -X 0.7123660266165851 -V 1.6190136968558754e-07 -W 10000,1000000 || exit $?
t1=$(date +%s.%N)
echo "synth $(python3 -c "print(round($t1 - $t0, 1))") s, $(stat -c %s $work/g.bam) bytes" | tee $out/synth.txt
cd $work
export GROM_FILEDATE=20260101 GROM_SEED=7
cat g.bam > /dev/null
for t in $threads; do
    { time GROM_PLAN_ONLY=1 GROM_DECODE_ONLY=1 GROM_VERBOSE=1 GROM_DECODE_THREADS=$t \
        timeout -k 10 300 $repo/grom_amd/bin/grom -i g.bam -r g.fa -o dec$t.vcf -M > $repo/$out/decode_$t.log 2>&1 ; } 2> $repo/$out/decode_$t.time || exit $?
    echo "decode $t threads: $(cat $repo/$out/decode_$t.time)"
    grep -h "streamed decode" $repo/$out/decode_$t.log
done
for t in ${WHOLE_THREADS:-16}; do
    { time GROM_VERBOSE=1 GROM_DECODE_THREADS=$t GROM_TRACE=$repo/$out/trace_$t.csv \
        timeout -k 10 300 $repo/grom_amd/bin/grom -i g.bam -r g.fa -o whole$t.vcf -M > $repo/$out/whole_$t.log 2>&1 ; } 2> $repo/$out/whole_$t.time || exit $?
    echo "whole run $t threads: $(cat $repo/$out/whole_$t.time)"
    grep -h "streamed decode\|cli " $repo/$out/whole_$t.log
    grep -vc '^#' whole$t.vcf
done
rm -rf $work
