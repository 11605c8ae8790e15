#!/bin/bash
# tools/record_sv_hits.sh -- on the gpurun box: record svcall.cpp's inputs and
# rows from real GPU scans (GROM_SV_HITS_DUMP) of the "sv" parity case, VCF
# rows and -f tab rows, into gpurun_out/svh/ (gzipped).  The records become
# tests/golden/svh_*.svh.gz, which tests/test_sanitize.py replays under ASan
# and TSan (san_driver svrows).
set -o pipefail
out=gpurun_out/svh
mkdir -p $out
repo=$(pwd)
work=$(mktemp -d)
cd $work
$repo/grom_amd/bin/grom_synth -o sv -L 600000,300000 -s 31 -X 30 -I 0.0003 -J 0.3 -Q 0.05 || exit 1
export GROM_FILEDATE=20260101 GROM_SEED=7
GROM_SV_HITS_DUMP=vcf timeout -k 10 120 $repo/grom_amd/bin/grom -i sv.bam -r sv.fa -o v.vcf > /dev/null || exit 1
GROM_SV_HITS_DUMP=tab timeout -k 10 120 $repo/grom_amd/bin/grom -i sv.bam -r sv.fa -o t.txt -f > /dev/null || exit 1
for f in *.svh; do gzip -9 -c $f > $repo/$out/svh_$f.gz; done
ls -la $repo/$out
rm -rf $work
