#!/bin/bash
# CNV path timing counters (GROM_TIMING) on one 150 Mb configs[2]-shape chromosome
set -o pipefail
mkdir -p gpurun_out/cnvt /tmp/ct
timeout -k 10 200 grom_amd/bin/grom_synth -o /tmp/ct/t -L 150000000 -s 3 -c 30.0 -l 150 -D 0.05 -X 0.7123660266165851 -V 1.6190136968558754e-07 -W 10000,1000000 > /dev/null || exit 1
cd /tmp/ct && export GROM_FILEDATE=20260101 GROM_SEED=7
for r in 1 2; do
  GROM_TIMING=1 GROM_VERBOSE=1 timeout -k 10 120 $GRAFT_REPO_ROOT/grom_amd/bin/grom -i t.bam -r t.fa -o g.vcf -M -g 1 > $GRAFT_REPO_ROOT/gpurun_out/cnvt/run$r.log 2>&1 || exit 1
done
grep -i "cnv\|timing\|chr" $GRAFT_REPO_ROOT/gpurun_out/cnvt/run2.log | head -60
