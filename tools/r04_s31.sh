#!/bin/bash
# CNV classify A/B on one 150 Mb configs[2]-shape chromosome: GROM_CNV_CLS
# 1 (per-wave queue) / 0 (lane per candidate), alternating, outputs compared
set -o pipefail
mkdir -p gpurun_out/s31 /tmp/ct
timeout -k 10 200 grom_amd/bin/grom_synth -o /tmp/ct/t -L 150000000 -s 3 -c 30.0 -l 150 -D 0.05 -X 0.7123660266165851 -V 1.6190136968558754e-07 -W 10000,1000000 > /dev/null || exit 1
cd /tmp/ct && export GROM_FILEDATE=20260101 GROM_SEED=7
GROM_VERBOSE=1 timeout -k 10 120 $GRAFT_REPO_ROOT/grom_amd/bin/grom -i t.bam -r t.fa -o w.vcf -M -g 1 > /dev/null 2>&1 || exit 1
for r in 1 2 3 4 5 6; do
  q=$(( r % 2 ))
  GROM_CNV_CLS=$q GROM_TIMING=1 GROM_VERBOSE=1 timeout -k 10 120 $GRAFT_REPO_ROOT/grom_amd/bin/grom -i t.bam -r t.fa -o g$r.vcf -M -g 1 > $GRAFT_REPO_ROOT/gpurun_out/s31/run$r.log 2>&1 || exit 1
  echo "run $r queue=$q: $(grep -h 'cnv phases' $GRAFT_REPO_ROOT/gpurun_out/s31/run$r.log) | $(grep -ho 'cnv [0-9.]* ms (device [0-9.]* ms' $GRAFT_REPO_ROOT/gpurun_out/s31/run$r.log)"
  cmp <(grep -v '^##' g1.vcf) <(grep -v '^##' g$r.vcf) || exit 1
done
