#!/bin/bash
# PMC passes of the pileup tile kernel (k_scan_tile) on the configs[1]-shape
# 100 Mb chromosome at 30x through the CLI: SQ occupancy / wait / instruction
# mix, LDS, and the HBM counters (FETCH_SIZE, WRITE_SIZE), one pass each
set -o pipefail
out=gpurun_out/s32
mkdir -p $out /tmp/p32
repo=$(pwd)
timeout -k 10 200 grom_amd/bin/grom_synth -o /tmp/p32/t -L 100000000 -s 3 -c 30.0 -l 150 -D 0.05 -X 0.7123660266165851 -V 1.6190136968558754e-07 -W 10000,1000000 > /dev/null || exit 1
cd /tmp/p32 && export GROM_FILEDATE=20260101 GROM_SEED=7
GROM_VERBOSE=1 timeout -k 10 120 $repo/grom_amd/bin/grom -i t.bam -r t.fa -o w.vcf -M -g 1 > $repo/$out/warm.log 2>&1 || exit 1
grep -h "pileup" $repo/$out/warm.log
cd /tmp && export TMPDIR=/tmp
export GROM_EXIT_HANDLERS=1
p=1
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 120 rocprofv3 --pmc $set -d $repo/$out/p$p -o run -- $repo/grom_amd/bin/grom -i /tmp/p32/t.bam -r /tmp/p32/t.fa -o /tmp/p32/p$p.vcf -M -g 1 > $repo/$out/p$p.log 2>&1 || { echo "pass $p failed"; tail -5 $repo/$out/p$p.log; exit 1; }
  db=$(find $repo/$out/p$p -name "*.db" | head -1)
  [ -n "$db" ] && python3 $repo/tools/pmc_summary.py $db $repo/$out/p$p.csv > /dev/null
  grep -h "scan_tile\|kernel,counter" $repo/$out/p$p.csv
  rm -rf $repo/$out/p$p
  p=$((p+1))
done
