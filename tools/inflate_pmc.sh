#!/bin/bash
# PMC counters of the GPU inflater (k_inflate) on a 2%-scale configs[2] BAM
set -o pipefail
mkdir -p gpurun_out/ipmc /tmp/ipmc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
L=$(python3 -c "import bench; print(','.join(str(max(int(l*0.02),1000000)) for _,l in bench.GRCH38))")
N=$(python3 -c "import bench; print(','.join(n for n,_ in bench.GRCH38))")
timeout -k 10 200 grom_amd/bin/grom_synth -o /tmp/ipmc/g -L $L -n $N -s 3 -c 30.0 -l 150 -D 0.05 -X 0.71 -V 1.6e-07 -W 10000,1000000 || exit 1
timeout -k 10 60 rocprofv3 -L > gpurun_out/ipmc/avail.txt 2>&1
grep -o "SQ_INSTS_[A-Z_]*\|SQ_WAIT[A-Z_]*\|TA_[A-Z_]*BUSY[A-Z_]*\|SQ_ACTIVE_INST_[A-Z]*\|SQ_INST_CYCLES_[A-Z_]*\|TCP_TOTAL[A-Z_]*" gpurun_out/ipmc/avail.txt | sort -u > gpurun_out/ipmc/names.txt
timeout -k 10 120 python tools/inflate_probe.py /tmp/ipmc/g.bam 0 0 > gpurun_out/ipmc/probe.json || exit 1
cat gpurun_out/ipmc/probe.json
p=1
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_ANY"; do
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/ipmc/p$p -o run -- python3 tools/inflate_probe.py /tmp/ipmc/g.bam 0 0 > gpurun_out/ipmc/p$p.log 2>&1 || { echo "pass $p failed"; tail -5 gpurun_out/ipmc/p$p.log; }
  db=$(find gpurun_out/ipmc/p$p -name "*.db" | head -1)
  [ -n "$db" ] && python3 tools/pmc_summary.py $db gpurun_out/ipmc/p$p.csv | grep -i inflate
  p=$((p+1))
done
