#!/bin/bash
# the CLI under a Python parent with / without a torch GPU context (0.3-scale genome)
set -o pipefail
mkdir -p gpurun_out/parent /tmp/gq
L=$(python3 -c "import bench; print(','.join(str(max(int(l*1.0),1000000)) for _,l in bench.GRCH38))")
N=$(python3 -c "import bench; print(','.join(n for n,_ in bench.GRCH38))")
timeout -k 10 300 grom_amd/bin/grom_synth -o /tmp/gq/g -L $L -n $N -s 3 -c 30.0 -l 150 -D 0.05 -X 0.71 -V 1.6e-07 -W 10000,1000000 > /dev/null || exit 1
for m in plain cuda; do
  timeout -k 10 200 python tools/r04_parent.py /tmp/gq/g.bam /tmp/gq/g.fa $m 2>&1 | tee -a gpurun_out/parent/log.txt || exit 1
done
