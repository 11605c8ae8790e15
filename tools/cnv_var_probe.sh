#!/bin/bash
# tools/cnv_var_probe.sh LIB... -- on the gpurun box: the 12 Mb configs[2]-style
# CNV probe chromosome through the CLI in-process with each library build
# (GROM_AMD_LIB), GROM_TIMING on; prints the CNV phase line per build.
set -o pipefail
t=/tmp/cnvprobe
mkdir -p $t gpurun_out
[ -f $t/g.bam ] || grom_amd/bin/grom_synth -o $t/g -L 12000000 -s 3 -D 0.05 -X 0.7 -V 1.6e-7 -W 10000,1000000 || exit $?
for lib in "$@"; do
  GROM_TIMING=1 GROM_AMD_LIB=$lib timeout -k 10 120 python3 -c "
import grom_amd, sys
sys.exit(grom_amd.cli_main(['-i', '$t/g.bam', '-r', '$t/g.fa', '-o', '$t/g.vcf', '-M']))" > gpurun_out/varprobe.log 2>&1 || exit $?
  echo "$lib: $(grep 'cnv phases' gpurun_out/varprobe.log)"
done
