#!/bin/bash
# tools/cnv_long_probe.sh LEN SECS [trace] -- on the gpurun box: one chromosome
# with configs[2]-style copy-number regions through the CLI with GROM_TIMING,
# to time the CNV window search (walk counters on stderr); with "trace", under
# rocprofv3 --kernel-trace --stats.  Data stays in /tmp (not merged back).
set -o pipefail
d=gpurun_out/cnvprobe
mkdir -p $d
t=/tmp/cnvprobe
mkdir -p $t
grom_amd/bin/grom_synth -o $t/g -L ${1:-12000000} -s 3 -D 0.05 -X 0.7 -V 1.6e-7 -W 10000,1000000 || exit $?
if [ "$3" = trace ]; then
    cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
    GROM_TIMING=1 timeout -k 10 ${2:-300} rocprofv3 --kernel-trace --stats -d $d/trace -o run -- \
        grom_amd/bin/grom -i $t/g.bam -r $t/g.fa -o $t/g.vcf -M > $d/run.log 2>&1
else
    GROM_TIMING=1 timeout -k 10 ${2:-300} grom_amd/bin/grom -i $t/g.bam -r $t/g.fa -o $t/g.vcf -M > $d/run.log 2>&1
fi
rc=$?
grep -E "cnv walk|cnv phases|grom timing" $d/run.log | cut -c1-400
exit $rc
