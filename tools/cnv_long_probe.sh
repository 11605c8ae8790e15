#!/bin/bash
# tools/cnv_long_probe.sh LEN SECS [trace] -- on the gpurun box: one chromosome
# with configs[2]-style copy-number regions through the CLI with GROM_TIMING,
# to time the CNV window search (walk counters on stderr); with "trace", a
# second run without GROM_TIMING under rocprofv3 --kernel-trace --stats.
# GROM_PROBE_LIBS="name=dir ...": also run the CLI with each variant library
# directory first on LD_LIBRARY_PATH.  Data stays in /tmp (not merged back).
set -o pipefail
d=gpurun_out/cnvprobe
mkdir -p $d
t=/tmp/cnvprobe
mkdir -p $t
grom_amd/bin/grom_synth -o $t/g -L ${1:-12000000} -s 3 -D 0.05 -X 0.7 -V 1.6e-7 -W 10000,1000000 || exit $?
GROM_TIMING=1 timeout -k 10 ${2:-300} grom_amd/bin/grom -i $t/g.bam -r $t/g.fa -o $t/g.vcf -M > $d/run.log 2>&1 || exit $?
grep -E "cnv walk|cnv phases|cnv classify|grom timing" $d/run.log | cut -c1-400
for v in $GROM_PROBE_LIBS; do
    n=${v%%=*}; dir=${v#*=}
    LD_LIBRARY_PATH=$dir:$LD_LIBRARY_PATH GROM_TIMING=1 timeout -k 10 ${2:-300} grom_amd/bin/grom -i $t/g.bam -r $t/g.fa -o $t/g_$n.vcf -M > $d/run_$n.log 2>&1 || exit $?
    echo "== variant $n"; grep -E "cycles|longest|cnv phases" $d/run_$n.log | cut -c1-400
    cmp $t/g.vcf $t/g_$n.vcf && echo "variant $n: same VCF"
done
if [ "$3" = trace ]; then
    cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
    timeout -k 10 ${2:-300} rocprofv3 --kernel-trace --stats -d $d/trace -o run -- \
        grom_amd/bin/grom -i $t/g.bam -r $t/g.fa -o $t/g.vcf -M > $d/trace.log 2>&1 || exit $?
    for v in $GROM_PROBE_LIBS; do
        n=${v%%=*}; dir=${v#*=}
        LD_LIBRARY_PATH=$dir:$LD_LIBRARY_PATH timeout -k 10 ${2:-300} rocprofv3 --kernel-trace --stats -d $d/trace_$n -o run -- \
            grom_amd/bin/grom -i $t/g.bam -r $t/g.fa -o $t/g.vcf -M > $d/trace_$n.log 2>&1 || exit $?
    done
fi
exit 0
