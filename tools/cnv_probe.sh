#!/bin/bash
# tools/cnv_probe.sh -- GPU probe of the CNV path: generate one synthetic
# genome, run the oracle and the product CLI on it, report timings and
# whether the VCFs are identical.  usage: tools/cnv_probe.sh <outdir> <grom args...> -- <synth args...>
set -u
out=$1; shift
gargs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do gargs+=("$1"); shift; done; shift
mkdir -p "$out"
./grom_amd/bin/grom_synth -o "$out/t" "$@" || exit 1
export GROM_FILEDATE=20260101 GROM_SEED=7
s=$(date +%s.%N)
(cd "$out" && ../../oracle/grom_oracle -i t.bam -r t.fa -o o.vcf "${gargs[@]}" > o.log 2>&1) || { echo "oracle failed"; exit 1; }
e=$(date +%s.%N); echo "oracle $(echo "$e - $s" | bc) s"
s=$(date +%s.%N)
(cd "$out" && GROM_TIMING=1 timeout -k 5 150 ../../grom_amd/bin/grom -i t.bam -r t.fa -o g.vcf "${gargs[@]}" > g.log 2>&1); rc=$?
e=$(date +%s.%N); echo "grom rc=$rc $(echo "$e - $s" | bc) s"
grep "timing\|cnv walk" "$out/g.log" | head -20
grep -c "<D" "$out/o.vcf"
cmp "$out/o.vcf" "$out/g.vcf" && echo IDENTICAL
exit $rc
