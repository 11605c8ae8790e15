#!/bin/bash
# tools/cli_trace.sh -- the whole-run CLI leg's BAM (bench.py --cli-scale 0.04)
# through the CLI with the host event trace (GROM_TRACE) and, in a second run,
# under rocprofv3 with kernel and memory-copy traces: the evidence that decode,
# host->device copies and scans overlap.  Outputs under gpurun_out/cli_trace/.
set -e
out=gpurun_out/cli_trace
mkdir -p $out
cd $out
L=9958256,9687741,7931822,7608582,7261530,6832239,6373838,5805545,5535788,5351896,5403464,5331012,4574573,4281748,4079647,3613533,3330297,3214931,2344704,2577766,1868399,2032738,6241635,2289096
N=chr1,chr2,chr3,chr4,chr5,chr6,chr7,chr8,chr9,chr10,chr11,chr12,chr13,chr14,chr15,chr16,chr17,chr18,chr19,chr20,chr21,chr22,chrX,chrY
../../grom_amd/bin/grom_synth -o cli -L $L -n $N -s 3 -c 30.0 -l 150 -D 0.05 -X 0.7123660266165851 -V 1.6190136968558754e-07 -W 10000,1000000
export GROM_FILEDATE=20260101 GROM_SEED=7
timeout -k 10 120 ../../grom_amd/bin/grom -i cli.bam -r cli.fa -o warm.vcf -M > warm.out
( time GROM_VERBOSE=1 GROM_TRACE=trace.csv timeout -k 10 120 ../../grom_amd/bin/grom -i cli.bam -r cli.fa -o t.vcf -M > run.out ) 2> time.out
for n in 2 4; do ( time GROM_SCANS_PER_GPU=$n GROM_VERBOSE=1 timeout -k 10 120 ../../grom_amd/bin/grom -i cli.bam -r cli.fa -o s$n.vcf -M > s$n.out ) 2> s$n.time; done
grep -h "cli \|real" run.out time.out s*.out s*.time
cd /tmp && export TMPDIR=/tmp
cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d prof -o cli -- ../../grom_amd/bin/grom -i cli.bam -r cli.fa -o p.vcf -M > prof.out 2>&1
ls -R prof | head -20
rm -f cli.bam cli.fa *.vcf
