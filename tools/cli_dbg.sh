set -x
mkdir -p gpurun_out/dbg && cd gpurun_out/dbg
../../grom_amd/bin/grom_synth -o cli -L 9958256,9687741,7931822,7608582,7261530,6832239,6373838,5805545,5535788,5351896,5403464,5331012,4574573,4281748,4079647,3613533,3330297,3214931,2344704,2577766,1868399,2032738,6241635,2289096 -s 3 -c 30.0 -l 150 -D 0.05 -X 0.7123660266165851 -V 1.6190136968558754e-07 -W 10000,1000000 -n chr1,chr2,chr3,chr4,chr5,chr6,chr7,chr8,chr9,chr10,chr11,chr12,chr13,chr14,chr15,chr16,chr17,chr18,chr19,chr20,chr21,chr22,chrX,chrY
for i in 1 2 3; do
  GROM_VERBOSE=1 GROM_FILEDATE=20260101 GROM_SEED=7 timeout -k 10 120 ../../grom_amd/bin/grom -i cli.bam -r cli.fa -o out$i.vcf -M > run$i.out 2> run$i.err
  echo "run $i rc=$?"
  tail -4 run$i.out; tail -5 run$i.err
done
md5sum out*.vcf out*.ctx.vcf
rm -f cli.bam cli.fa
