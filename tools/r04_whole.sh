#!/bin/bash
# tools/r04_whole.sh OUT SCALE RUNS [pytest node ids...] -- on the gpurun box:
# optional GPU tests first, then a configs[2]-shape genome at SCALE of GRCh38's
# lengths written by grom_synth and RUNS whole-run CLI calls (the first one
# writes <fasta>.info), each timed, with the CLI's phase/decode lines; the
# runs' outputs must be identical.  ALT_ENV="K=V ...": the last run with
# that environment (e.g. a decode variant, checked against the others).  Everything goes to gpurun_out/OUT.
set -o pipefail
out=gpurun_out/$1
scale=$2
runs=$3
shift 3
mkdir -p $out
repo=$(pwd)
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 250 --timeout-method thread "$@" > $out/pytest.log 2>&1 \
    || { tail -40 $out/pytest.log; exit 1; }
  tail -3 $out/pytest.log
fi
work=/tmp/gw
mkdir -p $work
export GROM_FILEDATE=20260101 GROM_SEED=7
TIMEFORMAT='%R s wall, %U s user, %S s sys'
L=$(python3 -c "import bench; print(','.join(str(max(int(l*$scale),1000000)) for _,l in bench.GRCH38))")
N=$(python3 -c "import bench; print(','.join(n for n,_ in bench.GRCH38))")
SY="-s 3 -c 30.0 -l 150 -D 0.05 -X 0.7123660266165851 -V 1.6190136968558754e-07 -W 10000,1000000"
t0=$(date +%s.%N)
timeout -k 10 400 $repo/grom_amd/bin/grom_synth -o $work/g -L $L -n $N $SY > /dev/null || exit 1
echo "synth $(python3 -c "print(round($(date +%s.%N) - $t0, 1))") s, $(stat -c %s $work/g.bam) bytes"
cd $work
for r in $(seq 1 $runs); do
  alt=""; [ $r -eq $runs ] && [ -n "$ALT_ENV" ] && alt="$ALT_ENV" && echo "== run $r with $ALT_ENV"
  { time env $alt GROM_VERBOSE=1 GROM_TRACE=$repo/$out/trace_$r.csv timeout -k 10 120 $repo/grom_amd/bin/grom \
      -i g.bam -r g.fa -o w_$r.vcf -M -g 1 ${GROM_EXTRA_FLAGS} > $repo/$out/whole_$r.log 2>&1 ; } 2> $repo/$out/whole_$r.time \
      || { tail $repo/$out/whole_$r.log; exit 1; }
  echo "== run $r: $(cat $repo/$out/whole_$r.time)"
  grep -h "decode\|cli " $repo/$out/whole_$r.log
  [ $r -gt 1 ] && { cmp w_1.vcf w_$r.vcf && cmp w_1.ctx.vcf w_$r.ctx.vcf || exit 1; }
done
sha256sum w_1.vcf w_1.ctx.vcf | tee $repo/$out/sha.txt
echo "rows $(grep -vc '^#' w_1.vcf)"
rm -rf $work
