#!/bin/bash
# tools/session.sh -- the GPU-box session steps, one script (replaces the
# round-4 one-off scripts).  Run as a chain of steps on one gpurun box; each
# step has its own time limit and a failing step ends the chain:
#
#   tools/session.sh STEP [args] [-- STEP [args] ...]
#
# steps (outputs under gpurun_out/$OUT, OUT defaults to "s"):
#   suite [pytest args]        the GPU suite in one pytest process
#   ksuite TAG K [K=V ...]     the GPU tests matching K under the environment K=V
#   genome SCALE               a configs[2]-shape genome at SCALE of GRCh38's
#                              lengths (grom_synth) in /tmp/gw (kept for the
#                              following steps of this call)
#   whole RUNS [K=V ...]       RUNS whole-run CLI calls on /tmp/gw (the first
#                              writes <fasta>.info); outputs compared run to run
#   trace [K=V ...]            one whole run under rocprofv3 --kernel-trace
#                              --stats; per-kernel summary kernel_stats.csv
#   pmc NAME "CTRS" [K=V ...]  one rocprofv3 --pmc pass (CTRS: one pass's
#                              counters) over a whole run; NAME.csv per kernel
#   bench [bench args]         python bench.py ... > bench.json
#   share CHROMS RUNS          a multi-GPU rank's share: the plan-only run that
#                              writes <bam>.mean, then RUNS runs over the
#                              chromosomes CHROMS (GROM_CHROMS, as bench.py's ranks)
#   probe CHECK [K=V ...]      the GPU inflater alone on /tmp/gw/g.bam
#                              (tools/inflate_probe.py; CHECK=1: against zlib;
#                              PROBE_MAX: a prefix of that many compressed bytes)
#
# environment: OUT (subdirectory of gpurun_out), FLAGS (CLI flags, default
# "-M -g 1"), SYNTH (extra grom_synth args, e.g. coverage for configs[4]).
set -o pipefail
repo=$(pwd)
out=gpurun_out/${OUT:-s}
mkdir -p $out
work=/tmp/gw
export GROM_FILEDATE=20260101 GROM_SEED=7
FLAGS=${FLAGS:-"-M -g 1"}
TIMEFORMAT='%R s wall, %U s user, %S s sys'

step_suite() {
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
      > $out/gputest.log 2>&1 || { tail -40 $out/gputest.log; return 1; }
  tail -3 $out/gputest.log
}

# the GPU suite's tests matching K under an environment (TAG names the log)
step_ksuite() {
  local tag=$1 k=$2; shift 2
  env "$@" timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$k" \
      > $out/gputest_$tag.log 2>&1
  local rc=$?
  tail -1 $out/gputest_$tag.log
  # (a failed assertion goes on to the next step; a crash or time limit ends the chain)
  [ $rc -ge 2 ] && return $rc
  return 0
}

step_genome() {
  local scale=$1
  mkdir -p $work
  local L N
  L=$(python3 -c "import bench; print(','.join(str(max(int(l*$scale),1000000)) for _,l in bench.GRCH38))")
  N=$(python3 -c "import bench; print(','.join(n for n,_ in bench.GRCH38))")
  local SY=${SYNTH:-"-s 3 -c 30.0 -l 150 -D 0.05 -X 0.7123660266165851 -V 1.6190136968558754e-07 -W 10000,1000000"}
  local t0=$(date +%s.%N)
  timeout -k 10 600 $repo/grom_amd/bin/grom_synth -o $work/g -L ${GLEN:-$L} -n ${GNAMES:-$N} $SY > /dev/null || return 1
  echo "synth $(python3 -c "print(round($(date +%s.%N) - $t0, 1))") s, $(stat -c %s $work/g.bam) bytes"
}

WN=0
step_whole() {
  local runs=$1; shift
  WN=$((WN + 1))
  local pre=""
  [ $WN -gt 1 ] && pre="w${WN}_"
  ( cd $work
    for r0 in $(seq 1 $runs); do
      r="${pre}${r0}"
      { time env "$@" GROM_VERBOSE=1 GROM_TRACE=$repo/$out/trace_$r.csv timeout -k 10 180 $repo/grom_amd/bin/grom -i g.bam -r g.fa -o w_$r.vcf $FLAGS \
          > $repo/$out/whole_$r.log 2>&1 ; } 2> $repo/$out/whole_$r.time || { tail $repo/$out/whole_$r.log; exit 1; }
      echo "== run $r: $(cat $repo/$out/whole_$r.time)"
      grep -h "decode:\|cli \|footprint\|took" $repo/$out/whole_$r.log
      if [ "$r" != "1" ]; then cmp w_1.vcf w_$r.vcf && cmp w_1.ctx.vcf w_$r.ctx.vcf || exit 1; fi
    done
    sha256sum w_1.vcf w_1.ctx.vcf | tee $repo/$out/sha.txt
    echo "rows sha256 vcf $(grep -v '^#' w_1.vcf | sha256sum | cut -c1-64) ctx $(grep -v '^#' w_1.ctx.vcf | sha256sum | cut -c1-64)" \
        | tee -a $repo/$out/sha.txt
    echo "rows $(grep -vc '^#' w_1.vcf)" )
}

step_trace() {
  ( cd /tmp && export TMPDIR=/tmp
    env "$@" GROM_EXIT_HANDLERS=1 GROM_VERBOSE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $repo/$out/trace -o run -- \
        $repo/grom_amd/bin/grom -i $work/g.bam -r $work/g.fa -o $work/t.vcf $FLAGS > $repo/$out/trace_run.log 2>&1 \
        || { tail $repo/$out/trace_run.log; exit 1; } )
  local db
  db=$(find $out/trace -name "*.db" | head -1)
  python3 tools/kstats.py $db $out/kernel_stats.csv $out/launches.csv | head -30
  find $out/trace -name "*kernel_stats.csv" -exec cp {} $out/rocprof_kernel_stats.csv \;
  rm -rf $out/trace
}

step_pmc() {
  local name=$1 ctrs=$2; shift 2
  ( cd /tmp && export TMPDIR=/tmp
    env "$@" GROM_EXIT_HANDLERS=1 timeout -s KILL 180 rocprofv3 --pmc $ctrs -d $repo/$out/pmc_$name -o run -- \
        $repo/grom_amd/bin/grom -i $work/g.bam -r $work/g.fa -o $work/p.vcf $FLAGS > $repo/$out/pmc_$name.log 2>&1 \
        || { echo "pmc pass $name failed"; tail -5 $repo/$out/pmc_$name.log; exit 1; } )
  local db
  db=$(find $out/pmc_$name -name "*.db" | head -1)
  [ -n "$db" ] && python3 tools/pmc_summary.py $db $out/pmc_$name.csv | head -12
  rm -rf $out/pmc_$name
}

step_share() {
  local chroms=$1 runs=$2
  ( cd $work
    GROM_PLAN_ONLY=1 GROM_CHROMS=- timeout -k 10 300 $repo/grom_amd/bin/grom -i g.bam -r g.fa -o prewarm.vcf $FLAGS \
        > $repo/$out/share_prewarm.log 2>&1 || { tail $repo/$out/share_prewarm.log; exit 1; }
    for r in $(seq 1 $runs); do
      { time env GROM_CHROMS=$chroms GROM_VERBOSE=1 timeout -k 10 300 $repo/grom_amd/bin/grom -i g.bam -r g.fa -o s_$r.vcf $FLAGS \
          > $repo/$out/share_$r.log 2>&1 ; } 2> $repo/$out/share_$r.time || { tail $repo/$out/share_$r.log; exit 1; }
      echo "== share run $r: $(cat $repo/$out/share_$r.time)"
      grep -h "decode:\|cli \|footprint\|took\|Loading" $repo/$out/share_$r.log
    done
    echo "rows $(grep -vc '^#' s_1.vcf)" )
}

step_probe() {
  local check=$1; shift
  env "$@" timeout -k 10 300 python3 tools/inflate_probe.py $work/g.bam ${PROBE_MAX:-0} $check | tee -a $out/probe.jsonl
}

step_bench() {
  timeout -k 10 1100 python -u bench.py "$@" > $out/bench.json 2> $out/bench_stderr.log \
      || { tail -20 $out/bench_stderr.log; return 1; }
  cat $out/bench.json
}

while [ $# -gt 0 ]; do
  name=$1; shift
  args=()
  while [ $# -gt 0 ] && [ "$1" != "--" ]; do args+=("$1"); shift; done
  [ "$1" == "--" ] && shift
  echo "== $name ${args[*]}"
  start=$(date +%s)
  step_$name "${args[@]}"
  rc=$?
  echo "== $name rc=$rc ($(( $(date +%s) - start )) s)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
