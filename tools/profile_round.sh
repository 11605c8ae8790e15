#!/bin/bash
# tools/profile_round.sh TAG [bench args] -- on the gpurun box: kernel-trace
# stats of the default bench (one timed pass), then the two HBM PMC passes
# (FETCH_SIZE, WRITE_SIZE) with one scan in flight, each its own run and time
# limit; outputs under gpurun_out/prof_TAG/.  Summaries are copied to
# profiles/ by hand (tools/kstats.py, tools/pmc_summary.py).
set -o pipefail
tag=${1:?tag}
shift
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $out/trace -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > $out/bench_trace.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 420 rocprofv3 --pmc $c -d $out/pmc_$c -o run -- \
        python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --inflight 1 "$@" > $out/pmc_$c.log 2>&1 || exit $?
done
ls $out
