#!/bin/bash
# tools/profile_round.sh TAG -- on the gpurun box: kernel-trace stats of the default
# bench and the two HBM PMC passes (FETCH_SIZE, WRITE_SIZE), each its own run and
# time limit, outputs under gpurun_out/prof_TAG/.  Copy the summaries to profiles/.
set -o pipefail
tag=${1:?tag}
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_trace.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c -d $out/pmc_$c -o run -- \
        python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --inflight 1 > $out/pmc_$c.log 2>&1 || exit $?
done
find $out -name "*.csv" | head -50
