#!/bin/bash
# tools/gpu_steps.sh -- run GPU steps on the gpurun box, each under its own time
# limit, logging to gpurun_out/<name>.log.  A step that fails normally (exit 1)
# is reported and the next step runs; a time-out, abort or signal ends the
# session at once (no further GPU work after a fault).
#   usage: tools/gpu_steps.sh name1 secs1 'cmd1' [name2 secs2 'cmd2' ...]
mkdir -p gpurun_out
status=0
while [ $# -ge 3 ]; do
    name=$1; secs=$2; cmd=$3; shift 3
    echo "== $name (limit ${secs}s): $cmd"
    start=$(date +%s)
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "== $name rc=$rc ($(( $(date +%s) - start ))s)"
    tail -n 5 "gpurun_out/$name.log"
    if [ $rc -ge 124 ]; then
        echo "FATAL: $name ended with $rc; stopping the session"
        exit $rc
    fi
    [ $rc -ne 0 ] && status=1
done
exit $status
