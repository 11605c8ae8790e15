# round-6 inflate probe: one-phase vs two-phase on the 5% configs[2] BAM
set -o pipefail
O=${O:-r06c}
OUT=$O tools/session.sh genome 0.05 -- probe 1 -- probe 0 GROM_INFLATE_TOKCAP=0 -- probe 0 -- probe 0 GROM_LZ_LANE=1 || exit 1
for t in 0 4096; do GROM_INFLATE_TOKCAP=$t PROBE_MAX=230000000 OUT=$O tools/session.sh probe 0 || exit 1; done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$O/ptrace -o p -- python3 $GRAFT_REPO_ROOT/tools/inflate_probe.py /tmp/gw/g.bam 0 0 > $GRAFT_REPO_ROOT/gpurun_out/$O/ptrace.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$O/ptrace2 -o p -- python3 $GRAFT_REPO_ROOT/tools/inflate_probe.py /tmp/gw/g.bam 230000000 0 > $GRAFT_REPO_ROOT/gpurun_out/$O/ptrace2.log 2>&1 || exit 1
