# bench A/B: the default and a variant (VARIANT: K=V list), STEPS each
set -o pipefail
O=${O:-r06v}
OUT=$O tools/session.sh bench --steps ${STEPS:-6} --warmup 1 --no-resident --no-cpu-baseline || exit 1
mv gpurun_out/$O/bench.json gpurun_out/$O/bench_default.json
env $VARIANT bash -c "OUT=$O tools/session.sh bench --steps ${STEPS:-6} --warmup 1 --no-resident --no-cpu-baseline" || exit 1
mv gpurun_out/$O/bench.json gpurun_out/$O/bench_variant.json
