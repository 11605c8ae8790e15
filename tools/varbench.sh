set -o pipefail
for v in ${VARIANTS:-base}; do
  if [ $v = base ]; then lib=""; else lib=grom_amd/lib/variants/libgrom_amd_$v.so; fi
  GROM_AMD_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/var_$v.log 2>&1 || exit $?
  echo $v $(grep -o '"launch_ms": [0-9.]*' gpurun_out/var_$v.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/var_$v.log)
done
