#!/bin/bash
# tools/varbench.sh -- on the gpurun box: the configs[1] bench with each kernel
# variant library (make variant V=... VFLAGS=...), one scan at a time; prints
# the pileup kernel's alone/mean launch time per variant.
set -o pipefail
for v in ${VARIANTS:-base}; do
  if [ $v = base ]; then lib=""; else lib=grom_amd/lib/variants/libgrom_amd_$v.so; fi
  GROM_AMD_LIB=$lib timeout -k 10 200 python bench.py --workload chrom --no-cpu-baseline --inflight 1 --steps 3 \
      --warmup 1 > gpurun_out/var_$v.log 2>&1 || exit $?
  echo $v $(grep -o '"launch_ms": [0-9.]*' gpurun_out/var_$v.log) $(grep -o '"launch_ms_mean": [0-9.]*' gpurun_out/var_$v.log) \
      $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/var_$v.log)
done
