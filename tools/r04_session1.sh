#!/bin/bash
# round-4 GPU session 1: new parity tests, SV-hit records for the sanitizer
# replay, a quick bench of the whole-run headline at 5% scale, the GPU
# inflater's throughput on that BAM
set -o pipefail
mkdir -p gpurun_out
T="tests/test_gpu_parity.py"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "$T::test_device_inflate_matches_zlib" \
  "$T::test_amplicon_depth_tiles" "$T::test_late_fallback_to_serial_reader" "$T::test_integration_stub" \
  "$T::test_rank_shares_merge_to_one_run" \
  "$T::test_counters_and_vcf_bit_exact[one_chr-p60]" "$T::test_counters_and_vcf_bit_exact[lowmapq_clip-q-1]" \
  "$T::test_cnv_rows_bit_exact[cnv-V1-p60]" "$T::test_sharded_cli_matches_one_gpu" \
  > gpurun_out/s1_pytest.log 2>&1 || { tail -60 gpurun_out/s1_pytest.log; exit 1; }
tail -15 gpurun_out/s1_pytest.log
timeout -k 10 300 tools/record_sv_hits.sh > gpurun_out/s1_svh.log 2>&1 || { cat gpurun_out/s1_svh.log; exit 1; }
timeout -k 10 400 python bench.py --scale 0.05 --steps 2 --warmup 1 --workdir /tmp/r04bench > gpurun_out/s1_bench.json \
  2> gpurun_out/s1_bench.err || { tail -30 gpurun_out/s1_bench.err; exit 1; }
cat gpurun_out/s1_bench.json
timeout -k 10 300 python tools/inflate_probe.py /tmp/r04bench/genome.bam 0 0 > gpurun_out/s1_inflate.json && \
timeout -k 10 300 python tools/inflate_probe.py /tmp/r04bench/genome.bam 3e8 1 >> gpurun_out/s1_inflate.json
cat gpurun_out/s1_inflate.json
