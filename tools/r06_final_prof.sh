# round-6 final profiles: the full genome, whole runs (default and without
# the explicit teardown), the kernel trace and the pileup's PMC passes
set -o pipefail
O=${O:-r06z}
OUT=$O tools/session.sh genome 1.0 -- whole 3 -- whole 2 GROM_CLI_PROCESS=1 -- trace \
  -- pmc fetch FETCH_SIZE -- pmc write WRITE_SIZE \
  -- pmc sq1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
