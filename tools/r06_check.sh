# round-6 check: the decode and merge GPU tests (the two-phase inflate
# forced on for a second pass), then a bench and a GROM_TIMING whole run
set -o pipefail
O=${O:-r06j}
OUT=$O tools/session.sh ksuite dec "inflate or device_decode or merge or workers_share" \
  -- ksuite dec2 "inflate or device_decode_matches" GROM_INFLATE_TOKCAP=4096 || exit 1
OUT=$O tools/session.sh bench --steps ${STEPS:-8} --warmup 2 || exit 1
