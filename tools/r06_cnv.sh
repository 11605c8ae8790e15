# round-6 CNV check: the CNV GPU tests and the oracle digests, then whole
# runs (one with the CNV counters, GROM_TIMING) and optionally a trace
set -o pipefail
O=${O:-r06l}
OUT=$O tools/session.sh ksuite cnv "cnv or oracle_digest" || exit 1
args=(genome 1.0 -- whole 2 -- whole 1 GROM_TIMING=1)
[ -n "$TRACE" ] && args+=(-- trace $TRACE)
OUT=$O tools/session.sh "${args[@]}"
