# round-6 whole-run session on the full configs[2] genome: runs under
# several settings (K=V lists separated by ';' in $VARIANTS), then a trace
set -o pipefail
O=${O:-r06e}
args=(genome 1.0 -- whole 2)
IFS=';' read -ra vs <<< "${VARIANTS:-}"
for v in "${vs[@]}"; do args+=(-- whole 1 $v); done
[ -n "$TRACE" ] && args+=(-- trace $TRACE)
OUT=$O tools/session.sh "${args[@]}"
