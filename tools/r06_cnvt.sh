# a 10% genome, one CNV-counter run
set -o pipefail
O=${O:-r06n}
OUT=$O tools/session.sh genome ${SCALE:-0.1} -- whole 1 -- whole 1 GROM_TIMING=1
