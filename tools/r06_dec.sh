# round-6 decode check: the decode GPU tests, then whole-run variants
set -o pipefail
O=${O:-r06u}
OUT=$O tools/session.sh ksuite dec "device_decode or inflate or oracle_digest_cases" || exit 1
O=$O bash tools/r06_whole.sh
