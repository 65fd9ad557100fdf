#!/bin/bash
# PMC counter passes (each pass its own rocprofv3 run, --pmc only; no tracing domains).
# Usage: scripts/pmc_session.sh TAG COUNTER_LIST_FILE [CONFIG]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=$1; CFG=${3:-1m_1080p_sh3}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
while read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/pmc$i" -o run -- \
     python3 "$ROOT/bench.py" --config "$CFG" --steps 3 --warmup 1 --no-cpu-baseline --no-census > "$OUT/pmc$i.log" 2>&1); rc=$?
  echo "pass $i ($ctrs) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done < "$2"
