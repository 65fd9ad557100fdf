#!/bin/bash
# SQ counters of the forward render variants (one --pmc pass per counter group and variant).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$1; mkdir -p "$OUT"; export TMPDIR=/tmp
for v in quad tile; do
  i=0
  while read -r ctrs; do
    [ -z "$ctrs" ] && continue; i=$((i+1))
    (cd /tmp && GSR_RENDER_FWD=$v timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/$v/pmc$i" -o run -- \
       python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/$v.pmc$i.log" 2>&1); rc=$?
    echo "$v pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done < scripts/pmc_sq.txt
done
