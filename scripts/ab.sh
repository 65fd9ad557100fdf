#!/bin/bash
# A/B of a runtime switch: parity tests (GPU, small) + bench stage times for each value.
# Usage: scripts/ab.sh TAG ENVVAR value1 value2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; VAR=$2; shift 2; mkdir -p "$OUT"
for v in "$@"; do
  env "$VAR=$v" timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "not fullsize" > "$OUT/pytest_$v.log" 2>&1; rc=$?
  echo "$VAR=$v tests rc=$rc: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
  env "$VAR=$v" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err"; rc=$?
  [ $rc -eq 0 ] || { tail -5 "$OUT/bench_$v.err"; exit $rc; }
  python -c "import json; d=json.load(open('$OUT/bench_$v.json')); print('  $v', round(d['ms_per_step'],4), d['stage_ms'])"
done
