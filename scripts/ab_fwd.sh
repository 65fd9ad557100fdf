#!/bin/bash
# A/B of the forward render variants: parity tests with each, bench stage times with each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
for v in quad tile; do
  GSR_RENDER_FWD=$v timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "not fullsize" > "$OUT/pytest_$v.log" 2>&1; rc=$?
  echo "$v tests rc=$rc: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
  GSR_RENDER_FWD=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err"; rc=$?
  python -c "import json; d=json.load(open('$OUT/bench_$v.json')); print('  $v', round(d['ms_per_step'],4), d['stage_ms'])"; [ $rc -eq 0 ] || exit $rc
done
for v in quad tile; do
  GSR_RENDER_FWD=$v GSR_LIBRARY=$PWD/gaussian_splatting_amd/lib/libgsr_stamps.so timeout -k 10 300 python tools/stamps.py > $OUT/stamps_$v.json 2>&1; rc=$?
  echo "stamps $v rc=$rc"; grep render_fwd $OUT/stamps_$v.json; [ $rc -eq 0 ] || exit $rc
done
