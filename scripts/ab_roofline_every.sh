#!/bin/bash
# A/B of bench.py --roofline-every (how often the timed region records the dominant kernel's event pair).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
for r in 1 2 3; do
  for e in 1 4 20; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-census --steps 40 --roofline-every $e > "$OUT/b${e}_$r.json" 2> "$OUT/b${e}_$r.err" || exit $?
    python -c "import json; d=json.load(open('$OUT/b${e}_$r.json')); rf=d['roofline']; print('$r every=$e', round(d['ms_per_step'],4), 'render_bwd', round(rf['mean_launch_ms'],4), rf['timed_launches'])"
  done
done
