#!/bin/bash
# Repeated short benches (alternating side-stream / same-stream zero fill): how often is a run slow?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
for r in 1 2 3 4 5 6; do
  for z in 1 2; do
    GSR_ZERO_FILL=$z timeout -k 10 300 python bench.py --no-cpu-baseline --no-census --steps 40 > "$OUT/b${z}_$r.json" 2> "$OUT/b${z}_$r.err" || exit $?
    python -c "import json; d=json.load(open('$OUT/b${z}_$r.json')); print('$r zero_fill=$z', round(d['ms_per_step'],4), round(d['roofline']['mean_launch_ms'],4))"
  done
done
