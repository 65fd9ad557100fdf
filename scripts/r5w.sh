#!/bin/bash
# r5w: what the bench line's own machinery costs inside the timed region: the census pass before it, and the
# live HIP events around the dominant kernel (every 4th step by default) -- interleaved, 3 rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5w; mkdir -p $OUT
for r in 1 2 3; do
  i=0
  for flags in "" "--no-census" "--roofline-every 10" "--no-census --roofline-every 1000"; do
    i=$((i+1))
    timeout -k 10 300 python bench.py --no-cpu-baseline $flags > $OUT/b${i}_$r.json 2> $OUT/b${i}_$r.err || exit $?
    python -c "import json; d=json.load(open('$OUT/b${i}_$r.json')); print('[$flags]', round(d['ms_per_step'],4), d['roofline']['timed_launches'])"
  done
done
