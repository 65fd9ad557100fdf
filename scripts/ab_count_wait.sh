#!/bin/bash
# Interleaved A/B of the forward's count wait (the "count_wait" option, GSR_COUNT_WAIT): ROUNDS rounds of
# (blocking wait, polling wait) default bench runs, as the driver runs them (--steps 20 --warmup 5); each
# line: ms/step and the run's slow steps (index, wall, forward call, backward call ms).
# Usage: scripts/ab_count_wait.sh TAG ROUNDS
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; R=${2:-8}; mkdir -p "$OUT"
for r in $(seq 1 $R); do
  for w in 0 1; do
    GSR_COUNT_WAIT=$w timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-census > "$OUT/bench_w${w}_$r.json" 2> "$OUT/bench_w${w}_$r.err"; rc=$?
    [ $rc -eq 0 ] || { tail -3 "$OUT/bench_w${w}_$r.err"; exit $rc; }
    python -c "import json; d=json.load(open('$OUT/bench_w${w}_$r.json')); h=d['host']; print('$r wait=$w', round(d['ms_per_step'],4), 'count_wait max', h['lib_count_wait_ms']['max'], 'slow', h.get('slow_steps'))"
  done
done
