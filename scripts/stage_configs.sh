#!/bin/bash
# bench.py stage times (ms) on each synthetic configuration (no CPU baseline).
# Usage: scripts/stage_configs.sh TAG [configs...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; shift; mkdir -p "$OUT"
CFGS=${*:-"500k_1080p_sh3 1m_1080p_sh3 5m_4k_sh3"}
for c in $CFGS; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --config $c --steps 20 > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || exit $?
  python -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['ms_per_step'],4), '%.3g' % d['value'], d['stage_ms'])"
done
