#!/bin/bash
# bench.py on each synthetic configuration (no CPU baseline), one JSON line per config.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
for c in 10k_256_sh0 500k_1080p_sh3 1m_1080p_sh3 5m_4k_sh3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --config $c --steps 20 > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || exit $?
  python -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['ms_per_step'],4), '%.3g' % d['value'])"
done
