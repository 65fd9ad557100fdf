#!/bin/bash
# A/B of runtime switches: bench.py under each "NAME=VAL ..." environment given, twice, alternating.
# Usage: scripts/ab_env.sh TAG "ENV1" "ENV2" ...   ("" = defaults)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; shift; mkdir -p "$OUT"
for rep in $(seq 1 ${REPS:-2}); do
  i=0
  for envs in "$@"; do
    i=$((i+1))
    env $envs timeout -k 10 300 python bench.py --config ${CFG:-1m_1080p_sh3} --no-cpu-baseline --no-census --steps 50 --warmup 5 > "$OUT/b${i}_$rep.json" 2> "$OUT/b${i}_$rep.err" || exit $?
    python -c "import json; d=json.load(open('$OUT/b${i}_$rep.json')); print('[$envs]', round(d['ms_per_step'],4), d.get('stage_ms'))"
  done
done
