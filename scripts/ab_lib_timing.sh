#!/bin/bash
# Timing-only A/B of side libraries whose results are deliberately wrong (no parity run):
# ROUNDS rounds of bench.py under the default library and each named libgsr_<v>.so.
# Usage: scripts/ab_lib_timing.sh TAG ROUNDS "v1 v2" [CONFIG]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$1; R=$2; CFG=${4:-1m_1080p_sh3}; mkdir -p "$OUT"
for r in $(seq 1 $R); do
  for v in default $3; do
    lib=$ROOT/gaussian_splatting_amd/lib/libgsr.so; [ "$v" = default ] || lib=$ROOT/gaussian_splatting_amd/lib/libgsr_$v.so
    GSR_LIBRARY=$lib timeout -k 10 300 python bench.py --config $CFG --no-cpu-baseline --no-census --steps 40 > "$OUT/t_${v}_$r.json" 2> "$OUT/t_${v}_$r.err" || exit $?
    python -c "import json; d=json.load(open('$OUT/t_${v}_$r.json')); s=d['stage_ms']; print('$r $v', round(d['ms_per_step'],4), ' '.join(f'{k}={x*1e3:.1f}' for k,x in s.items()))"
  done
done
