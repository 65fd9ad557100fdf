#!/bin/bash
# Repeated short benches under a kernel trace: is a slow run (~1.03 vs 0.82 ms/step) GPU-idle time or kernel time?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$1; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2 3 4 5; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/t$r" -o run -- \
     python3 "$ROOT/bench.py" --no-cpu-baseline --no-census --steps 40 > "$OUT/b$r.json" 2> "$OUT/b$r.err") || exit $?
  python -c "import json; d=json.load(open('$OUT/b$r.json')); print('$r', round(d['ms_per_step'],4))"
done
