#!/bin/bash
# rocprof kernel stats of bench.py on one synthetic config.  Usage: scripts/prof_config.sh TAG CONFIG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$1; mkdir -p "$OUT"; export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
   python3 "$ROOT/bench.py" --config "$2" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof.log" 2>&1) || exit 1
python3 tools/kstats.py "$OUT/prof/run_kernel_stats.csv" | head -20
