#!/bin/bash
# rocprof kernel stats of bench.py for each value of a runtime switch.
# Usage: scripts/prof_env.sh TAG ENVVAR value1 value2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$1; VAR=$2; shift 2; mkdir -p "$OUT"; export TMPDIR=/tmp
for v in "$@"; do
  (cd /tmp && env "$VAR=$v" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$v" -o run -- \
     python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/$v.log" 2>&1) || exit 1
  echo "== $VAR=$v"; python3 tools/kstats.py "$OUT/$v/run_kernel_stats.csv" | head -4
done
