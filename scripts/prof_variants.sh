#!/bin/bash
# rocprof kernel stats for each variant library
set -u
cd "${GRAFT_REPO_ROOT}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$1; shift; mkdir -p $OUT
export TMPDIR=/tmp
for lib in "$@"; do
  v=$(basename $lib .so)
  (cd /tmp && GSR_LIBRARY=$ROOT/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$v" -o run -- \
     python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/$v.log" 2>&1) || exit 1
  echo "== $v"; python3 tools/kstats.py $OUT/$v/run_kernel_stats.csv | head -3
done
