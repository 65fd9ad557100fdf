#!/bin/bash
# Kernel trace of a few bench steps under GSR_ environment settings, and whether the long-list sort kernels
# overlapped the per-tile sort.  Usage: scripts/trace_overlap.sh TAG CONFIG [NAME=VALUE ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=$1; CFG=$2; shift 2
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- \
   python3 "$ROOT/bench.py" --config "$CFG" --steps 5 --warmup 2 --no-cpu-baseline --no-census > "$OUT/trace.log" 2>&1) || exit 1
python3 - "$OUT/trace/run_kernel_trace.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = None
shown = 0
for i, r in enumerate(rows):
    n = r["Kernel_Name"]
    if "tile_sort_kernel" in n:
        last = r
    elif last is not None and ("tile_sort_window" in n or "tile_sort_class1" in n or "tile_sort_prefix" in n):
        s0, e0 = int(last["Start_Timestamp"]), int(last["End_Timestamp"])
        s1, e1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if shown < 12:
            print(f"{n.split('(')[0][-34:]:34s} start {(s1 - s0) / 1e3:8.2f} us after tile_sort start, tile_sort took "
                  f"{(e0 - s0) / 1e3:7.2f}, this {(e1 - s1) / 1e3:7.2f}; overlap {max(0, e0 - s1) / 1e3:7.2f} us")
            shown += 1
PY
