"""Summarise tools/launch_floor's rocprofv3 kernel trace: mean / median duration per kernel and grid.

usage: python tools/launch_floor_summary.py <dir holding *kernel_trace.csv>
"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def main(root):
    paths = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)
    if not paths:
        raise SystemExit(f"no kernel_trace.csv under {root}")
    dur = defaultdict(list)
    for p in paths:
        with open(p, newline="") as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"]
                if "floor" not in name:
                    continue
                grid = int(row.get("Grid_Size_X") or row.get("Grid_Size") or 0)
                wg = int(row.get("Workgroup_Size_X") or row.get("Workgroup_Size") or 0)
                lds = row.get("LDS_Block_Size") or row.get("Lds_Size") or "?"
                d = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                dur[(name.split("(")[0], grid // max(wg, 1), wg, lds)].append(d)
    print(f"{'kernel':<32} {'wgs':>6} {'wg':>4} {'lds':>7} {'n':>4} {'mean us':>8} {'median us':>9}")
    for k in sorted(dur, key=lambda k: (k[0], k[1])):
        v = dur[k][10:] or dur[k]  # drop the first launches (clock ramp)
        print(f"{k[0]:<32} {k[1]:>6} {k[2]:>4} {k[3]:>7} {len(v):>4} {statistics.mean(v) / 1e3:>8.2f} "
              f"{statistics.median(v) / 1e3:>9.2f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/launch_floor")
