"""Print one step's kernel timeline from a rocprofv3 kernel trace (development tool).

    python tools/trace_step.py gpurun_out/<tag>/prof/run_kernel_trace.csv [--step -2]
"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--step", type=int, default=-2, help="which preprocess-to-preprocess window (python index)")
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "preprocess" in r["Kernel_Name"]]
seq = rows[idx[a.step]:idx[a.step + 1]] if a.step + 1 < len(idx) and a.step + 1 != 0 else rows[idx[a.step]:]
t0 = int(seq[0]["Start_Timestamp"])
prev_end, busy = t0, 0
for r in seq:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    print(f"{(s - t0) / 1e3:8.1f} gap {(s - prev_end) / 1e3:6.1f}  {(e - s) / 1e3:7.1f} us  {r['Kernel_Name'][:90]}")
    prev_end = e
print(f"window {(prev_end - t0) / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us")
