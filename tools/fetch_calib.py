"""Ratios of rocprofv3's FETCH_SIZE / WRITE_SIZE to the known bytes of tools/fetch_calib.hip's kernels
(development tool; DESIGN.md section 4 "Counters").

    python tools/fetch_calib.py FETCH_DIR WRITE_DIR LOG [--json OUT]

FETCH_DIR / WRITE_DIR: the rocprofv3 output directories of the two --pmc passes; LOG: the program's
stdout (its "known ..." lines).  FETCH_SIZE and WRITE_SIZE are KiB per dispatch.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os


def counters(d, name):
    v = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name:
                k = r["Kernel_Name"].split("(")[0].strip()
                v[k].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(x) / len(x) for k, x in v.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("log")
    ap.add_argument("--json")
    a = ap.parse_args()
    known = {}
    for line in open(a.log):
        p = line.split()
        if p and p[0] == "known":
            known[p[1]] = {p[i]: float(p[i + 1]) for i in range(2, len(p), 2)}
    fetch, write = counters(a.fetch_dir, "FETCH_SIZE"), counters(a.write_dir, "WRITE_SIZE")
    out = {}
    print("| kernel | known read B | FETCH_SIZE B | known / FETCH | known write B | WRITE_SIZE B | known / WRITE |")
    print("|---|---|---|---|---|---|---|")
    for k, kn in known.items():
        f = next((v for n, v in fetch.items() if n.endswith(k)), None)
        w = next((v for n, v in write.items() if n.endswith(k)), None)
        rd = kn["read_table"] + kn["read_index"]
        row = {"known_read": rd, "fetch_size_bytes": f, "read_factor": rd / f if f else None,
               "known_write": kn["write"], "write_size_bytes": w,
               "write_factor": kn["write"] / w if w and kn["write"] else None}
        out[k] = row
        rf = f"{row['read_factor']:.3f}" if row["read_factor"] else "-"
        wf = f"{row['write_factor']:.3f}" if row["write_factor"] else "-"
        print(f"| {k} | {rd:.4g} | {f or 0:.4g} | {rf} | {kn['write']:.4g} | {w or 0:.4g} | {wf} |")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
