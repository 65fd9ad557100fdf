"""Summarise rocprofv3 --pmc passes (scripts/pmc_session.sh) per kernel: mean counter value per
dispatch, plus derived figures.  Development tool.

    python tools/pmc_summary.py gpurun_out/<tag> [--out profiles/r01/pmc_<tag>.md]

HBM bytes: FETCH_SIZE / WRITE_SIZE are in KiB.  MI355X_MICROARCH.md measured FETCH_SIZE at half the
bytes of a wide coalesced streaming read (16 B per lane); tools/fetch_calib.hip calibrated the other shapes
on the MI355X (profiles/r05/r5a/fetch_calib.md): a per-lane gather of a 64-byte record, of 48 bytes of one
or of 4 bytes of one is counted as one whole 64-byte line, exactly (known / FETCH = 1.03 for whole
records, the 0.03 being the coalesced index stream at half), and WRITE_SIZE counts a 48-byte scattered
record as its 64-byte line.  So the read factor is per kernel (READ_FACTOR): 1 where the reads are
record / line gathers (the render kernels), 2 where they are wide streams.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os

SHORT = [("render_bwd", "render_bwd"), ("render_fwd", "render_fwd"), ("gauss_bwd", "gauss_bwd"),
         ("gauss_reduce", "gauss_reduce"), ("gauss_live", "gauss_live"), ("preprocess", "preprocess"), ("tile_count", "tile_count"),
         ("tile_scan", "tile_scan"), ("tile_scatter", "tile_scatter"), ("tile_sort_class_kernel<128>", "tile_sort_c1"),
         ("tile_sort_class_kernel<512>", "tile_sort_c2"), ("tile_sort_global", "tile_sort_c3"),
         ("tile_sort_kernel", "tile_sort")]


def short(name: str) -> str:
    for k, v in SHORT:
        if k in name:
            return v
    return name[:40]


# read factor per kernel (bytes = factor x FETCH_SIZE x 1024) and why
_GATHER = "x1: per-lane 64-B record / line gathers dominate, counted exactly (tools/fetch_calib.hip, profiles/r05/r5a)"
_STREAM = "x2: wide coalesced streams dominate (MI355X_MICROARCH.md 'HBM'; tools/fetch_calib.hip stream16: 2.000)"
READ_FACTOR = {"render_bwd": (1.0, _GATHER), "render_fwd": (1.0, _GATHER)}


def read_factor(kernel: str):
    return READ_FACTOR.get(kernel, (2.0, _STREAM))


def load(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for f in glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = (r["VGPR_Count"], r["LDS_Block_Size"], r["Grid_Size"], r["Workgroup_Size"])
    return vals, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out")
    ap.add_argument("--json", help="also write {kernel: {hbm_read_bytes, hbm_write_bytes, ...}} here")
    ap.add_argument("--config", help="with --json: merge as configs[CONFIG] into the existing file (bench.py reads "
                                     "the entry of the config it runs)")
    a = ap.parse_args()
    vals, meta = load(a.dir)
    table = {}
    lines = ["| kernel | VGPR | LDS B | grid | VALU | SALU | LDS ops | VMEM rd | WAVE_CYC | ACTIVE_ANY | WAIT_INST | WAIT_ANY"
             " | LDS bank cf | HBM rd MB | HBM wr MB |", "|" + "---|" * 15]
    order = sorted(vals, key=lambda k: -sum(vals[k].get("SQ_WAVE_CYCLES", [0])) / max(1, len(vals[k].get("SQ_WAVE_CYCLES", [1]))))
    for k in order:
        v = vals[k]

        def m(c):
            x = v.get(c)
            return sum(x) / len(x) if x else float("nan")

        vg, lds, grid, wg = meta[k]
        rf, basis = read_factor(k)
        rd = rf * m("FETCH_SIZE") * 1024 / 1e6
        wr = m("WRITE_SIZE") * 1024 / 1e6
        table[k] = {"hbm_read_bytes": rd * 1e6, "hbm_write_bytes": wr * 1e6, "valu_insts": m("SQ_INSTS_VALU"),
                    "salu_insts": m("SQ_INSTS_SALU"), "wave_cycles": m("SQ_WAVE_CYCLES"),
                    "fetch_size_bytes": m("FETCH_SIZE") * 1024, "write_size_bytes": m("WRITE_SIZE") * 1024,
                    "read_factor": rf, "read_factor_basis": basis}
        lines.append(f"| {k} | {vg} | {lds} | {grid} | {m('SQ_INSTS_VALU'):.3g} | {m('SQ_INSTS_SALU'):.3g} | "
                     f"{m('SQ_INSTS_LDS'):.3g} | {m('SQ_INSTS_VMEM_RD'):.3g} | {m('SQ_WAVE_CYCLES'):.3g} | "
                     f"{m('SQ_ACTIVE_INST_ANY'):.3g} | {m('SQ_WAIT_INST_ANY'):.3g} | {m('SQ_WAIT_ANY'):.3g} | "
                     f"{m('SQ_LDS_BANK_CONFLICT'):.3g} | {rd:.1f} | {wr:.1f} |")
    text = "\n".join(lines)
    print(text)
    if a.json:
        import json

        entry = {"source": a.out or a.dir, "correction": "read = read_factor x FETCH_SIZE KiB (per kernel), write = "
                                                       "WRITE_SIZE KiB",
                 "kernels": table}
        if a.config:
            doc = json.load(open(a.json)) if os.path.exists(a.json) else {}
            doc.setdefault("configs", {})[a.config] = entry
            if a.config == "1m_1080p_sh3":  # the headline config also at the top level (older readers)
                doc.update(entry)
            entry = doc
        with open(a.json, "w") as f:
            json.dump(entry, f, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(f"# PMC summary ({a.dir}): mean per dispatch\n\n"
                    "HBM rd = read factor x FETCH_SIZE (x1 render kernels: 64-B gathers, x2 streams; tools/fetch_calib.hip), "
                    "KiB -> MB; "
                    "SQ cycle counters as reported (aggregated over SEs).\n\n" + text + "\n")


if __name__ == "__main__":
    main()
