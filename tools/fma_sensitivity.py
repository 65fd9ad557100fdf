#!/usr/bin/env python3
"""How sensitive are the rasterizer's INTEGER outputs to floating-point contraction?

The GPU's preprocess is compiled without contraction, and its integers (radii, tile rectangles,
num_rendered, the sorted tile lists) equal those of the uncontracted C oracle (`-ffp-contract=off`).
The reference is built by nvcc with its default `--fmad=true` (RI/setup.py:29 passes only `-I`), so
its decisions may come from fused multiply-adds.  This tool runs the f32 oracle twice on the same
full-size frame -- uncontracted (`liboracle_f32.so`) and contracted (`liboracle_f32fma.so`:
`-ffp-contract=fast -mfma`, gcc fusing every multiply-add it can) -- and counts the differences:
num_rendered, radii, tile-list lengths, tiles whose sorted list differs, and (beyond the integers)
pixels whose colour moves by more than 1e-5.  Which pairs nvcc fuses is not which pairs gcc fuses,
so this bounds the SIZE of the effect, not the reference's exact outputs.

    python tools/fma_sensitivity.py [--configs 500k_1080p_sh3,1m_1080p_sh3,5m_4k_sh3] [--json OUT]

Test / diagnostic infrastructure (imports oracle/); CPU only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gaussian_splatting_amd import synthetic as syn  # noqa: E402
from oracle import oracle  # noqa: E402


def run(cfg: str, precision: str, threads: int):
    scene, cam = syn.config_scene(cfg, seed=0)
    t0 = time.perf_counter()
    r = oracle.forward(scene.means3D, scene.opacities, cam.viewmatrix, cam.projmatrix, cam.campos, cam.tanfovx,
                       cam.tanfovy, cam.height, cam.width, shs=scene.shs, sh_degree=scene.sh_degree,
                       scales=scene.scales, rotations=scene.rotations, precision=precision, nthreads=threads)
    return r, time.perf_counter() - t0


def list_diff(a: dict, b: dict) -> dict:
    """Tiles whose list length differs, and tiles of equal length whose sorted entries differ."""
    ra, rb = a["ranges"].astype(np.int64), b["ranges"].astype(np.int64)
    la, lb = ra[:, 1] - ra[:, 0], rb[:, 1] - rb[:, 0]
    len_diff = la != lb
    same = (~len_diff) & (la > 0)
    content = np.zeros(len(la), bool)
    pa, pb = a["point_list"], b["point_list"]
    for t in np.flatnonzero(same):
        if not np.array_equal(pa[ra[t, 0]:ra[t, 1]], pb[rb[t, 0]:rb[t, 1]]):
            content[t] = True
    return {"tiles": int(len(la)), "tiles_length_differs": int(len_diff.sum()),
            "tiles_entries_differ": int(content.sum()),
            "instances_in_length_differing_tiles": int(np.abs(la - lb)[len_diff].sum())}


def compare(ra, rb) -> dict:
    out = {"num_rendered": [int(ra.num_rendered), int(rb.num_rendered)],
           "num_rendered_diff": int(rb.num_rendered) - int(ra.num_rendered)}
    rd = ra.radii != rb.radii
    out["radii_differ"] = int(rd.sum())
    out["radii_max_abs_diff"] = int(np.abs(ra.radii.astype(np.int64) - rb.radii.astype(np.int64)).max()) if rd.any() else 0
    ga, gb = ra.handle.geom(), rb.handle.geom()
    tt = ga["tiles_touched"] != gb["tiles_touched"]
    out["tiles_touched_differ"] = int(tt.sum())
    out.update(list_diff(ra.handle.binning(), rb.handle.binning()))
    d = np.maximum(np.abs(ra.color - rb.color).max(0), np.abs(ra.invdepth - rb.invdepth)[0])
    out["pixels_over_1e-5"] = int((d > 1e-5).sum())
    out["pixel_max_abs_diff"] = float(d.max())
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="500k_1080p_sh3,1m_1080p_sh3,5m_4k_sh3")
    ap.add_argument("--threads", type=int, default=len(os.sched_getaffinity(0)))
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    oracle.build()
    res = {"what": "uncontracted f32 oracle (-ffp-contract=off) vs contracted (-ffp-contract=fast -mfma), "
                   "same frame; counts of differing integer outputs", "configs": {}}
    for cfg in args.configs.split(","):
        a, ta = run(cfg, "f32", args.threads)
        b, tb = run(cfg, "f32fma", args.threads)
        c = compare(a, b)
        c["seconds"] = [round(ta, 1), round(tb, 1)]
        res["configs"][cfg] = c
        print(cfg, json.dumps(c), flush=True)
        del a, b
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
