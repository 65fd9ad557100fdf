#!/usr/bin/env python3
"""Cost of the screen-space backward (gsr_rasterize_backward_screen: render_bwd + the step that fills the view
block) on one MI355X, record path (bwd_atomic=0: records + gauss_reduce) against the atomic path (the default:
accumulator rows + gauss_live_views), interleaved (development tool).

    python tools/bench_screen.py [--config 1m_1080p_sh3] [--reps 20] [--rounds 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gaussian_splatting_amd import _C, _lib  # noqa: E402
from gaussian_splatting_amd import synthetic as syn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="1m_1080p_sh3")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = syn.CONFIGS[a.config]
    P, W, H, D = cfg["P"], cfg["width"], cfg["height"], cfg["sh_degree"]
    scene, cam = syn.config_scene(a.config, seed=0)
    scene, cam = scene.to(dev), cam.to(dev)
    gc, gd = syn.upstream_grads(H, W)
    gc, gd = gc.to(dev), gd.to(dev)
    bg, empty = torch.zeros(3, device=dev), torch.empty(0, device=dev)
    block = torch.empty(_C.view_block_floats(P), device=dev)
    setups = {}
    for mode in (0, 1):  # one forward per path: the forward decides (it zeroes and marks the rows)
        with _lib.options(bwd_atomic=mode):
            fwd = _C.rasterize_gaussians(bg, scene.means3D, empty, scene.opacities, scene.scales, scene.rotations, 1.0,
                                         empty, cam.viewmatrix, cam.projmatrix, cam.tanfovx, cam.tanfovy, H, W,
                                         scene.shs, D, cam.campos, False, False, False)
        nr, color, radii, geom, binning, img, invd = fwd
        setups[mode] = (fwd, (bg, scene.means3D, radii, empty, scene.opacities, scene.scales, scene.rotations, 1.0,
                              empty, cam.viewmatrix, cam.projmatrix, cam.tanfovx, cam.tanfovy, gc, gd, scene.shs, D,
                              cam.campos, geom, nr, binning, img, False, False))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = {"config": a.config, "reps": a.reps, "record_ms": [], "atomic_ms": []}
    for _ in range(a.rounds):
        for mode, key in ((0, "record_ms"), (1, "atomic_ms")):
            args = setups[mode][1]
            with _lib.options(bwd_atomic=mode):
                for _ in range(3):
                    _C.rasterize_gaussians_backward_screen(*args, view_block=block)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(a.reps):
                    _C.rasterize_gaussians_backward_screen(*args, view_block=block)
                e1.record()
                torch.cuda.synchronize()
            out[key].append(round(e0.elapsed_time(e1) / a.reps, 4))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
