#!/usr/bin/env python3
"""Estimate render work under different pixel-block granularities (development tool).

For a sample of tiles of a synthetic frame (the oracle's tile lists, per-pixel alpha and n_contrib),
count the backward's wave iterations
  * quadrant scheme (current render_bwd): one 64-lane evaluation per (entry, 8x8 quadrant) whose
    pixels the entry reaches (alpha >= 1/255 somewhere in it) before the quadrant's limit;
  * block scheme: the 16 4x4 blocks of a tile dealt to four 16-lane groups (group = block column,
    slot = block row); per batch of 64 entries and slot, the wave iterates max over the groups of
    the entries reaching that group's block -- the groups walk their own entries in order;
and the useful lanes (pixel, entry) pairs with a gradient term.

    python tools/sim_blocks.py [--config 1m_1080p_sh3] [--every 4]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="1m_1080p_sh3")
    ap.add_argument("--every", type=int, default=4)
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    from gaussian_splatting_amd import synthetic as syn
    from tests import common as C

    scene, cam = syn.config_scene(a.config, seed=0)
    inp = dict(bg=None, means3D=scene.means3D, opacities=scene.opacities, shs=scene.shs, sh_degree=scene.sh_degree,
               scales=scene.scales, rotations=scene.rotations, colors_precomp=None, cov3D_precomp=None,
               viewmatrix=cam.viewmatrix, projmatrix=cam.projmatrix, campos=cam.campos, tanfovx=cam.tanfovx,
               tanfovy=cam.tanfovy, H=cam.height, W=cam.width, scale_modifier=1.0, antialiasing=False)
    import torch
    inp["bg"] = torch.zeros(3)
    ref = C.run_oracle(inp, nthreads=a.threads)
    g = ref.handle.geom()
    b = ref.handle.binning()
    im = ref.handle.image()
    W, H = cam.width, cam.height
    gx = (W + 15) // 16
    gy = (H + 15) // 16
    xy, conic, op = g["means2D"], g["conic_opacity"][:, :3], g["conic_opacity"][:, 3]
    ranges, plist = b["ranges"].astype(np.int64), b["point_list"].astype(np.int64)
    nc = im["n_contrib"].reshape(H, W).astype(np.int64)
    ly, lx = np.mgrid[0:16, 0:16]
    lx, ly = lx.reshape(-1), ly.reshape(-1)
    quad = (ly // 8) * 2 + lx // 8       # 8x8 quadrant of each tile pixel
    blk = (ly // 4) * 4 + lx // 4        # 4x4 block
    blk8x4 = (ly // 4) * 2 + lx // 8     # 8x4 half-quadrant blocks: 8 per tile
    tot = dict(q_evals=0, b_iters=0, pairs=0, entries=0, b_lane_evals=0, h_iters=0, h_lane_evals=0)
    tiles = range(0, gx * gy, a.every)
    for t in tiles:
        s, e = ranges[t]
        if e <= s:
            continue
        tx, ty = (t % gx) * 16, (t // gx) * 16
        px, py = tx + lx, ty + ly
        inside = (px < W) & (py < H)
        ncp = np.where(inside, nc[np.minimum(py, H - 1), np.minimum(px, W - 1)], 0)
        lim = int(ncp.max())
        if lim == 0:
            continue
        ids = plist[s:s + lim]
        dx = xy[ids, 0][:, None] - px[None, :]
        dy = xy[ids, 1][:, None] - py[None, :]
        pw = -0.5 * (conic[ids, 0][:, None] * dx * dx + conic[ids, 2][:, None] * dy * dy) - conic[ids, 1][:, None] * dx * dy
        al = np.minimum(0.99, op[ids][:, None] * np.exp(pw))
        hit = (pw <= 0) & (al >= 1 / 255) & inside[None, :]
        pos = np.arange(lim)[:, None]
        grad = hit & (pos < ncp[None, :])           # (pixel, entry) pairs with a gradient term
        tot["pairs"] += int(grad.sum())
        tot["entries"] += lim
        # quadrant limits (slim) and blocks' limits
        qlim = np.array([ncp[quad == q].max() for q in range(4)])
        blim = np.array([ncp[blk == k].max() for k in range(16)])
        qh = np.stack([hit[:, quad == q].any(1) for q in range(4)], 1) & (pos < qlim[None, :])
        bh = np.stack([hit[:, blk == k].any(1) for k in range(16)], 1) & (pos < blim[None, :])
        tot["q_evals"] += int(qh.sum())
        tot["b_lane_evals"] += int(bh.sum()) * 16
        hlim = np.array([ncp[blk8x4 == k].max() for k in range(8)])
        hh = np.stack([hit[:, blk8x4 == k].any(1) for k in range(8)], 1) & (pos < hlim[None, :])
        tot["h_lane_evals"] += int(hh.sum()) * 32
        for b0 in range(0, lim, 64):
            bb = bh[b0:b0 + 64].reshape(-1, 4, 4)  # [entry, block row (slot), block column (group)]
            tot["b_iters"] += int(bb.sum(0).max(1).sum())
            # two 32-lane halves: half h owns the 8x4 blocks of column h (4 slots, one per block row)
            hb = hh[b0:b0 + 64].reshape(-1, 4, 2)
            tot["h_iters"] += int(hb.sum(0).max(1).sum())
    q_lanes = tot["q_evals"] * 64
    b_lanes = tot["b_iters"] * 64
    print(f"{a.config}, every {a.every}th tile: entries {tot['entries']}, pairs with a gradient {tot['pairs']}")
    print(f"  quadrant scheme: {tot['q_evals']} evaluations, useful lanes {tot['pairs'] / q_lanes:.3f}")
    print(f"  4x4 block scheme: {tot['b_iters']} wave iterations ({tot['b_iters'] / tot['q_evals']:.3f} of the quadrant "
          f"evaluations), useful lanes {tot['pairs'] / b_lanes:.3f}; lane-evaluations of touched blocks alone "
          f"{tot['b_lane_evals'] / q_lanes:.3f} of the quadrant scheme's")
    print(f"  8x4 blocks, two 32-lane halves: {tot['h_iters']} wave iterations ({tot['h_iters'] / tot['q_evals']:.3f}), "
          f"useful lanes {tot['pairs'] / (tot['h_iters'] * 64):.3f}; touched-block lane-evaluations "
          f"{tot['h_lane_evals'] / q_lanes:.3f}")


if __name__ == "__main__":
    main()
