#!/usr/bin/env python3
"""How many of a frame's tile-list instances the blend never reaches, and how much of them a cutoff
known BEFORE the key scatter (K3) could drop (development tool).

From the f32 oracle's tile lists and per-pixel state of one synthetic frame:
  * reach: per tile, the list prefix the forward walk must see -- up to the entry at which its last live
    pixel terminates (T (1 - alpha) < 1e-4, found by replaying the blend), or the whole list when a pixel
    never terminates.  n - reach is what an ideal per-tile cutoff would never emit or sort;
  * predictors a kernel could form before K3 from what preprocess / K1 already have, each giving a
    per-tile depth cutoff: entries at or below it are emitted, the rest not; a tile whose reach passes
    its emitted set is redone with its full list (the reachable-prefix sort's redo path).  Reported:
    the keys saved (net of the redone tiles' full lists) and the tiles redone.

    python tools/cutoff_estimate.py [--config 5m_4k_sh3] [--every 8] [--threads 8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def replay_reach(xy, conic, op, ids, tx0, ty0, W, H):
    """Entries the forward walk of one tile reads: it stops at the entry where its last live pixel
    terminates (CR/forward.cu:477-482), else reads the whole list.  Vectorised over the 256 pixels."""
    ly, lx = np.mgrid[0:16, 0:16]
    px, py = (tx0 + lx).reshape(-1).astype(np.float32), (ty0 + ly).reshape(-1).astype(np.float32)
    live = (px < W) & (py < H)
    T = np.ones(256, np.float32)
    n = len(ids)
    for k in range(0, n, 64):  # batches of entries, pixels x entries
        g = ids[k:k + 64]
        dx = xy[g, 0][None, :] - px[:, None]
        dy = xy[g, 1][None, :] - py[:, None]
        a, b, c = conic[g, 0][None, :], conic[g, 1][None, :], conic[g, 2][None, :]
        power = -0.5 * (a * dx * dx + c * dy * dy) - b * dx * dy
        alpha = np.minimum(np.float32(0.99), op[g][None, :] * np.exp(power))
        ok = (power <= 0) & (alpha >= 1.0 / 255.0)
        for j in range(len(g)):
            if not live.any():
                return k + j
            aj = np.where(ok[:, j] & live, alpha[:, j], 0.0).astype(np.float32)
            test = T * (1 - aj)
            term = live & (test < 1e-4)
            T = np.where(live & ~term, test, T)
            live &= ~term
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="5m_4k_sh3")
    ap.add_argument("--every", type=int, default=8, help="replay every k-th tile")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--json")
    a = ap.parse_args()
    import torch

    from gaussian_splatting_amd import synthetic as syn
    from tests import common as C

    scene, cam = syn.config_scene(a.config, seed=0)
    inp = dict(bg=torch.zeros(3), means3D=scene.means3D, opacities=scene.opacities, shs=scene.shs,
               sh_degree=scene.sh_degree, scales=scene.scales, rotations=scene.rotations, colors_precomp=None,
               cov3D_precomp=None, viewmatrix=cam.viewmatrix, projmatrix=cam.projmatrix, campos=cam.campos,
               tanfovx=cam.tanfovx, tanfovy=cam.tanfovy, H=cam.height, W=cam.width, scale_modifier=1.0,
               antialiasing=False)
    ref = C.run_oracle(inp, nthreads=a.threads)
    g, b = ref.handle.geom(), ref.handle.binning()
    W, H = cam.width, cam.height
    gx = (W + 15) // 16
    xy = g["means2D"].astype(np.float32)
    conic, op = g["conic_opacity"][:, :3].astype(np.float32), g["conic_opacity"][:, 3].astype(np.float32)
    depth = g["depths"].astype(np.float32)
    ranges, plist = b["ranges"].astype(np.int64), b["point_list"].astype(np.int64)
    radii = ref.radii.astype(np.int64)
    tiles = np.arange(0, len(ranges), a.every)
    n_t = ranges[tiles, 1] - ranges[tiles, 0]
    reach = np.zeros(len(tiles), np.int64)
    for i, t in enumerate(tiles):
        ids = plist[ranges[t, 0]:ranges[t, 1]]
        reach[i] = replay_reach(xy, conic, op, ids, (t % gx) * 16, (t // gx) * 16, W, H)
    # the depth of the last reached entry, per tile
    dreach = np.array([depth[plist[ranges[t, 0] + max(r - 1, 0)]] if r > 0 else 0.0
                       for t, r in zip(tiles, reach)], np.float32)
    out = {"config": a.config, "tiles_sampled": int(len(tiles)), "instances_sampled": int(n_t.sum()),
           "reached": int(reach.sum()), "reached_frac": float(reach.sum() / max(1, n_t.sum())),
           "whole_list_tiles": int((reach == n_t).sum()),
           "reach_depth_quantiles": {q: float(np.quantile(dreach[n_t > 0], q)) for q in (0.5, 0.9, 0.99, 1.0)}}

    def score(cut_depth, name):
        """keys emitted with a per-tile depth cutoff (entries with depth <= cut), a tile whose reach
        passes its emitted set redone with its whole list (emitted twice)."""
        emitted, redone = 0, 0
        for i, t in enumerate(tiles):
            ids = plist[ranges[t, 0]:ranges[t, 1]]
            k = int((depth[ids] <= cut_depth[i]).sum())
            if reach[i] > k or (reach[i] == k and k < len(ids) and reach[i] == len(ids)):
                emitted += k + len(ids)
                redone += 1
            else:
                emitted += k
        out[name] = {"emitted_frac": emitted / max(1, n_t.sum()), "tiles_redone": redone,
                     "tiles_redone_frac": redone / len(tiles)}

    # oracle-ideal: each tile cut at its own reach depth (no predictor can do better)
    score(dreach, "ideal_per_tile")
    # one global depth (the q-quantile of the tiles' reach depths): what a frame-wide bound would give
    for q in (0.9, 0.99, 1.0):
        score(np.full(len(tiles), out["reach_depth_quantiles"][q], np.float32), f"global_q{q}")
    # an opacity-mass predictor from data preprocess has: per tile, the depth at which the summed
    # -log(1 - a_min) of the Gaussians whose alpha >= a_min over the WHOLE tile reaches log(1e4) (then every
    # pixel of the tile has terminated: the mass is a sure bound, no redo)
    cut = np.full(len(tiles), np.inf, np.float32)
    for i, t in enumerate(tiles):
        ids = plist[ranges[t, 0]:ranges[t, 1]]
        tx0, ty0 = (t % gx) * 16, (t // gx) * 16
        # the tile corner farthest from each mean in the conic's metric bounds alpha from below (the
        # exponent is a concave quadratic: its minimum over the box is at a corner)
        cx = np.array([tx0, tx0 + 15, tx0, tx0 + 15], np.float32)
        cy = np.array([ty0, ty0, ty0 + 15, ty0 + 15], np.float32)
        dx = xy[ids, 0][:, None] - cx[None, :]
        dy = xy[ids, 1][:, None] - cy[None, :]
        A, B, Cc = conic[ids, 0][:, None], conic[ids, 1][:, None], conic[ids, 2][:, None]
        pw = (-0.5 * (A * dx * dx + Cc * dy * dy) - B * dx * dy).min(1)
        amin = np.minimum(0.99, op[ids] * np.exp(pw))
        amin = np.where(amin >= 1 / 255, amin, 0.0)
        mass = np.cumsum(-np.log1p(-amin))
        k = np.searchsorted(mass, np.log(1e4))
        if k < len(ids):
            cut[i] = depth[ids[k]]
    score(cut, "covering_mass_bound")
    # a frame-wide cutoff a kernel can form from preprocess's outputs alone: the depth at which the
    # screen-averaged opacity mass of the Gaussians in front (each o * 2 pi sqrt(det cov2D) / (W H), the
    # integral of its alpha over the plane) reaches `target` (saturation needs -ln 1e-4 = 9.2 per pixel)
    vis = radii > 0
    det_inv = conic[:, 0] * conic[:, 2] - conic[:, 1] ** 2  # det of the conic = 1 / det cov2D
    mass = np.where(vis & (det_inv > 0), op * 2 * np.pi / np.sqrt(np.maximum(det_inv, 1e-30)), 0.0) / (W * H)
    order = np.argsort(depth[vis], kind="stable")
    dz, cm = depth[vis][order], np.cumsum(mass[vis][order])
    out["mass_profile"] = {f"{q}": float(np.interp(q, cm, dz)) for q in (5, 9.2, 20, 40, 80) if q < cm[-1]}
    for target in (20, 40, 80):
        if target < cm[-1]:
            d = float(np.interp(target, cm, dz))
            score(np.full(len(tiles), d, np.float32), f"mass_target_{target}")
            out[f"mass_target_{target}"]["depth"] = d
    out["covering_mass_bound"]["note"] = ("sure bound (no redo by construction); needs per-(tile, Gaussian) "
                                          "corner tests in depth order before K3")
    print(json.dumps(out, indent=1))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
