"""K3 store-pattern statistics (development tool).

For a benchmark frame, rebuilds K0's spatial order (Gaussians counting-sorted by the 4x4-tile cell
of their tile rectangle's centre) and K3's chunks (256), and reports what K3's key stores look like:
tiles per chunk, instances per (chunk, tile) run, and the 128-byte lines the runs cover.
    python tools/k3_runs.py [--config 5m_4k_sh3]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402
from gaussian_splatting_amd import synthetic as syn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="5m_4k_sh3")
    ap.add_argument("--chunks", type=int, default=256)
    ap.add_argument("--order", choices=("row", "morton"), default="row",
                    help="cell order of K0's spatial sort: row-major cells or Z-order (Morton) cells")
    args = ap.parse_args()
    scene, cam = syn.config_scene(args.config, seed=0)
    W, H = cam.width, cam.height
    r = oracle.forward(scene.means3D, scene.opacities, cam.viewmatrix, cam.projmatrix, cam.campos, cam.tanfovx,
                       cam.tanfovy, H, W, shs=scene.shs, sh_degree=scene.sh_degree, scales=scene.scales,
                       rotations=scene.rotations, nthreads=8)
    g = r.handle.geom()
    gx, gy = (W + 15) // 16, (H + 15) // 16
    m = g["means2D"].astype(np.float32)
    rad = r.radii.astype(np.float32)
    x0 = np.clip(((m[:, 0] - rad) / 16).astype(np.int64), 0, gx)
    y0 = np.clip(((m[:, 1] - rad) / 16).astype(np.int64), 0, gy)
    x1 = np.clip(((m[:, 0] + rad + 15) / 16).astype(np.int64), 0, gx)
    y1 = np.clip(((m[:, 1] + rad + 15) / 16).astype(np.int64), 0, gy)
    n = (x1 - x0) * (y1 - y0) * (rad > 0)
    print("instances", n.sum(), "num_rendered", r.num_rendered)
    vis = np.nonzero(n > 0)[0]
    cgx = (gx + 3) // 4
    cx, cy = ((x0 + x1) >> 1) // 4, ((y0 + y1) >> 1) // 4
    if args.order == "row":
        cell = cy * cgx + cx
    else:
        cell = np.zeros_like(cx)
        for b in range(16):
            cell |= ((cx >> b) & 1) << (2 * b) | ((cy >> b) & 1) << (2 * b + 1)
    order = vis[np.argsort(cell[vis], kind="stable")]
    P = len(n)
    chunk = -(-P // args.chunks)
    tiles = gx * gy
    run_len = []
    tiles_per_chunk = []
    for c in range(args.chunks):
        idx = order[c * chunk:(c + 1) * chunk]
        if len(idx) == 0:
            continue
        cnt = np.zeros(tiles, np.int64)
        # vectorised: +1 over each rectangle by a 2-D difference array
        d = np.zeros((gy + 1, gx + 1), np.int64)
        np.add.at(d, (y0[idx], x0[idx]), 1)
        np.add.at(d, (y0[idx], x1[idx]), -1)
        np.add.at(d, (y1[idx], x0[idx]), -1)
        np.add.at(d, (y1[idx], x1[idx]), 1)
        cnt = d.cumsum(0).cumsum(1)[:gy, :gx].ravel()
        nz = cnt[cnt > 0]
        tiles_per_chunk.append(len(nz))
        run_len.append(nz)
    rl = np.concatenate(run_len)
    I = rl.sum()
    print(f"{args.config}: I={I} runs={len(rl)} mean run={rl.mean():.1f} keys; tiles/chunk mean {np.mean(tiles_per_chunk):.0f}"
          f" max {np.max(tiles_per_chunk)}")
    for q in (10, 25, 50, 75, 90, 99):
        print(f"  run length p{q}: {np.percentile(rl, q):.0f}")
    # instances by the length of the run they are in
    for lo, hi in ((1, 2), (2, 8), (8, 16), (16, 64), (64, 256), (256, 1 << 40)):
        sel = (rl >= lo) & (rl < hi)
        print(f"  runs [{lo},{hi}): {sel.sum()} runs, {rl[sel].sum() / I:.3f} of instances")
    # 128-B lines touched by the runs (8-B keys, run start uniformly aligned)
    b = rl * 8
    lines = np.floor(b / 128) + (np.mod(b, 128) > 0) + 0.5 * (np.mod(b, 128) != 0)  # rough: +1 partial crossing
    print(f"  key bytes {b.sum() / 1e9:.3f} GB; ~128-B lines covered {lines.sum() * 128 / 1e9:.3f} GB")


if __name__ == "__main__":
    main()
