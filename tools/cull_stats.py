"""Culling statistics for the render passes (development tool).

For a sample of tiles of a benchmark frame, counts per list entry and 8x8 quadrant:
  bbox   -- quadrants the alpha >= 1/255 footprint box overlaps (what the kernels test today)
  ellipse-- quadrants the alpha >= 1/255 ellipse itself overlaps (exact min of the quadratic form)
  hit    -- quadrants with at least one pixel the reference would blend (ignoring termination)
    python tools/cull_stats.py [--config 1m_1080p_sh3] [--tiles 200]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402
from gaussian_splatting_amd import synthetic as syn  # noqa: E402


def quad_min_form(mx, my, a, b, c, x0, x1, y0, y1):
    """min over the rectangle [x0,x1]x[y0,y1] of Q(d) = a dx^2 + 2 b dx dy + c dy^2, d = p - m (vectorised)."""
    inside = (mx >= x0) & (mx <= x1) & (my >= y0) & (my <= y1)
    best = np.full(mx.shape, np.inf)
    for fixed_x in (x0, x1):  # vertical edges: dx fixed, minimise over dy
        dx = fixed_x - mx
        dy = np.clip(-b * dx / c, y0 - my, y1 - my)
        best = np.minimum(best, a * dx * dx + 2 * b * dx * dy + c * dy * dy)
    for fixed_y in (y0, y1):
        dy = fixed_y - my
        dx = np.clip(-b * dy / a, x0 - mx, x1 - mx)
        best = np.minimum(best, a * dx * dx + 2 * b * dx * dy + c * dy * dy)
    return np.where(inside, 0.0, best)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="1m_1080p_sh3")
    ap.add_argument("--tiles", type=int, default=200)
    args = ap.parse_args()
    scene, cam = syn.config_scene(args.config, seed=0)
    r = oracle.forward(scene.means3D, scene.opacities, cam.viewmatrix, cam.projmatrix, cam.campos, cam.tanfovx,
                       cam.tanfovy, cam.height, cam.width, shs=scene.shs, sh_degree=scene.sh_degree,
                       scales=scene.scales, rotations=scene.rotations, nthreads=os.cpu_count())
    g = r.handle.geom()
    b = r.handle.binning()
    img = r.handle.image()
    W, H = cam.width, cam.height
    gx = (W + 15) // 16
    rng = np.random.default_rng(0)
    tiles = rng.choice(len(b["ranges"]), size=min(args.tiles, len(b["ranges"])), replace=False)
    tot = dict(entries=0, bbox=0, ellipse=0, hit=0, hit_live=0, bwd_wave=0, bwd_slot=0, bwd_slot_ell=0)
    for t in tiles:
        s, e = b["ranges"][t]
        if e <= s:
            continue
        ids = b["point_list"][s:e].astype(np.int64)
        tx0, ty0 = (t % gx) * 16, (t // gx) * 16
        m = g["means2D"][ids].astype(np.float64)
        co = g["conic_opacity"][ids].astype(np.float64)
        a, bb, c, o = co[:, 0], co[:, 1], co[:, 2], co[:, 3]
        tau = np.log(np.maximum(255.0 * o, 1e-30))
        nc = img["n_contrib"][ty0:ty0 + 16, tx0:tx0 + 16]
        tot["entries"] += len(ids)
        wave_lim = int(nc.max())
        for q in range(4):
            qx0, qy0 = tx0 + (q & 1) * 8, ty0 + (q >> 1) * 8
            if qx0 >= W or qy0 >= H:
                continue
            # bbox test, as preprocess builds it (tau * 1.001 + 0.01 margin; ex = sqrt(2 tau cov_xx) + 0.05)
            det = a * c - bb * bb
            cxx, cyy = c / det, a / det
            tm = np.maximum(tau, 0) * 1.001 + 0.01
            ex, ey = np.sqrt(2 * tm * cxx) + 0.05, np.sqrt(2 * tm * cyy) + 0.05
            bx0, bx1 = np.ceil(m[:, 0] - ex), np.floor(m[:, 0] + ex)
            by0, by1 = np.ceil(m[:, 1] - ey), np.floor(m[:, 1] + ey)
            in_bbox = (bx0 <= qx0 + 7) & (bx1 >= qx0) & (by0 <= qy0 + 7) & (by1 >= qy0) & (o * 255 >= 0.999)
            qmin = quad_min_form(m[:, 0], m[:, 1], a, bb, c, qx0, qx0 + 7, qy0, qy0 + 7)
            in_ell = (qmin <= 2 * tm) & (o * 255 >= 0.999)
            px = np.arange(8) + qx0
            py = np.arange(8) + qy0
            dx = m[:, 0, None, None] - px[None, None, :]
            dy = m[:, 1, None, None] - py[None, :, None]
            power = -0.5 * (a[:, None, None] * dx * dx + c[:, None, None] * dy * dy) - bb[:, None, None] * dx * dy
            alpha = np.minimum(0.99, o[:, None, None] * np.exp(np.minimum(power, 0)))
            valid = (px[None, None, :] < W) & (py[None, :, None] < H)
            hitpix = (power <= 0) & (alpha >= 1 / 255) & valid
            pos = np.arange(len(ids))[:, None, None]
            ncq = nc[(q >> 1) * 8:(q >> 1) * 8 + 8, (q & 1) * 8:(q & 1) * 8 + 8]
            ncq = np.pad(ncq, ((0, 8 - ncq.shape[0]), (0, 8 - ncq.shape[1])))
            live = hitpix & (pos < ncq[None])
            slot_lim = int(ncq.max())
            pos1 = np.arange(len(ids))
            tot["bwd_wave"] += int((in_bbox & (pos1 < wave_lim)).sum())
            tot["bwd_slot"] += int((in_bbox & (pos1 < slot_lim)).sum())
            tot["bwd_slot_ell"] += int((in_ell & (pos1 < slot_lim)).sum())
            tot["bbox"] += int(in_bbox.sum())
            tot["ellipse"] += int(in_ell.sum())
            tot["hit"] += int(hitpix.any(axis=(1, 2)).sum())
            tot["hit_live"] += int(live.any(axis=(1, 2)).sum())
            assert not (hitpix.any(axis=(1, 2)) & ~in_ell).any(), "ellipse test not conservative"
    n = tot["entries"]
    print({k: v for k, v in tot.items()})
    print("backward slot evals per entry: wave-limit %.3f slot-limit %.3f slot-limit+ellipse %.3f" %
          (tot["bwd_wave"] / n, tot["bwd_slot"] / n, tot["bwd_slot_ell"] / n))
    print("per entry: bbox %.3f ellipse %.3f hit %.3f hit-before-termination %.3f slots" %
          (tot["bbox"] / n, tot["ellipse"] / n, tot["hit"] / n, tot["hit_live"] / n))


if __name__ == "__main__":
    main()
