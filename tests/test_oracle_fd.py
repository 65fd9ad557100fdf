"""Central finite differences of the float64 oracle's forward against its own hand backward
(an autograd-free check).  CPU only.

L = <g_c, color> + <g_d, invdepth>.  Coordinates are perturbed one at a time by +-eps; eps
is small enough (1e-6 relative to typical magnitudes) that no discrete decision of the
forward (tile rectangles, the 1/255 and 1e-4 thresholds) flips for the sampled Gaussians,
which are drawn among those that are visible and not tiny.
"""
import numpy as np
import pytest
import torch

from tests import common as C

EPS = 1e-6


def _loss(inp, gc, gd):
    r = C.run_oracle(inp, precision="f64")
    return float((r.color * gc).sum() + (r.invdepth * gd).sum()), r


def _perturbed(inp, key, i, j, delta):
    out = dict(inp)
    t = inp[key].clone().double()
    t.view(t.shape[0], -1)[i, j] += delta
    out[key] = t
    return out


@pytest.mark.parametrize("case", [C.Case("fd_sh3", P=60, W=40, H=32, sh_degree=3),
                                  C.Case("fd_yaw_bg", P=60, W=40, H=32, yaw=20.0, bg=(0.3, 0.6, 0.1)),
                                  C.Case("fd_precomp", P=60, W=40, H=32, mode_color="precomp",
                                         mode_cov="precomp")], ids=lambda c: c.name)
def test_backward_matches_finite_differences(case):
    inp = C.build(case)
    inp = {k: (v.double() if torch.is_tensor(v) else v) for k, v in inp.items()}
    gc, gd = C.unit_grads(case.H, case.W, seed=9)
    gc, gd = gc.double().numpy(), gd.double().numpy()
    L0, r0 = _loss(inp, gc, gd)
    g = r0.handle.backward(gc, gd)
    rng = np.random.default_rng(0)
    # exclude Gaussians whose view-space x/z or y/z is clamped to 1.3 tan(fov): there the reference's
    # backward is deliberately not the true derivative (CR/backward.cu:193-194; pinned against autograd
    # with that convention in test_oracle_autograd.py)
    V = inp["viewmatrix"].double()
    pv = torch.cat([inp["means3D"], torch.ones(case.P, 1, dtype=torch.float64)], 1) @ V[:, :3]
    inside = ((pv[:, 0] / pv[:, 2]).abs() <= 1.3 * inp["tanfovx"]) & ((pv[:, 1] / pv[:, 2]).abs() <= 1.3 * inp["tanfovy"])
    vis = np.nonzero((r0.radii >= 2) & inside.numpy())[0]
    assert len(vis) >= 10
    keys = [("means3D", "dL_dmeans3D"), ("opacities", "dL_dopacity")]
    keys += [("colors_precomp", "dL_dcolors")] if inp["colors_precomp"] is not None else [("shs", "dL_dsh")]
    if inp["cov3D_precomp"] is not None:
        keys += [("cov3D_precomp", "dL_dcov3D")]
    else:
        keys += [("scales", "dL_dscales"), ("rotations", "dL_drotations")]
    checked = 0
    for key, gk in keys:
        width = inp[key].reshape(inp[key].shape[0], -1).shape[1]
        ana_all = g[gk].reshape(g[gk].shape[0], -1)
        for i in rng.choice(vis, size=6, replace=False):
            j = int(rng.integers(width))
            ana = ana_all[i, j]
            Lp, _ = _loss(_perturbed(inp, key, i, j, EPS), gc, gd)
            Lm, _ = _loss(_perturbed(inp, key, i, j, -EPS), gc, gd)
            fd = (Lp - Lm) / (2 * EPS)
            scale = max(np.abs(ana_all).max(), 1e-12)
            # dL/dscales omits scale_modifier (=1 here); cov3D grads of symmetric off-diagonals are per stored entry
            assert abs(fd - ana) <= 2e-4 * scale + 1e-7 * abs(ana), (key, i, j, fd, ana)
            checked += 1
    assert checked >= 24
