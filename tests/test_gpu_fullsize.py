"""Full-size parity at the benchmark configuration (1M Gaussians, 1920x1080, SH degree 3) and at
BASELINE.json's largest single-GPU configuration (5M Gaussians, 3840x2160, SH degree 3: ~115M
tile instances, lists of ~3,500 entries per tile -- the long-list sort classes and the tile-list
sizing).

The oracle (OpenMP C restatement of the reference) runs the same frame on the host.
At this size a handful of pixels sit exactly on a discrete threshold of the reference
algorithm (alpha = 1/255, T = 1e-4, integer radius rounding), where an fp32
rounding difference (FMA contraction, exp implementation) flips the decision; the
test therefore checks the 1e-5 bar on >= 99.9% of pixels and bounds the rest, and
checks size-independent properties exactly (determinism, tile-list invariants).
"""
import os

import numpy as np
import pytest
import torch

from tests import common as C
from gaussian_splatting_amd import synthetic as syn

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def _np(t):
    return t.detach().float().cpu().numpy()


@pytest.fixture(scope="module", params=["1m_1080p_sh3", "5m_4k_sh3"])
def fullsize(request):
    scene, cam = syn.config_scene(request.param, seed=0)
    inp = dict(bg=torch.zeros(3), means3D=scene.means3D, opacities=scene.opacities, shs=scene.shs,
               sh_degree=scene.sh_degree, scales=scene.scales, rotations=scene.rotations, colors_precomp=None,
               cov3D_precomp=None, viewmatrix=cam.viewmatrix, projmatrix=cam.projmatrix, campos=cam.campos,
               tanfovx=cam.tanfovx, tanfovy=cam.tanfovy, H=cam.height, W=cam.width, scale_modifier=1.0,
               antialiasing=False)
    threads = min(32, os.cpu_count() or 1)
    ref = C.run_oracle(inp, nthreads=threads)
    gc, gd = syn.upstream_grads(cam.height, cam.width)
    ref_g = ref.handle.backward(gc, gd, nthreads=threads)
    fwd = C.run_gpu_forward(inp)
    out = C.run_gpu_backward(inp, fwd, gc, gd)
    torch.cuda.synchronize()
    return inp, ref, ref_g, fwd, out, (gc, gd)


def test_fullsize_forward(fullsize):
    inp, ref, _, fwd, _, _ = fullsize
    nr, color, radii, *_, invd = fwd
    assert abs(nr - ref.num_rendered) <= 1e-4 * ref.num_rendered
    r = _np(radii).astype(np.int64)
    same = (r == ref.radii).mean()
    assert same >= 0.9999, same
    assert np.abs(r - ref.radii).max() <= 1
    for got, exp in ((_np(color), ref.color), (_np(invd), ref.invdepth)):
        d = np.abs(got - exp)
        assert (d <= 1e-5).mean() >= 0.999, (d <= 1e-5).mean()
        assert d.mean() <= 1e-6, d.mean()


def test_fullsize_backward(fullsize):
    _, _, ref_g, _, out, _ = fullsize
    for k, got in zip(C.GRAD_NAMES, out):
        g, e = _np(got), ref_g[k]
        assert g.shape == e.shape
        d = np.abs(g.astype(np.float64) - e)
        scale = np.abs(e).max()
        # 99.9% of entries within 1e-4 of the tensor's scale; the 1e-5 absolute bar with the L1 loss
        assert np.quantile(d, 0.999) <= 1e-4 * scale, (k, np.quantile(d, 0.999) / scale)
        assert d.max() <= 1e-5, (k, d.max())


def test_fullsize_deterministic(fullsize):
    inp, _, _, fwd, out, (gc, gd) = fullsize
    fwd2 = C.run_gpu_forward(inp)
    out2 = C.run_gpu_backward(inp, fwd2, gc, gd)
    assert fwd2[0] == fwd[0]
    assert torch.equal(fwd2[1], fwd[1]) and torch.equal(fwd2[6], fwd[6])
    for a, b in zip(out, out2):
        assert torch.equal(a, b)


def test_fullsize_colors_precomp_matches_sh(fullsize):
    """The reference's own consistency switch (gaussian_renderer/__init__.py:86-104): colours computed from
    the SHs outside the rasterizer give the same image as in-kernel SH evaluation."""
    inp, ref, _, fwd, _, _ = fullsize
    means = inp["means3D"]
    dirs = torch.nn.functional.normalize(means - inp["campos"][None], dim=1)
    rgb = _sh_eval(inp["shs"], dirs, inp["sh_degree"])
    inp2 = dict(inp, colors_precomp=torch.clamp_min(rgb + 0.5, 0.0), shs=None)
    fwd2 = C.run_gpu_forward(inp2)
    d = (fwd2[1] - fwd[1]).abs()
    assert (d <= 1e-5).float().mean() >= 0.999
    assert float(d.mean()) <= 1e-6


def _sh_eval(sh, dirs, deg):
    """utils/sh_utils.py:57-112 restated (same polynomial and constants as CR/auxiliary.h:23-40)."""
    C0, C1 = 0.28209479177387814, 0.4886025119029199
    C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
    C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
          1.445305721320277, -0.5900435899266435]
    x, y, z = dirs[:, 0:1], dirs[:, 1:2], dirs[:, 2:3]
    res = C0 * sh[:, 0]
    if deg > 0:
        res = res - C1 * y * sh[:, 1] + C1 * z * sh[:, 2] - C1 * x * sh[:, 3]
        if deg > 1:
            xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
            res = (res + C2[0] * xy * sh[:, 4] + C2[1] * yz * sh[:, 5] + C2[2] * (2.0 * zz - xx - yy) * sh[:, 6]
                   + C2[3] * xz * sh[:, 7] + C2[4] * (xx - yy) * sh[:, 8])
            if deg > 2:
                res = (res + C3[0] * y * (3 * xx - yy) * sh[:, 9] + C3[1] * xy * z * sh[:, 10]
                       + C3[2] * y * (4 * zz - xx - yy) * sh[:, 11]
                       + C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 12]
                       + C3[4] * x * (4 * zz - xx - yy) * sh[:, 13] + C3[5] * z * (xx - yy) * sh[:, 14]
                       + C3[6] * x * (xx - 3 * yy) * sh[:, 15])
    return res
