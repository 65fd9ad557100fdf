"""Separate-DC SH input: the 3DGS-accel interface (dc + rest, gsr_rasterize_forward_dc /
gsr_rasterize_backward_dc) that the reference's callers select with separate_sh=True
(train.py:41-45,105,144; gaussian_renderer/__init__.py:106-125).

The accel build is not vendored by the reference, so there
is no reference vector for it; what pins it is its definition -- the split arrays hold
the same coefficients as one [P, M+1, 3] array, and the colour polynomial does not care
where coefficient 0 lives.  The GPU tests therefore demand BITWISE equality between the
split path and the combined path (same arithmetic on the same values, both of which are
checked against the oracle in test_gpu_parity.py), plus the oracle on the concatenation.
"""
import numpy as np
import pytest
import torch

from tests import common as C

CASES = [
    C.Case("sep_sh3", P=300, W=64, H=48),                       # LDS path (M = 16), one ragged wave
    C.Case("sep_sh3_P64k", P=64 * 7 + 33, W=80, H=64),          # several waves, ragged 32-row half
    C.Case("sep_sh1_of_16", P=250, W=64, H=64, sh_degree=1),    # M = 16 but D < 3: generic preprocess path
    C.Case("sep_sh2_M9", P=250, W=48, H=40, sh_degree=2, M=9),  # generic path, rest of 8
    C.Case("sep_sh0_M1", P=250, W=48, H=40, sh_degree=0, M=1),  # dc only, empty rest
    C.Case("sep_antialiasing", P=300, W=64, H=48, antialiasing=True),
]


def _split(inp, device):
    sh = inp["shs"].to(device)
    return sh[:, :1, :].contiguous(), sh[:, 1:, :].contiguous()


def _accel_forward(inp, dc, rest, device):
    from gaussian_splatting_amd import _C

    d = lambda k: C._dev(inp[k], device)  # noqa: E731
    return _C.rasterize_gaussians(
        d("bg"), d("means3D"), d("colors_precomp"), d("opacities"), d("scales"), d("rotations"),
        inp["scale_modifier"], d("cov3D_precomp"), d("viewmatrix"), d("projmatrix"), inp["tanfovx"],
        inp["tanfovy"], inp["H"], inp["W"], dc, rest, inp["sh_degree"], d("campos"), False,
        inp["antialiasing"], False)


def _accel_backward(inp, fwd, dc, rest, gc, gd, device):
    from gaussian_splatting_amd import _C

    d = lambda k: C._dev(inp[k], device)  # noqa: E731
    nr, color, radii, geom, binning, img, invd = fwd
    return _C.rasterize_gaussians_backward(
        d("bg"), d("means3D"), radii, d("colors_precomp"), d("opacities"), d("scales"), d("rotations"),
        inp["scale_modifier"], d("cov3D_precomp"), d("viewmatrix"), d("projmatrix"), inp["tanfovx"],
        inp["tanfovy"], gc.to(device), gd.to(device), dc, rest, inp["sh_degree"], d("campos"), geom, nr, binning,
        img, inp["antialiasing"], False)


def test_arity_is_checked():
    from gaussian_splatting_amd import _C

    with pytest.raises(TypeError, match="20 or 21"):
        _C.rasterize_gaussians(*([None] * 19))
    with pytest.raises(TypeError, match="24 or 25"):
        _C.rasterize_gaussians_backward(*([None] * 23))


def test_dropin_exports_sparse_adam():
    import diff_gaussian_rasterization as dgr

    assert hasattr(dgr, "SparseGaussianAdam")  # train.py:41-45 then selects separate_sh=True
    assert hasattr(dgr._C, "adamUpdate")


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=lambda c: c.name)
@pytest.mark.record_path
def test_split_equals_combined_bitwise(case):
    dev = "cuda"
    inp = C.build(case)
    gc, gd = C.unit_grads(case.H, case.W)
    comb = C.run_gpu_forward(inp, device=dev)
    comb_g = C.run_gpu_backward(inp, comb, gc, gd, device=dev)
    dc, rest = _split(inp, dev)
    sep = _accel_forward(inp, dc, rest, dev)
    sep_g = _accel_backward(inp, sep, dc, rest, gc, gd, dev)
    torch.cuda.synchronize()
    assert sep[0] == comb[0]
    for i in (1, 2, 6):  # color, radii, invdepth
        assert torch.equal(sep[i], comb[i]), i
    assert len(sep_g) == 9 and len(comb_g) == 8
    names = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D"]
    for k, name in enumerate(names):
        assert torch.equal(sep_g[k], comb_g[k]), name
    assert tuple(sep_g[5].shape) == (case.P, 1, 3)
    assert tuple(sep_g[6].shape) == (case.P, rest.size(1), 3)
    assert torch.equal(sep_g[5], comb_g[5][:, :1]), "dL_ddc"
    assert torch.equal(sep_g[6], comb_g[5][:, 1:]), "dL_dsh (rest)"
    assert torch.equal(sep_g[7], comb_g[6]) and torch.equal(sep_g[8], comb_g[7])
    # and the oracle on the concatenated coefficients (the combined path's own parity contract)
    ref = C.run_oracle(inp)
    assert sep[0] == ref.num_rendered
    assert float(np.abs(sep[1].cpu().numpy() - ref.color).max()) <= 1e-5


@pytest.mark.gpu
@pytest.mark.record_path
def test_rasterizer_module_separate_sh_autograd():
    """GaussianRasterizer(dc=..., shs=...) as gaussian_renderer/__init__.py:115-125 calls it: gradients land on
    dc and shs, equal to the combined path's split gradient."""
    from gaussian_splatting_amd.rasterizer import GaussianRasterizationSettings, GaussianRasterizer

    case = C.Case("module", P=400, W=64, H=48)
    inp = C.build(case)
    dev = "cuda"
    s = GaussianRasterizationSettings(
        image_height=case.H, image_width=case.W, tanfovx=inp["tanfovx"], tanfovy=inp["tanfovy"],
        bg=inp["bg"].to(dev), scale_modifier=1.0, viewmatrix=inp["viewmatrix"].to(dev),
        projmatrix=inp["projmatrix"].to(dev), sh_degree=3, campos=inp["campos"].to(dev), prefiltered=False,
        debug=False, antialiasing=False)
    r = GaussianRasterizer(s)

    def leaf(t):
        return t.to(dev).clone().requires_grad_(True)

    means, opac, sc, rot = (leaf(inp[k]) for k in ("means3D", "opacities", "scales", "rotations"))
    sh = leaf(inp["shs"])
    m2d = torch.zeros_like(means, requires_grad=True)
    img, radii, depth = r(means3D=means, means2D=m2d, opacities=opac, shs=sh, scales=sc, rotations=rot)
    (img.sum() + depth.sum()).backward()
    g_comb = [t.grad.clone() for t in (means, m2d, opac, sc, rot, sh)]

    means2, opac2, sc2, rot2 = (leaf(inp[k]) for k in ("means3D", "opacities", "scales", "rotations"))
    dc, rest = leaf(inp["shs"][:, :1]), leaf(inp["shs"][:, 1:])
    m2d2 = torch.zeros_like(means2, requires_grad=True)
    img2, radii2, depth2 = r(means3D=means2, means2D=m2d2, dc=dc, shs=rest, colors_precomp=None,
                             opacities=opac2, scales=sc2, rotations=rot2, cov3D_precomp=None)
    (img2.sum() + depth2.sum()).backward()
    assert torch.equal(img, img2) and torch.equal(radii, radii2) and torch.equal(depth, depth2)
    for a, b in zip(g_comb[:5], (means2, m2d2, opac2, sc2, rot2)):
        assert torch.equal(a, b.grad)
    assert torch.equal(g_comb[5][:, :1], dc.grad) and torch.equal(g_comb[5][:, 1:], rest.grad)


@pytest.mark.gpu
def test_accel_precomputed_colours_zero_dc_grad():
    case = C.Case("precomp", P=200, W=48, H=40, mode_color="precomp")
    inp = C.build(case)
    dev = "cuda"
    empty = torch.Tensor([])
    fwd = _accel_forward(inp, empty, empty, dev)
    comb = C.run_gpu_forward(inp, device=dev)
    assert torch.equal(fwd[1], comb[1])
    gc, gd = C.unit_grads(case.H, case.W)
    g = _accel_backward(inp, fwd, empty, empty, gc, gd, dev)
    assert len(g) == 9
    assert tuple(g[5].shape) == (case.P, 1, 3) and not g[5].any()
