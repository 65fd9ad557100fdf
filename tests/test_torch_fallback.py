"""The pure-PyTorch CPU fallback rasterizer (oracle/torch_fallback.py) -- north_star's CPU
baseline and BASELINE.json configs[0] ("10k random Gaussians, 256x256, SH degree 0, forward-only
via PyTorch CPU fallback") -- against the C oracle (oracle/gsr_oracle.c) on the same inputs.

CPU only.  Bars: integers (num_rendered, radii, n_contrib) identical; colour / inverse depth / final T
within 1e-5 abs; gradients with a unit upstream gradient within 1e-4 relative (Frobenius).  In the
antialiasing case only the gradients the AA chain does not touch are compared (colours, SH, means2D):
the reference's AA gradient formula (CR/backward.cu:256-270) is not the derivative of its forward, so
autograd of the fallback legitimately differs in opacity / cov3D / scales / rotations / means3D."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from gaussian_splatting_amd import synthetic as syn
from oracle import torch_fallback as tf
from tests import common as C


def _fallback(inp, gc=None, gd=None, **kw):
    return tf.rasterize(inp["means3D"], inp["opacities"], inp["viewmatrix"], inp["projmatrix"], inp["campos"],
                        inp["tanfovx"], inp["tanfovy"], inp["H"], inp["W"], bg=inp["bg"], shs=inp["shs"],
                        sh_degree=inp["sh_degree"], colors_precomp=inp["colors_precomp"], scales=inp["scales"],
                        rotations=inp["rotations"], cov3D_precomp=inp["cov3D_precomp"],
                        scale_modifier=inp["scale_modifier"], antialiasing=inp["antialiasing"], dL_dcolor=gc,
                        dL_dinvdepth=gd, **kw)


def _check_forward(res, ref):
    assert res["num_rendered"] == ref.num_rendered
    np.testing.assert_array_equal(res["radii"].numpy(), ref.radii)
    img = ref.handle.image()
    np.testing.assert_array_equal(res["n_contrib"].numpy(), img["n_contrib"])
    assert np.abs(res["color"].numpy() - ref.color).max() <= 1e-5
    assert np.abs(res["invdepth"].numpy() - ref.invdepth).max() <= 1e-5
    assert np.abs(res["final_T"].numpy() - img["final_T"]).max() <= 1e-5


def test_config1_forward_10k_256_sh0():
    """BASELINE.json configs[0]: the forward-only CPU plumbing case, full frame."""
    scene, cam = syn.config_scene("10k_256_sh0", seed=0)
    inp = dict(bg=torch.zeros(3), means3D=scene.means3D, opacities=scene.opacities, shs=scene.shs, sh_degree=0,
               scales=scene.scales, rotations=scene.rotations, colors_precomp=None, cov3D_precomp=None,
               viewmatrix=cam.viewmatrix, projmatrix=cam.projmatrix, campos=cam.campos, tanfovx=cam.tanfovx,
               tanfovy=cam.tanfovy, H=cam.height, W=cam.width, scale_modifier=1.0, antialiasing=False)
    res = _fallback(inp)
    assert "grads" not in res and res["num_rendered"] > 10_000
    _check_forward(res, C.run_oracle(inp, nthreads=4))


@pytest.mark.parametrize("case", [c for c in C.SMALL_CASES if c.P <= 2000], ids=lambda c: c.name)
def test_forward_backward_matches_oracle(case):
    inp = C.build(case)
    gc, gd = C.unit_grads(case.H, case.W)
    res = _fallback(inp, gc, gd)
    ref = C.run_oracle(inp)
    _check_forward(res, ref)
    rg = ref.handle.backward(gc, gd)
    names = ("dL_dmeans2D", "dL_dcolors", "dL_dsh") if case.antialiasing else C.GRAD_NAMES
    for k in names:
        got, exp = res["grads"][k].numpy(), rg[k]
        err = np.linalg.norm(got - exp) / max(np.linalg.norm(exp), 1e-30)
        assert err <= 1e-4, (k, err)


def test_rounds_cross_256_entries():
    """Lists longer than one 256-entry round: the transmittance and the autograd state carry over."""
    case = next(c for c in C.SMALL_CASES if c.name == "lists_1k_2k")
    inp = C.build(case)
    gc, gd = C.unit_grads(case.H, case.W)
    res = _fallback(inp, gc, gd)
    ref = C.run_oracle(inp)
    _check_forward(res, ref)
    rg = ref.handle.backward(gc, gd)
    for k in ("dL_dmeans2D", "dL_dopacity", "dL_dcolors"):
        err = np.linalg.norm(res["grads"][k].numpy() - rg[k]) / np.linalg.norm(rg[k])
        assert err <= 1e-4, (k, err)


def test_tile_sample_renders_a_subset():
    """The bounded timing mode (bench.py cpu_baseline) renders every k-th tile only."""
    case = C.Case("sample", P=600, W=96, H=64)
    inp = C.build(case)
    full = _fallback(inp)
    half = _fallback(inp, tile_fraction=0.5)
    none = _fallback(inp, tile_fraction=0.0)
    assert full["rendered_instances"] == full["num_rendered"]
    assert 0 < half["rendered_instances"] < full["rendered_instances"]
    assert none["rendered_instances"] == 0
    assert set(full["timings"]) == {"preprocess", "binning", "render", "preprocess_backward"}


@pytest.mark.parametrize("cfg", ["500k_1080p_sh3", "1m_1080p_sh3"])
def test_fullsize_integers_match_oracle(cfg):
    """The CPU baseline's workload is the GPU's: at BASELINE's full 1080p sizes the fallback's radii, tile
    rectangles (hence num_rendered) and sorted tile lists equal the f32 C oracle's, which the GPU's equal
    (test_gpu_fullsize.py).  (The focal length is formed in float32 as the reference forms it; a double
    quotient rounded once moved two radii and 6 instances at 1M.)"""
    scene, cam = syn.config_scene(cfg, seed=0)
    with torch.no_grad():
        pre = tf.preprocess(scene.means3D, scene.opacities, cam.viewmatrix, cam.projmatrix, cam.campos, cam.tanfovx,
                            cam.tanfovy, cam.height, cam.width, shs=scene.shs, sh_degree=scene.sh_degree,
                            scales=scene.scales, rotations=scene.rotations)
        point_list, starts, counts = tf.binning(pre)
    inp = dict(bg=torch.zeros(3), means3D=scene.means3D, opacities=scene.opacities, shs=scene.shs,
               sh_degree=scene.sh_degree, scales=scene.scales, rotations=scene.rotations, colors_precomp=None,
               cov3D_precomp=None, viewmatrix=cam.viewmatrix, projmatrix=cam.projmatrix, campos=cam.campos,
               tanfovx=cam.tanfovx, tanfovy=cam.tanfovy, H=cam.height, W=cam.width, scale_modifier=1.0,
               antialiasing=False)
    ref = C.run_oracle(inp, nthreads=8)
    np.testing.assert_array_equal(pre["radii"].numpy(), ref.radii.astype(np.int64))
    assert int(counts.sum()) == ref.num_rendered
    rb = ref.handle.binning()
    np.testing.assert_array_equal(point_list.numpy(), rb["point_list"].astype(np.int64))
    er = rb["ranges"].astype(np.int64)
    np.testing.assert_array_equal(counts.numpy(), er[:, 1] - er[:, 0])
