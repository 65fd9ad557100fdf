"""The oracle and the host-side conventions against the golden vectors (CPU, no GPU needed).

Reference vectors (tests/golden/make_golden.py, produced by the reference's own Python):
camera matrices, the SH polynomial as used by the renderer's convert_SHs_python switch, and
the L1 loss gradient.  Rasterizer vectors: the float64 oracle's outputs, which the oracle
must keep reproducing (in f64 and in f32) -- the GPU tests compare the HIP path with them.
"""
import os

import numpy as np
import pytest
import torch

from tests import common as C
from tests import torch_ref as TR
from gaussian_splatting_amd import synthetic as syn

GOLDEN = C.GOLDEN


def _npz(name):
    return np.load(os.path.join(GOLDEN, name))


# ---------------------------------------------------------------------------- reference vectors
@pytest.mark.parametrize("tag", ["", "_mod"])
def test_cov3d_matches_reference_get_covariance(tag):
    """The oracle's computeCov3D (CR/forward.cu:149-190), fed the normalised quaternion the rasterizer gets
    (get_rotation), equals the reference's own GaussianModel.get_covariance (build_scaling_rotation +
    strip_symmetric on the raw quaternion) to float32 rounding; so does tests/common.py's restatement."""
    from oracle import oracle

    z = _npz("cov3d.npz")
    mod = float(z["modifier" + tag])
    exp = z["cov3D" + tag]
    scale = np.abs(exp).max(1, keepdims=True)
    got = oracle.cov3d(z["scales"], z["rotations"], mod)
    assert float((np.abs(got - exp) / scale).max()) <= 1e-6
    res = C.cov3d_reference(torch.tensor(z["scales"]) * mod, torch.tensor(z["raw_rotations"])).numpy()
    assert float((np.abs(res - exp) / scale).max()) <= 1e-6
    # the quaternion convention: build_rotation's matrix is the one the oracle's cov3D is made of
    R = z["R"]
    S = z["scales"] * mod
    M = R * S[:, None, :]
    full = M @ M.transpose(0, 2, 1)
    tri = np.stack([full[:, 0, 0], full[:, 0, 1], full[:, 0, 2], full[:, 1, 1], full[:, 1, 2], full[:, 2, 2]], 1)
    np.testing.assert_allclose(tri, exp, rtol=1e-5, atol=1e-9)


def test_camera_matrices_match_reference():
    """syn.world2view / syn.projection / make_camera follow getWorld2View2 + getProjectionMatrix composed as
    scene/cameras.py:86-89 (transposed view, full projection = view @ proj^T, campos = inverse(view)[3,:3])."""
    z = _npz("camera.npz")
    i = 0
    while f"cam{i}_inputs" in z.files:
        W, H, f, yaw, fovx, fovy = z[f"cam{i}_inputs"]
        wv = torch.tensor(syn.world2view(z[f"cam{i}_R"], z[f"cam{i}_T"])).transpose(0, 1)
        np.testing.assert_allclose(wv.numpy(), z[f"cam{i}_viewmatrix"], rtol=0, atol=2e-6)
        pm = torch.tensor(syn.projection(syn.ZNEAR, syn.ZFAR, fovx, fovy)).transpose(0, 1)
        full = (wv.unsqueeze(0).bmm(pm.unsqueeze(0))).squeeze(0)
        np.testing.assert_allclose(full.numpy(), z[f"cam{i}_projmatrix"], rtol=1e-6, atol=1e-6)
        cam = syn.make_camera(int(W), int(H), float(f), float(yaw))
        np.testing.assert_allclose(cam.viewmatrix.numpy(), z[f"cam{i}_viewmatrix"], rtol=0, atol=2e-6)
        np.testing.assert_allclose(cam.projmatrix.numpy(), z[f"cam{i}_projmatrix"], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(cam.campos.numpy(), z[f"cam{i}_campos"], rtol=0, atol=1e-5)
        assert abs(cam.tanfovx - np.tan(fovx / 2)) < 1e-12 and abs(cam.tanfovy - np.tan(fovy / 2)) < 1e-12
        i += 1
    assert i >= 3


def _sh_inputs(z, deg, precomp):
    W, H, tx, ty = z["camera"]
    inp = dict(bg=torch.zeros(3), means3D=torch.from_numpy(z["means3D"]), opacities=torch.from_numpy(z["opacities"]),
               shs=None if precomp else torch.from_numpy(z["features"]), sh_degree=deg,
               colors_precomp=torch.from_numpy(z[f"colors_deg{deg}"]) if precomp else None,
               scales=torch.from_numpy(z["scales"]), rotations=torch.from_numpy(z["rotations"]), cov3D_precomp=None,
               viewmatrix=torch.from_numpy(z["viewmatrix"]), projmatrix=torch.from_numpy(z["projmatrix"]),
               campos=torch.from_numpy(z["campos"]), tanfovx=float(tx), tanfovy=float(ty), H=int(H), W=int(W),
               scale_modifier=1.0, antialiasing=False)
    return inp


@pytest.mark.parametrize("deg", [0, 1, 2, 3])
def test_sh_colours_match_reference_eval_sh(deg):
    """The in-rasterizer SH evaluation (computeColorFromSH, CR/forward.cu:22-80) equals the reference's
    convert_SHs_python path (gaussian_renderer/__init__.py:86-96 over utils/sh_utils.eval_sh): the same
    image whether colours come from shs= or colors_precomp=."""
    z = _npz("sh_eval.npz")
    # the torch restatement's polynomial, directly
    means, campos = torch.from_numpy(z["means3D"]).double(), torch.from_numpy(z["campos"]).double()
    d = torch.nn.functional.normalize(means - campos[None], dim=1)
    rgb = torch.clamp_min(TR.eval_sh(deg, torch.from_numpy(z["features"]).double(), d) + 0.5, 0.0)
    np.testing.assert_allclose(rgb.numpy(), z[f"colors_deg{deg}"], rtol=0, atol=2e-6)
    # the oracle, both precisions
    for prec, tol in (("f64", 2e-6), ("f32", 5e-6)):
        a = C.run_oracle(_sh_inputs(z, deg, precomp=False), precision=prec)
        b = C.run_oracle(_sh_inputs(z, deg, precomp=True), precision=prec)
        assert a.num_rendered == b.num_rendered > 0
        np.testing.assert_array_equal(a.radii, b.radii)
        np.testing.assert_allclose(a.color, b.color, rtol=0, atol=tol)


def test_rgb2sh_constant():
    z = _npz("sh_eval.npz")
    np.testing.assert_allclose((z["rgb2sh_in"] - 0.5) / TR.SH_C0, z["rgb2sh_out"], rtol=1e-6, atol=1e-7)


def test_l1_upstream_gradient_convention():
    """dL/dimage of l1_loss (utils/loss_utils.py:16-19) is sign(image - gt) / numel -- the form of the
    synthetic upstream gradient the benchmark and the tests use (synthetic.upstream_grads)."""
    z = _npz("l1_grad.npz")
    img, gt = z["image"], z["gt"]
    np.testing.assert_allclose(np.sign(img - gt) / img.size, z["grad"], rtol=1e-6, atol=0)
    np.testing.assert_allclose(np.abs(img - gt).mean(), z["loss"], rtol=1e-6)
    gc, _ = syn.upstream_grads(12, 10)
    assert set(np.unique(np.abs(gc.numpy()) * gc.numel()).round(5)) == {1.0}


def test_cov3d_precomp_switch():
    """compute_cov3D_python (gaussian_renderer/__init__.py:97-104 with GaussianModel.get_covariance,
    scene/gaussian_model.py:34-42) gives the same image as in-rasterizer computeCov3D."""
    case = C.Case("cov_switch", P=200, W=64, H=48, scale_modifier=0.8)
    a_inp = C.build(case)
    b_inp = dict(a_inp, cov3D_precomp=C.cov3d_reference(a_inp["scales"] * 0.8, a_inp["rotations"]), scales=None,
                 rotations=None)
    for prec, tol in (("f64", 1e-6), ("f32", 1e-5)):
        a, b = C.run_oracle(a_inp, prec), C.run_oracle(b_inp, prec)
        assert a.num_rendered == b.num_rendered
        np.testing.assert_allclose(a.color, b.color, rtol=0, atol=tol)


# ---------------------------------------------------------------------------- rasterizer vectors
@pytest.mark.parametrize("name", C.RASTER_FIXTURES)
def test_oracle_reproduces_raster_fixture(name):
    inp, exp, grads = C.load_raster(name)
    for prec, tol in (("f64", 2e-7), ("f32", 1e-5)):
        r = C.run_oracle(inp, precision=prec, nthreads=min(8, os.cpu_count() or 1))
        assert abs(r.num_rendered - exp["num_rendered"]) <= (0 if prec == "f64" else 2)
        assert (r.radii != exp["radii"]).sum() <= (0 if prec == "f64" else 2)
        d = np.abs(r.color - exp["color"])
        assert (d <= tol).mean() >= (1.0 if prec == "f64" else 0.999), (prec, d.max())
        if grads is None:
            continue
        g = r.handle.backward(grads[0].numpy(), grads[1].numpy())
        for k in C.GRAD_NAMES:
            err = C.rel_err(g[k], exp[k])
            assert err <= (1e-6 if prec == "f64" else 2e-3), (prec, k, err)
