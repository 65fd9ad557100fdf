"""Known-answer cases of the reference's blending rule (CR/forward.cu:367-513), on the oracle.
CPU only; the GPU path is held to the same cases in tests/test_gpu_parity.py.
"""
import math

import numpy as np
import torch

from tests import common as C
from gaussian_splatting_amd import synthetic as syn


def _scene(means, colors, opac, cov, W=32, H=32, focal=40.0, bg=(0.0, 0.0, 0.0)):
    cam = syn.make_camera(W, H, focal)
    P = means.shape[0]
    return dict(bg=torch.tensor(bg, dtype=torch.float32), means3D=means.float(), opacities=opac.float().reshape(P, 1),
                shs=None, sh_degree=0, scales=None, rotations=None, colors_precomp=colors.float(),
                cov3D_precomp=cov.float(), viewmatrix=cam.viewmatrix, projmatrix=cam.projmatrix, campos=cam.campos,
                tanfovx=cam.tanfovx, tanfovy=cam.tanfovy, H=H, W=W, scale_modifier=1.0, antialiasing=False)


def _pixel_center_mean(px, py, z, W=32, H=32, focal=40.0):
    """World point (camera at origin looking +z) that projects exactly onto pixel (px, py)."""
    x = (px - (W - 1) / 2.0) / focal * z
    y = (py - (H - 1) / 2.0) / focal * z
    return torch.tensor([[x, y, z]], dtype=torch.float64)


def test_single_gaussian_at_pixel_centre():
    """power = 0 at the centre pixel: alpha = min(0.99, o); C = c alpha + (1 - alpha) bg."""
    for o in (0.5, 0.999):
        bg = (0.1, 0.2, 0.3)
        inp = _scene(_pixel_center_mean(10, 12, 4.0), torch.tensor([[0.9, 0.4, 0.2]]), torch.tensor([o]),
                     torch.tensor([[1e-3, 0, 0, 1e-3, 0, 1e-3]]), bg=bg)
        r = C.run_oracle(inp, precision="f64")
        a = min(0.99, o)
        exp = np.array([0.9, 0.4, 0.2]) * a + (1 - a) * np.array(bg)
        np.testing.assert_allclose(r.color[:, 12, 10], exp, rtol=0, atol=1e-5)
        np.testing.assert_allclose(r.invdepth[0, 12, 10], a / 4.0, rtol=1e-5)
        assert r.handle.image()["n_contrib"][12, 10] == 1


def test_alpha_below_threshold_gives_background():
    """o * G < 1/255 everywhere: the Gaussian is skipped and every pixel shows the background."""
    bg = (0.25, 0.5, 0.75)
    inp = _scene(_pixel_center_mean(16, 16, 4.0), torch.tensor([[1.0, 1.0, 1.0]]), torch.tensor([1.0 / 300.0]),
                 torch.tensor([[1e-2, 0, 0, 1e-2, 0, 1e-2]]), bg=bg)
    r = C.run_oracle(inp, precision="f64")
    assert r.num_rendered > 0
    np.testing.assert_allclose(r.color, np.broadcast_to(np.array(bg)[:, None, None], r.color.shape), atol=0)
    assert (r.invdepth == 0).all()


def test_opaque_stack_terminates_early():
    """Ten co-located opaque Gaussians: T goes 1, 0.01, 1e-4 ... the third would make T < 1e-4, so the pixel
    stops after two contributors (the third is not added) and the rest are never visited."""
    P = 10
    means = _pixel_center_mean(8, 8, 3.0).repeat(P, 1)
    means[:, 2] += torch.arange(P, dtype=torch.float64) * 0.01  # strictly increasing depth
    means[:, :2] *= (means[:, 2:3] / 3.0)  # keep them on the same pixel ray
    cols = torch.rand(P, 3, generator=torch.Generator().manual_seed(0))
    inp = _scene(means, cols, torch.full((P,), 0.999), torch.tensor([[1e-3, 0, 0, 1e-3, 0, 1e-3]]).repeat(P, 1))
    r = C.run_oracle(inp, precision="f64")
    img = r.handle.image()
    assert img["n_contrib"][8, 8] == 2
    exp = cols[0].double().numpy() * 0.99 + cols[1].double().numpy() * 0.99 * 0.01
    np.testing.assert_allclose(r.color[:, 8, 8], exp, rtol=0, atol=1e-6)
    np.testing.assert_allclose(img["final_T"][8, 8], 0.01 * 0.01, rtol=1e-6)


def test_culled_behind_near_plane():
    """view-space z <= 0.2 (in_frustum, CR/auxiliary.h:164-190): radius 0, nothing rendered."""
    inp = _scene(torch.tensor([[0.0, 0.0, 0.15]], dtype=torch.float64), torch.tensor([[1.0, 0, 0]]),
                 torch.tensor([0.9]), torch.tensor([[1e-3, 0, 0, 1e-3, 0, 1e-3]]))
    r = C.run_oracle(inp, precision="f64")
    assert r.radii[0] == 0 and r.num_rendered == 0 and (r.color == 0).all()


def test_radius_is_three_sigma_ceiling():
    """radius = ceil(3 sqrt(lambda_max)) of the dilated 2-D covariance (CR/forward.cu:314-318)."""
    z, s2, focal = 4.0, 0.01, 40.0
    inp = _scene(_pixel_center_mean(16, 16, z), torch.tensor([[1.0, 1, 1]]), torch.tensor([0.9]),
                 torch.tensor([[s2, 0, 0, s2, 0, s2]]), focal=focal)
    r = C.run_oracle(inp, precision="f64")
    lam = (focal / z) ** 2 * s2 + 0.3  # isotropic: J W Sigma W^T J^T = (f/z)^2 s2 I (+ tiny off-centre terms)
    assert r.radii[0] == math.ceil(3 * math.sqrt(lam))
