"""Shared helpers for the parity tests: small seeded scenes, the oracle call and the
GPU call with the same arguments, and comparison utilities."""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch

from gaussian_splatting_amd import synthetic as syn


@dataclass
class Case:
    """One rasterizer invocation, in the positional vocabulary of _C.rasterize_gaussians."""

    name: str
    P: int
    W: int
    H: int
    focal: float = 60.0
    sh_degree: int = 3
    M: Optional[int] = None  # SH coefficients stored (default (max degree 3 + 1)^2 = 16)
    mode_color: str = "sh"  # "sh" | "precomp"
    mode_cov: str = "scalerot"  # "scalerot" | "precomp"
    antialiasing: bool = False
    bg: tuple = (0.0, 0.0, 0.0)
    scale_modifier: float = 1.0
    yaw: float = 0.0
    seed: int = 0
    scale_range: tuple = (0.02, 0.25)
    z_range: tuple = (2.0, 8.0)
    opacity_std: float = 1.5
    extra: dict = field(default_factory=dict)


def build(case: Case):
    """Inputs as torch CPU float32 tensors (scene + camera + settings)."""
    cam = syn.make_camera(case.W, case.H, case.focal, case.yaw)
    base = syn.make_camera(case.W, case.H, case.focal, 0.0)
    sc = syn.make_scene(case.P, base, sh_degree=3, seed=case.seed, scale_range=case.scale_range,
                        opacity_std=case.opacity_std, z_range=case.z_range)
    M = case.M if case.M is not None else 16
    shs = sc.shs[:, :M, :].contiguous()
    inp = dict(
        bg=torch.tensor(case.bg, dtype=torch.float32),
        means3D=sc.means3D, opacities=sc.opacities, shs=shs, sh_degree=case.sh_degree,
        scales=sc.scales, rotations=sc.rotations, colors_precomp=None, cov3D_precomp=None,
        viewmatrix=cam.viewmatrix, projmatrix=cam.projmatrix, campos=cam.campos,
        tanfovx=cam.tanfovx, tanfovy=cam.tanfovy, H=case.H, W=case.W, scale_modifier=case.scale_modifier,
        antialiasing=case.antialiasing,
    )
    if case.mode_color == "precomp":
        g = torch.Generator().manual_seed(case.seed + 7)
        inp["colors_precomp"] = torch.rand(case.P, 3, generator=g)
        inp["shs"] = None
    if case.mode_cov == "precomp":
        inp["cov3D_precomp"] = cov3d_reference(sc.scales * case.scale_modifier, sc.rotations)
        inp["scales"] = None
        inp["rotations"] = None
    return inp


def cov3d_reference(s: torch.Tensor, r: torch.Tensor) -> torch.Tensor:
    """build_scaling_rotation + strip_symmetric (utils/general_utils.py:78-110), restated on CPU."""
    q = torch.nn.functional.normalize(r, dim=1)
    w, x, y, z = q.unbind(1)
    R = torch.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
        2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
        2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], 1).reshape(-1, 3, 3)
    L = R * s[:, None, :]
    S = L @ L.transpose(1, 2)
    return torch.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1], S[:, 1, 2], S[:, 2, 2]], 1).contiguous()


def run_oracle(inp, precision="f32", nthreads=1):
    from oracle import oracle

    return oracle.forward(
        inp["means3D"], inp["opacities"], inp["viewmatrix"], inp["projmatrix"], inp["campos"], inp["tanfovx"],
        inp["tanfovy"], inp["H"], inp["W"], bg=inp["bg"], shs=inp["shs"], sh_degree=inp["sh_degree"],
        colors_precomp=inp["colors_precomp"], scales=inp["scales"], rotations=inp["rotations"],
        cov3D_precomp=inp["cov3D_precomp"], scale_modifier=inp["scale_modifier"],
        antialiasing=inp["antialiasing"], precision=precision, nthreads=nthreads)


def _dev(t, device):
    return torch.Tensor([]) if t is None else t.to(device)


def run_gpu_forward(inp, device="cuda", prefiltered=False, debug=False):
    from gaussian_splatting_amd import _C

    d = lambda k: _dev(inp[k], device)  # noqa: E731
    return _C.rasterize_gaussians(
        d("bg"), d("means3D"), d("colors_precomp"), d("opacities"), d("scales"), d("rotations"),
        inp["scale_modifier"], d("cov3D_precomp"), d("viewmatrix"), d("projmatrix"), inp["tanfovx"],
        inp["tanfovy"], inp["H"], inp["W"], d("shs"), inp["sh_degree"], d("campos"), prefiltered,
        inp["antialiasing"], debug)


def run_gpu_backward(inp, fwd, grad_color, grad_invdepth, device="cuda", debug=False, out=None):
    from gaussian_splatting_amd import _C

    d = lambda k: _dev(inp[k], device)  # noqa: E731
    num_rendered, color, radii, geom, binning, img, invdepth = fwd
    gi = torch.Tensor([]) if grad_invdepth is None else grad_invdepth.to(device)
    return _C.rasterize_gaussians_backward(
        d("bg"), d("means3D"), radii, d("colors_precomp"), d("opacities"), d("scales"), d("rotations"),
        inp["scale_modifier"], d("cov3D_precomp"), d("viewmatrix"), d("projmatrix"), inp["tanfovx"],
        inp["tanfovy"], grad_color.to(device), gi, d("shs"), inp["sh_degree"], d("campos"), geom, num_rendered,
        binning, img, inp["antialiasing"], debug, out=out)


GRAD_NAMES = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
              "dL_drotations"]


def rel_err(a: np.ndarray, b: np.ndarray) -> float:
    """max |a-b| / max(|b|, tiny): a scale-free error for gradient tensors."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    if a.size == 0:
        return 0.0
    den = max(np.abs(b).max(), 1e-30)
    return float(np.abs(a - b).max() / den)


def unit_grads(H, W, seed=3):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(3, H, W, generator=g), torch.randn(1, H, W, generator=g)


def l1_grads(H, W, seed=3):
    return syn.upstream_grads(H, W, seed)


SMALL_CASES = [
    Case("sh3_scalerot", P=300, W=64, H=48),
    Case("ragged_37x23", P=120, W=37, H=23, focal=30.0),
    Case("sh1_of_16", P=250, W=64, H=64, sh_degree=1),
    Case("sh0_M1", P=250, W=48, H=40, sh_degree=0, M=1),
    Case("sh2_M9", P=250, W=48, H=40, sh_degree=2, M=9),
    Case("colors_precomp", P=300, W=64, H=48, mode_color="precomp"),
    Case("cov3d_precomp", P=300, W=64, H=48, mode_cov="precomp"),
    Case("antialiasing", P=300, W=64, H=48, antialiasing=True),
    Case("background", P=200, W=64, H=48, bg=(0.2, 0.5, 0.9)),
    Case("scale_modifier", P=200, W=64, H=48, scale_modifier=0.7),
    Case("yawed_view", P=300, W=64, H=48, yaw=15.0),
    Case("dense_opaque", P=2000, W=64, H=64, opacity_std=3.0, scale_range=(0.05, 0.3)),
    # tile lists past one wave's sort (binning.hip K4 classes): (1024, 2048], (2048, 4096], (4096, 8192],
    # > 8192 entries
    Case("lists_1k_2k", P=1800, W=32, H=32, scale_range=(0.1, 0.4)),
    Case("lists_2k_4k", P=5000, W=32, H=32, scale_range=(0.1, 0.4)),
    Case("lists_4k_8k", P=10000, W=32, H=32, scale_range=(0.1, 0.4)),
    Case("lists_over_8k", P=10000, W=16, H=16, scale_range=(0.1, 0.4)),
]


GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
RASTER_FIXTURES = sorted(f[len("raster_"):-len(".npz")] for f in os.listdir(GOLDEN)
                         if f.startswith("raster_") and f.endswith(".npz"))


def load_raster(name):
    """A rasterizer golden vector (tests/golden/make_golden.py): (inp, expected, (grad_color, grad_invdepth))."""
    z = np.load(os.path.join(GOLDEN, f"raster_{name}.npz"))
    inp = dict(bg=None, means3D=None, opacities=None, shs=None, sh_degree=0, scales=None, rotations=None,
               colors_precomp=None, cov3D_precomp=None)
    for k in z.files:
        if k.startswith("in_"):
            v = z[k]
            inp[k[3:]] = torch.from_numpy(v.copy()) if v.ndim > 0 else v.item()
    for k in ("H", "W", "sh_degree"):
        inp[k] = int(inp[k])
    for k in ("tanfovx", "tanfovy", "scale_modifier"):
        inp[k] = float(inp[k])
    inp["antialiasing"] = bool(inp["antialiasing"])
    exp = {k[4:]: z[k] for k in z.files if k.startswith("out_")}
    exp["num_rendered"] = int(exp["num_rendered"])
    grads = None
    if "grad_color" in z.files:
        grads = (torch.from_numpy(z["grad_color"].copy()), torch.from_numpy(z["grad_invdepth"].copy()))
    return inp, exp, grads
