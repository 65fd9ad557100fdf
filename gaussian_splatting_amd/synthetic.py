"""Synthetic scenes and cameras for the benchmark and the tests.

Camera matrices restate the reference's conventions (``utils/graphics_utils.py:38-71``,
``scene/cameras.py:86-89``):

* ``viewmatrix``  = ``getWorld2View2(R, T)^T``  (the tensor the rasterizer reads as
  16 floats in column-major order),
* ``projmatrix``  = ``viewmatrix @ getProjectionMatrix(...)^T``,
* ``campos``      = ``inverse(viewmatrix)[3, :3]``.

Gaussians mirror the reference's random initialisation (uniform points,
``scene/dataset_readers.py:290-296``) with post-activation scales, rotations and
opacities, exactly as ``GaussianModel.get_*`` hand them to the rasterizer.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

ZNEAR = 0.01  # scene/cameras.py:80-81
ZFAR = 100.0


def world2view(R: np.ndarray, t: np.ndarray) -> np.ndarray:
    """World-to-camera 4x4 [R^T | t] (COLMAP convention, utils/graphics_utils.py:38-49 with translate=0, scale=1)."""
    Rt = np.zeros((4, 4))
    Rt[:3, :3] = R.transpose()
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    return Rt.astype(np.float32)


def projection(znear: float, zfar: float, fovx: float, fovy: float) -> np.ndarray:
    """OpenGL-style perspective with z in [0, 1] (utils/graphics_utils.py:51-71)."""
    tan_y, tan_x = math.tan(fovy / 2), math.tan(fovx / 2)
    top, right = tan_y * znear, tan_x * znear
    bottom, left = -top, -right
    P = np.zeros((4, 4), np.float32)
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = 1.0
    P[2, 2] = zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


@dataclass
class Camera:
    width: int
    height: int
    tanfovx: float
    tanfovy: float
    viewmatrix: torch.Tensor  # [4,4] float32
    projmatrix: torch.Tensor  # [4,4] float32
    campos: torch.Tensor  # [3] float32

    def to(self, device) -> "Camera":
        return Camera(self.width, self.height, self.tanfovx, self.tanfovy, self.viewmatrix.to(device),
                      self.projmatrix.to(device), self.campos.to(device))


def make_camera(width: int, height: int, focal: float, yaw_deg: float = 0.0, pivot_z: float = 7.0) -> Camera:
    """Pinhole camera looking down +z; ``yaw_deg`` rotates it about +y around (0, 0, pivot_z).

    View k of the 8-view config uses ``yaw_deg = 5 * k``.
    """
    fovx = 2 * math.atan(width / (2 * focal))  # focal2fov
    fovy = 2 * math.atan(height / (2 * focal))
    th = math.radians(yaw_deg)
    c, s = math.cos(th), math.sin(th)
    R_c2w = np.array([[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]])
    center = np.array([0.0, 0.0, pivot_z]) + R_c2w @ np.array([0.0, 0.0, -pivot_z])
    T = -R_c2w.T @ center
    wv = torch.tensor(world2view(R_c2w, T)).transpose(0, 1).contiguous()
    pm = torch.tensor(projection(ZNEAR, ZFAR, fovx, fovy)).transpose(0, 1)
    full = (wv.unsqueeze(0).bmm(pm.unsqueeze(0))).squeeze(0).contiguous()
    campos = wv.inverse()[3, :3].contiguous()
    return Camera(width, height, math.tan(fovx * 0.5), math.tan(fovy * 0.5), wv, full, campos)


@dataclass
class Scene:
    means3D: torch.Tensor  # [P,3]
    shs: torch.Tensor  # [P,M,3]
    opacities: torch.Tensor  # [P,1]
    scales: torch.Tensor  # [P,3]
    rotations: torch.Tensor  # [P,4]
    sh_degree: int

    @property
    def P(self) -> int:
        return self.means3D.shape[0]

    def to(self, device) -> "Scene":
        return Scene(*(t.to(device) for t in (self.means3D, self.shs, self.opacities, self.scales, self.rotations)),
                     self.sh_degree)


def make_scene(P: int, cam: Camera, sh_degree: int = 3, seed: int = 0,
               scale_range=(0.003, 0.03), opacity_std: float = 1.5, z_range=(2.0, 12.0)) -> Scene:
    """Frustum-uniform Gaussians generated on the CPU with torch's RNG."""
    g = torch.Generator().manual_seed(seed)
    z = torch.empty(P).uniform_(z_range[0], z_range[1], generator=g)
    x = torch.empty(P).uniform_(-1.1, 1.1, generator=g) * cam.tanfovx * z
    y = torch.empty(P).uniform_(-1.1, 1.1, generator=g) * cam.tanfovy * z
    means = torch.stack([x, y, z], 1)
    lo, hi = math.log(scale_range[0]), math.log(scale_range[1])
    scales = torch.exp(torch.empty(P, 3).uniform_(lo, hi, generator=g))
    rots = torch.nn.functional.normalize(torch.randn(P, 4, generator=g), dim=1)
    opac = torch.sigmoid(torch.randn(P, 1, generator=g) * opacity_std)
    M = (sh_degree + 1) ** 2
    shs = torch.randn(P, M, 3, generator=g) * 0.05
    shs[:, 0, :] = torch.randn(P, 3, generator=g) * 0.5
    return Scene(means.contiguous(), shs.contiguous(), opac.contiguous(), scales.contiguous(), rots.contiguous(),
                 sh_degree)


def upstream_grads(H: int, W: int, seed: int = 1):
    """dL/dcolor = sign(N)/(3HW) (an L1-mean loss, train.py:155) and dL/dinvdepth = N(0,1)/(HW)."""
    g = torch.Generator().manual_seed(seed)
    gc = torch.sign(torch.randn(3, H, W, generator=g)) / (3 * H * W)
    gd = torch.randn(1, H, W, generator=g) / (H * W)
    return gc.contiguous(), gd.contiguous()


# Named configurations of BASELINE.json "configs"
CONFIGS = {
    "10k_256_sh0": dict(P=10_000, width=256, height=256, focal=213.0, sh_degree=0),
    "500k_1080p_sh3": dict(P=500_000, width=1920, height=1080, focal=1600.0, sh_degree=3),
    "1m_1080p_sh3": dict(P=1_000_000, width=1920, height=1080, focal=1600.0, sh_degree=3),
    "5m_4k_sh3": dict(P=5_000_000, width=3840, height=2160, focal=3200.0, sh_degree=3),
}


def config_scene(name: str, seed: int = 0, yaw_deg: float = 0.0, P: Optional[int] = None):
    c = CONFIGS[name]
    cam = make_camera(c["width"], c["height"], c["focal"], yaw_deg)
    base_cam = make_camera(c["width"], c["height"], c["focal"], 0.0)
    scene = make_scene(P or c["P"], base_cam, c["sh_degree"], seed)
    return scene, cam
