"""ctypes front-end for the CPU restatement in ``gsr_oracle.c``.

TEST INFRASTRUCTURE ONLY -- imported by ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py``, never by the product package.

The C restatement follows the reference rasterizer file by file (see the header
of ``gsr_oracle.c``).  This wrapper only marshals numpy arrays; the
``float32`` build is the reference's arithmetic, the ``float64`` build is used
for finite-difference gradient checks.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_BUILD = os.path.join(_HERE, "_build")
_LIBS: dict = {}


def build(force: bool = False) -> None:
    """Compile the variants with the committed Makefile (gcc + OpenMP): f32 and f64 without FP
    contraction (the oracle), and f32fma -- float32 with every multiply-add the compiler can fuse
    contracted into an FMA, as nvcc's default --fmad=true builds the reference (RI/setup.py passes
    only -I).  f32fma only measures how sensitive the integer outputs are to contraction
    (tools/fma_sensitivity.py); it is not a parity oracle."""
    targets = [os.path.join(_BUILD, f"liboracle_{p}.so") for p in ("f32", "f64", "f32fma")]
    src = os.path.join(_HERE, "gsr_oracle.c")
    if not force and all(os.path.exists(t) and os.path.getmtime(t) >= os.path.getmtime(src) for t in targets):
        return
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _lib(precision: str):
    if precision in _LIBS:
        return _LIBS[precision]
    build()
    lib = ctypes.CDLL(os.path.join(_BUILD, f"liboracle_{precision}.so"))
    pre = "oracle32_" if precision.startswith("f32") else "oracle64_"
    vp = ctypes.c_void_p
    i = ctypes.c_int
    r = ctypes.c_float if precision.startswith("f32") else ctypes.c_double
    fwd = getattr(lib, pre + "forward")
    fwd.restype = vp
    fwd.argtypes = [i, i, i, vp, i, i, vp, vp, vp, vp, vp, r, vp, vp, vp, vp, vp, r, r, i, i, vp, vp, vp, vp, i]
    bwd = getattr(lib, pre + "backward")
    bwd.restype = None
    bwd.argtypes = [vp] + [vp] * 12 + [i]
    for name, args in (("get_geom", [vp] * 7), ("get_binning", [vp] * 3), ("get_image", [vp] * 3)):
        f = getattr(lib, pre + name)
        f.restype = None
        f.argtypes = args
    for name in ("prefilter_violation", "num_rendered"):
        f = getattr(lib, pre + name)
        f.restype = i
        f.argtypes = [vp]
    pm = getattr(lib, pre + "pixel_margins")
    pm.restype = None
    pm.argtypes = [vp, vp, vp, vp, i]
    tg = getattr(lib, pre + "threshold_gaussians")
    tg.restype = None
    tg.argtypes = [vp, r, r, r, vp, i]
    c3 = getattr(lib, pre + "cov3d")
    c3.restype = None
    c3.argtypes = [i, vp, r, vp, vp]
    mv = getattr(lib, pre + "mark_visible")
    mv.restype = None
    mv.argtypes = [i, vp, vp, vp]
    fr = getattr(lib, pre + "free")
    fr.restype = None
    fr.argtypes = [vp]
    _LIBS[precision] = (lib, pre, r)
    return _LIBS[precision]


def _ptr(a: Optional[np.ndarray]):
    if a is None or a.size == 0:
        return None
    return a.ctypes.data_as(ctypes.c_void_p)


def _arr(x, dtype) -> Optional[np.ndarray]:
    if x is None:
        return None
    if hasattr(x, "detach"):  # torch tensor
        x = x.detach().cpu().numpy()
    a = np.ascontiguousarray(np.asarray(x, dtype=dtype))
    return None if a.size == 0 else a


@dataclass
class ForwardResult:
    color: np.ndarray  # [3,H,W]
    invdepth: np.ndarray  # [1,H,W]
    radii: np.ndarray  # [P] int32
    num_rendered: int
    handle: "OracleHandle"


class OracleHandle:
    """Owns the C-side state (the reference's geom/binning/image buffers)."""

    def __init__(self, precision, h, P, M, W, H):
        self.precision, self.h, self.P, self.M, self.W, self.H = precision, h, P, M, W, H
        self._lib, self._pre, _ = _lib(precision)
        self.dtype = np.float32 if precision.startswith("f32") else np.float64

    def __del__(self):
        try:
            if self.h:
                getattr(self._lib, self._pre + "free")(self.h)
                self.h = None
        except Exception:
            pass

    def geom(self):
        P = self.P
        d = dict(
            depths=np.zeros(P, self.dtype),
            means2D=np.zeros((P, 2), self.dtype),
            conic_opacity=np.zeros((P, 4), self.dtype),
            rgb=np.zeros((P, 3), self.dtype),
            tiles_touched=np.zeros(P, np.uint32),
            clamped=np.zeros(P, np.uint8),
        )
        getattr(self._lib, self._pre + "get_geom")(
            self.h, *[_ptr(d[k]) for k in ("depths", "means2D", "conic_opacity", "rgb", "tiles_touched", "clamped")]
        )
        return d

    def binning(self):
        R = getattr(self._lib, self._pre + "num_rendered")(self.h)
        gx, gy = (self.W + 15) // 16, (self.H + 15) // 16
        pl = np.zeros(max(R, 1), np.uint32)
        ranges = np.zeros((gx * gy, 2), np.uint32)
        getattr(self._lib, self._pre + "get_binning")(self.h, _ptr(pl), _ptr(ranges))
        return dict(point_list=pl[:R], ranges=ranges)

    def image(self):
        N = self.W * self.H
        fT = np.zeros(N, self.dtype)
        nc = np.zeros(N, np.uint32)
        getattr(self._lib, self._pre + "get_image")(self.h, _ptr(fT), _ptr(nc))
        return dict(final_T=fT.reshape(self.H, self.W), n_contrib=nc.reshape(self.H, self.W))

    def pixel_margins(self, nthreads: int = 1):
        """Per pixel [H, W]: the blend's smallest distances to the reference's discrete thresholds
        (|power| vs the power > 0 skip, |255 alpha - 1| vs the alpha skip, |1e4 test_T - 1| vs the
        termination), over the entries the reference's loop visits (gsr_oracle.c pixel_margins)."""
        N = self.W * self.H
        out = [np.zeros(N, self.dtype) for _ in range(3)]
        getattr(self._lib, self._pre + "pixel_margins")(self.h, *[_ptr(o) for o in out], int(nthreads))
        return {k: o.reshape(self.H, self.W) for k, o in zip(("power", "alpha", "T"), out)}

    def threshold_gaussians(self, m_power: float, m_alpha: float, m_T: float, nthreads: int = 1) -> np.ndarray:
        """bool [P]: Gaussians whose own blend at some pixel lies within the margins of a discrete
        threshold of the reference (power > 0 / alpha < 1/255 skips, T < 1e-4 termination at it)."""
        _, _, rtype = _lib(self.precision)
        flags = np.zeros(max(self.P, 1), np.uint8)
        getattr(self._lib, self._pre + "threshold_gaussians")(self.h, rtype(m_power), rtype(m_alpha), rtype(m_T),
                                                              _ptr(flags), int(nthreads))
        return flags[:self.P].astype(bool)

    def prefilter_violation(self) -> bool:
        return bool(getattr(self._lib, self._pre + "prefilter_violation")(self.h))

    def backward(self, dL_dpix, dL_dinvdepth=None, nthreads: int = 1):
        P, M, dt = self.P, self.M, self.dtype
        g = _arr(dL_dpix, dt)
        gi = _arr(dL_dinvdepth, dt)
        out = dict(
            dL_dmeans2D=np.zeros((P, 3), dt),
            dL_dconic=np.zeros((P, 4), dt),
            dL_dopacity=np.zeros((P, 1), dt),
            dL_dcolors=np.zeros((P, 3), dt),
            dL_dinvdepths=np.zeros((P, 1), dt) if gi is not None else None,
            dL_dmeans3D=np.zeros((P, 3), dt),
            dL_dcov3D=np.zeros((P, 6), dt),
            dL_dsh=np.zeros((P, M, 3), dt),
            dL_dscales=np.zeros((P, 3), dt),
            dL_drotations=np.zeros((P, 4), dt),
        )
        keys = ["dL_dmeans2D", "dL_dconic", "dL_dopacity", "dL_dcolors", "dL_dinvdepths", "dL_dmeans3D",
                "dL_dcov3D", "dL_dsh", "dL_dscales", "dL_drotations"]
        ptrs = [_ptr(out[k]) if out[k] is not None else None for k in keys]
        getattr(self._lib, self._pre + "backward")(self.h, _ptr(g), _ptr(gi), *ptrs, int(nthreads))
        return out


def forward(
    means3D,
    opacities,
    viewmatrix,
    projmatrix,
    campos,
    tanfovx: float,
    tanfovy: float,
    image_height: int,
    image_width: int,
    bg=(0.0, 0.0, 0.0),
    shs=None,
    sh_degree: int = 0,
    colors_precomp=None,
    scales=None,
    rotations=None,
    cov3D_precomp=None,
    scale_modifier: float = 1.0,
    prefiltered: bool = False,
    antialiasing: bool = False,
    precision: str = "f32",
    nthreads: int = 1,
) -> ForwardResult:
    """Forward pass of the restatement; argument meaning follows GaussianRasterizer / _C.rasterize_gaussians."""
    lib, pre, rtype = _lib(precision)
    dt = np.float32 if precision.startswith("f32") else np.float64
    m3 = _arr(means3D, dt)
    P = 0 if m3 is None else m3.reshape(-1, 3).shape[0]
    sh = _arr(shs, dt)
    M = 0 if sh is None else sh.reshape(P, -1, 3).shape[1]
    W, H = int(image_width), int(image_height)
    color = np.zeros((3, H, W), dt)
    invd = np.zeros((1, H, W), dt)
    radii = np.zeros(max(P, 1), np.int32)
    nr = ctypes.c_int(0)
    ins = [_arr(bg, dt), m3, sh, _arr(colors_precomp, dt), _arr(opacities, dt), _arr(scales, dt)]
    more = [_arr(rotations, dt), _arr(cov3D_precomp, dt), _arr(viewmatrix, dt), _arr(projmatrix, dt), _arr(campos, dt)]
    h = getattr(lib, pre + "forward")(
        P, int(sh_degree), M, _ptr(ins[0]), W, H, _ptr(ins[1]), _ptr(ins[2]), _ptr(ins[3]), _ptr(ins[4]),
        _ptr(ins[5]), rtype(scale_modifier), _ptr(more[0]), _ptr(more[1]), _ptr(more[2]), _ptr(more[3]),
        _ptr(more[4]), rtype(tanfovx), rtype(tanfovy), int(bool(prefiltered)), int(bool(antialiasing)),
        _ptr(color), _ptr(invd), _ptr(radii), ctypes.byref(nr), int(nthreads),
    )
    handle = OracleHandle(precision, h, P, M, W, H)
    return ForwardResult(color, invd, radii[:P], int(nr.value), handle)


def cov3d(scales, rotations, scale_modifier: float = 1.0, precision: str = "f32") -> np.ndarray:
    """computeCov3D (CR/forward.cu:149-190): upper triangle [P, 6] of (S R)^T (S R); rotations are used
    as given (the reference's kernel does not normalise them)."""
    lib, pre, rtype = _lib(precision)
    dt = np.float32 if precision.startswith("f32") else np.float64
    s = _arr(scales, dt)
    q = _arr(rotations, dt)
    P = 0 if s is None else s.reshape(-1, 3).shape[0]
    out = np.zeros((max(P, 1), 6), dt)
    getattr(lib, pre + "cov3d")(P, _ptr(s), rtype(scale_modifier), _ptr(q), _ptr(out))
    return out[:P]


def mark_visible(means3D, viewmatrix, precision: str = "f32") -> np.ndarray:
    lib, pre, _ = _lib(precision)
    dt = np.float32 if precision.startswith("f32") else np.float64
    m3 = _arr(means3D, dt)
    P = 0 if m3 is None else m3.reshape(-1, 3).shape[0]
    out = np.zeros(max(P, 1), np.uint8)
    getattr(lib, pre + "mark_visible")(P, _ptr(m3), _ptr(_arr(viewmatrix, dt)), _ptr(out))
    return out[:P].astype(bool)
