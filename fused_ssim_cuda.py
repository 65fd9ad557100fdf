"""``fused_ssim_cuda`` -- the reference's compiled fused-SSIM module (submodules/fused-ssim,
pybind ext.cpp:4-7; C++ ssim.cu:368-444), implemented over libgsr.so (include/gsr_ssim.h,
gaussian_splatting_amd/csrc/ssim.hip).  Same two functions, same arguments, same returns.
HIP device tensors only; there is no CPU path.
"""
from __future__ import annotations

import ctypes

import torch

from gaussian_splatting_amd import _lib

__all__ = ["fusedssim", "fusedssim_backward"]


def _check(img: torch.Tensor, name: str) -> torch.Tensor:
    if img.dim() != 4:
        raise RuntimeError(f"{name}: expected a 4-D [B, CH, H, W] tensor, got {img.dim()}-D")
    if img.device.type != "cuda":
        raise RuntimeError(f"{name}: the MI355X fused SSIM needs HIP device tensors, got {img.device.type} "
                           "(there is no CPU implementation)")
    if img.dtype != torch.float32:
        raise RuntimeError(f"{name}: expected float32, got {img.dtype}")
    return img.contiguous()


def _stream(dev: torch.device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def fusedssim(C1: float, C2: float, img1: torch.Tensor, img2: torch.Tensor, train: bool = True):
    """ssim.cu:368-404: returns (ssim_map, dm_dmu1, dm_dsigma1_sq, dm_dsigma12); the last three are
    empty tensors when ``train`` is False (the reference returns torch.empty(0) then)."""
    a, b = _check(img1, "img1"), _check(img2, "img2")
    if a.shape != b.shape:
        raise RuntimeError(f"fusedssim: image shapes differ: {tuple(a.shape)} vs {tuple(b.shape)}")
    B, CH, H, W = a.shape
    out = torch.empty_like(a)
    dms = [torch.empty_like(a) for _ in range(3)] if train else [torch.empty(0, device=a.device) for _ in range(3)]
    ptr = [d.data_ptr() if train else None for d in dms]
    with torch.cuda.device(a.device):
        rc = _lib.load().gsr_fused_ssim_forward(B, CH, H, W, float(C1), float(C2), a.data_ptr(), b.data_ptr(),
                                                out.data_ptr(), ptr[0], ptr[1], ptr[2], _stream(a.device))
    _lib.check(rc, "fusedssim")
    return out, dms[0], dms[1], dms[2]


def fusedssim_backward(C1: float, C2: float, img1: torch.Tensor, img2: torch.Tensor, dL_dmap: torch.Tensor,
                       dm_dmu1: torch.Tensor, dm_dsigma1_sq: torch.Tensor, dm_dsigma12: torch.Tensor) -> torch.Tensor:
    """ssim.cu:406-444: dL/dimg1."""
    a, b = _check(img1, "img1"), _check(img2, "img2")
    g = _check(dL_dmap, "dL_dmap")
    d = [_check(t, n) for t, n in ((dm_dmu1, "dm_dmu1"), (dm_dsigma1_sq, "dm_dsigma1_sq"),
                                   (dm_dsigma12, "dm_dsigma12"))]
    for t in [b, g] + d:
        if t.shape != a.shape:
            raise RuntimeError(f"fusedssim_backward: shape {tuple(t.shape)} differs from img1 {tuple(a.shape)}")
    B, CH, H, W = a.shape
    grad = torch.empty_like(a)
    with torch.cuda.device(a.device):
        rc = _lib.load().gsr_fused_ssim_backward(B, CH, H, W, float(C1), float(C2), a.data_ptr(), b.data_ptr(),
                                                 g.data_ptr(), d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(),
                                                 grad.data_ptr(), _stream(a.device))
    _lib.check(rc, "fusedssim_backward")
    return grad
