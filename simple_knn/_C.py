"""``simple_knn._C`` over libgsr.so: the one function of the reference's pybind module
(submodules/simple-knn/ext.cpp:14-17).

distCUDA2(points) -> mean squared distance to the 3 nearest other points, one value per
point (spatial.cu:14-25).  HIP device tensors only; there is no CPU path.
"""
from __future__ import annotations

import ctypes

import torch

from gaussian_splatting_amd import _lib

__all__ = ["distCUDA2"]


def distCUDA2(points: torch.Tensor) -> torch.Tensor:
    """spatial.cu:14-25: ``points`` [P, 3] float32 on a HIP device -> float32 [P] on the same device."""
    if points.dim() != 2 or points.size(1) != 3:
        raise RuntimeError("distCUDA2: points must have dimensions (num_points, 3)")
    if points.device.type != "cuda":
        raise RuntimeError("distCUDA2: the MI355X implementation needs a HIP device tensor "
                           f"(got {points.device.type}); there is no CPU implementation")
    if points.dtype != torch.float32:
        raise RuntimeError(f"distCUDA2: expected a float32 tensor, got {points.dtype}")
    lib = _lib.load()
    pts = points.contiguous()
    P = pts.size(0)
    means = torch.empty(P, dtype=torch.float32, device=pts.device)
    if P == 0:
        return means
    scratch = torch.empty(0, dtype=torch.uint8, device=pts.device)

    def _resize(_ctx, nbytes):
        try:
            scratch.resize_(int(nbytes))
            return scratch.data_ptr()
        except Exception:
            return None

    cb = _lib.ALLOC_FN(_resize)
    with torch.cuda.device(pts.device):
        stream = ctypes.c_void_p(torch.cuda.current_stream(pts.device).cuda_stream)
        rc = lib.gsr_knn_mean_dist2(P, pts.data_ptr(), means.data_ptr(), cb, None, stream)
    _lib.check(rc, "distCUDA2")
    return means
