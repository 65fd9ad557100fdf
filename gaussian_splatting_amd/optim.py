"""SparseGaussianAdam on MI355X: the optimizer the reference's ``train.py`` uses with
``--optimizer_type sparse_adam`` (train.py:41-45,74,240-246; scene/gaussian_model.py:246-251).

The class belongs to the 3DGS-accel build of ``diff_gaussian_rasterization``, which the
reference imports but does not vendor.  Its contract, kept
here: a ``torch.optim.Adam`` subclass constructed as ``SparseGaussianAdam(param_groups,
lr=0.0, eps=1e-15)`` with one parameter per group, whose ``step(visibility, N)`` updates
only the rows of Gaussians with ``visibility[g]`` true (``radii > 0``), with betas
(0.9, 0.999), no bias correction, and the state keys ``exp_avg`` / ``exp_avg_sq`` /
``step`` that ``GaussianModel``'s densification code edits in place
(scene/gaussian_model.py:508-600).

Native path: every group of one step goes to libgsr in one launch
(``gsr_adam_update_multi``, include/gsr_adam.h; kernel csrc/adam.hip).  There is no
CPU implementation: CPU tensors raise.
"""
from __future__ import annotations

import ctypes
from typing import List

import torch

from . import _lib

__all__ = ["SparseGaussianAdam", "adam_update"]

BETA1, BETA2 = 0.9, 0.999


_Group = _lib.AdamGroup
_MAX_GROUPS = 8  # GSR_ADAM_MAX_GROUPS


def _check_tensor(t: torch.Tensor, name: str, device) -> None:
    if t.device.type != "cuda":
        raise RuntimeError(f"{name}: SparseGaussianAdam needs HIP device tensors, got {t.device.type} "
                           "(there is no CPU implementation)")
    if t.dtype != torch.float32 or not t.is_contiguous():
        raise RuntimeError(f"{name}: expected a contiguous float32 tensor")
    if t.device != device:
        raise RuntimeError(f"{name}: tensor on {t.device}, expected {device}")


def _visibility(visibility: torch.Tensor, N: int, device) -> torch.Tensor:
    if visibility.device != device:
        raise RuntimeError(f"visibility: tensor on {visibility.device}, expected {device}")
    if visibility.numel() != N:
        raise RuntimeError(f"visibility has {visibility.numel()} entries, expected N={N}")
    if visibility.dtype != torch.bool:
        visibility = visibility != 0
    return visibility.contiguous()


def adam_update(param, param_grad, exp_avg, exp_avg_sq, visibility, lr, b1, b2, eps, N, M) -> None:
    """``_C.adamUpdate``: one sparse Adam step of one parameter tensor (include/gsr_adam.h)."""
    device = param.device
    for t, n in ((param, "param"), (param_grad, "param_grad"), (exp_avg, "exp_avg"), (exp_avg_sq, "exp_avg_sq")):
        _check_tensor(t, n, device)
    vis = _visibility(visibility, int(N), device)
    lib = _lib.load()
    with torch.cuda.device(device):
        rc = lib.gsr_adam_update(param.data_ptr(), param_grad.data_ptr(), exp_avg.data_ptr(), exp_avg_sq.data_ptr(),
                                 vis.data_ptr(), float(lr), float(b1), float(b2), float(eps), int(N), int(M),
                                 ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream))
    _lib.check(rc, "adamUpdate")


class SparseGaussianAdam(torch.optim.Adam):
    """Adam over the Gaussians visible in the current view only (see the module docstring)."""

    def __init__(self, params, lr, eps):
        super().__init__(params=params, lr=lr, eps=eps)

    @torch.no_grad()
    def step(self, visibility, N):
        todo: List[tuple] = []
        for group in self.param_groups:
            lr = group["lr"]
            eps = group["eps"]
            assert len(group["params"]) == 1, "more than one tensor in group"
            param = group["params"][0]
            if param.grad is None:
                continue
            state = self.state[param]
            if len(state) == 0:  # lazy state initialisation, as torch's Adam
                state["step"] = torch.tensor(0.0, dtype=torch.float32)
                state["exp_avg"] = torch.zeros_like(param, memory_format=torch.preserve_format)
                state["exp_avg_sq"] = torch.zeros_like(param, memory_format=torch.preserve_format)
            M = param.numel() // N
            todo.append((param, param.grad, state["exp_avg"], state["exp_avg_sq"], lr, eps, M))
        if not todo:
            return
        device = todo[0][0].device
        vis = _visibility(visibility, int(N), device)
        fused = len(todo) <= _MAX_GROUPS and all(
            p.device == device and all(t.dtype == torch.float32 and t.is_contiguous() for t in (p, g, m, v))
            and p.numel() == N * M for p, g, m, v, _, _, M in todo)
        if not fused:  # one launch per group (still the HIP kernel)
            for p, g, m, v, lr, eps, M in todo:
                adam_update(p, g.contiguous(), m, v, vis, lr, BETA1, BETA2, eps, N, M)
            return
        for p, g, m, v, _, _, _ in todo:
            for t, name in ((p, "param"), (g, "grad"), (m, "exp_avg"), (v, "exp_avg_sq")):
                _check_tensor(t, name, device)
        groups = (_Group * len(todo))(*[
            _Group(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(), M, float(lr), float(eps))
            for p, g, m, v, lr, eps, M in todo])
        lib = _lib.load()
        with torch.cuda.device(device):
            rc = lib.gsr_adam_update_multi(groups, len(todo), vis.data_ptr(), int(N), BETA1, BETA2,
                                           ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream))
        _lib.check(rc, "SparseGaussianAdam.step")
