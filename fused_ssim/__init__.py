"""Drop-in for the reference's ``fused_ssim`` package (submodules/fused-ssim), over the gfx950
kernels of ``fused_ssim_cuda`` (libgsr.so, csrc/ssim.hip).

Callers use one function: ``fused_ssim(img1, img2, padding="same", train=True)`` -> the mean SSIM
of img1 against img2 (train.py:34-39 imports it, :157 calls it as the loss).  The package also
exports the map-level autograd function (``FusedSSIMMap``) and ``allowed_padding`` under the
reference's names.

Design: the loss is what training differentiates, so it has its own autograd function.  Its
upstream gradient is one scalar, so dL/dmap is that scalar / n on the kept window (all pixels for
"same", the map minus a 5-pixel border for "valid": the 11-tap window's half width) -- one constant
map built in the backward instead of a padded copy of an upstream map.  The kernels compute dL/dimg1
only (img2 is the fixed ground truth), from the three derivative maps the forward leaves behind;
``train=False`` skips them (evaluation).
"""
from __future__ import annotations

import torch

import fused_ssim_cuda as _native

__all__ = ["fused_ssim", "FusedSSIMMap", "allowed_padding"]

allowed_padding = ["same", "valid"]
_HALF = 5                      # half width of the 11x11 Gaussian window (ssim.hip)
_C1, _C2 = 0.01 ** 2, 0.03 ** 2  # the constants fused_ssim uses (K1 = 0.01, K2 = 0.03, L = 1)


class PaddingError(ValueError, AssertionError):
    """An unknown padding mode (the reference asserts on it, so this is also an AssertionError)."""


def _kept(t: torch.Tensor, padding: str) -> torch.Tensor:
    """The part of a [B, C, H, W] map a padding mode keeps (a view)."""
    if padding == "same":
        return t
    if padding == "valid":
        return t[..., _HALF:-_HALF, _HALF:-_HALF]
    raise PaddingError(f"padding must be one of {allowed_padding}, got {padding!r}")


def _grad_img1(state, dL_dmap: torch.Tensor) -> torch.Tensor:
    img1, img2, dmu, dsig11, dsig12, c1, c2 = state
    return _native.fusedssim_backward(c1, c2, img1, img2, dL_dmap.contiguous(), dmu, dsig11, dsig12)


class _MeanSSIM(torch.autograd.Function):
    """mean(SSIM map over the kept window); gradient with respect to img1."""

    @staticmethod
    def forward(ctx, img1, img2, padding, train, c1, c2):
        ssim, dmu, dsig11, dsig12 = _native.fusedssim(c1, c2, img1, img2, train)
        kept = _kept(ssim, padding)
        ctx.padding = padding
        ctx.n = kept.numel()
        ctx.consts = (c1, c2)
        if train:
            ctx.save_for_backward(img1.detach(), img2, dmu, dsig11, dsig12)
        return kept.mean()

    @staticmethod
    def backward(ctx, g):
        if not ctx.needs_input_grad[0]:
            return None, None, None, None, None, None
        if len(ctx.saved_tensors) == 0:
            raise RuntimeError("fused_ssim: called with train=False, no gradient is available")
        img1, img2, dmu, dsig11, dsig12 = ctx.saved_tensors
        dL_dmap = torch.zeros_like(img1) if ctx.padding == "valid" else torch.empty_like(img1)
        _kept(dL_dmap, ctx.padding).copy_((g / ctx.n).expand_as(_kept(dL_dmap, ctx.padding)))
        grad = _grad_img1((img1, img2, dmu, dsig11, dsig12) + ctx.consts, dL_dmap)
        return grad, None, None, None, None, None


class FusedSSIMMap(torch.autograd.Function):
    """The SSIM map itself, ``apply(C1, C2, img1, img2, padding="same", train=True)`` (the
    reference package's map-level function); its gradient flows to img1."""

    @staticmethod
    def forward(ctx, C1, C2, img1, img2, padding="same", train=True):
        ssim, dmu, dsig11, dsig12 = _native.fusedssim(C1, C2, img1, img2, train)
        ctx.padding = padding
        ctx.consts = (C1, C2)
        if train:
            ctx.save_for_backward(img1.detach(), img2, dmu, dsig11, dsig12)
        return _kept(ssim, padding)

    @staticmethod
    def backward(ctx, g):
        if len(ctx.saved_tensors) == 0:
            raise RuntimeError("FusedSSIMMap: called with train=False, no gradient is available")
        img1 = ctx.saved_tensors[0]
        if ctx.padding == "valid":  # the border of the map was dropped: it receives no gradient
            full = torch.zeros_like(img1)
            _kept(full, "valid").copy_(g)
            g = full
        grad = _grad_img1(tuple(ctx.saved_tensors) + ctx.consts, g)
        return None, None, grad, None, None, None


def fused_ssim(img1: torch.Tensor, img2: torch.Tensor, padding: str = "same", train: bool = True) -> torch.Tensor:
    """Mean SSIM of img1 against img2 ([B, C, H, W] float32 on the GPU), 11x11 Gaussian window,
    sigma 1.5; ``padding`` "same" (zero padding, every pixel) or "valid" (the map without its
    5-pixel border).  Differentiable with respect to img1 when ``train``."""
    if padding not in allowed_padding:
        raise PaddingError(f"padding must be one of {allowed_padding}, got {padding!r}")
    return _MeanSSIM.apply(img1, img2, padding, train, _C1, _C2)
