"""Python surface of the rasterizer: the same names and behaviour as the reference's
``diff_gaussian_rasterization/__init__.py`` (``GaussianRasterizationSettings`` :151-180,
``GaussianRasterizer`` :183-274, ``rasterize_gaussians`` :24-46, ``_RasterizeGaussians``
:48-148), running on libgsr through the ``_C`` module of this package.
"""
from __future__ import annotations

import threading
from typing import NamedTuple

import torch
import torch.nn as nn

from . import _C

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "_RasterizeGaussians",
           "cpu_deep_copy_tuple"]


def cpu_deep_copy_tuple(input_tuple):
    """Copy every tensor of a tuple to the host (debug helper kept from the reference surface)."""
    return tuple(item.cpu().clone() if isinstance(item, torch.Tensor) else item for item in input_tuple)


class GaussianRasterizationSettings(NamedTuple):
    """Per-view settings, field for field the reference's NamedTuple."""

    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool
    antialiasing: bool


def rasterize_gaussians(*args):
    """``rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
    raster_settings)`` (vendored, :24-46), or the 3DGS-accel form with ``dc`` before ``sh``."""
    if len(args) not in (9, 10):
        raise TypeError(f"rasterize_gaussians(): expected 9 or 10 arguments, got {len(args)}")
    # (a render no backward can follow -- grad disabled, or no input requires grad -- skips the atomic backward's
    # accumulator zeroing; autograd's needs_input_grad cannot tell, it ignores the grad mode)
    _RasterizeGaussians._no_backward.value = not (torch.is_grad_enabled() and any(
        isinstance(a, torch.Tensor) and a.requires_grad for a in args[:-1]))
    return _RasterizeGaussians.apply(*args)


class _RasterizeGaussians(torch.autograd.Function):
    """Autograd node: forward = _C.rasterize_gaussians, backward = _C.rasterize_gaussians_backward.

    Inputs ``(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, raster_settings)``
    as in the vendored rasterizer (:48-148), or ``(means3D, means2D, dc, sh, ...)`` as in the 3DGS-accel build
    (separate_sh=True callers, gaussian_renderer/__init__.py:106-125): ``dc`` is ``_features_dc`` [P,1,3] and
    ``sh`` then ``_features_rest`` [P,M,3]; the two get their own gradients, with no concatenation.
    ``means2D`` only carries the screen-space gradient (the reference's trick for densification statistics);
    its value is never read.
    """

    _no_backward = threading.local()

    @staticmethod
    def forward(ctx, *args):
        if len(args) == 10:
            means3D, means2D, dc, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, s = args
        else:
            means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, s = args
            dc = None
        head = (s.bg, means3D, colors_precomp, opacities, scales, rotations, s.scale_modifier, cov3Ds_precomp,
                s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width)
        tail = (s.sh_degree, s.campos, s.prefiltered, s.antialiasing, s.debug)
        sh_args = (sh,) if dc is None else (dc, sh)
        no_backward = getattr(_RasterizeGaussians._no_backward, "value", False)
        _RasterizeGaussians._no_backward.value = False  # (set by rasterize_gaussians for this call only)
        num_rendered, color, radii, geom, binning, img, invdepths = _C.rasterize_gaussians(
            *head, *sh_args, *tail, no_backward=no_backward)
        ctx.raster_settings = s
        ctx.num_rendered = num_rendered
        ctx.separate_sh = dc is not None
        saved = (colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, opacities, geom, binning, img)
        ctx.save_for_backward(*saved, *(() if dc is None else (dc,)))
        ctx.mark_non_differentiable(radii)
        return color, radii, invdepths

    @staticmethod
    def backward(ctx, grad_out_color, _grad_radii, grad_out_depth):
        s = ctx.raster_settings
        saved = ctx.saved_tensors
        (colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, opacities, geom, binning,
         img) = saved[:11]
        dc = saved[11] if ctx.separate_sh else None
        head = (s.bg, means3D, radii, colors_precomp, opacities, scales, rotations, s.scale_modifier, cov3Ds_precomp,
                s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, grad_out_color, grad_out_depth)
        tail = (s.sh_degree, s.campos, geom, ctx.num_rendered, binning, img, s.antialiasing, s.debug)

        def fit(g, like):  # inputs given as empty tensors get no gradient
            return None if like is None or like.numel() == 0 else g

        if dc is None:
            (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp, grad_sh,
             grad_scales, grad_rotations) = _C.rasterize_gaussians_backward(*head, sh, *tail)
            return (grad_means3D, grad_means2D, fit(grad_sh, sh), fit(grad_colors_precomp, colors_precomp),
                    grad_opacities, fit(grad_scales, scales), fit(grad_rotations, rotations),
                    fit(grad_cov3Ds_precomp, cov3Ds_precomp), None)
        (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp, grad_dc, grad_sh,
         grad_scales, grad_rotations) = _C.rasterize_gaussians_backward(*head, dc, sh, *tail)
        return (grad_means3D, grad_means2D, fit(grad_dc, dc), fit(grad_sh, sh),
                fit(grad_colors_precomp, colors_precomp), grad_opacities, fit(grad_scales, scales),
                fit(grad_rotations, rotations), fit(grad_cov3Ds_precomp, cov3Ds_precomp), None)


class GaussianRasterizer(nn.Module):
    """nn.Module front-end; argument checks and empty-tensor placeholders as in the reference (:242-261)."""

    def __init__(self, raster_settings: GaussianRasterizationSettings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        with torch.no_grad():
            s = self.raster_settings
            return _C.mark_visible(positions, s.viewmatrix, s.projmatrix)

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None, dc=None):
        """Same checks as the reference (:242-261).  ``dc=`` (keyword) selects the 3DGS-accel separate-SH
        input: ``dc`` = ``_features_dc`` [P,1,3] and ``shs`` = ``_features_rest`` [P,M,3]
        (gaussian_renderer/__init__.py:115-125)."""
        s = self.raster_settings
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception("Please provide exactly one of either SHs or precomputed colors!")
        if ((scales is None or rotations is None) and cov3D_precomp is None) or (
                (scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!")
        empty = torch.Tensor([])
        shs = empty if shs is None else shs
        colors_precomp = empty if colors_precomp is None else colors_precomp
        scales = empty if scales is None else scales
        rotations = empty if rotations is None else rotations
        cov3D_precomp = empty if cov3D_precomp is None else cov3D_precomp
        if dc is None:
            return rasterize_gaussians(means3D, means2D, shs, colors_precomp, opacities, scales, rotations,
                                       cov3D_precomp, s)
        dc = empty if colors_precomp.numel() != 0 else dc
        return rasterize_gaussians(means3D, means2D, dc, shs, colors_precomp, opacities, scales, rotations,
                                   cov3D_precomp, s)
