"""Python surface of the rasterizer: the same names and behaviour as the reference's
``diff_gaussian_rasterization/__init__.py`` (``GaussianRasterizationSettings`` :151-180,
``GaussianRasterizer`` :183-274, ``rasterize_gaussians`` :24-46, ``_RasterizeGaussians``
:48-148), running on libgsr through the ``_C`` module of this package.
"""
from __future__ import annotations

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


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings):
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings)


class _RasterizeGaussians(torch.autograd.Function):
    """Autograd node: forward = _C.rasterize_gaussians, backward = _C.rasterize_gaussians_backward.

    ``means2D`` only carries the screen-space gradient (the reference's trick for
    densification statistics); its value is never read.
    """

    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings):
        s = raster_settings
        num_rendered, color, radii, geom, binning, img, invdepths = _C.rasterize_gaussians(
            s.bg, means3D, colors_precomp, opacities, scales, rotations, s.scale_modifier, cov3Ds_precomp,
            s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width, sh, s.sh_degree,
            s.campos, s.prefiltered, s.antialiasing, s.debug)
        ctx.raster_settings = s
        ctx.num_rendered = num_rendered
        ctx.save_for_backward(colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, opacities, geom,
                              binning, img)
        ctx.mark_non_differentiable(radii)
        return color, radii, invdepths

    @staticmethod
    def backward(ctx, grad_out_color, _grad_radii, grad_out_depth):
        s = ctx.raster_settings
        (colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, opacities, geom, binning,
         img) = ctx.saved_tensors
        (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp, grad_sh, grad_scales,
         grad_rotations) = _C.rasterize_gaussians_backward(
            s.bg, means3D, radii, colors_precomp, opacities, scales, rotations, s.scale_modifier, cov3Ds_precomp,
            s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, grad_out_color, grad_out_depth, sh, s.sh_degree,
            s.campos, geom, ctx.num_rendered, binning, img, s.antialiasing, s.debug)

        def fit(g, like):  # inputs given as empty tensors get no gradient
            return None if like is None or like.numel() == 0 else g

        return (grad_means3D, grad_means2D, fit(grad_sh, sh), fit(grad_colors_precomp, colors_precomp),
                grad_opacities, fit(grad_scales, scales), fit(grad_rotations, rotations),
                fit(grad_cov3Ds_precomp, cov3Ds_precomp), None)


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
                cov3D_precomp=None):
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
        return rasterize_gaussians(means3D, means2D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp,
                                   s)
