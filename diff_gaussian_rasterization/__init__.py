"""Drop-in ``diff_gaussian_rasterization`` package backed by the MI355X rasterizer.

``gaussian_renderer/__init__.py:14`` imports ``GaussianRasterizationSettings`` and
``GaussianRasterizer`` from here; ``_C`` exposes the three native entry points with
the reference's signatures.  ``SparseGaussianAdam`` is deliberately not exported,
so ``train.py:41-45`` keeps the default (non-separate-SH) path.
"""
from gaussian_splatting_amd import _C  # noqa: F401
from gaussian_splatting_amd.rasterizer import (  # noqa: F401
    GaussianRasterizationSettings,
    GaussianRasterizer,
    _RasterizeGaussians,
    cpu_deep_copy_tuple,
    rasterize_gaussians,
)

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "_RasterizeGaussians",
           "cpu_deep_copy_tuple", "_C"]
