"""Drop-in ``diff_gaussian_rasterization`` package backed by the MI355X rasterizer.

``gaussian_renderer/__init__.py:14`` imports ``GaussianRasterizationSettings`` and
``GaussianRasterizer`` from here; ``_C`` exposes the native entry points with the
reference's signatures.  Both interfaces the reference's callers can meet are served:

* the vendored rasterizer's (``submodules/diff-gaussian-rasterization``): one
  ``shs`` tensor, ``_C.rasterize_gaussians`` with 20 arguments;
* the 3DGS-accel build's, which ``train.py:41-45`` detects by importing
  ``SparseGaussianAdam``: with it importable, ``train.py`` / ``render.py`` call the
  renderer with ``separate_sh=True`` (``dc=`` + ``shs=``,
  gaussian_renderer/__init__.py:106-125) and ``--optimizer_type sparse_adam`` steps
  only the visible Gaussians (train.py:240-246).
"""
from gaussian_splatting_amd import _C  # noqa: F401
from gaussian_splatting_amd.optim import SparseGaussianAdam  # noqa: F401
from gaussian_splatting_amd.rasterizer import (  # noqa: F401
    GaussianRasterizationSettings,
    GaussianRasterizer,
    _RasterizeGaussians,
    cpu_deep_copy_tuple,
    rasterize_gaussians,
)

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "_RasterizeGaussians",
           "SparseGaussianAdam", "cpu_deep_copy_tuple", "_C"]
