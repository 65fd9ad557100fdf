"""MI355X-native differentiable Gaussian tile rasterizer (HIP/CDNA4, gfx950).

The hot path -- preprocess, binning, radix sort, tile blending and the matching
backward -- lives in libgsr.so (gaussian_splatting_amd/csrc, C ABI in
include/gsr.h).  ``rasterizer`` and ``_C`` mirror the reference's
``diff_gaussian_rasterization`` Python surface; ``distributed`` shards training
views over GPUs with one RCCL gradient all-reduce.
"""
__version__ = "0.1.0"

from .rasterizer import (  # noqa: E402,F401
    GaussianRasterizationSettings,
    GaussianRasterizer,
    rasterize_gaussians,
)
