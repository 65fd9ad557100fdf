"""Drop-in replacement of the reference's ``simple_knn`` package (submodules/simple-knn).

The reference's only use is ``from simple_knn._C import distCUDA2``
(scene/gaussian_model.py:21, called at :198); ``_C`` here implements it over the C ABI
of libgsr.so (include/gsr_knn.h, csrc/knn.hip).
"""
from . import _C  # noqa: F401
