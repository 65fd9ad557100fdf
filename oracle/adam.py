"""CPU oracle of the sparse Adam step (SparseGaussianAdam / _C.adamUpdate): TEST
INFRASTRUCTURE ONLY -- imported by tests/ and never by the product path.

The 3DGS-accel rasterizer that provides SparseGaussianAdam is not vendored by the
reference (it only calls it: train.py:41-45,240-246, scene/gaussian_model.py:246-251;
SURVEY.md section 8f row 3).  This restates its published per-element update, float32,
in its operation order (the accel build's adamUpdate kernel):

    if visible[i // M]:
        m = b1 * m + (1 - b1) * g
        v = b2 * v + (1 - b2) * g * g
        p = p + (-lr * m / (sqrt(v) + eps))

with b1 = 0.9, b2 = 0.999 passed by SparseGaussianAdam.step, no bias correction, no
step counter, and untouched rows for invisible Gaussians.  numpy float32 arithmetic is
IEEE round-to-nearest per operation (no fused multiply-add), so the HIP kernel, built
without contraction, must match it bit for bit.  Parity unpinned by reference tests (the
reference ships none for this path); pinned by definition and by the float64 restatement
in tests/test_adam.py.
"""
from __future__ import annotations

import numpy as np


def adam_update(param, grad, exp_avg, exp_avg_sq, visible, lr, b1, b2, eps, N, M):
    """One step on float32 numpy arrays of N*M values; returns new (param, exp_avg, exp_avg_sq)."""
    f = np.float32
    p = np.asarray(param, f).reshape(-1).copy()
    g = np.asarray(grad, f).reshape(-1)
    m = np.asarray(exp_avg, f).reshape(-1).copy()
    v = np.asarray(exp_avg_sq, f).reshape(-1).copy()
    vis = np.repeat(np.asarray(visible, bool).reshape(-1)[:N], M)
    lr, b1, b2, eps = f(lr), f(b1), f(b2), f(eps)
    with np.errstate(all="ignore"):
        m_new = b1 * m + (f(1) - b1) * g
        v_new = b2 * v + ((f(1) - b2) * g) * g
        step = (-lr * m_new) / (np.sqrt(v_new) + eps)
        p_new = p + step
    p[vis], m[vis], v[vis] = p_new[vis], m_new[vis], v_new[vis]
    return p, m, v
