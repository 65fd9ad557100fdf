"""Pin the C oracle's hand-written backward with torch autograd over an independent
float64 restatement of the forward (tests/torch_ref.py).  CPU only.

The reference's backward source is incomplete (BACKWARD::render's launcher and the tail
of computeCov2DCUDA are missing), so this is the check that the
re-derived parts are the derivative of the reference's forward.  Tolerances:
  * gradients that do not pass through the conic inverse: 1e-10 relative;
  * gradients through it: 1e-5 relative, because the reference divides by
    (det^2 + 1e-7) instead of det^2 (CR/backward.cu:273-283) -- a deviation that shrinks
    as 1e-7/det^2, see test_conic_epsilon_is_the_only_difference;
  * antialiasing: the reference's d(h_scaling)/d(cov2D) is evaluated at the dilated
    covariance (CR/backward.cu:256-270) and is not the derivative of its forward; only the
    gradients that do not depend on it are compared.
"""
import numpy as np
import pytest

from tests import common as C
from tests import torch_ref as TR

TIGHT = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dsh"]
CONIC = ["dL_dmeans3D", "dL_dcov3D", "dL_dscales", "dL_drotations"]
CASES = [c for c in C.SMALL_CASES if c.name != "dense_opaque"] + [
    C.Case("dense_small", P=600, W=32, H=32, opacity_std=3.0, scale_range=(0.05, 0.3)),
    C.Case("clamped_fov", P=150, W=40, H=40, yaw=35.0),
    C.Case("near_plane", P=150, W=48, H=48, z_range=(0.1, 3.0)),
]


def _run(case):
    inp = C.build(case)
    o = C.run_oracle(inp, precision="f64")
    r = TR.render(inp)
    gc, gd = C.unit_grads(case.H, case.W)
    og = o.handle.backward(gc.double().numpy(), gd.double().numpy())
    tg = TR.grads(r, gc, gd)
    return inp, o, r, og, tg


@pytest.mark.parametrize("case", CASES, ids=lambda c: c.name)
def test_forward_matches_restatement(case):
    _, o, r, _, _ = _run(case)
    assert o.num_rendered == r["num_rendered"]
    np.testing.assert_array_equal(o.radii, r["radii"].numpy())
    np.testing.assert_allclose(o.color, r["color"].detach().numpy(), rtol=0, atol=1e-12)
    np.testing.assert_allclose(o.invdepth, r["invdepth"].detach().numpy(), rtol=0, atol=1e-12)
    img = o.handle.image()
    np.testing.assert_array_equal(img["n_contrib"], r["n_contrib"].numpy())
    np.testing.assert_allclose(img["final_T"], r["final_T"].detach().numpy(), rtol=0, atol=1e-12)


@pytest.mark.parametrize("case", CASES, ids=lambda c: c.name)
def test_backward_matches_autograd(case):
    _, _, _, og, tg = _run(case)
    for k in TIGHT:
        assert C.rel_err(og[k], tg[k]) <= 1e-10, (k, C.rel_err(og[k], tg[k]))
    if case.antialiasing:
        return
    for k in CONIC:
        assert C.rel_err(og[k], tg[k]) <= 1e-5, (k, C.rel_err(og[k], tg[k]))


def test_conic_epsilon_is_the_only_difference():
    """Scaling every Gaussian up by s scales det(cov2D) by ~s^4, so the (det^2 + 1e-7) deviation must
    fall by orders of magnitude -- which would not happen for a genuine derivation error."""
    errs = []
    for s in (1.0, 4.0):
        case = C.Case("eps", P=120, W=48, H=48, scale_range=(0.02 * s, 0.1 * s))
        _, _, _, og, tg = _run(case)
        errs.append(C.rel_err(og["dL_dcov3D"], tg["dL_dcov3D"]))
    assert errs[1] < errs[0] / 20, errs


def test_f32_oracle_close_to_f64():
    case = C.Case("prec", P=300, W=64, H=48)
    inp = C.build(case)
    a, b = C.run_oracle(inp, "f32"), C.run_oracle(inp, "f64")
    d = np.abs(a.color - b.color)
    assert (d <= 1e-5).mean() >= 0.999 and d.mean() < 1e-6
