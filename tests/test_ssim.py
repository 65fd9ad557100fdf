"""Fused SSIM (fused_ssim / fused_ssim_cuda over libgsr, csrc/ssim.hip).

Reference: submodules/fused-ssim (ssim.cu, fused_ssim/__init__.py).  Its own test
(tests/test.py:57-91) checks the fused value and gradient against the conv2d SSIM of
utils/loss_utils.py with torch.isclose; tests/golden/ssim.npz holds that conv2d SSIM's value
and autograd gradient (float64, generated from the reference's Python), which pin
oracle/ssim.py (float64 restatement of the kernels, including the per-pixel map and the three
derivative maps).  GPU tolerances (fp32 kernels vs float64 oracle): map 1e-5 abs (values are
O(1); the variance terms E[x^2] - mu^2 cancel in fp32); derivative maps and gradients 1e-4 of
the tensor's max magnitude; the mean value 1e-6 abs.
"""
import os

import numpy as np
import pytest
import torch

from oracle import ssim as ossim

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ssim.npz")


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def test_oracle_matches_reference_conv2d_ssim():
    z = np.load(GOLDEN)
    for i in range(3):
        v, g = ossim.fused_ssim(z[f"img1_{i}"], z[f"img2_{i}"])
        assert abs(v - float(z[f"value_{i}"])) <= 1e-8, i
        assert _rel(g, z[f"grad_{i}"]) <= 1e-6, i


def test_oracle_backward_is_gradient_of_forward():
    """Central differences of the float64 oracle's mean SSIM."""
    rng = np.random.default_rng(3)
    a, b = rng.random((1, 2, 12, 15)), rng.random((1, 2, 12, 15))
    for padding in ("same", "valid"):
        _, g = ossim.fused_ssim(a, b, padding)
        for idx in [(0, 0, 0, 0), (0, 1, 6, 7), (0, 0, 11, 14), (0, 1, 3, 12)]:
            e = np.zeros_like(a)
            e[idx] = 1e-6
            fd = (ossim.fused_ssim(a + e, b, padding)[0] - ossim.fused_ssim(a - e, b, padding)[0]) / 2e-6
            assert abs(fd - g[idx]) <= 1e-7 + 1e-5 * abs(fd), (padding, idx, fd, g[idx])


def test_fused_ssim_rejects_cpu():
    from fused_ssim import fused_ssim

    with pytest.raises(RuntimeError, match="HIP device"):
        fused_ssim(torch.rand(1, 3, 16, 16), torch.rand(1, 3, 16, 16))


# ---- GPU parity ---------------------------------------------------------------------
SHAPES = [(1, 3, 37, 53), (2, 3, 64, 64), (1, 3, 65, 130), (1, 1, 9, 7), (3, 1, 128, 70)]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_fusedssim_maps_match_oracle(shape):
    import fused_ssim_cuda

    rng = np.random.default_rng(sum(shape))
    a = rng.random(shape).astype(np.float32)
    b = np.clip(0.6 * a + 0.4 * rng.random(shape), 0, 1).astype(np.float32)
    m, d1, d2, d3 = fused_ssim_cuda.fusedssim(0.01 ** 2, 0.03 ** 2, torch.from_numpy(a).cuda(),
                                              torch.from_numpy(b).cuda(), True)
    em, e1, e2, e3 = ossim.forward(a, b)
    np.testing.assert_allclose(m.cpu().numpy(), em, atol=1e-5, rtol=0)
    for got, exp in ((d1, e1), (d2, e2), (d3, e3)):
        assert _rel(got.cpu().numpy(), exp) <= 1e-4
    # backward with a random upstream map
    g = rng.standard_normal(shape).astype(np.float32)
    grad = fused_ssim_cuda.fusedssim_backward(0.01 ** 2, 0.03 ** 2, torch.from_numpy(a).cuda(),
                                              torch.from_numpy(b).cuda(), torch.from_numpy(g).cuda(), d1, d2, d3)
    assert _rel(grad.cpu().numpy(), ossim.backward(a, b, g, e1, e2, e3)) <= 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("padding", ["same", "valid"])
def test_fused_ssim_autograd_matches_reference_golden(padding):
    from fused_ssim import fused_ssim

    z = np.load(GOLDEN)
    for i in range(3):
        if padding == "valid" and min(z[f"img1_{i}"].shape[-2:]) <= 10:
            continue  # nothing left after the 5-pixel crop
        a = torch.from_numpy(z[f"img1_{i}"].astype(np.float32)).cuda().requires_grad_(True)
        b = torch.from_numpy(z[f"img2_{i}"].astype(np.float32)).cuda()
        v = fused_ssim(a, b, padding)
        v.backward()
        ev, eg = ossim.fused_ssim(z[f"img1_{i}"].astype(np.float32), z[f"img2_{i}"].astype(np.float32), padding)
        assert abs(float(v) - ev) <= 1e-6
        assert _rel(a.grad.cpu().numpy(), eg) <= 1e-4
        if padding == "same":  # the reference's conv2d SSIM itself (torch.isclose in fused-ssim tests/test.py:79-87)
            assert abs(float(v) - float(z[f"value_{i}"])) <= 1e-6
            assert _rel(a.grad.cpu().numpy(), z[f"grad_{i}"]) <= 1e-4


@pytest.mark.gpu
def test_train_false_and_accel_variant():
    """train=False returns empty derivative maps; the two-function variant loss_utils.py:16-37 imports from
    diff_gaussian_rasterization._C gives the same map and gradient."""
    import fused_ssim_cuda
    from diff_gaussian_rasterization import _C

    rng = np.random.default_rng(1)
    a = torch.from_numpy(rng.random((3, 40, 50)).astype(np.float32)).cuda()
    b = torch.from_numpy(rng.random((3, 40, 50)).astype(np.float32)).cuda()
    m, d1, d2, d3 = fused_ssim_cuda.fusedssim(1e-4, 9e-4, a[None], b[None], False)
    assert d1.numel() == d2.numel() == d3.numel() == 0
    m2 = _C.fusedssim(1e-4, 9e-4, a, b)
    assert torch.equal(m[0], m2)
    g = torch.randn_like(a)
    _, e1, e2, e3 = fused_ssim_cuda.fusedssim(1e-4, 9e-4, a[None], b[None], True)
    ref = fused_ssim_cuda.fusedssim_backward(1e-4, 9e-4, a[None], b[None], g[None], e1, e2, e3)[0]
    assert torch.equal(_C.fusedssim_backward(1e-4, 9e-4, a, b, g), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("padding", ["same", "valid"])
def test_map_function_agrees_with_loss(padding):
    """The package's two autograd functions: the map-level FusedSSIMMap, averaged, gives the loss
    fused_ssim computes and the same dL/dimg1; train=False gives the value and refuses a backward;
    an unknown padding raises (an AssertionError, as the reference's assert)."""
    from fused_ssim import FusedSSIMMap, fused_ssim

    g = torch.Generator().manual_seed(5)
    a0 = torch.rand(2, 3, 37, 53, generator=g).cuda()
    b = torch.rand(2, 3, 37, 53, generator=g).cuda()
    a1 = a0.clone().requires_grad_(True)
    a2 = a0.clone().requires_grad_(True)
    loss = fused_ssim(a1, b, padding)
    loss.backward()
    m = FusedSSIMMap.apply(0.01 ** 2, 0.03 ** 2, a2, b, padding, True).mean()
    m.backward()
    torch.testing.assert_close(loss, m, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(a1.grad, a2.grad, rtol=1e-5, atol=1e-9)
    with torch.no_grad():
        v = fused_ssim(a0, b, padding, train=False)
    torch.testing.assert_close(v, loss.detach(), rtol=1e-6, atol=1e-7)
    a3 = a0.clone().requires_grad_(True)
    with pytest.raises(RuntimeError, match="train=False"):
        fused_ssim(a3, b, padding, train=False).backward()
    with pytest.raises(AssertionError):
        fused_ssim(a0, b, "full")
