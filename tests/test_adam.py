"""SparseGaussianAdam / _C.adamUpdate (include/gsr_adam.h, csrc/adam.hip).

Oracle: oracle/adam.py, the float32 restatement of the 3DGS-accel adamUpdate (not vendored
by the reference).  CPU tests pin the oracle against a float64
restatement and its sparsity contract; GPU tests demand BITWISE equality of the HIP kernel
with the oracle (both are IEEE float32 per operation, no FMA contraction), for every M the
GaussianModel's groups use (3, 3, 45, 1, 3, 4: scene/gaussian_model.py:235-242), ragged N,
all-visible / none / random / alternating visibility, unaligned views (scalar path), and
several steps through the optimizer API as train.py:240-246 drives it.
"""
import numpy as np
import pytest
import torch

from oracle import adam as oadam

GROUP_M = {"xyz": 3, "f_dc": 3, "f_rest": 45, "opacity": 1, "scaling": 3, "rotation": 4}
LRS = {"xyz": 1.6e-4, "f_dc": 2.5e-3, "f_rest": 2.5e-3 / 20.0, "opacity": 2.5e-2, "scaling": 5e-3, "rotation": 1e-3}


def _rand_state(N, M, rng):
    p = rng.standard_normal(N * M).astype(np.float32)
    g = (rng.standard_normal(N * M) * 1e-3).astype(np.float32)
    m = (rng.standard_normal(N * M) * 1e-4).astype(np.float32)
    v = (rng.random(N * M) * 1e-6).astype(np.float32)
    return p, g, m, v


def test_oracle_matches_float64_definition():
    rng = np.random.default_rng(0)
    N, M = 500, 3
    p, g, m, v = _rand_state(N, M, rng)
    vis = rng.random(N) < 0.7
    p1, m1, v1 = oadam.adam_update(p, g, m, v, vis, 1e-3, 0.9, 0.999, 1e-15, N, M)
    P, G, Mm, V = (x.astype(np.float64) for x in (p, g, m, v))
    b1, b2 = float(np.float32(0.9)), float(np.float32(0.999))  # the kernel's float32 constants
    m_ref = b1 * Mm + (1 - b1) * G
    v_ref = b2 * V + (1 - b2) * G * G
    p_ref = P - float(np.float32(1e-3)) * m_ref / (np.sqrt(v_ref) + 1e-15)
    sel = np.repeat(vis, M)
    np.testing.assert_allclose(m1[sel], m_ref[sel], rtol=2e-6, atol=5e-11)  # cancellation: a few ulp of |b1 m|
    np.testing.assert_allclose(v1[sel], v_ref[sel], rtol=1e-5, atol=1e-15)
    np.testing.assert_allclose(p1[sel], p_ref[sel], rtol=1e-6, atol=1e-6)
    # invisible Gaussians: every value untouched, bit for bit
    assert np.array_equal(p1[~sel].view(np.uint32), p[~sel].view(np.uint32))
    assert np.array_equal(m1[~sel].view(np.uint32), m[~sel].view(np.uint32))
    assert np.array_equal(v1[~sel].view(np.uint32), v[~sel].view(np.uint32))


def test_oracle_first_step_known_answer():
    """From zero state the first step moves every visible value by -lr * (1-b1) g / (sqrt((1-b2) g^2) + eps)
    = -lr * 0.1 / sqrt(0.001) * sign(g) ~ -3.1623 lr sign(g) (no bias correction, unlike torch.optim.Adam)."""
    g = np.array([2.0, -0.5, 1e-3], np.float32)
    z = np.zeros(3, np.float32)
    p1, _, _ = oadam.adam_update(z, g, z, z, [True, True, True], 1e-2, 0.9, 0.999, 1e-15, 3, 1)
    np.testing.assert_allclose(p1, -1e-2 * 0.1 / np.sqrt(0.001) * np.sign(g), rtol=1e-5)


def test_rejects_cpu_tensors():
    from gaussian_splatting_amd.optim import SparseGaussianAdam

    p = torch.nn.Parameter(torch.zeros(4, 3))
    opt = SparseGaussianAdam([{"params": [p], "lr": 0.1, "name": "xyz"}], lr=0.0, eps=1e-15)
    p.grad = torch.ones(4, 3)
    with pytest.raises(RuntimeError, match="HIP device"):
        opt.step(torch.ones(4, dtype=torch.bool), 4)


# ---- GPU ------------------------------------------------------------------------------
def _bits(t):
    return t.detach().cpu().contiguous().view(torch.int32).numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 3, 4, 45])
@pytest.mark.parametrize("N", [1, 5, 2049, 100003])
@pytest.mark.parametrize("pattern", ["all", "none", "random", "alternate"])
def test_adam_update_bitwise(M, N, pattern):
    from gaussian_splatting_amd import _C

    rng = np.random.default_rng(N * 7 + M)
    p, g, m, v = _rand_state(N, M, rng)
    vis = {"all": np.ones(N, bool), "none": np.zeros(N, bool), "random": rng.random(N) < 0.6,
           "alternate": np.arange(N) % 2 == 0}[pattern]
    ep, em, ev = oadam.adam_update(p, g, m, v, vis, 2.5e-3, 0.9, 0.999, 1e-15, N, M)
    dev = "cuda"
    tp, tg, tm, tv = (torch.from_numpy(x).to(dev) for x in (p, g, m, v))
    _C.adamUpdate(tp, tg, tm, tv, torch.from_numpy(vis).to(dev), 2.5e-3, 0.9, 0.999, 1e-15, N, M)
    torch.cuda.synchronize()
    assert np.array_equal(_bits(tp), ep.view(np.int32))
    assert np.array_equal(_bits(tm), em.view(np.int32))
    assert np.array_equal(_bits(tv), ev.view(np.int32))


@pytest.mark.gpu
def test_adam_unaligned_views_scalar_path():
    """Parameter views at a 4-byte offset take the kernel's scalar path; same bits."""
    from gaussian_splatting_amd import _C

    N, M = 3001, 3
    rng = np.random.default_rng(5)
    p, g, m, v = _rand_state(N, M, rng)
    vis = rng.random(N) < 0.5
    ep, em, ev = oadam.adam_update(p, g, m, v, vis, 1e-3, 0.9, 0.999, 1e-15, N, M)

    def shifted(x):
        buf = torch.zeros(x.size + 1, dtype=torch.float32, device="cuda")
        buf[1:] = torch.from_numpy(x).cuda()
        return buf[1:]

    tp, tg, tm, tv = (shifted(x) for x in (p, g, m, v))
    assert tp.data_ptr() % 16 != 0
    _C.adamUpdate(tp, tg, tm, tv, torch.from_numpy(vis).cuda(), 1e-3, 0.9, 0.999, 1e-15, N, M)
    torch.cuda.synchronize()
    assert np.array_equal(_bits(tp), ep.view(np.int32))
    assert np.array_equal(_bits(tm), em.view(np.int32))
    assert np.array_equal(_bits(tv), ev.view(np.int32))


@pytest.mark.gpu
@pytest.mark.parametrize("N", [777, 200000])
def test_sparse_gaussian_adam_steps_like_gaussian_model(N):
    """Six groups shaped like GaussianModel.training_setup (gaussian_model.py:235-251), stepped three times
    with train.py:240-246's call; one fused launch per step, bitwise equal to the oracle per group."""
    from diff_gaussian_rasterization import SparseGaussianAdam

    rng = np.random.default_rng(N)
    shapes = {"xyz": (N, 3), "f_dc": (N, 1, 3), "f_rest": (N, 15, 3), "opacity": (N, 1), "scaling": (N, 3),
              "rotation": (N, 4)}
    host = {k: rng.standard_normal(int(np.prod(s))).astype(np.float32) for k, s in shapes.items()}
    params = {k: torch.nn.Parameter(torch.from_numpy(host[k].copy()).reshape(s).cuda())
              for k, s in shapes.items()}
    groups = [{"params": [params[k]], "lr": LRS[k], "name": k} for k in shapes]
    opt = SparseGaussianAdam(groups, lr=0.0, eps=1e-15)
    state = {k: (host[k].copy(), np.zeros_like(host[k]), np.zeros_like(host[k])) for k in shapes}
    for it in range(3):
        vis = rng.random(N) < 0.8
        for k in shapes:
            gr = (rng.standard_normal(host[k].size) * 1e-2).astype(np.float32)
            params[k].grad = torch.from_numpy(gr).reshape(shapes[k]).cuda()
            state[k] = oadam.adam_update(*state[k][:1], gr, *state[k][1:], vis, LRS[k], 0.9, 0.999, 1e-15, N,
                                         GROUP_M[k])
        radii = torch.from_numpy(np.where(vis, 3, 0).astype(np.int32)).cuda()
        visible = radii > 0
        opt.step(visible, radii.shape[0])
        opt.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        for k in shapes:
            st = opt.state[params[k]]
            assert np.array_equal(_bits(params[k]).reshape(-1), state[k][0].view(np.int32)), (it, k)
            assert np.array_equal(_bits(st["exp_avg"]).reshape(-1), state[k][1].view(np.int32)), (it, k)
            assert np.array_equal(_bits(st["exp_avg_sq"]).reshape(-1), state[k][2].view(np.int32)), (it, k)
