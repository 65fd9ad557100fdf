"""simple-knn replacement (simple_knn._C.distCUDA2 over libgsr's gsr_knn_mean_dist2).

Reference: submodules/simple-knn (distCUDA2, spatial.cu:14-25; SimpleKNN::knn,
simple_knn.cu:172-221); the reference ships no test for it, so parity rests on the
oracle's restatement of its definition (oracle/knn.py: exact 3-NN mean in float32 with
the FLT_MAX fill for fewer than three neighbours) and on an independent float64 k-d
tree.  Tolerance: the GPU and the oracle form the same float32 distances, so values
agree to a few ulps (rtol 2e-6); infinities and the FLT_MAX fill agree exactly.
"""
import numpy as np
import pytest
import torch

from oracle import knn as oknn


def _clouds():
    rng = np.random.default_rng(7)
    uniform = rng.random((5000, 3)).astype(np.float32) * 10 - 5
    blobs = np.concatenate([rng.normal(c, s, (800, 3)) for c, s in
                            [((0, 0, 0), 0.01), ((3, 1, -2), 0.5), ((-4, 2, 8), 2.0), ((1, 1, 1), 1e-3)]])
    dup = np.repeat(rng.random((700, 3)), 3, axis=0)  # every point three times: distances 0
    flat = rng.random((3000, 3)) * 4
    flat[:, 2] = 0.0  # a degenerate bounding-box axis (0/0 in the Morton scale, simple_knn.cu:57-59)
    shifted = rng.random((2000, 3)) * 0.1 + 100.0  # far from the origin: the {0,0,0}-clamped box is loose
    return {"uniform": uniform, "blobs": blobs.astype(np.float32), "duplicates": dup.astype(np.float32),
            "flat": flat.astype(np.float32), "shifted": shifted.astype(np.float32)}


# ---- CPU: the oracle itself --------------------------------------------------------
def test_oracle_matches_kdtree():
    for name, p in _clouds().items():
        a = oknn.mean_dist2(p).astype(np.float64)
        b = oknn.mean_dist2_kdtree(p)
        scale = max(b.max(), 1e-30)
        assert np.abs(a - b).max() <= 1e-5 * scale + 1e-12, name


def test_oracle_fewer_than_four_points():
    flt = np.float32(np.finfo(np.float32).max)
    assert np.isinf(oknn.mean_dist2(np.zeros((1, 3), np.float32))).all()
    assert np.isinf(oknn.mean_dist2(np.eye(2, 3, dtype=np.float32))).all()
    three = oknn.mean_dist2(np.eye(3, dtype=np.float32))
    np.testing.assert_array_equal(three, np.float32((np.float32(2) + np.float32(2) + flt) / np.float32(3)))


def test_distcuda2_rejects_cpu_and_bad_shapes():
    from simple_knn._C import distCUDA2

    with pytest.raises(RuntimeError, match="HIP device"):
        distCUDA2(torch.zeros(10, 3))
    with pytest.raises(RuntimeError, match="num_points, 3"):
        distCUDA2(torch.zeros(10, 2))


# ---- GPU: parity ---------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(_clouds()))
def test_distcuda2_matches_oracle(name):
    from simple_knn._C import distCUDA2

    p = _clouds()[name]
    got = distCUDA2(torch.from_numpy(p).cuda()).cpu().numpy()
    exp = oknn.mean_dist2(p)
    np.testing.assert_allclose(got, exp, rtol=2e-6, atol=1e-30)


@pytest.mark.gpu
@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 1023, 1024, 1025])
def test_distcuda2_small_and_box_edges(P):
    from simple_knn._C import distCUDA2

    p = np.random.default_rng(P).random((P, 3)).astype(np.float32)
    got = distCUDA2(torch.from_numpy(p).cuda()).cpu().numpy()
    np.testing.assert_allclose(got, oknn.mean_dist2(p), rtol=2e-6, atol=1e-30)


@pytest.mark.gpu
def test_distcuda2_large_against_kdtree_and_deterministic():
    """200k points (196 boxes of 1024), float64 k-d tree reference, bitwise repeatable."""
    from simple_knn._C import distCUDA2

    rng = np.random.default_rng(11)
    p = np.concatenate([rng.normal(0, 1, (150_000, 3)), rng.random((50_000, 3)) * 20 - 10]).astype(np.float32)
    t = torch.from_numpy(p).cuda()
    a = distCUDA2(t)
    b = distCUDA2(t)
    assert torch.equal(a, b)
    exp = oknn.mean_dist2_kdtree(p)
    np.testing.assert_allclose(a.cpu().numpy().astype(np.float64), exp, rtol=1e-5, atol=1e-12)
