"""CPU oracle of the reference's simple-knn (submodules/simple-knn): TEST INFRASTRUCTURE
ONLY -- imported by tests/ and never by the product path.

distCUDA2 (spatial.cu:14-25 -> SimpleKNN::knn, simple_knn.cu:172-221) returns, per
point, the mean of the squared distances to its 3 nearest other points.  The CUDA
code's Morton order, boxes and the +-3 neighbour bound only prune: every candidate that
can enter the best three is visited (boxMeanDist, simple_knn.cu:137-170), so the result
is the exact 3-NN mean.  Restated here by brute force:
  * distances in float32 as d.x*d.x + d.y*d.y + d.z*d.z (simple_knn.cu:123-124);
  * the three smallest over j != i (duplicates of a point count as distance 0);
  * fewer than three other points: the missing entries stay FLT_MAX (the initial value
    of best[], simple_knn.cu:143,152-154);
  * mean = (b0 + b1 + b2) / 3 in float32 (simple_knn.cu:169).
The reference ships no test for simple-knn; parity rests on this definition ("parity
unpinned" by reference tests) plus an independent float64 k-d tree (scipy) in tests/.
"""
from __future__ import annotations

import numpy as np

FLT_MAX = np.float32(np.finfo(np.float32).max)


def mean_dist2(points: np.ndarray, block: int = 1024) -> np.ndarray:
    """Exact brute-force oracle, O(P^2): fine for P up to a few thousand."""
    p = np.ascontiguousarray(points, dtype=np.float32)
    P = p.shape[0]
    out = np.empty(P, np.float32)
    for s in range(0, P, block):
        q = p[s:s + block]
        d = q[:, None, :] - p[None, :, :]
        d2 = (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]
        idx = np.arange(s, s + q.shape[0])
        d2[np.arange(q.shape[0]), idx] = np.inf  # j != i
        k = min(3, P - 1)
        best = np.full((q.shape[0], 3), FLT_MAX, np.float32)
        if k > 0:
            best[:, :k] = np.sort(np.partition(d2, k - 1, axis=1)[:, :k], axis=1) if k < P else np.sort(d2, axis=1)[:, :k]
        with np.errstate(over="ignore"):
            out[s:s + q.shape[0]] = ((best[:, 0] + best[:, 1]) + best[:, 2]) / np.float32(3.0)
    return out


def mean_dist2_kdtree(points: np.ndarray) -> np.ndarray:
    """Independent float64 check for large P (scipy k-d tree); P >= 4."""
    from scipy.spatial import cKDTree

    p = np.asarray(points, np.float64)
    d, _ = cKDTree(p).query(p, k=4)
    return (d[:, 1:] ** 2).mean(axis=1)
