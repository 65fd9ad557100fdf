#!/usr/bin/env python3
"""Measure simple_knn._C.distCUDA2 (libgsr's gsr_knn_mean_dist2) on one MI355X.

    python tools/bench_knn.py [--points 1000000] [--reps 5]

Prints one JSON line: points/s on the GPU (inputs resident in HBM, mean of --reps calls
after a warm-up; the call includes its scratch allocation and its final stream sync, as the
reference's does), and the CPU baseline: the oracle (oracle/knn.py, the brute-force
restatement) on a bounded sample of the same cloud, one core (numpy).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from simple_knn._C import distCUDA2  # noqa: E402


def cloud(n, seed=0):
    """COLMAP-like synthetic cloud: dense blobs plus a uniform background."""
    rng = np.random.default_rng(seed)
    k = n * 3 // 4
    centres = rng.random((64, 3)) * 20 - 10
    blobs = centres[rng.integers(0, 64, k)] + rng.normal(0, 0.3, (k, 3))
    return np.concatenate([blobs, rng.random((n - k, 3)) * 24 - 12]).astype(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu-sample", type=int, default=20_000)
    a = ap.parse_args()
    p = cloud(a.points)
    t = torch.from_numpy(p).cuda()
    distCUDA2(t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        distCUDA2(t)
    torch.cuda.synchronize()
    gpu_s = (time.perf_counter() - t0) / a.reps
    from oracle import knn as oknn

    sample = cloud(a.cpu_sample, seed=1)
    c0 = time.perf_counter()
    oknn.mean_dist2(sample)
    cpu_s = time.perf_counter() - c0
    print(json.dumps({"metric": "simple-knn distCUDA2 points/s", "points": a.points, "ms_per_call": gpu_s * 1e3,
                      "value": a.points / gpu_s, "unit": "points/s", "data": "synthetic blobs + uniform",
                      "cpu_baseline": {"value": a.cpu_sample / cpu_s, "unit": "points/s", "cores": 1, "kind": "port",
                                       "sample": f"{a.cpu_sample} points, brute force (oracle/knn.py), {cpu_s:.1f} s"}}))


if __name__ == "__main__":
    main()
