#!/usr/bin/env python3
"""Measure SparseGaussianAdam's step (libgsr csrc/adam.hip, one launch for all groups) on one MI355X.

    python tools/bench_adam.py [--P 1000000 --visible 0.87 --reps 50]

One step = ``optimizer.step(radii > 0, N)`` over GaussianModel's six parameter groups at SH
degree 3 (59 floats per Gaussian: scene/gaussian_model.py:235-242), as train.py:240-246 calls it.
Algorithmic HBM bytes per step: each value of a visible Gaussian reads param, grad, exp_avg,
exp_avg_sq (16 B) and writes param, exp_avg, exp_avg_sq (12 B); an invisible one costs nothing;
plus one visibility byte per Gaussian per group.  Beside it: torch.optim.Adam (foreach, the
reference's dense default optimizer, gaussian_model.py:245) on the same tensors, and the CPU
port (oracle/adam.py, numpy float32, one core) on a bounded sample.
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

from gaussian_splatting_amd.optim import SparseGaussianAdam  # noqa: E402

SHAPES = {"xyz": (3,), "f_dc": (1, 3), "f_rest": (15, 3), "opacity": (1,), "scaling": (3,), "rotation": (4,)}
LRS = {"xyz": 1.6e-4, "f_dc": 2.5e-3, "f_rest": 1.25e-4, "opacity": 2.5e-2, "scaling": 5e-3, "rotation": 1e-3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--visible", type=float, default=0.87)  # 87% of the synthetic Gaussians
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    P = a.P
    g = torch.Generator(device="cuda").manual_seed(0)
    params = {k: torch.nn.Parameter(torch.randn((P,) + s, device="cuda", generator=g)) for k, s in SHAPES.items()}
    for p in params.values():
        p.grad = torch.randn(p.shape, device="cuda", generator=g) * 1e-2
    visible = torch.rand(P, device="cuda", generator=g) < a.visible
    groups = [{"params": [params[k]], "lr": LRS[k], "name": k} for k in SHAPES]
    opt = SparseGaussianAdam(groups, lr=0.0, eps=1e-15)
    for _ in range(5):
        opt.step(visible, P)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(a.reps):
        opt.step(visible, P)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    floats = sum(int(np.prod(s)) for s in SHAPES.values())
    n_vis = int(visible.sum())
    alg = 28 * floats * n_vis + len(SHAPES) * P
    gbs = alg / (ms * 1e-3) / 1e9

    # the dense default (torch.optim.Adam, foreach) on the same tensors
    dense = torch.optim.Adam(groups, lr=0.0, eps=1e-15)
    for _ in range(3):
        dense.step()
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(a.reps):
        dense.step()
    e1.record(stream)
    torch.cuda.synchronize()
    ms_dense = e0.elapsed_time(e1) / a.reps

    # CPU port on a bounded sample (one group of 45 floats per Gaussian, 200k Gaussians)
    from oracle import adam as oadam

    n = min(P, 200_000)
    rng = np.random.default_rng(0)
    x = rng.standard_normal(n * 45).astype(np.float32)
    vis = rng.random(n) < a.visible
    t0, reps = time.perf_counter(), 0
    while time.perf_counter() - t0 < 3.0:
        oadam.adam_update(x, x, x, np.abs(x), vis, 1e-3, 0.9, 0.999, 1e-15, n, 45)
        reps += 1
    cpu_s = (time.perf_counter() - t0) / reps
    cpu_gauss_per_s = n / cpu_s * 45 / floats
    print(json.dumps({
        "metric": "SparseGaussianAdam step, 1 MI355X", "P": P, "visible": n_vis, "floats_per_gaussian": floats,
        "ms_per_step": ms, "gaussians_per_s": P / (ms * 1e-3), "algorithmic_bytes": alg, "achieved_GBs": gbs,
        "hbm_frac": gbs / 8000.0, "torch_adam_dense_ms": ms_dense,
        "cpu_port": {"gaussians_per_s": cpu_gauss_per_s, "cores": 1, "kind": "port",
                     "sample": f"oracle/adam.py on {n} Gaussians x 45 floats, scaled to 59 floats"}}))


if __name__ == "__main__":
    main()
