#!/usr/bin/env python3
"""Measure the fused SSIM (fused_ssim over libgsr's csrc/ssim.hip) on one MI355X.

    python tools/bench_ssim.py [--H 1080 --W 1920 --C 3 --reps 50]

One "step" = fused_ssim(img, gt) + backward, the loss term train.py:157 evaluates every
iteration.  Reported beside it: the reference's fallback (utils/loss_utils.py ssim, conv2d,
restated here as torch ops on the same GPU) and a CPU baseline (oracle/ssim.py, float64 numpy,
one core).  Algorithmic HBM bytes per step: forward reads 2 images and writes 4 maps, backward
reads 2 images + 4 maps and writes 1: 13 floats per pixel-channel.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from fused_ssim import fused_ssim  # noqa: E402


def conv2d_ssim(img1, img2, window):
    """utils/loss_utils.py:66-87 restated (the reference's non-fused path)."""
    ch = img1.size(-3)
    mu1 = F.conv2d(img1, window, padding=5, groups=ch)
    mu2 = F.conv2d(img2, window, padding=5, groups=ch)
    s11 = F.conv2d(img1 * img1, window, padding=5, groups=ch) - mu1 * mu1
    s22 = F.conv2d(img2 * img2, window, padding=5, groups=ch) - mu2 * mu2
    s12 = F.conv2d(img1 * img2, window, padding=5, groups=ch) - mu1 * mu2
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    m = ((2 * mu1 * mu2 + C1) * (2 * s12 + C2)) / ((mu1 * mu1 + mu2 * mu2 + C1) * (s11 + s22 + C2))
    return m.mean()


def timeit(fn, reps, warm_s=0.2):
    """Mean seconds per call; calls fn for ~warm_s first (clock ramp-up, allocator caching)."""
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < warm_s:
        fn()
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--C", type=int, default=3)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    img = torch.rand(1, a.C, a.H, a.W, device="cuda", generator=g).requires_grad_(True)
    gt = torch.rand(1, a.C, a.H, a.W, device="cuda", generator=g)

    def fused_step():
        v = fused_ssim(img, gt)
        v.backward()

    from oracle import ssim as ossim

    gauss = torch.tensor(ossim.G, dtype=torch.float32, device="cuda")
    window = (gauss[:, None] * gauss[None, :]).expand(a.C, 1, 11, 11).contiguous()

    def conv_step():
        v = conv2d_ssim(img, gt, window)
        v.backward()

    t_fused = timeit(fused_step, a.reps)
    import fused_ssim_cuda

    C1, C2 = 0.01 ** 2, 0.03 ** 2
    m, d1, d2, d3 = fused_ssim_cuda.fusedssim(C1, C2, img.detach(), gt, True)
    t_kfwd = timeit(lambda: fused_ssim_cuda.fusedssim(C1, C2, img.detach(), gt, True), a.reps)
    t_kbwd = timeit(lambda: fused_ssim_cuda.fusedssim_backward(C1, C2, img.detach(), gt, m, d1, d2, d3), a.reps)
    t_conv = timeit(conv_step, max(5, a.reps // 5))
    n = a.C * a.H * a.W
    x, y = img.detach().cpu().numpy(), gt.cpu().numpy()
    c0 = time.perf_counter()
    ossim.fused_ssim(x, y)
    t_cpu = time.perf_counter() - c0
    print(json.dumps({"metric": "fused SSIM fwd+bwd pixel-channels/s", "shape": [1, a.C, a.H, a.W],
                      "ms_per_step": t_fused * 1e3, "value": n / t_fused, "unit": "pixel-channels/s",
                      "algorithmic_GBs": 13 * 4 * n / t_fused / 1e9,
                      "fusedssim_call_ms": t_kfwd * 1e3, "fusedssim_backward_call_ms": t_kbwd * 1e3,
                      "reference_conv2d_path_ms": t_conv * 1e3,
                      "cpu_baseline": {"value": n / t_cpu, "unit": "pixel-channels/s", "cores": 1, "kind": "port",
                                       "sample": f"one {a.C}x{a.H}x{a.W} image pair, oracle/ssim.py (float64 numpy), "
                                                 f"{t_cpu:.1f} s"}}))


if __name__ == "__main__":
    main()
