#!/usr/bin/env python3
"""Host-side time of one forward and one backward call, with torch allocator counters
(development tool): separates host stalls (allocation, synchronisation) from kernel time.

    python tools/host_time.py [--config 5m_4k_sh3] [--steps 4]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gaussian_splatting_amd import _C  # noqa: E402
from gaussian_splatting_amd import synthetic as syn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="5m_4k_sh3")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--burst", type=int, default=0, help="then this many steps back to back, no synchronisation")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    scene, cam = syn.config_scene(a.config, seed=0)
    scene, cam = scene.to(dev), cam.to(dev)
    gc, gd = syn.upstream_grads(cam.height, cam.width)
    gc, gd = gc.to(dev), gd.to(dev)
    bg = torch.zeros(3, device=dev)
    empty = torch.empty(0, device=dev)
    for i in range(a.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fwd = _C.rasterize_gaussians(bg, scene.means3D, empty, scene.opacities, scene.scales, scene.rotations, 1.0,
                                     empty, cam.viewmatrix, cam.projmatrix, cam.tanfovx, cam.tanfovy, cam.height,
                                     cam.width, scene.shs, scene.sh_degree, cam.campos, False, False, False)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        nr, color, radii, geom, binning, img, invd = fwd
        _C.rasterize_gaussians_backward(bg, scene.means3D, radii, empty, scene.opacities, scene.scales,
                                        scene.rotations, 1.0, empty, cam.viewmatrix, cam.projmatrix, cam.tanfovx,
                                        cam.tanfovy, gc, gd, scene.shs, scene.sh_degree, cam.campos, geom, nr,
                                        binning, img, False, False)
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        st = torch.cuda.memory_stats(dev)
        print(json.dumps({"step": i, "fwd_host_ms": round((t1 - t0) * 1e3, 3), "fwd_gpu_ms": round((t2 - t0) * 1e3, 3),
                          "bwd_host_ms": round((t3 - t2) * 1e3, 3), "bwd_gpu_ms": round((t4 - t2) * 1e3, 3),
                          "num_rendered": int(nr), "binning_bytes": binning.numel(),
                          "reserved_gb": round(st["reserved_bytes.all.current"] / 2**30, 2),
                          "segments": st["segment.all.current"], "alloc_retries": st["num_alloc_retries"],
                          "cuda_mallocs": st.get("num_device_alloc", -1), "cuda_frees": st.get("num_device_free", -1)}))
        del fwd, nr, color, radii, geom, binning, img, invd
    t0 = time.perf_counter()
    for i in range(a.burst):
        fwd = _C.rasterize_gaussians(bg, scene.means3D, empty, scene.opacities, scene.scales, scene.rotations, 1.0,
                                     empty, cam.viewmatrix, cam.projmatrix, cam.tanfovx, cam.tanfovy, cam.height,
                                     cam.width, scene.shs, scene.sh_degree, cam.campos, False, False, False)
        nr, color, radii, geom, binning, img, invd = fwd
        _C.rasterize_gaussians_backward(bg, scene.means3D, radii, empty, scene.opacities, scene.scales,
                                        scene.rotations, 1.0, empty, cam.viewmatrix, cam.projmatrix, cam.tanfovx,
                                        cam.tanfovy, gc, gd, scene.shs, scene.sh_degree, cam.campos, geom, nr,
                                        binning, img, False, False)
        if i % 5 == 4 or i == a.burst - 1:
            st = torch.cuda.memory_stats(dev)
            print(json.dumps({"burst_step": i, "elapsed_ms": round((time.perf_counter() - t0) * 1e3, 1),
                              "binning_bytes": binning.numel(),
                              "reserved_gb": round(st["reserved_bytes.all.current"] / 2**30, 2),
                              "segments": st["segment.all.current"], "alloc_retries": st["num_alloc_retries"],
                              "cuda_mallocs": st.get("num_device_alloc", -1), "cuda_frees": st.get("num_device_free", -1)}))
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
