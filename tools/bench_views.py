#!/usr/bin/env python3
"""Cost of the multi-GPU view exchange's compute side on one MI355X (development tool).

    python tools/bench_views.py [--config 1m_1080p_sh3]

Renders N = 1, 2, 4, 8 distinct views (yaw 5 deg apart, as bench.py's ranks) and times
gauss_backward_views over their view blocks (the gathered buffer an N-rank job holds after the
all-gather), next to the single-view backward's gauss_bwd stage; then the same for the sparse
form (pack, unpack at the largest count, gauss_backward_views over the unpacked blocks).  Also
prints the exchange volumes per rank: all-gather of dense / sparse view blocks vs all-reduce
of the 59-float parameter gradients.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gaussian_splatting_amd import _C, _lib  # noqa: E402
from gaussian_splatting_amd import synthetic as syn  # noqa: E402
from gaussian_splatting_amd.distributed import GradArena  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="1m_1080p_sh3")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = syn.CONFIGS[a.config]
    P, W, H, D = cfg["P"], cfg["width"], cfg["height"], cfg["sh_degree"]
    scene, cam = syn.config_scene(a.config, seed=0)
    scene, cam = scene.to(dev), cam.to(dev)
    gc, gd = syn.upstream_grads(H, W)
    gc, gd = gc.to(dev), gd.to(dev)
    bg, empty = torch.zeros(3, device=dev), torch.empty(0, device=dev)
    arena = GradArena(P, scene.shs.shape[1], dev)
    fwd = _C.rasterize_gaussians(bg, scene.means3D, empty, scene.opacities, scene.scales, scene.rotations, 1.0, empty,
                                 cam.viewmatrix, cam.projmatrix, cam.tanfovx, cam.tanfovy, H, W, scene.shs, D,
                                 cam.campos, False, False, False)
    nr, color, radii, geom, binning, img, invd = fwd
    bwd = (bg, scene.means3D, radii, empty, scene.opacities, scene.scales, scene.rotations, 1.0, empty, cam.viewmatrix,
           cam.projmatrix, cam.tanfovx, cam.tanfovy, gc, gd, scene.shs, D, cam.campos, geom, nr, binning, img, False,
           False)
    nb = _C.view_block_floats(P)
    block = torch.empty(nb, device=dev)
    _C.rasterize_gaussians_backward_screen(*bwd, view_block=block)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps

    _lib.profile_reset()
    _lib.profile_enable(True, stages=["gauss_bwd"])
    for _ in range(a.reps):
        _C.rasterize_gaussians_backward(*bwd, out=arena.views())
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    t, n = _lib.profile_collect()["gauss_bwd"]
    res = {"config": a.config, "P": P, "gauss_bwd_single_ms": t / n, "views_ms": {}, "exchange_MB_per_rank": {}}
    # N distinct views, as an N-rank job has them (bench.py: yaw 5 deg x rank): their dense blocks
    # and their packed forms (pack timed on view 0), all packed at the largest count
    view_blocks = [block]
    for v in range(1, 8):
        _, cam_v = syn.config_scene(a.config, seed=0, yaw_deg=5.0 * v)
        cam_v = cam_v.to(dev)
        fv = _C.rasterize_gaussians(bg, scene.means3D, empty, scene.opacities, scene.scales, scene.rotations, 1.0,
                                    empty, cam_v.viewmatrix, cam_v.projmatrix, cam_v.tanfovx, cam_v.tanfovy, H, W,
                                    scene.shs, D, cam_v.campos, False, False, False)
        bv = torch.empty(nb, device=dev)
        _C.rasterize_gaussians_backward_screen(bg, scene.means3D, fv[2], empty, scene.opacities, scene.scales,
                                               scene.rotations, 1.0, empty, cam_v.viewmatrix, cam_v.projmatrix,
                                               cam_v.tanfovx, cam_v.tanfovy, gc, gd, scene.shs, D, cam_v.campos,
                                               fv[3], fv[0], fv[4], fv[5], False, False, view_block=bv)
        view_blocks.append(bv)
    packed = torch.empty(8, _C.view_pack_floats(P), device=dev)
    scratch = torch.empty(4 * ((P + 255) // 256), dtype=torch.uint8, device=dev)
    count = torch.zeros(1, dtype=torch.int32, device=dev)
    res["pack_ms"] = timed(lambda: _C.view_block_pack(block, packed[0], scratch, count, P))
    counts = []
    for v, bv in enumerate(view_blocks):
        _C.view_block_pack(bv, packed[v], scratch, count, P)
        counts.append(int(count.item()))
    res["live_entries"], res["live_fraction"] = counts, [c / P for c in counts]
    res["views_sparse_ms"], res["unpack_ms"] = {}, {}
    for N in (1, 2, 4, 8):
        blocks = torch.stack(view_blocks[:N])
        res["views_ms"][N] = timed(lambda: _C.gauss_backward_views(scene.means3D, None, scene.shs, D, scene.opacities,
                                                                  scene.scales, scene.rotations, 1.0, blocks,
                                                                  arena.views()))
        size = _C.view_pack_floats(max(counts[:N]))
        recv = packed[:N, :size].contiguous()
        res["unpack_ms"][N] = timed(lambda: _C.view_block_unpack(recv, blocks, P))
        flags = torch.empty(N, P, dtype=torch.int32, device=dev)
        res.setdefault("index_ms", {})[N] = timed(lambda: _C.view_block_index(recv, flags, P))
        res.setdefault("views_packed_ms", {})[N] = timed(lambda: _C.gauss_backward_views(
            scene.means3D, None, scene.shs, D, scene.opacities, scene.scales, scene.rotations, 1.0, recv,
            arena.views(), flags=flags))
        live = torch.empty(_C.views_live_floats(P), dtype=torch.int32, device=dev)
        res.setdefault("live_list_ms", {})[N] = timed(lambda: _C.views_live_list(flags, live, P))
        res.setdefault("zero_ms", {})[N] = timed(lambda: arena.flat.zero_())
        res.setdefault("views_live_ms", {})[N] = timed(lambda: _C.gauss_backward_views(
            scene.means3D, None, scene.shs, D, scene.opacities, scene.scales, scene.rotations, 1.0, recv,
            arena.views(), flags=flags, live=live))
        res["views_sparse_ms"][N] = timed(lambda: _C.gauss_backward_views(scene.means3D, None, scene.shs, D,
                                                                         scene.opacities, scene.scales,
                                                                         scene.rotations, 1.0, blocks, arena.views()))
        res["exchange_MB_per_rank"][N] = {"allgather_view_blocks": (N - 1) * nb * 4 / 1e6,
                                          "allgather_sparse_blocks": (N - 1) * _C.view_pack_floats(max(counts[:N])) * 4 / 1e6,
                                          "allreduce_param_grads": 2 * (N - 1) / N * arena.flat.numel() * 4 / 1e6}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
