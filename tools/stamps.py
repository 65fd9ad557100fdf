#!/usr/bin/env python3
"""Per-workgroup timeline of the binning and render kernels (development tool).

Needs the diagnostic variant library (s_memtime stamps, -DGSR_STAMPS):

    python -m gaussian_splatting_amd.build --variant stamps --cflags=-DGSR_STAMPS
    GSR_LIBRARY=gaussian_splatting_amd/lib/libgsr_stamps.so python tools/stamps.py [--config 1m_1080p_sh3]

For every instrumented kernel it prints the span (first start to last end, shader
clocks), the per-workgroup duration distribution, the per-phase means, and the
"tail": when 50/90/99% of workgroups had finished, relative to the span.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gaussian_splatting_amd import _C, _lib  # noqa: E402
from gaussian_splatting_amd import synthetic as syn  # noqa: E402

SLOTS = 8


def read(fn, which, nwg):
    buf = (ctypes.c_ulonglong * (nwg * SLOTS))()
    rc = fn(which, buf, nwg * SLOTS)
    assert rc == 0, rc
    return np.frombuffer(buf, dtype=np.uint64).reshape(nwg, SLOTS).astype(np.int64)


def timeline(name, st, phases, extra=None):
    t0 = st[:, 0]
    tend = st[:, phases[-1]]
    ok = (t0 > 0) & (tend >= t0)
    st, t0, tend = st[ok], t0[ok], tend[ok]
    span = tend.max() - t0.min()
    dur = tend - t0
    fin = np.sort(tend - t0.min())
    out = {"kernel": name, "workgroups": int(ok.sum()), "span_clk": int(span),
           "dur_mean": float(dur.mean()), "dur_p50": float(np.median(dur)), "dur_max": int(dur.max()),
           "finish_p50": float(fin[len(fin) // 2] / span), "finish_p90": float(fin[int(len(fin) * 0.9)] / span),
           "finish_p99": float(fin[int(len(fin) * 0.99)] / span),
           "start_p90": float(np.quantile(t0 - t0.min(), 0.9) / span)}
    prev = 0
    for k, ph in enumerate(phases):
        if k == 0:
            continue
        d = st[:, ph] - st[:, phases[k - 1]]
        out[f"phase{k}_mean"] = float(d.mean())
    if extra:
        for k, col in extra.items():
            v = st[:, col].astype(np.float64)
            out[f"{k}_mean"] = float(v.mean())
            out[f"{k}_max"] = float(v.max())
            out[f"corr_dur_{k}"] = float(np.corrcoef(v, dur)[0, 1]) if v.std() > 0 else 0.0
    return out


def occupancy(name, st):
    """Device timeline from slots 4/5 (s_memrealtime, 100 MHz) and 7 (placement): per XCD the
    span and the number of running workgroups at 10%, 20%, .. of the kernel's span."""
    hw = st[:, 7]
    xcc = (hw >> 32) & 0xF
    t0, t1 = st[:, 4], st[:, 5]
    ok = (t0 > 0) & (t1 >= t0)
    rows = []
    base, span = t0[ok].min(), t1[ok].max() - t0[ok].min()
    grid = np.linspace(0, span, 11)[1:-1]
    for x in sorted(set(xcc[ok].tolist())):
        m = ok & (xcc == x)
        a, b = t0[m] - base, t1[m] - base
        running = [int(((a <= t) & (b > t)).sum()) for t in grid]
        simd = (hw[m] >> 4) & 3
        cu = (hw[m] >> 8) & 0xF
        se = (hw[m] >> 13) & 0x7
        rows.append({"kernel": name, "xcc": int(x), "wgs": int(m.sum()), "kernel_us": float(span / 100.0),
                     "xcc_end_us": float((b.max()) / 100.0), "wg_us_mean": float((b - a).mean() / 100.0),
                     "running_at_10pct_steps": running,
                     "distinct_simds": int(len(set(zip(se.tolist(), cu.tolist(), simd.tolist()))))})
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="1m_1080p_sh3")
    a = ap.parse_args()
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    cfg = syn.CONFIGS[a.config]
    scene, cam = syn.config_scene(a.config, seed=0)
    scene, cam = scene.to(dev), cam.to(dev)
    gc, gd = syn.upstream_grads(cam.height, cam.width)
    gc, gd = gc.to(dev), gd.to(dev)
    bg = torch.zeros(3, device=dev)
    empty = torch.empty(0, device=dev)
    for _ in range(3):
        fwd = _C.rasterize_gaussians(bg, scene.means3D, empty, scene.opacities, scene.scales, scene.rotations, 1.0,
                                     empty, cam.viewmatrix, cam.projmatrix, cam.tanfovx, cam.tanfovy, cam.height,
                                     cam.width, scene.shs, scene.sh_degree, cam.campos, False, False, False)
        nr, color, radii, geom, binning, img, invd = fwd
        _C.rasterize_gaussians_backward(bg, scene.means3D, radii, empty, scene.opacities, scene.scales,
                                        scene.rotations, 1.0, empty, cam.viewmatrix, cam.projmatrix, cam.tanfovx,
                                        cam.tanfovy, gc, gd, scene.shs, scene.sh_degree, cam.campos, geom, nr,
                                        binning, img, False, False)
    torch.cuda.synchronize()
    tiles = ((cam.width + 15) // 16) * ((cam.height + 15) // 16)
    P = cfg["P"]
    units = int(nr) // 256 + tiles  # bwd_max_units (render.hip), checkpoint stride 256
    nchunks = min(256, max(1, (P + 1023) // 1024))
    fb = lib.gsr_diag_stamps_binning
    fr = lib.gsr_diag_stamps_render
    for f in (fb, fr):
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_size_t]
    res = [
        timeline("tile_count", read(fb, 0, nchunks), [0, 1, 2, 3]),
        timeline("tile_scatter", read(fb, 1, nchunks), [0, 1, 2]),
        timeline("tile_sort", read(fb, 2, tiles), [0, 1], extra={"n": 2}),
        timeline("render_fwd", read(fr, 0, tiles),
                 [0, 1], extra={"n": 2}),
        timeline("render_bwd", read(fr, 1, units), [0, 1], extra={"len": 3}),
    ]
    for r in res:
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}))
    # K2 (tile_scan, one workgroup) stamps its phases at workgroup slot 1000 of the count buffer
    k2 = read(fb, 0, 1001)[1000, :5]
    if k2[0] > 0:
        print(json.dumps({"kernel": "tile_scan", "phase_clk": [int(x) for x in np.diff(k2)],
                          "labels": ["tile scan", "chunk scan", "barrier", "class counts + zeroing"]}))
    # backward: one workgroup per (tile, segment) unit; per-tile sums of the unit durations
    sf, sb = read(fr, 0, tiles), read(fr, 1, units)
    okb = (sb[:, 0] > 0) & (sb[:, 1] >= sb[:, 0])
    fwd_tile = (sf[:, 1] - sf[:, 0]).astype(np.float64)
    bwd_tile = np.bincount(sb[okb, 2], weights=(sb[okb, 1] - sb[okb, 0]).astype(np.float64), minlength=tiles)
    print(json.dumps({"bwd_units": int(okb.sum()),
                      "corr_fwd_bwd_tile_duration": float(np.corrcoef(fwd_tile, bwd_tile[:tiles])[0, 1]),
                      "bwd_tile_cv": float(bwd_tile.std() / bwd_tile.mean()),
                      "fwd_dur_cv": float(fwd_tile.std() / fwd_tile.mean())}))
    for r in occupancy("render_fwd", sf)[:3] + occupancy("render_bwd", sb)[:3]:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
