#!/usr/bin/env python3
"""Time adaptive density control on one MI355X (development tool).

    python tools/bench_densify.py [--P 1000000] [--reps 10]

A GaussianModel-shaped state (SH3: 59 floats per Gaussian, Adam moments for all six groups),
statistics chosen so ~10% of the Gaussians clone, ~10% split and ~5% are pruned, as in a
mid-training densification step.  Measures:
  * native: gaussian_splatting_amd.densify.densify_and_prune (plan + one host read + apply),
    including the torch.normal draw and the optimizer bookkeeping, as train.py calls it;
  * torch: the reference's own tensor formulation (scene/gaussian_model.py:400-640, restated
    here with torch ops on the same GPU: boolean indexing, cat, repeat, bmm);
  * the stats update (train.py:212-215) natively vs the reference's indexed torch ops;
  * cpu_port: oracle/densify.py (numpy) on a bounded sample, one core.
Algorithmic bytes of the apply: each old row and its moments read once (3 x 236 B), each new
row written once (kept rows with moments, new rows with zero moments).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
from torch import nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gaussian_splatting_amd import densify  # noqa: E402

ATTR = {"xyz": "_xyz", "f_dc": "_features_dc", "f_rest": "_features_rest", "opacity": "_opacity",
        "scaling": "_scaling", "rotation": "_rotation"}
SHAPE = {"xyz": (3,), "f_dc": (1, 3), "f_rest": (15, 3), "opacity": (1,), "scaling": (3,), "rotation": (4,)}


class Model:
    def __init__(self, P, dev, seed=0):
        g = torch.Generator(device=dev).manual_seed(seed)
        r = lambda *s: torch.rand(*s, device=dev, generator=g)  # noqa: E731
        self._xyz = nn.Parameter(r(P, 3) * 6 - 3)
        self._features_dc = nn.Parameter(r(P, 1, 3))
        self._features_rest = nn.Parameter(r(P, 15, 3) * 0.1)
        self._opacity = nn.Parameter(torch.logit(r(P, 1) * 0.9 + 0.0047))   # ~5% below 0.005 + 0.0047
        self._scaling = nn.Parameter(torch.log(r(P, 3) * 0.04 + 1e-3))      # max scale ~ half above 0.02
        self._rotation = nn.Parameter(r(P, 4) - 0.5)
        groups = [{"params": [getattr(self, a)], "lr": 1e-3, "name": k} for k, a in ATTR.items()]
        self.optimizer = torch.optim.Adam(groups, lr=0.0, eps=1e-15)
        for k, a in ATTR.items():
            p = getattr(self, a)
            self.optimizer.state[p] = {"step": torch.tensor(1.0), "exp_avg": torch.zeros_like(p) + 1e-4,
                                       "exp_avg_sq": torch.zeros_like(p) + 1e-8}
        self.xyz_gradient_accum = (r(P, 1) < 0.2).float() * 3e-4  # 20% above the threshold
        self.denom = torch.ones(P, 1, device=dev)
        self.max_radii2D = torch.zeros(P, device=dev)
        self.tmp_radii = None
        self.percent_dense = 0.01

    @property
    def get_scaling(self):
        return torch.exp(self._scaling)

    @property
    def get_opacity(self):
        return torch.sigmoid(self._opacity)


# ---- the reference's formulation (scene/gaussian_model.py:400-640), torch ops on the GPU ----
def _build_rotation(r):
    norm = torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])
    q = r / norm[:, None]
    R = torch.zeros((q.size(0), 3, 3), device=r.device)
    r0, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R[:, 0, 0] = 1 - 2 * (y * y + z * z); R[:, 0, 1] = 2 * (x * y - r0 * z); R[:, 0, 2] = 2 * (x * z + r0 * y)
    R[:, 1, 0] = 2 * (x * y + r0 * z); R[:, 1, 1] = 1 - 2 * (x * x + z * z); R[:, 1, 2] = 2 * (y * z - r0 * x)
    R[:, 2, 0] = 2 * (x * z - r0 * y); R[:, 2, 1] = 2 * (y * z + r0 * x); R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    return R


def _cat(m, d):
    out = {}
    for group in m.optimizer.param_groups:
        ext = d[group["name"]]
        st = m.optimizer.state.get(group["params"][0], None)
        if st is not None:
            st["exp_avg"] = torch.cat((st["exp_avg"], torch.zeros_like(ext)), dim=0)
            st["exp_avg_sq"] = torch.cat((st["exp_avg_sq"], torch.zeros_like(ext)), dim=0)
            del m.optimizer.state[group["params"][0]]
            group["params"][0] = nn.Parameter(torch.cat((group["params"][0], ext), dim=0).requires_grad_(True))
            m.optimizer.state[group["params"][0]] = st
        else:
            group["params"][0] = nn.Parameter(torch.cat((group["params"][0], ext), dim=0).requires_grad_(True))
        out[group["name"]] = group["params"][0]
    for k, a in ATTR.items():
        setattr(m, a, out[k])
    P = m._xyz.shape[0]
    m.xyz_gradient_accum = torch.zeros((P, 1), device="cuda")
    m.denom = torch.zeros((P, 1), device="cuda")
    m.max_radii2D = torch.zeros((P), device="cuda")


def _prune(m, mask):
    valid = ~mask
    out = {}
    for group in m.optimizer.param_groups:
        st = m.optimizer.state.get(group["params"][0], None)
        if st is not None:
            st["exp_avg"] = st["exp_avg"][valid]
            st["exp_avg_sq"] = st["exp_avg_sq"][valid]
            del m.optimizer.state[group["params"][0]]
            group["params"][0] = nn.Parameter(group["params"][0][valid].requires_grad_(True))
            m.optimizer.state[group["params"][0]] = st
        else:
            group["params"][0] = nn.Parameter(group["params"][0][valid].requires_grad_(True))
        out[group["name"]] = group["params"][0]
    for k, a in ATTR.items():
        setattr(m, a, out[k])
    m.xyz_gradient_accum = m.xyz_gradient_accum[valid]
    m.denom = m.denom[valid]
    m.max_radii2D = m.max_radii2D[valid]


def torch_densify_and_prune(m, max_grad, min_opacity, extent, max_screen_size, N=2):
    grads = m.xyz_gradient_accum / m.denom
    grads[grads.isnan()] = 0.0
    sel = torch.where(torch.norm(grads, dim=-1) >= max_grad, True, False)
    sel = torch.logical_and(sel, torch.max(m.get_scaling, dim=1).values <= m.percent_dense * extent)
    _cat(m, {k: getattr(m, a)[sel] for k, a in ATTR.items()})
    n_init = m._xyz.shape[0]
    padded = torch.zeros((n_init), device="cuda")
    padded[:grads.shape[0]] = grads.squeeze()
    sel = torch.where(padded >= max_grad, True, False)
    sel = torch.logical_and(sel, torch.max(m.get_scaling, dim=1).values > m.percent_dense * extent)
    stds = m.get_scaling[sel].repeat(N, 1)
    samples = torch.normal(mean=torch.zeros((stds.size(0), 3), device="cuda"), std=stds)
    rots = _build_rotation(m._rotation[sel]).repeat(N, 1, 1)
    new = {"xyz": torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1) + m._xyz[sel].repeat(N, 1),
           "scaling": torch.log(m.get_scaling[sel].repeat(N, 1) / (0.8 * N)),
           "rotation": m._rotation[sel].repeat(N, 1), "f_dc": m._features_dc[sel].repeat(N, 1, 1),
           "f_rest": m._features_rest[sel].repeat(N, 1, 1), "opacity": m._opacity[sel].repeat(N, 1)}
    _cat(m, new)
    _prune(m, torch.cat((sel, torch.zeros(N * sel.sum(), device="cuda", dtype=bool))))
    prune = (m.get_opacity < min_opacity).squeeze()
    if max_screen_size:
        prune = torch.logical_or(torch.logical_or(prune, m.max_radii2D > max_screen_size),
                                 m.get_scaling.max(dim=1).values > 0.1 * extent)
    _prune(m, prune)


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    args = (2e-4, 0.005, 2.0, 20)

    counts = {}

    def native():
        m = Model(a.P, dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        densify.densify_and_prune(m, *args, radii=None)
        torch.cuda.synchronize()
        counts["P_new"] = m._xyz.shape[0]
        return time.perf_counter() - t0

    def reference():
        m = Model(a.P, dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch_densify_and_prune(m, *args)
        torch.cuda.synchronize()
        counts["P_new_torch"] = m._xyz.shape[0]
        return time.perf_counter() - t0

    for _ in range(2):
        native(), reference()
    t_nat = float(np.median([native() for _ in range(a.reps)])) * 1e3
    t_ref = float(np.median([reference() for _ in range(a.reps)])) * 1e3

    # statistics update, every iteration of the densification phase
    m = Model(a.P, dev)
    vg = torch.randn(a.P, 3, device=dev)
    vpt = torch.zeros(a.P, 3, device=dev, requires_grad=True)
    vpt.grad = vg
    radii = (torch.rand(a.P, device=dev) * 40 - 5).int()
    vis = radii > 0

    def stats_native():
        densify.update_max_radii(m, radii)
        densify.densification_stats(vg, m.xyz_gradient_accum, m.denom, visible=vis)

    def stats_torch():
        idx = vis.nonzero()
        m.max_radii2D[vis] = torch.max(m.max_radii2D[vis], radii[vis])
        m.xyz_gradient_accum[idx] += torch.norm(vpt.grad[idx, :2], dim=-1, keepdim=True)
        m.denom[idx] += 1

    for f in (stats_native, stats_torch):
        f()
    t_sn, t_st = timed(stats_native, 20), timed(stats_torch, 20)

    # CPU port on a bounded sample
    from oracle import densify as od

    n = min(a.P, 200_000)
    rng = np.random.default_rng(0)
    params = {k: rng.random((n,) + s).astype(np.float32) for k, s in SHAPE.items()}
    params["scaling"] = np.log(rng.random((n, 3)) * 0.04 + 1e-3).astype(np.float32)
    moms = {k: (np.zeros_like(v), np.zeros_like(v)) for k, v in params.items()}
    accum = ((rng.random(n) < 0.2) * 3e-4).astype(np.float32)
    st = od.State(params, moms, accum, np.ones(n, np.float32))
    with np.errstate(all="ignore"):
        grads = st.accum / st.denom
    st_c = od.State(params, moms, accum, np.ones(n, np.float32))
    od.densify_and_clone(st_c, grads, 2e-4, 2.0, 0.01)
    ns = int(od.split_mask(st_c, grads, 2e-4, 2.0, 0.01).sum())
    t0 = time.perf_counter()
    od.densify_and_prune(st, 2e-4, 0.005, 2.0, 20, 0.01, rng.standard_normal((2 * ns, 3)).astype(np.float32))
    cpu_s = time.perf_counter() - t0

    floats = 59
    alg = a.P * floats * 4 * 3 + counts["P_new"] * floats * 4 * 3
    print(json.dumps({
        "metric": "densify_and_prune, 1 MI355X", "P": a.P, "P_new": counts["P_new"],
        "P_new_torch_formulation": counts.get("P_new_torch"),
        "native_ms": t_nat, "torch_formulation_ms": t_ref, "speedup": t_ref / t_nat,
        "apply_algorithmic_bytes": alg, "native_GBs_incl_host": alg / (t_nat * 1e-3) / 1e9,
        "stats_native_ms": t_sn, "stats_torch_ms": t_st,
        "cpu_port": {"gaussians_per_s": n / cpu_s, "cores": 1, "kind": "port",
                     "sample": f"oracle/densify.py on {n} Gaussians"}}))


if __name__ == "__main__":
    main()
