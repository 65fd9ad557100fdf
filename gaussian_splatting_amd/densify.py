"""Adaptive density control on MI355X: the reference's ``GaussianModel`` densification
methods over the HIP kernels of ``csrc/densify.hip`` (C ABI: include/gsr_densify.h).

Reference (``scene/gaussian_model.py``): ``add_densification_stats`` (:643-654) and the
``max_radii2D`` update of ``train.py:212-213``; ``densify_and_prune`` (:574-640) with
``densify_and_clone`` (:552-571), ``densify_and_split`` (:508-550), ``prune_points``
(:420-437), ``_prune_optimizer`` (:400-418), ``cat_tensors_to_optimizer`` (:439-481) and
``densification_postfix`` (:483-506).  SURVEY.md section 8f row 4.

The functions take the model as their first argument and touch exactly the attributes the
reference's methods touch (``_xyz``, ``_features_dc``, ``_features_rest``, ``_opacity``,
``_scaling``, ``_rotation``, ``optimizer``, ``xyz_gradient_accum``, ``denom``,
``max_radii2D``, ``tmp_radii``, ``percent_dense``), so ``install(GaussianModel)`` binds them
as the class's methods and ``train.py`` runs unchanged.

Semantics kept from the reference, including its quirks:
* the output order: kept originals, kept clones, kept children of the first split copy,
  kept children of the second (clone appends, split appends and drops its parents, prune
  compacts);
* clones and children start with zero Adam moments; kept rows keep theirs; a group without
  optimizer state yet gets none;
* the split samples are drawn with ``torch.normal(mean=zeros, std=get_scaling[split].repeat(N, 1))``
  (gaussian_model.py:520-528): same shape, same generator, so a seeded run draws the same
  numbers; with ``torch.distributed`` initialised (world > 1) rank 0's samples are broadcast
  so every replica densifies identically;
* the screen-size prune compares ``max_radii2D`` after ``densification_postfix`` zeroed it,
  so it never fires; only the world-space size test does (``max_screen_size`` truthy);
* afterwards ``xyz_gradient_accum``, ``denom`` and ``max_radii2D`` are zeros of the new size
  and ``tmp_radii`` is ``None``.

There is no CPU implementation: CPU tensors raise.
"""
from __future__ import annotations

import ctypes
import math

import torch
import torch.distributed as dist
from torch import nn

from . import _lib

__all__ = ["add_densification_stats", "update_max_radii", "densification_stats", "densify_and_prune", "install",
           "GROUPS"]

COPY, XYZ, SCALING = 0, 1, 2  # GSR_DENSIFY_COPY / _XYZ / _SCALING
# optimizer group name, model attribute, how children rows are made
GROUPS = (("xyz", "_xyz", XYZ), ("f_dc", "_features_dc", COPY), ("f_rest", "_features_rest", COPY),
          ("opacity", "_opacity", COPY), ("scaling", "_scaling", SCALING), ("rotation", "_rotation", COPY))


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _dev_check(t: torch.Tensor, name: str) -> None:
    if t.device.type != "cuda":
        raise RuntimeError(f"{name}: densification runs on HIP device tensors, got {t.device.type} "
                           "(there is no CPU implementation)")


def _f32(t: torch.Tensor, name: str) -> torch.Tensor:
    _dev_check(t, name)
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name}: expected float32, got {t.dtype}")
    return t.contiguous()


def densification_stats(viewspace_grad, grad_accum: torch.Tensor = None, denom: torch.Tensor = None,
                        max_radii2D: torch.Tensor = None, radii: torch.Tensor = None,
                        visible: torch.Tensor = None) -> None:
    """In place: ``grad_accum[v] += ||viewspace_grad[v, :2]||``, ``denom[v] += 1`` (skipped when
    ``viewspace_grad`` is None) and, with ``radii`` and ``max_radii2D``,
    ``max_radii2D[v] = max(max_radii2D[v], radii[v])``; v = ``visible`` (bool mask) or
    ``radii > 0``.  The accumulators are [P] or [P, 1] contiguous float32."""
    ref = viewspace_grad if viewspace_grad is not None else radii
    if ref is None:
        raise RuntimeError("densification_stats: need the viewspace gradient or radii")
    P = ref.shape[0]
    g = None
    if viewspace_grad is not None:
        g = _f32(viewspace_grad, "viewspace grad")
        if g.dim() != 2 or g.shape[1] < 2:
            raise RuntimeError("viewspace grad must be [P, 3]")
        if g.shape[1] != 3:
            g = torch.nn.functional.pad(g[:, :2], (0, 1)).contiguous()
        for t, n in ((grad_accum, "xyz_gradient_accum"), (denom, "denom")):
            if t is None:
                raise RuntimeError(f"densification_stats: {n} missing")
            _f32(t, n)
            if t.numel() != P or not t.is_contiguous():
                raise RuntimeError(f"{n}: expected {P} contiguous values, got {tuple(t.shape)}")
    r = None
    if radii is not None:
        _dev_check(radii, "radii")
        r = radii.to(torch.int32).contiguous()
        if max_radii2D is not None:
            _f32(max_radii2D, "max_radii2D")
            if max_radii2D.numel() != P or not max_radii2D.is_contiguous():
                raise RuntimeError("max_radii2D: expected P contiguous values")
    vis = None
    if visible is not None:
        _dev_check(visible, "visibility")
        vis = visible.to(torch.uint8).contiguous()
    if r is None and vis is None:
        raise RuntimeError("densification_stats: need radii or a visibility mask")
    device = ref.device
    lib = _lib.load()
    ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    with torch.cuda.device(device):
        rc = lib.gsr_densify_stats(P, ptr(g), ptr(r), ptr(vis), ptr(grad_accum) if g is not None else None,
                                   ptr(denom) if g is not None else None,
                                   ptr(max_radii2D) if r is not None else None, _stream(device))
    _lib.check(rc, "densify_stats")


def _filter_mask(update_filter: torch.Tensor, P: int, device) -> torch.Tensor:
    if update_filter.dtype == torch.bool:
        m = update_filter.reshape(-1)
        if m.numel() != P:
            raise RuntimeError(f"update_filter has {m.numel()} entries, expected {P}")
        return m.to(device)
    m = torch.zeros(P, dtype=torch.bool, device=device)  # index tensor ((radii > 0).nonzero())
    m[update_filter.reshape(-1).to(device)] = True
    return m


def add_densification_stats(model, viewspace_point_tensor, update_filter) -> None:
    """``GaussianModel.add_densification_stats`` (gaussian_model.py:643-654)."""
    P = model.xyz_gradient_accum.shape[0]
    mask = _filter_mask(update_filter, P, model.xyz_gradient_accum.device)
    densification_stats(viewspace_point_tensor.grad, model.xyz_gradient_accum, model.denom, visible=mask)


def update_max_radii(model, radii: torch.Tensor, visibility_filter=None) -> None:
    """``train.py:212-213``: max_radii2D[v] = max(max_radii2D[v], radii[v]), v = the renderer's
    visibility_filter (radii > 0)."""
    vis = None
    if visibility_filter is not None:
        vis = _filter_mask(visibility_filter, model.max_radii2D.shape[0], radii.device)
    densification_stats(None, max_radii2D=model.max_radii2D, radii=radii, visible=vis)


def _params(max_grad, min_opacity, extent, max_screen_size, percent_dense, N):
    # scalars compare against float32 tensors in float32 (torch casts the Python scalar), and the
    # products the reference forms in Python (percent_dense * extent, 0.1 * extent, 0.8 * N) are
    # doubles rounded once
    return _lib.DensifyParams(float(max_grad), float(percent_dense * extent), float(min_opacity), float(0.1 * extent),
                              1 if max_screen_size else 0, int(N), float(0.8 * N))


def _replace_in_optimizer(optimizer, new: dict) -> dict:
    """The optimizer-side halves of cat_tensors_to_optimizer / _prune_optimizer: each group's
    parameter becomes a fresh ``nn.Parameter``; its state (if any) moves with it."""
    out = {}
    for group in optimizer.param_groups:
        assert len(group["params"]) == 1
        name = group["name"]
        tensor, m, v = new[name]
        old = group["params"][0]
        stored_state = optimizer.state.get(old, None)
        param = nn.Parameter(tensor.requires_grad_(True))
        if stored_state is not None:
            stored_state["exp_avg"] = m
            stored_state["exp_avg_sq"] = v
            del optimizer.state[old]
            optimizer.state[param] = stored_state
        group["params"][0] = param
        out[name] = param
    return out


def densify_and_prune(model, max_grad, min_opacity, extent, max_screen_size, radii, N: int = 2,
                      generator: torch.Generator = None) -> None:
    """``GaussianModel.densify_and_prune`` (gaussian_model.py:574-640) on MI355X."""
    model.tmp_radii = radii
    xyz = model._xyz
    _dev_check(xyz, "_xyz")
    device = xyz.device
    P = xyz.shape[0]
    names = {g["name"] for g in model.optimizer.param_groups}
    if names != {n for n, _, _ in GROUPS}:
        raise RuntimeError(f"densify_and_prune: optimizer groups {sorted(names)}, expected the six of "
                           "GaussianModel.training_setup")
    src = {name: _f32(getattr(model, attr), attr) for name, attr, _ in GROUPS}
    accum = _f32(model.xyz_gradient_accum, "xyz_gradient_accum").reshape(-1)
    denom = _f32(model.denom, "denom").reshape(-1)
    prm = _params(max_grad, min_opacity, extent, max_screen_size, model.percent_dense, N)
    lib = _lib.load()
    scratch = torch.empty(int(lib.gsr_densify_scratch_bytes(P)), dtype=torch.uint8, device=device)
    split_mask = torch.empty(P, dtype=torch.uint8, device=device)
    counts = (ctypes.c_longlong * 5)()
    with torch.cuda.device(device):
        rc = lib.gsr_densify_plan(P, accum.data_ptr(), denom.data_ptr(), src["opacity"].data_ptr(),
                                  src["scaling"].data_ptr(), ctypes.byref(prm), scratch.data_ptr(),
                                  split_mask.data_ptr(), counts, _stream(device))
    _lib.check(rc, "densify_and_prune (plan)")
    n_split, P_new = int(counts[3]), int(counts[4])

    # the split's samples, drawn as the reference draws them (gaussian_model.py:520-528)
    stds = torch.exp(src["scaling"][split_mask.bool()]).repeat(N, 1)
    means = torch.zeros((stds.size(0), 3), device=device)
    samples = torch.normal(mean=means, std=stds, generator=generator) if generator is not None else \
        torch.normal(mean=means, std=stds)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(samples, src=0)  # identical replicas
    samples = samples.contiguous()
    assert samples.shape[0] == N * n_split

    state = {g["name"]: model.optimizer.state.get(g["params"][0], None) for g in model.optimizer.param_groups}
    new, keep = [], {}
    for name, attr, role in GROUPS:
        s = src[name]
        width = int(math.prod(s.shape[1:]))
        dst = torch.empty((P_new,) + tuple(s.shape[1:]), dtype=torch.float32, device=device)
        st = state[name]
        m = v = dm = dv = None
        if st is not None and "exp_avg" in st:
            m, v = _f32(st["exp_avg"], f"{name} exp_avg"), _f32(st["exp_avg_sq"], f"{name} exp_avg_sq")
            dm, dv = torch.empty_like(dst), torch.empty_like(dst)
        keep[name] = (dst, dm, dv, (m, v))
        new.append(_lib.DensifyGroup(s.data_ptr(), dst.data_ptr(), m.data_ptr() if m is not None else None,
                                     v.data_ptr() if v is not None else None, dm.data_ptr() if dm is not None else None,
                                     dv.data_ptr() if dv is not None else None, int(width), role))
    groups = (_lib.DensifyGroup * len(new))(*new)
    with torch.cuda.device(device):
        rc = lib.gsr_densify_apply(P, scratch.data_ptr(), groups, len(new), src["rotation"].data_ptr(),
                                   samples.data_ptr() if samples.numel() else None, None, None, ctypes.byref(prm),
                                   _stream(device))
    _lib.check(rc, "densify_and_prune (apply)")

    replaced = _replace_in_optimizer(model.optimizer, {
        name: (dst, dm if dm is not None else None, dv if dv is not None else None)
        for name, (dst, dm, dv, _) in keep.items()})
    for name, attr, _ in GROUPS:
        setattr(model, attr, replaced[name])
    model.xyz_gradient_accum = torch.zeros((P_new, 1), device=device)
    model.denom = torch.zeros((P_new, 1), device=device)
    model.max_radii2D = torch.zeros((P_new), device=device)
    model.tmp_radii = None


def install(cls) -> None:
    """Bind the native densification as ``cls``'s methods (cls = the reference's GaussianModel)."""
    cls.add_densification_stats = add_densification_stats
    cls.densify_and_prune = densify_and_prune
