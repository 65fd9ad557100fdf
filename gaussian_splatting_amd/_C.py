"""Drop-in replacement of the reference's ``diff_gaussian_rasterization._C`` module.

Same three functions, same positional arguments, same return tuples as the
pybind11 module of the reference (``ext.cpp:15-19``; tensor handling in
``rasterize_points.cu:45-274``), implemented over the C ABI of libgsr.so
(include/gsr.h).  Only HIP-device tensors are accepted: there is no CPU path.

Error behaviour follows the reference: a malformed ``means3D`` raises
``RuntimeError("means3D must have dimensions (num_points, 3)")``
(rasterize_points.cu:69-71) and any failure inside the native library raises
``RuntimeError`` with the library's message.
"""
from __future__ import annotations

import ctypes
import os
import weakref
from typing import Optional, Tuple

import torch

from . import _lib

__all__ = ["rasterize_gaussians", "rasterize_gaussians_backward", "rasterize_gaussians_backward_screen",
           "gauss_backward_views", "view_block_floats", "view_pack_floats", "view_block_pack", "view_block_unpack", "view_block_index",
           "views_live_floats", "views_live_list",
           "mark_visible", "adamUpdate", "fusedssim",
           "fusedssim_backward", "forward_rebuilds", "debug_forward_state"]


# Sync-free forward (gsr_rasterize_forward_ex): the binning buffer is sized from a capacity
# hint -- a decaying maximum of recent num_rendered for the same (device, W, H) and point
# count, plus a margin -- so the forward never waits for the host mid-way.  A hint that
# turns out too small only costs a redo of the binning stage inside the library
# (forward_rebuilds() counts them).  One entry per (device, W, H): a new point count (after
# densification) replaces the old entry instead of piling up next to it.
# GSR_SYNC_FORWARD=1 restores the reference's synchronising forward.
_capacity: dict = {}
_CAP_MARGIN = 1.05
_CAP_DECAY = 0.98  # per forward; with the 1.05 margin a view 7% smaller than the last does not shrink the hint below the next
_INT_MAX = 2**31 - 1


def _capacity_hint(key, P: int) -> int:
    if os.environ.get("GSR_SYNC_FORWARD", "0") == "1":
        return 0
    p, last = _capacity.get(key, (P, 0))
    if p != P:
        return 0
    return min(_INT_MAX, int(last * _CAP_MARGIN) + 1024) if last > 0 else 0


def _note_rendered(key, P: int, nr: int) -> None:
    p, last = _capacity.get(key, (P, 0))
    _capacity[key] = (P, max(int(nr), int(last * _CAP_DECAY)) if p == P else int(nr))


def forward_rebuilds() -> int:
    """Forwards (process-wide) whose capacity hint was too small, so the binning stage was redone."""
    return int(_lib.load().gsr_forward_rebuilds())


# GSR_POISON=1 (the GPU test suite sets it): every scratch buffer the library requests is
# filled with 0xff bytes and every output the kernels are meant to overwrite completely is
# filled with NaN before the call, so a read of memory no kernel wrote, or an output element
# no kernel wrote, shows up in the parity tests instead of depending on what the caching
# allocator happened to hand out.
def _poison() -> bool:
    return os.environ.get("GSR_POISON", "0") == "1"


def _empty(shape, **kw) -> torch.Tensor:
    t = torch.empty(shape, **kw)
    if _poison():
        t.fill_(float("nan") if t.dtype.is_floating_point else -1)
    return t


def _stream_handle(device: torch.device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _require_device(t: torch.Tensor, name: str) -> None:
    if t.device.type != "cuda":
        raise RuntimeError(f"{name}: the MI355X rasterizer needs HIP device tensors, got a {t.device.type} tensor "
                           "(there is no CPU implementation)")


class _Inputs:
    """Keeps contiguous fp32 views alive for the duration of a native call."""

    def __init__(self, device: torch.device):
        self.device = device
        self.keep = []

    def opt(self, t: Optional[torch.Tensor], name: str, align16: bool = False) -> Optional[int]:
        """Device pointer of an optional input; an empty tensor means 'absent' (data_ptr()==nullptr)."""
        if t is None or t.numel() == 0:
            return None
        return self.req(t, name, align16)

    def radii(self, t: torch.Tensor) -> int:
        """Device pointer of the int32 radii, kept alive (a contiguous copy if needed) for the call."""
        _require_device(t, "radii")
        if t.dtype != torch.int32:
            raise RuntimeError(f"radii: expected an int32 tensor, got {t.dtype}")
        if t.device != self.device:
            raise RuntimeError(f"radii: tensor on {t.device}, expected {self.device}")
        t = t.contiguous()
        self.keep.append(t)
        return t.data_ptr()

    def req(self, t: torch.Tensor, name: str, align16: bool = False, small: bool = False) -> int:
        if small and t.device.type != "cuda":
            t = t.to(self.device)  # bg / matrices / campos: 3-16 floats
        _require_device(t, name)
        if t.dtype != torch.float32:
            raise RuntimeError(f"{name}: expected a float32 tensor, got {t.dtype}")
        if t.device != self.device:
            raise RuntimeError(f"{name}: tensor on {t.device}, expected {self.device}")
        t = t.contiguous()
        if align16 and t.data_ptr() % 16:
            t = t.clone()
        self.keep.append(t)
        return t.data_ptr()


class _Resizer:
    """The reference's resizeFunctional (rasterize_points.cu:29-43) as a C callback."""

    def __init__(self, tensor: torch.Tensor):
        # The callback closes over the tensor, not over self: a bound method would make a
        # reference cycle (self -> cb -> method -> self), so the multi-GB buffers would live
        # until Python's cyclic GC ran -- about twenty steps of them at 5M@4K (200 GB reserved).
        def resize(_ctx, nbytes):
            try:
                tensor.resize_(int(nbytes))
                if _poison():
                    tensor.fill_(255)
                return tensor.data_ptr()
            except Exception:  # e.g. out of memory: the library reports GSR_ERR_ALLOC
                return None

        self.cb = _lib.ALLOC_FN(resize)


def _present(t) -> bool:
    return t is not None and t.numel() != 0 and t.size(0) != 0


# The geometry buffers this process's forwards returned, by device address (weak: a freed buffer drops out).
# A backward given any other tensor at such an address -- a copy, a buffer restored from a checkpoint, a
# view -- makes the library forget that address's forward state first (include/gsr.h gsr_geom_forget), so
# the backward takes the record path after writing the record inputs instead of trusting a stale mark.
_FORWARD_GEOMS: "weakref.WeakValueDictionary[int, torch.Tensor]" = weakref.WeakValueDictionary()


def _own_geometry(geomBuffer: torch.Tensor) -> None:
    if geomBuffer.numel() == 0:
        return
    t = _FORWARD_GEOMS.get(geomBuffer.data_ptr())
    if t is None or t._cdata != geomBuffer._cdata:
        _lib.load().gsr_geom_forget(geomBuffer.data_ptr())


def rasterize_gaussians(*args, no_backward: bool = False) -> Tuple[int, torch.Tensor, torch.Tensor, torch.Tensor,
                                                                     torch.Tensor, torch.Tensor, torch.Tensor]:
    """RasterizeGaussiansCUDA (rasterize_points.cu:45-146).

    Positional arguments, as the pybind function takes them:
    ``(bg, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix, projmatrix,
    tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos, prefiltered, antialiasing, debug)``
    -- the vendored rasterizer's 20 -- or the 3DGS-accel build's 21, which insert ``dc`` ([P,1,3]) before ``sh``
    (then the rest coefficients [P,M,3]); see include/gsr.h gsr_rasterize_forward_dc.

    Returns ``(num_rendered, color[3,H,W], radii[P] int32, geomBuffer, binningBuffer, imgBuffer, invdepth[1,H,W])``.

    ``no_backward`` (an extension): no backward will follow (an eval / no_grad render), so the forward does not
    zero the atomic backward's accumulator rows beside its render ("bwd_atomic" 0 for this call; a backward
    of it would take the record path).
    """
    if len(args) == 21:
        (background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
         projmatrix, tan_fovx, tan_fovy, image_height, image_width, dc, sh, degree, campos, prefiltered,
         antialiasing, debug) = args
    elif len(args) == 20:
        (background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
         projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos, prefiltered, antialiasing,
         debug) = args
        dc = None
    else:
        raise TypeError(f"rasterize_gaussians(): expected 20 or 21 positional arguments, got {len(args)}")
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    _require_device(means3D, "means3D")
    device = means3D.device
    lib = _lib.load()
    P = means3D.size(0)
    H, W = int(image_height), int(image_width)
    f32 = dict(dtype=torch.float32, device=device)
    alloc = _empty if P > 0 else torch.zeros  # every pixel / Gaussian is written when P > 0
    out_color = alloc((3, H, W), **f32)
    out_invdepth = alloc((1, H, W), **f32)
    radii = alloc((P,), dtype=torch.int32, device=device)
    geom = torch.empty(0, dtype=torch.uint8, device=device)
    binning = torch.empty(0, dtype=torch.uint8, device=device)
    img = torch.empty(0, dtype=torch.uint8, device=device)
    if P == 0:
        return 0, out_color, radii, geom, binning, img, out_invdepth

    M = sh.size(1) if _present(sh) else 0
    split = dc is not None and _present(dc) and not _present(colors)
    ins = _Inputs(device)
    rg, rb, ri = _Resizer(geom), _Resizer(binning), _Resizer(img)
    nr = ctypes.c_int(0)
    cap = ctypes.c_int(0)
    key = (device.index, W, H)
    common_head = (rg.cb, None, rb.cb, None, ri.cb, None, P, int(degree), M,
                   ins.req(background, "bg", small=True), W, H, ins.req(means3D, "means3D"))
    sh_args = ((ins.req(dc, "dc"), ins.opt(sh, "sh", align16=True)) if split else (ins.opt(sh, "sh", align16=True),))
    common_tail = (
        ins.opt(colors, "colors_precomp"), ins.req(opacity, "opacities"), ins.opt(scales, "scales"),
        float(scale_modifier), ins.opt(rotations, "rotations", align16=True), ins.opt(cov3D_precomp, "cov3D_precomp"),
        ins.req(viewmatrix, "viewmatrix", small=True), ins.req(projmatrix, "projmatrix", small=True),
        ins.opt(campos if campos is not None and campos.device.type == "cuda" else
                (campos.to(device) if campos is not None else None), "campos"),
        float(tan_fovx), float(tan_fovy), int(bool(prefiltered)), out_color.data_ptr(), out_invdepth.data_ptr(),
        int(bool(antialiasing)), radii.data_ptr(), int(bool(debug)), _stream_handle(device), ctypes.byref(nr),
        _capacity_hint(key, P), ctypes.byref(cap))
    fn = lib.gsr_rasterize_forward_dc if split else lib.gsr_rasterize_forward_ex
    with torch.cuda.device(device):
        if no_backward:
            with _lib.thread_options(bwd_atomic=0):
                rc = fn(*common_head, *sh_args, *common_tail)
        else:
            rc = fn(*common_head, *sh_args, *common_tail)
    _lib.check(rc, "rasterize_gaussians")
    _FORWARD_GEOMS[geom.data_ptr()] = geom
    _note_rendered(key, P, nr.value)
    # The binning buffer's layout (its capacity) is recovered by the backward from the buffer's
    # size (include/gsr.h gsr_rasterize_backward_ex), so nothing rides on the tensor object.
    return int(nr.value), out_color, radii, geom, binning, img, out_invdepth


def rasterize_gaussians_backward(*args, out=None):
    """RasterizeGaussiansBackwardCUDA (rasterize_points.cu:149-248).

    Positional arguments: the vendored rasterizer's 24 ``(bg, means3D, radii, colors, opacities, scales,
    rotations, scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color,
    dL_dout_invdepth, sh, degree, campos, geomBuffer, R, binningBuffer, imageBuffer, antialiasing, debug)``,
    or the 3DGS-accel build's 25 with ``dc`` before ``sh``.

    Returns ``(dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations)``,
    or, with ``dc``, ``(..., dL_dcov3D, dL_ddc, dL_dsh, ...)`` (9 tensors, as the accel build returns them).
    ``out`` (an extension, not in the reference) may map any of the names ``dL_dmeans3D, dL_ddc, dL_dsh,
    dL_dopacity, dL_dscales, dL_drotations`` to preallocated contiguous float32 tensors of the right shape --
    e.g. views of one flat gradient arena that is then all-reduced without a copy.
    """
    if len(args) == 25:
        (background, means3D, radii, colors, opacities, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
         projmatrix, tan_fovx, tan_fovy, dL_dout_color, dL_dout_invdepth, dc, sh, degree, campos, geomBuffer, R,
         binningBuffer, imageBuffer, antialiasing, debug) = args
        accel = True
    elif len(args) == 24:
        (background, means3D, radii, colors, opacities, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
         projmatrix, tan_fovx, tan_fovy, dL_dout_color, dL_dout_invdepth, sh, degree, campos, geomBuffer, R,
         binningBuffer, imageBuffer, antialiasing, debug) = args
        dc, accel = None, False
    else:
        raise TypeError(f"rasterize_gaussians_backward(): expected 24 or 25 positional arguments, got {len(args)}")
    _require_device(means3D, "means3D")
    device = means3D.device
    lib = _lib.load()
    P = means3D.size(0)
    H, W = int(dL_dout_color.size(1)), int(dL_dout_color.size(2))
    M = sh.size(1) if _present(sh) else 0
    split = accel and dc is not None and _present(dc) and not _present(colors)
    f32 = dict(dtype=torch.float32, device=device)
    alloc = _empty if P > 0 else torch.zeros
    out = dict(out or {})

    def buf(name, shape):
        t = out.get(name)
        if t is None:
            return alloc(shape, **f32)
        if tuple(t.shape) != tuple(shape) or t.dtype != torch.float32 or not t.is_contiguous() or t.device != device:
            raise RuntimeError(f"out[{name}] must be a contiguous float32 {tuple(shape)} tensor on {device}")
        return t

    dL_dmeans2D = alloc((P, 3), **f32)
    dL_dcolors = alloc((P, 3), **f32)
    dL_dopacity = buf("dL_dopacity", (P, 1))
    dL_dmeans3D = buf("dL_dmeans3D", (P, 3))
    dL_dcov3D = alloc((P, 6), **f32)
    # the accel build always returns a [P,1,3] dc gradient (zeros when colours were precomputed)
    dL_ddc = buf("dL_ddc", (P, 1, 3)) if accel else None
    dL_dsh = buf("dL_dsh", (P, M, 3))
    dL_dscales = buf("dL_dscales", (P, 3))
    dL_drotations = buf("dL_drotations", (P, 4))
    has_inv = dL_dout_invdepth is not None and dL_dout_invdepth.numel() != 0 and dL_dout_invdepth.size(0) != 0
    dL_dinvdepths = alloc((P, 1), **f32) if has_inv else None
    if accel:
        result = (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_ddc, dL_dsh, dL_dscales,
                  dL_drotations)
    else:
        result = (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations)
    if P == 0:
        return result
    if accel and not split:
        dL_ddc.zero_()  # no SH evaluation: the dc gradient is zero, as the accel build's zero-initialised tensor

    ins = _Inputs(device)
    scratch = torch.empty(0, dtype=torch.uint8, device=device)
    rs = _Resizer(scratch)
    _own_geometry(geomBuffer)
    head = (P, int(degree), M, int(R), ins.req(background, "bg", small=True), W, H, ins.req(means3D, "means3D"))
    sh_args = ((ins.req(dc, "dc"), ins.opt(sh, "sh")) if split else (ins.opt(sh, "sh"),))
    mid = (ins.opt(colors, "colors_precomp"),
           ins.req(opacities, "opacities"), ins.opt(scales, "scales"), float(scale_modifier),
           ins.opt(rotations, "rotations", align16=True), ins.opt(cov3D_precomp, "cov3D_precomp"),
           ins.req(viewmatrix, "viewmatrix", small=True), ins.req(projmatrix, "projmatrix", small=True),
           ins.opt(campos if campos is not None and campos.device.type == "cuda" else
                   (campos.to(device) if campos is not None else None), "campos"),
           float(tan_fovx), float(tan_fovy), ins.radii(radii), geomBuffer.data_ptr(),
           binningBuffer.data_ptr() if binningBuffer.numel() else None, imageBuffer.data_ptr(),
           ins.req(dL_dout_color, "dL_dout_color"),
           ins.req(dL_dout_invdepth, "dL_dout_invdepth") if has_inv else None,
           dL_dmeans2D.data_ptr(), None, dL_dopacity.data_ptr(), dL_dcolors.data_ptr(),
           dL_dinvdepths.data_ptr() if has_inv else None, dL_dmeans3D.data_ptr(), dL_dcov3D.data_ptr())
    sh_grads = ((dL_ddc.data_ptr(), dL_dsh.data_ptr() if M > 0 else None) if split else
                (dL_dsh.data_ptr() if M > 0 else None,))
    tail = (dL_dscales.data_ptr(), dL_drotations.data_ptr(), int(bool(antialiasing)), int(bool(debug)), rs.cb, None,
            _stream_handle(device), 0, int(binningBuffer.numel()))
    fn = lib.gsr_rasterize_backward_dc if split else lib.gsr_rasterize_backward_ex
    with torch.cuda.device(device):
        rc = fn(*head, *sh_args, *mid, *sh_grads, *tail)
    _lib.check(rc, "rasterize_gaussians_backward")
    return result


def debug_forward_state(fwd, P: int) -> dict:
    """The forward's private tile lists and per-pixel state (include/gsr.h gsr_debug_forward_state),
    for parity tests: ``ranges`` [tiles, 2], ``point_list`` [R] (Gaussian indices, tile-major, each
    tile in (depth, index) order), ``n_contrib`` [H, W], ``final_T`` [H, W]; int64 / float32 CPU
    tensors.  ``fwd`` is the tuple ``rasterize_gaussians`` returned."""
    num_rendered, color, _radii, geom, binning, img, _inv = fwd
    H, W = int(color.size(1)), int(color.size(2))
    device = color.device
    tiles = ((W + 15) // 16) * ((H + 15) // 16)
    i32 = dict(dtype=torch.int32, device=device)
    ranges = torch.zeros((tiles, 2), **i32)
    plist = torch.zeros((max(int(num_rendered), 1),), **i32)
    n_contrib = torch.zeros((H, W), **i32)
    final_T = torch.zeros((H, W), dtype=torch.float32, device=device)
    lib = _lib.load()
    with torch.cuda.device(device):
        rc = lib.gsr_debug_forward_state(int(P), W, H, int(num_rendered), 0, int(binning.numel()), geom.data_ptr(),
                                         binning.data_ptr() if binning.numel() else None, img.data_ptr(),
                                         ranges.data_ptr(), plist.data_ptr(), n_contrib.data_ptr(),
                                         final_T.data_ptr(), _stream_handle(device))
    _lib.check(rc, "debug_forward_state")
    u = lambda t: t.cpu().numpy().view("uint32").astype("int64")  # noqa: E731
    return {"ranges": torch.from_numpy(u(ranges)), "point_list": torch.from_numpy(u(plist)[:int(num_rendered)] >> 4),
            "n_contrib": torch.from_numpy(u(n_contrib)), "final_T": final_T.cpu()}


def debug_sort_state(fwd, P: int) -> dict:
    """The forward's reachable-prefix sort state (include/gsr.h gsr_debug_sort_state): ``sorted_len``
    [tiles] (entries of each tile list in final order) and ``redo_count`` (tiles the forward
    rendered again because a wave passed its sorted prefix); int64 CPU tensor / int."""
    num_rendered, color, _radii, geom, binning, img, _inv = fwd
    H, W = int(color.size(1)), int(color.size(2))
    device = color.device
    tiles = ((W + 15) // 16) * ((H + 15) // 16)
    sl = torch.zeros(tiles, dtype=torch.int32, device=device)
    rc = torch.zeros(1, dtype=torch.int32, device=device)
    with torch.cuda.device(device):
        r = _lib.load().gsr_debug_sort_state(int(P), W, H, geom.data_ptr(), sl.data_ptr(), rc.data_ptr(),
                                             _stream_handle(device))
    _lib.check(r, "debug_sort_state")
    return {"sorted_len": sl.cpu().long(), "redo_count": int(rc.item())}


def debug_near_state(fwd, P: int) -> dict:
    """The forward's near-first binning state (include/gsr.h gsr_debug_near_state): ``zcut`` (the depth bin
    of its cut, None when there was none) and ``near_len`` [tiles] (entries keyed and sorted per tile;
    the whole list lengths when there was no cut); int / int64 CPU tensor."""
    num_rendered, color, _radii, geom, binning, img, _inv = fwd
    H, W = int(color.size(1)), int(color.size(2))
    device = color.device
    tiles = ((W + 15) // 16) * ((H + 15) // 16)
    zc = torch.zeros(1, dtype=torch.int32, device=device)
    nr = torch.zeros((tiles, 2), dtype=torch.int32, device=device)
    with torch.cuda.device(device):
        r = _lib.load().gsr_debug_near_state(int(P), W, H, geom.data_ptr(), zc.data_ptr(), nr.data_ptr(),
                                             _stream_handle(device))
    _lib.check(r, "debug_near_state")
    cut = int(zc.item()) & 0xFFFFFFFF
    st = debug_forward_state(fwd, P)
    rg = st["ranges"]
    if cut == 0xFFFFFFFF:
        return {"zcut": None, "near_len": rg[:, 1] - rg[:, 0]}
    n = nr.cpu().numpy().view("uint32").astype("int64")
    return {"zcut": cut, "near_len": torch.from_numpy(n[:, 1] - n[:, 0])}


def view_block_floats(P: int) -> int:
    """Floats in one view block (include/gsr.h, multi-GPU view exchange)."""
    return int(_lib.load().gsr_view_block_floats(int(P)))


def view_pack_floats(entries: int) -> int:
    """Floats of a packed (sparse) view block holding ``entries`` entries (include/gsr.h)."""
    return int(_lib.load().gsr_view_pack_floats(int(entries)))


def _range(P, rng):
    g0, g1 = (0, P) if rng is None else (int(rng[0]), int(rng[1]))
    if not 0 <= g0 <= g1 <= P:
        raise RuntimeError(f"Gaussian range [{g0}, {g1}) outside [0, {P})")
    return g0, g1


def view_block_pack(view_block: torch.Tensor, packed: torch.Tensor, scratch: torch.Tensor, count: torch.Tensor,
                    P: int, rng=None) -> None:
    """Pack a dense view block into ``packed`` (capacity from its size); the entry count lands in
    ``count`` (an int32 device tensor of one element) and in the packed header (include/gsr.h
    gsr_view_block_pack).  Only Gaussians with a non-zero render gradient are kept; with ``rng`` =
    (g0, g1) only those of Gaussians [g0, g1) (one chunk of a chunked exchange)."""
    g0, g1 = _range(P, rng)
    _require_device(view_block, "view_block")
    nb = view_block_floats(P)
    if view_block.numel() != nb or view_block.dtype != torch.float32 or not view_block.is_contiguous():
        raise RuntimeError(f"view_block must be a contiguous float32 tensor of {nb} values")
    cap = (packed.numel() - 64) // 12
    if packed.dtype != torch.float32 or not packed.is_contiguous() or cap < 0:
        raise RuntimeError("packed must be a contiguous float32 tensor of at least 64 values")
    need = int(_lib.load().gsr_view_pack_scratch_bytes(int(P)))
    if scratch.numel() * scratch.element_size() < need or count.numel() != 1 or count.dtype != torch.int32:
        raise RuntimeError("view_block_pack: scratch too small or count not an int32 scalar tensor")
    lib = _lib.load()
    with torch.cuda.device(view_block.device):
        rc = lib.gsr_view_block_pack_range(int(P), g0, g1, view_block.data_ptr(), packed.data_ptr(), int(cap),
                                           scratch.data_ptr(), count.data_ptr(), _stream_handle(view_block.device))
    _lib.check(rc, "view_block_pack")


def view_block_unpack(packed: torch.Tensor, blocks: torch.Tensor, P: int) -> None:
    """Unpack ``packed`` ([n_views, packed_floats]) into dense view blocks ``blocks``
    ([n_views, view_block_floats(P)]; include/gsr.h gsr_view_block_unpack)."""
    _require_device(packed, "packed")
    nb = view_block_floats(P)
    if packed.dim() != 2 or blocks.dim() != 2 or blocks.size(1) != nb or packed.size(0) != blocks.size(0):
        raise RuntimeError(f"packed [n_views, k] and blocks [n_views, {nb}] expected")
    if not (packed.is_contiguous() and blocks.is_contiguous()):
        raise RuntimeError("packed and blocks must be contiguous")
    cap = (packed.size(1) - 64) // 12
    lib = _lib.load()
    with torch.cuda.device(packed.device):
        rc = lib.gsr_view_block_unpack(int(P), int(packed.size(0)), packed.data_ptr(), int(packed.size(1)),
                                       blocks.data_ptr(), int(cap), _stream_handle(packed.device))
    _lib.check(rc, "view_block_unpack")


def view_block_index(packed: torch.Tensor, flags: torch.Tensor, P: int, rng=None) -> None:
    """Index ``packed`` ([n_views, packed_floats]) for ``gauss_backward_views(..., flags=flags)``:
    ``flags`` ([n_views, P] int32) is cleared and, for each packed entry i of view v, flags[v, g] =
    i << 4 | its flag bits (include/gsr.h gsr_view_block_index); with ``rng`` = (g0, g1) only the
    flags of Gaussians [g0, g1) (the packed blocks of one chunk)."""
    g0, g1 = _range(P, rng)
    _require_device(packed, "packed")
    if packed.dim() != 2 or flags.dim() != 2 or tuple(flags.shape) != (packed.size(0), P):
        raise RuntimeError(f"packed [n_views, k] and flags [n_views, {P}] expected")
    if flags.dtype != torch.int32 or not (packed.is_contiguous() and flags.is_contiguous()):
        raise RuntimeError("packed (float32) and flags (int32) must be contiguous")
    cap = (packed.size(1) - 64) // 12
    lib = _lib.load()
    with torch.cuda.device(packed.device):
        rc = lib.gsr_view_block_index_range(int(P), g0, g1, int(packed.size(0)), packed.data_ptr(),
                                            int(packed.size(1)), flags.data_ptr(), int(cap),
                                            _stream_handle(packed.device))
    _lib.check(rc, "view_block_index")


def views_live_floats(P: int) -> int:
    """int32 words of a live-list buffer for ``views_live_list`` (include/gsr.h)."""
    return int(_lib.load().gsr_views_live_floats(int(P)))


def views_live_list(flags: torch.Tensor, live: torch.Tensor, P: int, rng=None) -> None:
    """The Gaussians some view flags (``flags`` from ``view_block_index``) into ``live``
    (int32, ``views_live_floats(P)`` words), for ``gauss_backward_views(..., live=live)``; with
    ``rng`` = (g0, g1) only Gaussians [g0, g1)."""
    g0, g1 = _range(P, rng)
    _require_device(flags, "flags")
    if flags.dim() != 2 or flags.size(1) != P or flags.dtype != torch.int32 or not flags.is_contiguous():
        raise RuntimeError(f"flags must be a contiguous int32 [n_views, {P}] tensor")
    if live.dtype != torch.int32 or live.numel() < views_live_floats(P) or not live.is_contiguous():
        raise RuntimeError(f"live must be a contiguous int32 tensor of {views_live_floats(P)} words")
    lib = _lib.load()
    with torch.cuda.device(flags.device):
        rc = lib.gsr_views_live_list_range(int(P), g0, g1, int(flags.size(0)), flags.data_ptr(), live.data_ptr(),
                                           _stream_handle(flags.device))
    _lib.check(rc, "views_live_list")


def rasterize_gaussians_backward_screen(*args, view_block: torch.Tensor) -> None:
    """The backward of ``rasterize_gaussians_backward`` up to the per-Gaussian render-gradient
    sums, written with the camera into ``view_block`` (a float32 tensor of
    ``view_block_floats(P)`` values; include/gsr.h ``gsr_rasterize_backward_screen``).
    Arguments as ``rasterize_gaussians_backward`` (24, or 25 with ``dc``); colours from SH and
    cov3D from scales / rotations.  The rest of the backward, over any number of gathered
    views, is ``gauss_backward_views``."""
    if len(args) == 25:
        (background, means3D, radii, colors, opacities, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
         projmatrix, tan_fovx, tan_fovy, dL_dout_color, dL_dout_invdepth, dc, sh, degree, campos, geomBuffer, R,
         binningBuffer, imageBuffer, antialiasing, debug) = args
    elif len(args) == 24:
        (background, means3D, radii, colors, opacities, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
         projmatrix, tan_fovx, tan_fovy, dL_dout_color, dL_dout_invdepth, sh, degree, campos, geomBuffer, R,
         binningBuffer, imageBuffer, antialiasing, debug) = args
        dc = None
    else:
        raise TypeError(f"rasterize_gaussians_backward_screen(): expected 24 or 25 positional arguments, got {len(args)}")
    if _present(colors) or _present(cov3D_precomp):
        raise RuntimeError("rasterize_gaussians_backward_screen: precomputed colours / cov3D are per view; "
                           "use rasterize_gaussians_backward")
    _require_device(means3D, "means3D")
    device = means3D.device
    P = means3D.size(0)
    nb = view_block_floats(P)
    if (view_block.dtype != torch.float32 or not view_block.is_contiguous() or view_block.numel() != nb
            or view_block.device != device):
        raise RuntimeError(f"view_block must be a contiguous float32 tensor of {nb} values on {device}")
    if P == 0:
        return
    lib = _lib.load()
    H, W = int(dL_dout_color.size(1)), int(dL_dout_color.size(2))
    M = sh.size(1) if _present(sh) else 0
    has_inv = dL_dout_invdepth is not None and dL_dout_invdepth.numel() != 0 and dL_dout_invdepth.size(0) != 0
    ins = _Inputs(device)
    scratch = torch.empty(0, dtype=torch.uint8, device=device)
    rs = _Resizer(scratch)
    _own_geometry(geomBuffer)
    with torch.cuda.device(device):
        rc = lib.gsr_rasterize_backward_screen(
            P, int(degree), M, int(R), ins.req(background, "bg", small=True), W, H, ins.req(means3D, "means3D"),
            ins.opt(dc, "dc") if _present(dc) else None, ins.opt(sh, "sh"), ins.req(opacities, "opacities"),
            ins.req(scales, "scales"), float(scale_modifier), ins.req(rotations, "rotations", align16=True),
            ins.req(viewmatrix, "viewmatrix", small=True), ins.req(projmatrix, "projmatrix", small=True),
            ins.req(campos if campos.device.type == "cuda" else campos.to(device), "campos"),
            float(tan_fovx), float(tan_fovy), ins.radii(radii), geomBuffer.data_ptr(),
            binningBuffer.data_ptr() if binningBuffer.numel() else None, imageBuffer.data_ptr(),
            ins.req(dL_dout_color, "dL_dout_color"),
            ins.req(dL_dout_invdepth, "dL_dout_invdepth") if has_inv else None,
            int(bool(antialiasing)), int(bool(debug)), rs.cb, None, _stream_handle(device),
            0, int(binningBuffer.numel()), view_block.data_ptr())
    _lib.check(rc, "rasterize_gaussians_backward_screen")


def gauss_backward_views(means3D, dc, sh, degree, opacities, scales, rotations, scale_modifier, blocks, out,
                         flags=None, live=None) -> None:
    """The per-Gaussian backward summed over ``blocks`` ([n_views, view_block_floats(P)] float32,
    e.g. an all-gathered exchange buffer), written into ``out`` (names as the ``out=`` of
    ``rasterize_gaussians_backward``: dL_dmeans3D, dL_ddc (when dc is given), dL_dsh,
    dL_dopacity, dL_dscales, dL_drotations; contiguous float32).  With ``flags`` (from
    ``view_block_index``), ``blocks`` are packed blocks ([n_views, packed_floats]) read in place;
    with ``live`` too (``views_live_list``) only the listed Gaussians' rows are written -- the
    caller zeroes ``out`` beforehand."""
    _require_device(means3D, "means3D")
    device = means3D.device
    P = means3D.size(0)
    nb = view_block_floats(P) if flags is None else int(blocks.size(1)) if blocks.dim() == 2 else -1
    if blocks.dim() != 2 or blocks.size(1) != nb or blocks.dtype != torch.float32 or not blocks.is_contiguous():
        raise RuntimeError(f"blocks must be a contiguous float32 [n_views, {nb}] tensor")
    if flags is not None and (tuple(flags.shape) != (blocks.size(0), P) or flags.dtype != torch.int32 or
                              not flags.is_contiguous()):
        raise RuntimeError(f"flags must be a contiguous int32 [{blocks.size(0)}, {P}] tensor")
    M = sh.size(1) if _present(sh) else 0
    need = {"dL_dmeans3D": (P, 3), "dL_dsh": (P, M, 3), "dL_dopacity": (P, 1), "dL_dscales": (P, 3),
            "dL_drotations": (P, 4)}
    if _present(dc):
        need["dL_ddc"] = (P, 1, 3)
    for k, shp in need.items():
        t = out.get(k)
        if t is None or tuple(t.shape) != shp or t.dtype != torch.float32 or not t.is_contiguous() or t.device != device:
            raise RuntimeError(f"out[{k}] must be a contiguous float32 {shp} tensor on {device}")
    if P == 0:
        return
    lib = _lib.load()
    ins = _Inputs(device)
    geo = (P, int(degree), M, ins.req(means3D, "means3D"), ins.opt(dc, "dc") if _present(dc) else None,
           ins.opt(sh, "sh"), ins.req(opacities, "opacities"), ins.req(scales, "scales"),
           ins.req(rotations, "rotations", align16=True), float(scale_modifier), int(blocks.size(0)),
           blocks.data_ptr(), nb)
    outs = (out["dL_dmeans3D"].data_ptr(), out["dL_ddc"].data_ptr() if _present(dc) else None,
            out["dL_dsh"].data_ptr() if M > 0 else None, out["dL_dopacity"].data_ptr(), out["dL_dscales"].data_ptr(),
            out["dL_drotations"].data_ptr(), _stream_handle(device))
    with torch.cuda.device(device):
        if flags is None:
            rc = lib.gsr_gauss_backward_views(*geo, *outs)
        elif live is None:
            rc = lib.gsr_gauss_backward_views_packed(*geo, flags.data_ptr(), *outs)
        else:
            rc = lib.gsr_gauss_backward_views_live(*geo, flags.data_ptr(), live.data_ptr(), *outs)
    _lib.check(rc, "gauss_backward_views")


def mark_visible(means3D, viewmatrix, projmatrix) -> torch.Tensor:
    """markVisible (rasterize_points.cu:250-274): bool[P], view-space z > 0.2."""
    _require_device(means3D, "means3D")
    device = means3D.device
    lib = _lib.load()
    P = means3D.size(0)
    present = torch.zeros(P, dtype=torch.bool, device=device)
    if P == 0:
        return present
    ins = _Inputs(device)
    with torch.cuda.device(device):
        rc = lib.gsr_mark_visible(P, ins.req(means3D, "means3D"), ins.req(viewmatrix, "viewmatrix", small=True),
                                  ins.req(projmatrix, "projmatrix", small=True), present.data_ptr(),
                                  _stream_handle(device))
    _lib.check(rc, "mark_visible")
    return present


def adamUpdate(param, param_grad, exp_avg, exp_avg_sq, visible, lr, b1, b2, eps, N, M):
    """The 3DGS-accel build's ``_C.adamUpdate`` (SparseGaussianAdam's per-group call; include/gsr_adam.h)."""
    from .optim import adam_update

    adam_update(param, param_grad, exp_avg, exp_avg_sq, visible, lr, b1, b2, eps, N, M)


# ---- fused SSIM as utils/loss_utils.py:16-37 expects it from this module ------------------
# The reference's loss_utils tries ``from diff_gaussian_rasterization._C import fusedssim,
# fusedssim_backward`` (the 3DGS-accel rasterizer's two-function variant: the forward returns
# only the map, the backward takes the upstream gradient and recomputes what it needs).  Both
# run on the same gfx950 kernels as fused_ssim_cuda (csrc/ssim.hip).
def fusedssim(C1, C2, img1, img2):
    """SSIM map of img1 vs img2 ([C,H,W] or [B,C,H,W], float32, HIP device), 'same' padding."""
    import fused_ssim_cuda

    a, b = (img1.unsqueeze(0), img2.unsqueeze(0)) if img1.dim() == 3 else (img1, img2)
    ssim_map = fused_ssim_cuda.fusedssim(C1, C2, a, b, False)[0]
    return ssim_map[0] if img1.dim() == 3 else ssim_map


def fusedssim_backward(C1, C2, img1, img2, opt_grad):
    """dL/dimg1 given dL/dmap; the derivative maps are recomputed (one extra forward pass)."""
    import fused_ssim_cuda

    squeeze = img1.dim() == 3
    a, b, g = (t.unsqueeze(0) for t in (img1, img2, opt_grad)) if squeeze else (img1, img2, opt_grad)
    _, d1, d2, d3 = fused_ssim_cuda.fusedssim(C1, C2, a, b, True)
    grad = fused_ssim_cuda.fusedssim_backward(C1, C2, a, b, g, d1, d2, d3)
    return grad[0] if squeeze else grad
