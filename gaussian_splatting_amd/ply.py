"""PLY scene I/O of the reference, over the native reader/writer of ``csrc/ply.cpp``
(C ABI: include/gsr_ply.h).  The reference uses the ``plyfile`` package, which this image
does not have (loading trained ``point_cloud.ply`` scenes).

* ``save_ply(model, path)`` / ``load_ply(model, path, use_train_test_exp=False)`` /
  ``construct_list_of_attributes(model)``: ``GaussianModel``'s methods
  (scene/gaussian_model.py:288-376), same property names and order, same SH layout
  (``f_dc`` / ``f_rest`` stored channel-major: ``transpose(1, 2).flatten(1)``), float32
  binary little-endian, the same header plyfile writes;
* ``store_ply(path, xyz, rgb)`` / ``fetch_ply(path)``: ``storePly`` / ``fetchPly``
  (scene/dataset_readers.py:120-143), uint8 colours;
* ``install(GaussianModel)`` binds the three methods; ``install_dataset_readers(module)``
  replaces ``storePly`` / ``fetchPly`` in ``scene.dataset_readers``.

The file work is host code (no GPU): the model's tensors are copied to and from the device
around it, as the reference does.
"""
from __future__ import annotations

import ctypes
import json
import os
from typing import Dict, List, NamedTuple, Sequence, Tuple

import numpy as np

from . import _lib

__all__ = ["read_vertex", "read_vertex_raw", "vertex_properties", "vertex_schema", "write_vertex", "construct_list_of_attributes", "save_ply", "load_ply",
           "store_ply", "fetch_ply", "BasicPointCloud", "install", "install_dataset_readers"]


class BasicPointCloud(NamedTuple):  # utils/graphics_utils.py's tuple
    points: np.ndarray
    colors: np.ndarray
    normals: np.ndarray


def _open(path: str):
    lib = _lib.load()
    h = ctypes.c_void_p()
    _lib.check(lib.gsr_ply_open(os.fsencode(path), ctypes.byref(h)), f"ply open {path}")
    return lib, h


def vertex_properties(path: str) -> Tuple[int, List[str]]:
    """(vertex count, vertex property names in file order)."""
    lib, h = _open(path)
    try:
        n = lib.gsr_ply_vertex_count(h)
        names = [lib.gsr_ply_property_name(h, i).decode() for i in range(lib.gsr_ply_property_count(h))]
        return int(n), names
    finally:
        lib.gsr_ply_close(h)


def vertex_schema(path: str) -> Tuple[int, List[str], List[Tuple[int, str]]]:
    """(vertex count, property names, (bytes, kind) per property: kind 'i' / 'u' / 'f', or
    'l' for a list property)."""
    lib, h = _open(path)
    try:
        n = int(lib.gsr_ply_vertex_count(h))
        names, types = [], []
        for i in range(lib.gsr_ply_property_count(h)):
            names.append(lib.gsr_ply_property_name(h, i).decode())
            b, k = ctypes.c_int(), ctypes.c_char()
            _lib.check(lib.gsr_ply_property_type(h, i, ctypes.byref(b), ctypes.byref(k)), "ply property type")
            types.append((b.value, k.value.decode()))
        return n, names, types
    finally:
        lib.gsr_ply_close(h)


def read_vertex_raw(path: str, names: Sequence[str], out: Dict[str, np.ndarray]) -> None:
    """Fill ``out[name]`` (1-D arrays, possibly strided, of the property's own size) with the
    named vertex properties in their file types, host byte order."""
    lib, h = _open(path)
    try:
        N = int(lib.gsr_ply_vertex_count(h))
        k = len(names)
        for n in names:
            if out[n].ndim != 1 or out[n].shape[0] != N:
                raise ValueError(f"output for '{n}' must be a vector of {N}")
        c_names = (ctypes.c_char_p * k)(*[n.encode() for n in names])
        ptrs = (ctypes.c_void_p * k)(*[out[n].ctypes.data for n in names])
        strides = (ctypes.c_longlong * k)(*[out[n].strides[0] for n in names])
        _lib.check(lib.gsr_ply_read_raw(h, k, c_names, ptrs, strides), f"ply read {path}")
    finally:
        lib.gsr_ply_close(h)


def read_vertex(path: str, names: Sequence[str], out: Dict[str, np.ndarray] = None) -> Dict[str, np.ndarray]:
    """The named vertex properties as float32 columns (``out[name]`` may supply strided float32
    views of length N to fill in place)."""
    lib, h = _open(path)
    try:
        N = int(lib.gsr_ply_vertex_count(h))
        cols = {}
        for n in names:
            a = out[n] if out is not None and n in out else np.empty(N, np.float32)
            if a.dtype != np.float32 or a.ndim != 1 or a.shape[0] != N:
                raise ValueError(f"output for '{n}' must be a float32 vector of {N}")
            cols[n] = a
        k = len(names)
        c_names = (ctypes.c_char_p * k)(*[n.encode() for n in names])
        ptrs = (ctypes.c_void_p * k)(*[cols[n].ctypes.data for n in names])
        strides = (ctypes.c_longlong * k)(*[cols[n].strides[0] for n in names])
        _lib.check(lib.gsr_ply_read_float(h, k, c_names, ptrs, strides), f"ply read {path}")
        return cols
    finally:
        lib.gsr_ply_close(h)


_CODES = {"i1": b"b", "u1": b"B", "i2": b"h", "u2": b"H", "i4": b"i", "u4": b"I", "f4": b"f", "f8": b"d"}


def write_vertex(path: str, columns: Sequence[Tuple[str, np.ndarray]], element: str = "vertex") -> None:
    """One vertex element; each column a 1-D numeric array of a PLY scalar type (int8 ... float64;
    strided views such as structured-array fields are fine)."""
    if element != "vertex":
        raise NotImplementedError(f"only a 'vertex' element can be written, not '{element}'")
    if not columns:
        raise ValueError("write_vertex: no columns")
    N = columns[0][1].shape[0]
    names, types, ptrs, strides, keep = [], b"", [], [], []
    for name, a in columns:
        if a.ndim != 1 or a.shape[0] != N:
            raise ValueError(f"column '{name}' must be 1-D of length {N}")
        code = _CODES.get(a.dtype.str[1:]) if a.dtype.byteorder in "=<|" else None
        if code is None:
            raise ValueError(f"column '{name}': dtype {a.dtype} is not a little-endian PLY scalar type")
        types += code
        keep.append(a)
        names.append(name.encode())
        ptrs.append(a.ctypes.data)
        strides.append(a.strides[0])
    k = len(columns)
    lib = _lib.load()
    rc = lib.gsr_ply_write(os.fsencode(path), N, k, (ctypes.c_char_p * k)(*names), types,
                           (ctypes.c_void_p * k)(*ptrs), (ctypes.c_longlong * k)(*strides))
    _lib.check(rc, f"ply write {path}")


# ---- GaussianModel (scene/gaussian_model.py:288-376) ------------------------------------
def construct_list_of_attributes(model) -> List[str]:
    l = ["x", "y", "z", "nx", "ny", "nz"]
    for i in range(model._features_dc.shape[1] * model._features_dc.shape[2]):
        l.append(f"f_dc_{i}")
    for i in range(model._features_rest.shape[1] * model._features_rest.shape[2]):
        l.append(f"f_rest_{i}")
    l.append("opacity")
    for i in range(model._scaling.shape[1]):
        l.append(f"scale_{i}")
    for i in range(model._rotation.shape[1]):
        l.append(f"rot_{i}")
    return l


def save_ply(model, path: str) -> None:
    """``GaussianModel.save_ply``: x y z, zero normals, f_dc_*, f_rest_* (channel-major),
    opacity, scale_*, rot_*, float32."""
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)  # mkdir_p
    xyz = model._xyz.detach().cpu().numpy().astype(np.float32, copy=False)
    normals = np.zeros_like(xyz)
    f_dc = model._features_dc.detach().transpose(1, 2).flatten(start_dim=1).contiguous().cpu().numpy()
    f_rest = model._features_rest.detach().transpose(1, 2).flatten(start_dim=1).contiguous().cpu().numpy()
    opacities = model._opacity.detach().cpu().numpy()
    scale = model._scaling.detach().cpu().numpy()
    rotation = model._rotation.detach().cpu().numpy()
    attributes = [xyz, normals, f_dc, f_rest, opacities, scale, rotation]
    names = construct_list_of_attributes(model)
    cols, j = [], 0
    for block in attributes:
        block = np.asarray(block, np.float32).reshape(block.shape[0], -1)
        for c in range(block.shape[1]):
            cols.append((names[j], block[:, c]))
            j += 1
    assert j == len(names)
    write_vertex(path, cols)


def _sorted_by_suffix(names, prefix):
    sel = [n for n in names if n.startswith(prefix)]
    return sorted(sel, key=lambda x: int(x.split("_")[-1]))


def load_ply(model, path: str, use_train_test_exp: bool = False) -> None:
    """``GaussianModel.load_ply``: properties found by name, f_rest_* / scale_* / rot* ordered
    by suffix, parameters created on the GPU, active_sh_degree = max_sh_degree."""
    import torch
    from torch import nn

    if use_train_test_exp:
        exposure_file = os.path.join(os.path.dirname(path), os.pardir, os.pardir, "exposure.json")
        if os.path.exists(exposure_file):
            with open(exposure_file, "r") as f:
                exposures = json.load(f)
            model.pretrained_exposures = {name: torch.FloatTensor(exposures[name]).requires_grad_(False).cuda()
                                          for name in exposures}
            print("Pretrained exposures loaded.")
        else:
            print(f"No exposure to be loaded at {exposure_file}")
            model.pretrained_exposures = None

    N, names = vertex_properties(path)
    extra = _sorted_by_suffix(names, "f_rest_")
    assert len(extra) == 3 * (model.max_sh_degree + 1) ** 2 - 3
    scale_names = _sorted_by_suffix(names, "scale_")
    rot_names = _sorted_by_suffix(names, "rot")
    want = ["x", "y", "z", "opacity", "f_dc_0", "f_dc_1", "f_dc_2"] + extra + scale_names + rot_names
    # read straight into the final host layouts (strided views)
    xyz = np.empty((N, 3), np.float32)
    opac = np.empty((N, 1), np.float32)
    fdc = np.empty((N, 3, 1), np.float32)
    fextra = np.empty((N, len(extra)), np.float32)
    scales = np.empty((N, len(scale_names)), np.float32)
    rots = np.empty((N, len(rot_names)), np.float32)
    out = {"x": xyz[:, 0], "y": xyz[:, 1], "z": xyz[:, 2], "opacity": opac[:, 0],
           "f_dc_0": fdc[:, 0, 0], "f_dc_1": fdc[:, 1, 0], "f_dc_2": fdc[:, 2, 0]}
    out.update({n: fextra[:, i] for i, n in enumerate(extra)})
    out.update({n: scales[:, i] for i, n in enumerate(scale_names)})
    out.update({n: rots[:, i] for i, n in enumerate(rot_names)})
    read_vertex(path, want, out)
    fextra = fextra.reshape((N, 3, (model.max_sh_degree + 1) ** 2 - 1))

    dev = "cuda"
    model._xyz = nn.Parameter(torch.tensor(xyz, dtype=torch.float, device=dev).requires_grad_(True))
    model._features_dc = nn.Parameter(torch.tensor(fdc, dtype=torch.float, device=dev).transpose(1, 2)
                                      .contiguous().requires_grad_(True))
    model._features_rest = nn.Parameter(torch.tensor(fextra, dtype=torch.float, device=dev).transpose(1, 2)
                                        .contiguous().requires_grad_(True))
    model._opacity = nn.Parameter(torch.tensor(opac, dtype=torch.float, device=dev).requires_grad_(True))
    model._scaling = nn.Parameter(torch.tensor(scales, dtype=torch.float, device=dev).requires_grad_(True))
    model._rotation = nn.Parameter(torch.tensor(rots, dtype=torch.float, device=dev).requires_grad_(True))
    model.active_sh_degree = model.max_sh_degree


# ---- scene/dataset_readers.py:120-143 -------------------------------------------------
def fetch_ply(path: str) -> BasicPointCloud:
    """``fetchPly``: positions and normals float32, colours / 255 float64 (the dtypes numpy
    gives for plyfile's f4 / u1 columns)."""
    c = read_vertex(path, ["x", "y", "z", "red", "green", "blue", "nx", "ny", "nz"])
    positions = np.vstack([c["x"], c["y"], c["z"]]).T
    # plyfile yields the uchar columns as uint8 arrays: uint8 / 255.0 is float64
    colors = np.vstack([c["red"], c["green"], c["blue"]]).T.astype(np.uint8) / 255.0
    normals = np.vstack([c["nx"], c["ny"], c["nz"]]).T
    return BasicPointCloud(points=positions, colors=colors, normals=normals)


def store_ply(path: str, xyz, rgb) -> None:
    """``storePly``: x y z nx ny nz (zero normals) float32, red green blue uint8."""
    xyz = np.asarray(xyz)
    rgb = np.asarray(rgb)
    normals = np.zeros_like(xyz)
    # the reference fills a structured array from float rows: values cast to f4 / u1
    f = np.concatenate((xyz, normals), axis=1).astype(np.float32)
    u = rgb.astype(np.uint8)
    write_vertex(path, [("x", f[:, 0]), ("y", f[:, 1]), ("z", f[:, 2]), ("nx", f[:, 3]), ("ny", f[:, 4]),
                        ("nz", f[:, 5]), ("red", u[:, 0]), ("green", u[:, 1]), ("blue", u[:, 2])])


def install(cls) -> None:
    """Bind save_ply / load_ply / construct_list_of_attributes as ``cls``'s methods."""
    cls.save_ply = save_ply
    cls.load_ply = load_ply
    cls.construct_list_of_attributes = construct_list_of_attributes


def install_dataset_readers(module) -> None:
    """Replace ``storePly`` / ``fetchPly`` of the reference's ``scene.dataset_readers`` module."""
    module.storePly = store_ply
    module.fetchPly = fetch_ply
