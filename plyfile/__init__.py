"""Drop-in ``plyfile`` for the reference, over libgsr's native PLY reader/writer
(include/gsr_ply.h, gaussian_splatting_amd/csrc/ply.cpp).

The reference imports ``from plyfile import PlyData, PlyElement`` at module level in
``scene/gaussian_model.py:16`` and ``scene/dataset_readers.py:22``; the package is not in
this image, so without this module neither file imports.  The subset the reference uses
(scene/gaussian_model.py:303-376, scene/dataset_readers.py:120-143) behaves as plyfile's:

* ``PlyData.read(path)``: ``.elements`` in file order, ``plydata['vertex']``,
  ``element['x']`` -> a numpy array of the property's own type (``f4``, ``u1``, ...),
  ``element.properties`` with ``.name``, ``len(element)``, ``element.data`` (a structured
  array of the scalar properties);
* ``PlyElement.describe(structured_array, 'vertex')`` and ``PlyData([el]).write(path)``:
  binary little-endian, one element, scalar properties, the header plyfile writes.

Only vertex-element data is readable (other elements are listed, with their properties);
ascii output, list properties and multi-element output are not implemented and raise.
"""
from __future__ import annotations

import os
from typing import Dict, List, Sequence

import numpy as np

from gaussian_splatting_amd import ply as _ply

__all__ = ["PlyData", "PlyElement", "PlyProperty", "PlyListProperty", "PlyParseError"]

_DTYPE = {("i", 1): "i1", ("u", 1): "u1", ("i", 2): "i2", ("u", 2): "u2", ("i", 4): "i4", ("u", 4): "u4",
          ("f", 4): "f4", ("f", 8): "f8"}


class PlyParseError(Exception):
    pass


class PlyProperty:
    def __init__(self, name: str, val_dtype: str):
        self.name = name
        self.val_dtype = val_dtype

    def __repr__(self):
        return f"PlyProperty({self.name!r}, {self.val_dtype!r})"


class PlyListProperty(PlyProperty):
    pass


def _path(stream) -> str:
    if isinstance(stream, (str, bytes, os.PathLike)):
        return os.fsdecode(stream)
    name = getattr(stream, "name", None)
    if isinstance(name, str):
        return name
    raise NotImplementedError("plyfile (libgsr): streams without a file name are not supported")


class PlyElement:
    def __init__(self, name: str, properties: Sequence[PlyProperty], count: int, data=None, source=None):
        self.name = name
        self.properties = tuple(properties)
        self.count = int(count)
        self._data = data
        self._source = source  # path of the file this vertex element is read from (lazily)
        self._cols: Dict[str, np.ndarray] = {}

    def __len__(self):
        return self.count

    def __contains__(self, name):
        return any(p.name == name for p in self.properties)

    @property
    def data(self) -> np.ndarray:
        if self._data is None:
            scalar = [p for p in self.properties if not isinstance(p, PlyListProperty)]
            arr = np.empty(self.count, dtype=[(p.name, "<" + p.val_dtype) for p in scalar])
            self._read([p.name for p in scalar], {p.name: arr[p.name] for p in scalar})
            self._data = arr
        return self._data

    def _read(self, names: List[str], out: Dict[str, np.ndarray]) -> None:
        if self._source is None:
            raise NotImplementedError(f"plyfile (libgsr): element '{self.name}' data is not readable")
        _ply.read_vertex_raw(self._source, names, out)

    def __getitem__(self, key: str) -> np.ndarray:
        if self._data is not None:
            return self._data[key]
        if key not in self._cols:
            prop = next((p for p in self.properties if p.name == key), None)
            if prop is None:
                raise KeyError(key)
            if isinstance(prop, PlyListProperty):
                raise NotImplementedError("plyfile (libgsr): list properties are not readable")
            col = np.empty(self.count, "<" + prop.val_dtype)
            self._read([key], {key: col})
            self._cols[key] = col
        return self._cols[key]

    @staticmethod
    def describe(data: np.ndarray, name: str, len_types=None, val_types=None, comments=None) -> "PlyElement":
        if not isinstance(data, np.ndarray) or data.dtype.names is None or data.ndim != 1:
            raise TypeError("only one-dimensional structured arrays are supported")
        props = []
        for f in data.dtype.names:
            dt = data.dtype.fields[f][0]
            if dt.kind not in "iuf" or dt.shape != ():
                raise NotImplementedError(f"plyfile (libgsr): field '{f}' of dtype {dt} (scalar fields only)")
            props.append(PlyProperty(f, dt.str[1:]))
        return PlyElement(name, props, len(data), data=data)

    def __repr__(self):
        return f"PlyElement({self.name!r}, {self.properties!r}, count={self.count})"


class PlyData:
    def __init__(self, elements=(), text: bool = False, byte_order: str = "=", comments=(), obj_info=()):
        self.elements = list(elements)
        self.text = text
        self.byte_order = byte_order
        self.comments = list(comments)
        self.obj_info = list(obj_info)

    def __getitem__(self, name: str) -> PlyElement:
        for e in self.elements:
            if e.name == name:
                return e
        raise KeyError(name)

    def __contains__(self, name):
        return any(e.name == name for e in self.elements)

    def __len__(self):
        return len(self.elements)

    def __iter__(self):
        return iter(self.elements)

    @staticmethod
    def read(stream, known_list_len=None, mmap=None) -> "PlyData":
        path = _path(stream)
        n, names, types = _ply.vertex_schema(path)
        props = []
        for nm, (b, k) in zip(names, types):
            props.append(PlyListProperty(nm, "f4") if k == "l" else PlyProperty(nm, _DTYPE[(k, b)]))
        # only the vertex element is exposed with data; the C reader skips the others
        return PlyData([PlyElement("vertex", props, n, source=path)])

    def write(self, stream) -> None:
        if self.text:
            raise NotImplementedError("plyfile (libgsr): ascii output is not supported")
        if self.byte_order not in ("=", "<"):
            raise NotImplementedError("plyfile (libgsr): only little-endian output is supported")
        if len(self.elements) != 1:
            raise NotImplementedError("plyfile (libgsr): exactly one element can be written")
        el = self.elements[0]
        data = el.data
        cols = [(p.name, data[p.name]) for p in el.properties]
        _ply.write_vertex(_path(stream), cols, element=el.name)
