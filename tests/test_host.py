"""Host-side checks that need no GPU: the C-ABI library builds, loads and exports every entry
point include/gsr.h declares; the Python surface mirrors the reference's (names, argument
validation, error messages); the product path refuses to run without a HIP device instead of
falling back to any CPU code.
"""
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    from gaussian_splatting_amd import build, _lib

    build.build(verbose=False)
    return _lib.load()


def test_library_exports_every_header_symbol(lib):
    from gaussian_splatting_amd import _lib

    names = _lib.header_symbols()
    assert {"gsr_rasterize_forward", "gsr_rasterize_backward", "gsr_mark_visible"} <= set(names)
    for n in names:
        assert hasattr(lib, n), n
    # and the dynamic symbol table says the same (extern "C", unmangled)
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert set(names) <= exported
    # every Python signature corresponds to a declared symbol and vice versa
    assert set(_lib.SIGNATURES) == set(names)


def test_library_is_gfx950(lib, tmp_path):
    assert lib.gsr_version().decode().endswith("gfx950")
    import shutil

    from gaussian_splatting_amd import _lib

    # (on a copy: `--offloading` extracts the device images next to the file it reads)
    copy = tmp_path / "libgsr.so"
    shutil.copy(_lib.LIB_PATH, copy)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(copy), "-d", "--no-show-raw-insn"],
                         capture_output=True, text=True, cwd=tmp_path)
    if out.returncode == 0 and out.stdout:
        assert "gfx950" in out.stdout or "gfx950" in out.stderr


def test_header_documents_reference_interfaces():
    """Each entry point in include/gsr.h cites the reference interface it replaces."""
    text = open(os.path.join(ROOT, "include", "gsr.h")).read()
    for cite in ("rasterizer_impl.cu", "rasterize_points.cu"):
        assert cite in text


def test_missing_library_fails_loudly():
    code = ("import os, sys; sys.path.insert(0, %r); os.environ['GSR_LIBRARY'] = '/nonexistent/libgsr.so'\n"
            "from gaussian_splatting_amd import _lib\n"
            "try:\n    _lib.load()\nexcept _lib.GsrError as e:\n    print('raised', e)\n" % ROOT)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                         env=dict(os.environ, GSR_LIBRARY="/nonexistent/libgsr.so"))
    assert "raised" in out.stdout and "not found" in out.stdout


def test_cpu_tensors_are_refused(lib):
    """No CPU fallback: host tensors raise RuntimeError at the boundary (the reference's module would
    fail inside CUDA; ours says why)."""
    from gaussian_splatting_amd import _C

    e = torch.empty(0)
    with pytest.raises(RuntimeError, match="HIP device"):
        _C.mark_visible(torch.zeros(4, 3), torch.eye(4), torch.eye(4))
    with pytest.raises(RuntimeError):
        _C.rasterize_gaussians(torch.zeros(3), torch.zeros(4, 3), e, torch.ones(4, 1), torch.ones(4, 3),
                               torch.ones(4, 4), 1.0, e, torch.eye(4), torch.eye(4), 0.5, 0.5, 16, 16,
                               torch.zeros(4, 1, 3), 0, torch.zeros(3), False, False, False)


def test_means3d_shape_error_message():
    """RI/rasterize_points.cu:69-71: 'means3D must have dimensions (num_points, 3)'."""
    from gaussian_splatting_amd import _C

    e = torch.empty(0)
    with pytest.raises(RuntimeError, match=r"means3D must have dimensions \(num_points, 3\)"):
        _C.rasterize_gaussians(torch.zeros(3), torch.zeros(4, 2), e, torch.ones(4, 1), e, e, 1.0, e, torch.eye(4),
                               torch.eye(4), 0.5, 0.5, 16, 16, e, 0, torch.zeros(3), False, False, False)


def _settings(**kw):
    from gaussian_splatting_amd import GaussianRasterizationSettings

    base = dict(image_height=16, image_width=16, tanfovx=0.5, tanfovy=0.5, bg=torch.zeros(3), scale_modifier=1.0,
                viewmatrix=torch.eye(4), projmatrix=torch.eye(4), sh_degree=0, campos=torch.zeros(3),
                prefiltered=False, debug=False, antialiasing=False)
    base.update(kw)
    return GaussianRasterizationSettings(**base)


def test_settings_fields_match_reference():
    """RI/diff_gaussian_rasterization/__init__.py:151-180 (13 fields, in order)."""
    from gaussian_splatting_amd import GaussianRasterizationSettings

    assert GaussianRasterizationSettings._fields == (
        "image_height", "image_width", "tanfovx", "tanfovy", "bg", "scale_modifier", "viewmatrix", "projmatrix",
        "sh_degree", "campos", "prefiltered", "debug", "antialiasing")


def test_rasterizer_argument_validation():
    """GaussianRasterizer.forward's checks and messages (RI/diff_gaussian_rasterization/__init__.py:242-247)."""
    from gaussian_splatting_amd import GaussianRasterizer

    r = GaussianRasterizer(_settings())
    P = 4
    m = torch.zeros(P, 3)
    with pytest.raises(Exception, match="Please provide exactly one of either SHs or precomputed colors!"):
        r(means3D=m, means2D=m, opacities=torch.ones(P, 1), shs=None, colors_precomp=None,
          scales=torch.ones(P, 3), rotations=torch.ones(P, 4))
    with pytest.raises(Exception, match="Please provide exactly one of either scale/rotation pair or "
                                        "precomputed 3D covariance!"):
        r(means3D=m, means2D=m, opacities=torch.ones(P, 1), colors_precomp=torch.ones(P, 3))


def test_drop_in_package_surface():
    """diff_gaussian_rasterization exports what gaussian_renderer imports, plus the 3DGS-accel surface:
    SparseGaussianAdam (train.py:41-45 then passes dc=/shs= separately, which GaussianRasterizer.forward accepts)."""
    import diff_gaussian_rasterization as d

    for name in ("GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "_RasterizeGaussians",
                 "_C"):
        assert hasattr(d, name), name
    assert hasattr(d, "SparseGaussianAdam")
    import inspect

    assert "dc" in inspect.signature(d.GaussianRasterizer.forward).parameters
    for fn in ("rasterize_gaussians", "rasterize_gaussians_backward", "mark_visible", "adamUpdate"):
        assert callable(getattr(d._C, fn))


def test_grad_arena_layout():
    """59 floats per Gaussian at SH degree 3, parameter-group order of GaussianModel (gaussian_model.py:235-242)."""
    from gaussian_splatting_amd.distributed import GradArena

    a = GradArena(5, 16, "cpu")
    assert a.floats_per_gaussian == 59 and a.flat.numel() == 5 * 59
    v = a.views()
    assert v["dL_dmeans3D"].shape == (5, 3) and v["dL_dsh"].shape == (5, 16, 3)
    assert v["dL_dopacity"].shape == (5, 1) and v["dL_dscales"].shape == (5, 3) and v["dL_drotations"].shape == (5, 4)
    ptrs = sorted((t.data_ptr(), t.numel()) for t in v.values())
    for (p0, n0), (p1, _) in zip(ptrs, ptrs[1:]):
        assert p1 == p0 + 4 * n0  # back to back, no gaps
    dc, rest = a.split_features()
    assert dc.shape == (5, 1, 3) and rest.shape == (5, 15, 3)


def test_resizer_frees_without_cyclic_gc():
    """The scratch-buffer callback must not form a reference cycle: the multi-GB geometry,
    binning and backward buffers are freed by reference counting as soon as the caller drops
    them, not at the next cyclic GC (which let ~20 steps of buffers pile up at 5M@4K)."""
    import gc
    import weakref

    import torch

    from gaussian_splatting_amd import _C

    gc.disable()
    try:
        t = torch.empty(0, dtype=torch.uint8)
        ref = weakref.ref(t)
        rs = _C._Resizer(t)
        assert rs.cb(None, 4096) == t.data_ptr() and t.numel() == 4096
        del rs, t
        assert ref() is None
    finally:
        gc.enable()


def test_product_path_never_touches_the_oracle():
    """The oracle is the checker only: no product module (the packages a user imports, and the
    native sources behind them) may import, load or link anything under oracle/."""
    import re

    product = ["gaussian_splatting_amd", "diff_gaussian_rasterization", "simple_knn", "fused_ssim",
               "plyfile", "fused_ssim_cuda.py"]
    pat = re.compile(r"(^|\s)(import\s+oracle|from\s+oracle)\b|oracle/|gsr_oracle|liboracle")
    offenders = []
    for entry in product:
        path = os.path.join(ROOT, entry)
        files = [path] if os.path.isfile(path) else [
            os.path.join(d, f) for d, _, fs in os.walk(path) for f in fs
            if f.endswith((".py", ".hip", ".cpp", ".h"))]
        for f in files:
            with open(f, encoding="utf-8", errors="replace") as fh:
                for n, line in enumerate(fh, 1):
                    code = line.split("#")[0] if f.endswith(".py") else line.split("//")[0]
                    if pat.search(code):
                        offenders.append("%s:%d: %s" % (os.path.relpath(f, ROOT), n, line.strip()))
    assert not offenders, "\n".join(offenders)


def test_option_errors_and_restore():
    """libgsr's runtime options (include/gsr.h gsr_option_set): range checks and the restoring
    context manager; no GPU work (the paths themselves: tests/test_gpu_options.py)."""
    from gaussian_splatting_amd import _lib

    before = {k: _lib.option_get(k) for k in _lib.OPTIONS}
    with pytest.raises(_lib.GsrError, match="unknown option"):
        _lib.option_set("no_such_option", 1)
    with pytest.raises(_lib.GsrError, match="out of range"):
        _lib.option_set("fwd_quads", 3)
    with pytest.raises(_lib.GsrError, match="out of range"):
        _lib.option_set("zero_fill", 4)
    with pytest.raises(_lib.GsrError, match="out of range"):
        _lib.option_set("bwd_grid", 3)
    assert before["bwd_grid"] == 0  # auto: the strided grid only where the worst case is far larger
    # the reachable prefix is bounded by the prefix sort's LDS buffer: 1024 at most
    _lib.option_set("sort_prefix", 1024)
    with pytest.raises(_lib.GsrError, match="out of range"):
        _lib.option_set("sort_prefix", 1025)
    _lib.option_set("sort_prefix", before["sort_prefix"])
    with _lib.options(zero_fill=2, live_list=0):
        assert _lib.option_get("zero_fill") == 2 and _lib.option_get("live_list") == 0
    assert {k: _lib.option_get(k) for k in _lib.OPTIONS} == before


def test_library_is_the_build_of_this_tree():
    """freshness is decided by a hash of the sources, headers and flags (not by
    mtimes), stored beside the library and compiled into it; the loaded library carries this tree's."""
    from gaussian_splatting_amd import _lib, build

    if _lib.LIB_PATH != _lib.DEFAULT_LIB:
        pytest.skip("GSR_LIBRARY selects a variant build")
    want = build.input_hash()
    assert _lib.build_id() == want
    with open(_lib.DEFAULT_LIB + ".inputs") as f:
        assert f.read().strip() == want
    assert build.input_hash(extra=("-DX=1",)) != want  # flags are part of the identity


def test_build_identity_ignores_the_compiler_path(monkeypatch):
    """the identity is the sources, flags and target, not the compiler's path -- a library
    built with HIPCC=/custom/hipcc loads in a shell without that variable."""
    from gaussian_splatting_amd import build

    want = build.input_hash()
    monkeypatch.setattr(build, "HIPCC", "/somewhere/else/hipcc")
    assert build.input_hash() == want
    monkeypatch.setattr(build, "ARCH", "gfx942")
    assert build.input_hash() != want  # the target is part of it


def test_build_id_check_without_sources(monkeypatch):
    """an install without the csrc sources skips the build-id check with a warning instead
    of raising FileNotFoundError from load()."""
    from gaussian_splatting_amd import _lib, build

    if _lib.LIB_PATH != _lib.DEFAULT_LIB:
        pytest.skip("GSR_LIBRARY selects a variant build")
    monkeypatch.setattr(build, "CSRC", "/nonexistent/csrc")
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.warns(UserWarning, match="build-id check skipped"):
        _lib.load()
