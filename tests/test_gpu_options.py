"""Every alternative kernel path libgsr ships (include/gsr.h gsr_option_set) against the oracle.

The library's runtime options select alternative paths of the forward and backward -- binning
without the fused scan, whole-tile forward waves, longer backward work units, a queued copy of the
instance count, the three zero-fill modes of the backward outputs and gauss_bwd without the live
list.  Each path is a way a user can run the rasterizer, so each is held to the same bars as the
default path (tests/test_gpu_parity.py), on cases that reach every binning sort class, in both the
synchronising and the capacity-hint forward:
  * integers identical to the f32 oracle: num_rendered, radii, the sorted tile lists;
  * colour / inverse depth within 1e-5; gradients within 1e-5 absolute with the L1 upstream
    gradient and 2e-4 of max |ref| with a unit one;
  * and against the record path with the other defaults (bwd_atomic=0 is the base here, whatever the
    library's default, tests/conftest.py record_path): bitwise equal, except the backward of "bwd_seg_ck",
    whose work units start from other blend checkpoints (the same sums in another rounding), the
    backward of "bwd_atomic", whose per-Gaussian sums are added in the hardware's order (and whose
    second backward of one forward checks that the first restored its accumulators to zero), and
    "fwd_quads=4", a separate instantiation of the forward kernel in which the compiler contracts
    other multiply-adds into FMAs (the oracle bars above still hold it).
"""
import numpy as np
import pytest
import torch

from tests import common as C

pytestmark = pytest.mark.gpu

VARIANTS = {
    "fused_bin=0": dict(fused_bin=0),
    "fwd_quads=4": dict(fwd_quads=4),
    "bwd_seg_ck=2": dict(bwd_seg_ck=2),
    "bwd_seg_ck=max": dict(bwd_seg_ck=1 << 20),
    "host_total=0": dict(host_total=0),
    "zero_fill=0": dict(zero_fill=0),
    "zero_fill=1": dict(zero_fill=1),         # side stream, forked / joined by events
    "zero_fill=2": dict(zero_fill=2),
    "live_list=0": dict(live_list=0),
    "sort_prefix=0": dict(sort_prefix=0),     # whole lists sorted
    "sort_prefix=64": dict(sort_prefix=64),   # long lists sorted to 64 entries: most of their tiles redone
    "count_wait=0": dict(count_wait=0),       # the blocking wait for the instance count
    "count_wait=1": dict(count_wait=1),       # the host polls an event behind the count (default 2: the slot)
    "bwd_grid=1": dict(bwd_grid=1),           # render_bwd: one block per possible unit
    "bwd_grid=2": dict(bwd_grid=2),           # render_bwd: two blocks per tile walking units i, i + G, ...
    "bwd_atomic=1": dict(bwd_atomic=1),       # per-Gaussian float-atomic rows instead of records + gauss_reduce
    "near_mass=0": dict(near_mass=0),         # no near-first binning: every instance keyed and sorted
    "near_mass=1": dict(near_mass=1),         # a very early depth cut: far fills and redos in dense tiles
    "bwd_atomic=1,near_mass=1": dict(bwd_atomic=1, near_mass=1),  # the far fill zeroes the far rows it files
    # gauss_bwd over runs of 512 / 4096 Gaussians: several flushes of 128 per workgroup, a ring list in LDS
    "bwd_atomic=1,touched_run=4": dict(bwd_atomic=1, touched_run=4),
    "bwd_atomic=1,touched_run=32": dict(bwd_atomic=1, touched_run=32),
}
CASES = ["sh3_scalerot", "antialiasing", "dense_opaque", "lists_1k_2k", "lists_4k_8k", "lists_over_8k"]


def _np(t):
    return t.detach().float().cpu().numpy()


def _run(inp, case, grads, hint):
    """Forward (synchronising, or with a capacity hint of the exact count) + two backwards."""
    from gaussian_splatting_amd import _C as CM

    key = (torch.cuda.current_device(), case.W, case.H)
    CM._capacity.pop(key, None)
    if hint:
        ref = C.run_oracle(inp)
        CM._capacity[key] = (case.P, ref.num_rendered)
    fwd = C.run_gpu_forward(inp)
    outs = [C.run_gpu_backward(inp, fwd, *g) for g in grads]
    torch.cuda.synchronize()
    CM._capacity.pop(key, None)
    return fwd, outs


@pytest.mark.parametrize("hint", [False, True], ids=["sync", "hint"])
@pytest.mark.parametrize("case_name", CASES)
@pytest.mark.parametrize("variant", sorted(VARIANTS))
@pytest.mark.record_path
def test_option_path_matches_oracle(variant, case_name, hint):
    from gaussian_splatting_amd import _C as CM
    from gaussian_splatting_amd import _lib

    case = next(c for c in C.SMALL_CASES if c.name == case_name)
    inp = C.build(case)
    ref = C.run_oracle(inp)
    grads = (C.unit_grads(case.H, case.W), C.l1_grads(case.H, case.W))
    base_fwd, base_outs = _run(inp, case, grads, hint)
    with _lib.options(**VARIANTS[variant]):
        fwd, outs = _run(inp, case, grads, hint)
        st = CM.debug_forward_state(fwd, case.P)
    nr, color, radii, *_, invd = fwd
    assert nr == ref.num_rendered
    np.testing.assert_array_equal(_np(radii).astype(np.int32), ref.radii)
    np.testing.assert_array_equal(st["point_list"].numpy(), ref.handle.binning()["point_list"].astype(np.int64))
    np.testing.assert_allclose(_np(color), ref.color, atol=1e-5, rtol=0)
    np.testing.assert_allclose(_np(invd), ref.invdepth, atol=1e-5, rtol=0)
    for (gc, gd), out, mode in zip(grads, outs, ("unit", "l1")):
        r = ref.handle.backward(gc, gd)
        for k, got in zip(C.GRAD_NAMES, out):
            if mode == "l1":
                np.testing.assert_allclose(_np(got), r[k], atol=1e-5, rtol=0, err_msg=f"{variant} {k}")
            else:
                assert C.rel_err(_np(got), r[k]) <= 2e-4, (variant, k, C.rel_err(_np(got), r[k]))
    # against the default path
    assert torch.equal(fwd[2], base_fwd[2])
    if variant == "fwd_quads=4":
        assert float((fwd[1] - base_fwd[1]).abs().max()) <= 1e-6
        return
    assert torch.equal(fwd[1], base_fwd[1]) and torch.equal(fwd[6], base_fwd[6])
    if not variant.startswith(("bwd_seg_ck", "bwd_atomic")):
        for out, base in zip(outs, base_outs):
            for a, b in zip(out, base):
                assert torch.equal(a, b), variant



@pytest.mark.parametrize("seg_ck", [2, 1 << 20])
@pytest.mark.parametrize("case_name", ["lists_1k_2k", "lists_over_8k"])
@pytest.mark.record_path
def test_seg_ck_set_around_forward_only(seg_ck, case_name):
    """the backward walks the work units its OWN forward wrote.  A forward run with
    bwd_seg_ck = k and a backward run after the option is restored (and the reverse) must give the
    gradients of a forward + backward both run with k -- no segment counted twice, none left out."""
    from gaussian_splatting_amd import _lib

    case = next(c for c in C.SMALL_CASES if c.name == case_name)
    inp = C.build(case)
    ref = C.run_oracle(inp)
    gc, gd = C.l1_grads(case.H, case.W)
    with _lib.options(bwd_seg_ck=seg_ck):
        fwd_k = C.run_gpu_forward(inp)
        both_k = C.run_gpu_backward(inp, fwd_k, gc, gd)
    split_k = C.run_gpu_backward(inp, fwd_k, gc, gd)  # option back at the default
    fwd_1 = C.run_gpu_forward(inp)
    with _lib.options(bwd_seg_ck=seg_ck):
        split_1 = C.run_gpu_backward(inp, fwd_1, gc, gd)  # forward at the default, backward under k
    both_1 = C.run_gpu_backward(inp, fwd_1, gc, gd)
    torch.cuda.synchronize()
    r = ref.handle.backward(gc, gd)
    for a, b in zip(split_k, both_k):
        assert torch.equal(a, b)
    for a, b in zip(split_1, both_1):
        assert torch.equal(a, b)
    for k, got in zip(C.GRAD_NAMES, split_k):
        np.testing.assert_allclose(_np(got), r[k], atol=1e-5, rtol=0, err_msg=k)


@pytest.mark.parametrize("run", [1, 16], ids=["run128", "run2048"])
@pytest.mark.parametrize("case_name", ["sh3_scalerot", "lists_4k_8k"])
def test_atomic_backward_repeats(case_name, run):
    """bwd_atomic: the forward zeroes the accumulator rows and touched bits, and each backward restores
    what it used to zero (gauss_bwd the bits and the rows), so three backwards of one forward
    agree to float rounding of the add order (a row left over would double a Gaussian's gradient);
    a record-path backward of a forward run with the option on equals the record path bitwise, and so
    does a backward with the option on of a forward without it (its buffer is not marked: no rows zeroed)."""
    from gaussian_splatting_amd import _lib

    case = next(c for c in C.SMALL_CASES if c.name == case_name)
    inp = C.build(case)
    gc, gd = C.l1_grads(case.H, case.W)
    with _lib.options(bwd_atomic=0):
        base_fwd = C.run_gpu_forward(inp)
    with _lib.options(bwd_atomic=1, touched_run=run):
        fwd = C.run_gpu_forward(inp)
        outs = [C.run_gpu_backward(inp, fwd, gc, gd) for _ in range(3)]
    with _lib.options(bwd_atomic=0):
        rec = C.run_gpu_backward(inp, fwd, gc, gd)  # the record path on the same buffers
        base = C.run_gpu_backward(inp, C.run_gpu_forward(inp), gc, gd)
    with _lib.options(bwd_atomic=1):  # a forward without the option: its backward takes the record path
        unmarked = C.run_gpu_backward(inp, base_fwd, gc, gd)
    torch.cuda.synchronize()
    for a, b, u in zip(rec, base, unmarked):
        assert torch.equal(a, b) and torch.equal(u, b)
    for o in outs:
        for k, a, b in zip(C.GRAD_NAMES, o, base):
            scale = float(b.abs().max()) or 1.0
            assert float((a - b).abs().max()) <= 1e-5 * scale, (k, float((a - b).abs().max()), scale)


def test_foreign_geometry_buffer_takes_record_path():
    """A geometry tensor the forward did not return (here a view of it: the same address, another tensor) makes
    the library forget that address's forward state (include/gsr.h gsr_geom_forget, _C._own_geometry): its
    backward writes the record inputs and takes the deterministic record path -- bitwise the record path's
    gradients -- instead of trusting the mark of the atomic forward that wrote the address."""
    from gaussian_splatting_amd import _lib

    case = next(c for c in C.SMALL_CASES if c.name == "sh3_scalerot")
    inp = C.build(case)
    gc, gd = C.unit_grads(case.H, case.W)
    with _lib.options(bwd_atomic=0):
        ref = C.run_gpu_backward(inp, C.run_gpu_forward(inp), gc, gd)
    with _lib.options(bwd_atomic=1):
        fwd = C.run_gpu_forward(inp)
        nr, color, radii, geom, binning, img, invd = fwd
        view = geom[:]
        assert view.data_ptr() == geom.data_ptr() and view._cdata != geom._cdata
        got = C.run_gpu_backward(inp, (nr, color, radii, view, binning, img, invd), gc, gd)
        # the address is forgotten for the original tensor too: the record path again
        again = C.run_gpu_backward(inp, fwd, gc, gd)
    torch.cuda.synchronize()
    for a, b, r in zip(got, again, ref):
        assert torch.equal(a, r) and torch.equal(b, r)


def test_no_backward_forward():
    """_C.rasterize_gaussians(..., no_backward=True) (an eval render: rasterizer.py passes it when grad is off or
    no input requires grad) skips zeroing the atomic backward's rows: the same image, and a backward of it anyway
    takes the record path (bitwise the record path's gradients)."""
    from gaussian_splatting_amd import _C, _lib
    from gaussian_splatting_amd.rasterizer import GaussianRasterizationSettings, GaussianRasterizer

    case = next(c for c in C.SMALL_CASES if c.name == "sh3_scalerot")
    inp = C.build(case)
    gc, gd = C.unit_grads(case.H, case.W)
    dev = torch.device("cuda", 0)
    d = lambda k: C._dev(inp[k], dev)  # noqa: E731
    args = (d("bg"), d("means3D"), d("colors_precomp"), d("opacities"), d("scales"), d("rotations"), 1.0,
            d("cov3D_precomp"), d("viewmatrix"), d("projmatrix"), inp["tanfovx"], inp["tanfovy"], inp["H"], inp["W"],
            d("shs"), inp["sh_degree"], d("campos"), False, False, False)
    with _lib.options(bwd_atomic=0):
        ref_fwd = C.run_gpu_forward(inp)
        ref = C.run_gpu_backward(inp, ref_fwd, gc, gd)
    with _lib.options(bwd_atomic=1):
        fwd = _C.rasterize_gaussians(*args, no_backward=True)
        assert _lib.option_get("bwd_atomic") == 1  # (the override was this call's only)
        got = C.run_gpu_backward(inp, fwd, gc, gd)
    torch.cuda.synchronize()
    assert fwd[0] == ref_fwd[0] and torch.equal(fwd[1], ref_fwd[1]) and torch.equal(fwd[6], ref_fwd[6])
    for a, r in zip(got, ref):
        assert torch.equal(a, r)
    # the autograd module under no_grad renders the same image
    s = GaussianRasterizationSettings(image_height=inp["H"], image_width=inp["W"], tanfovx=inp["tanfovx"],
                                      tanfovy=inp["tanfovy"], bg=d("bg"), scale_modifier=1.0,
                                      viewmatrix=d("viewmatrix"), projmatrix=d("projmatrix"), sh_degree=inp["sh_degree"],
                                      campos=d("campos"), prefiltered=False, debug=False, antialiasing=False)
    with torch.no_grad():
        color, radii, invd = GaussianRasterizer(s)(means3D=d("means3D"), means2D=torch.zeros_like(d("means3D")),
                                                   opacities=d("opacities"), shs=d("shs"), scales=d("scales"),
                                                   rotations=d("rotations"))
    assert torch.equal(color, ref_fwd[1])
