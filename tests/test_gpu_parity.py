"""GPU parity: libgsr (HIP, gfx950) against the CPU restatement of the reference (oracle/).

Bars:
* integer outputs (num_rendered, radii) -- exact;
* forward colour / inverse depth -- 1e-5 absolute (fp32);
* backward, with the reference's L1-mean upstream gradient -- 1e-5 absolute, and with
  a unit-scale upstream gradient -- max |gpu - oracle| / max |oracle| <= 2e-4 per tensor
  (the reference's own backward sums with unordered float atomics; ours sums in a
  different, fixed order).
"""
import numpy as np
import pytest
import torch

from tests import common as C

pytestmark = pytest.mark.gpu

ATOL_FWD = 1e-5
RTOL_BWD = 2e-4


def _to_np(t):
    return t.detach().float().cpu().numpy()


@pytest.mark.parametrize("case", C.SMALL_CASES, ids=lambda c: c.name)
def test_forward_matches_oracle(case):
    inp = C.build(case)
    ref = C.run_oracle(inp)
    nr, color, radii, geom, binning, img, invd = C.run_gpu_forward(inp)
    torch.cuda.synchronize()
    assert nr == ref.num_rendered
    np.testing.assert_array_equal(_to_np(radii).astype(np.int32), ref.radii)
    # the tile lists themselves (identifyTileRanges + the sorted point_list): identical
    from gaussian_splatting_amd import _C as CM
    st = CM.debug_forward_state((nr, color, radii, geom, binning, img, invd), case.P)
    rb = ref.handle.binning()
    np.testing.assert_array_equal(st["point_list"].numpy(), rb["point_list"].astype(np.int64))
    glen = st["ranges"][:, 1] - st["ranges"][:, 0]
    np.testing.assert_array_equal(glen.numpy(), (rb["ranges"][:, 1].astype(np.int64) - rb["ranges"][:, 0]))
    np.testing.assert_array_equal(st["n_contrib"].numpy(), ref.handle.image()["n_contrib"].astype(np.int64))
    np.testing.assert_allclose(_to_np(color), ref.color, atol=ATOL_FWD, rtol=0)
    np.testing.assert_allclose(_to_np(invd), ref.invdepth, atol=ATOL_FWD, rtol=0)


@pytest.mark.parametrize("case", C.SMALL_CASES, ids=lambda c: c.name)
def test_backward_matches_oracle(case):
    inp = C.build(case)
    ref = C.run_oracle(inp)
    fwd = C.run_gpu_forward(inp)
    for grads, mode in ((C.unit_grads(case.H, case.W), "unit"), (C.l1_grads(case.H, case.W), "l1")):
        gc, gd = grads
        out = C.run_gpu_backward(inp, fwd, gc, gd)
        torch.cuda.synchronize()
        r = ref.handle.backward(gc, gd)
        names = dict(zip(C.GRAD_NAMES, out))
        for k in C.GRAD_NAMES:
            got = _to_np(names[k])
            exp = r[k]
            if k in ("dL_dscales", "dL_drotations") and inp["scales"] is None:
                exp = np.zeros_like(got)
            assert got.shape == exp.shape, (k, got.shape, exp.shape)
            if mode == "l1":
                np.testing.assert_allclose(got, exp, atol=1e-5, rtol=0, err_msg=k)
            else:
                assert C.rel_err(got, exp) <= RTOL_BWD, (k, C.rel_err(got, exp))


def test_backward_without_invdepth_grad():
    case = C.SMALL_CASES[0]
    inp = C.build(case)
    ref = C.run_oracle(inp)
    fwd = C.run_gpu_forward(inp)
    gc, _ = C.unit_grads(case.H, case.W)
    out = C.run_gpu_backward(inp, fwd, gc, None)
    r = ref.handle.backward(gc, None)
    for k, got in zip(C.GRAD_NAMES, out):
        assert C.rel_err(_to_np(got), r[k]) <= RTOL_BWD, k


@pytest.mark.record_path
def test_deterministic_bitwise():
    """The record path (bwd_atomic=0, this module's default by the record_path marker) uses no float atomics --
    its one atomic, an OR of a record's content bit, is order-free -- so two runs give bit-identical images and
    gradients.  (The default atomic path adds in the hardware's order: tests/test_gpu_options.py.)"""
    case = C.SMALL_CASES[-1]
    inp = C.build(case)
    gc, gd = C.unit_grads(case.H, case.W)
    runs = []
    for _ in range(2):
        fwd = C.run_gpu_forward(inp)
        out = C.run_gpu_backward(inp, fwd, gc, gd)
        runs.append([_to_np(fwd[1]), _to_np(fwd[6])] + [_to_np(o) for o in out])
    for a, b in zip(*runs):
        np.testing.assert_array_equal(a, b)


def test_empty_and_culled():
    from gaussian_splatting_amd import _C

    case = C.Case("empty", P=0, W=32, H=32)
    inp = C.build(C.Case("tmp", P=10, W=32, H=32))
    for k in ("means3D", "opacities", "shs", "scales", "rotations"):
        inp[k] = inp[k][:0]
    nr, color, radii, *_ , invd = C.run_gpu_forward(inp)
    assert nr == 0 and radii.numel() == 0
    assert float(color.abs().max()) == 0.0  # P == 0: nothing launched, zero image (RI/rasterize_points.cu:108)
    # every point behind the camera: num_rendered == 0, image == background
    inp = C.build(C.Case("behind", P=50, W=32, H=32, bg=(0.1, 0.2, 0.3)))
    inp["means3D"] = inp["means3D"].clone()
    inp["means3D"][:, 2] = -5.0
    fwd = C.run_gpu_forward(inp)
    assert fwd[0] == 0
    assert int(fwd[2].abs().sum()) == 0
    exp = torch.tensor([0.1, 0.2, 0.3]).view(3, 1, 1).expand(3, 32, 32)
    torch.testing.assert_close(fwd[1].cpu(), exp)
    gc, gd = C.unit_grads(32, 32)
    out = C.run_gpu_backward(inp, fwd, gc, gd)
    for t in out:
        assert float(t.abs().max()) == 0.0
    del _C, case


def test_prefiltered_violation_raises():
    inp = C.build(C.Case("pref", P=20, W=32, H=32))
    inp["means3D"] = inp["means3D"].clone()
    inp["means3D"][0, 2] = -1.0
    with pytest.raises(RuntimeError, match="prefiltered"):
        C.run_gpu_forward(inp, prefiltered=True)


def test_debug_mode_runs():
    case = C.SMALL_CASES[0]
    inp = C.build(case)
    ref = C.run_oracle(inp)
    fwd = C.run_gpu_forward(inp, debug=True)
    np.testing.assert_allclose(_to_np(fwd[1]), ref.color, atol=ATOL_FWD)
    gc, gd = C.unit_grads(case.H, case.W)
    C.run_gpu_backward(inp, fwd, gc, gd, debug=True)


def test_known_answer_single_gaussian():
    """One isotropic Gaussian centred on a pixel: C = c * min(0.99, o) + (1 - alpha) * bg."""
    from gaussian_splatting_amd import _C
    from gaussian_splatting_amd import synthetic as syn

    W = H = 33
    cam = syn.make_camera(W, H, 40.0)
    dev = "cuda"
    means = torch.tensor([[0.0, 0.0, 4.0]])
    colors = torch.tensor([[0.3, 0.6, 0.9]])
    op = torch.tensor([[0.5]])
    cov = torch.tensor([[0.01, 0.0, 0.0, 0.01, 0.0, 0.01]])
    bg = torch.tensor([0.1, 0.1, 0.1])
    nr, color, radii, *_ = _C.rasterize_gaussians(
        bg.to(dev), means.to(dev), colors.to(dev), op.to(dev), torch.Tensor([]), torch.Tensor([]), 1.0, cov.to(dev),
        cam.viewmatrix.to(dev), cam.projmatrix.to(dev), cam.tanfovx, cam.tanfovy, H, W, torch.Tensor([]), 0,
        cam.campos.to(dev), False, False, False)
    c = color.cpu()[:, 16, 16]
    exp = colors[0] * 0.5 + 0.5 * bg
    torch.testing.assert_close(c, exp, atol=1e-6, rtol=0)
    assert nr > 0 and int(radii[0]) > 0


def test_mark_visible():
    from gaussian_splatting_amd import _C
    from oracle import oracle

    inp = C.build(C.Case("mv", P=500, W=64, H=48, z_range=(-3.0, 6.0)))
    vis = _C.mark_visible(inp["means3D"].cuda(), inp["viewmatrix"].cuda(), inp["projmatrix"].cuda())
    exp = oracle.mark_visible(inp["means3D"], inp["viewmatrix"])
    np.testing.assert_array_equal(vis.cpu().numpy(), exp)


@pytest.mark.record_path
def test_autograd_module_matches_direct_calls():
    """GaussianRasterizer through autograd == _C forward/backward, incl. means2D gradient."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer

    case = C.SMALL_CASES[0]
    inp = C.build(case)
    dev = "cuda"
    settings = GaussianRasterizationSettings(
        image_height=case.H, image_width=case.W, tanfovx=inp["tanfovx"], tanfovy=inp["tanfovy"],
        bg=inp["bg"].to(dev), scale_modifier=1.0, viewmatrix=inp["viewmatrix"].to(dev),
        projmatrix=inp["projmatrix"].to(dev), sh_degree=inp["sh_degree"], campos=inp["campos"].to(dev),
        prefiltered=False, debug=False, antialiasing=False)
    leaves = {k: inp[k].to(dev).requires_grad_(True) for k in ("means3D", "shs", "opacities", "scales", "rotations")}
    means2D = torch.zeros_like(leaves["means3D"], requires_grad=True)
    color, radii, invd = GaussianRasterizer(settings)(
        means3D=leaves["means3D"], means2D=means2D, shs=leaves["shs"], opacities=leaves["opacities"],
        scales=leaves["scales"], rotations=leaves["rotations"])
    gc, gd = C.unit_grads(case.H, case.W)
    torch.autograd.backward([color, invd], [gc.to(dev), gd.to(dev)])
    fwd = C.run_gpu_forward(inp)
    out = dict(zip(C.GRAD_NAMES, C.run_gpu_backward(inp, fwd, gc, gd)))
    torch.testing.assert_close(color, fwd[1])
    torch.testing.assert_close(means2D.grad, out["dL_dmeans2D"])
    torch.testing.assert_close(leaves["means3D"].grad, out["dL_dmeans3D"])
    torch.testing.assert_close(leaves["shs"].grad, out["dL_dsh"])
    torch.testing.assert_close(leaves["opacities"].grad, out["dL_dopacity"])
    torch.testing.assert_close(leaves["scales"].grad, out["dL_dscales"])
    torch.testing.assert_close(leaves["rotations"].grad, out["dL_drotations"])


def _module_grads(case, inp, gc, gd):
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer

    dev = "cuda"
    settings = GaussianRasterizationSettings(
        image_height=case.H, image_width=case.W, tanfovx=inp["tanfovx"], tanfovy=inp["tanfovy"],
        bg=inp["bg"].to(dev), scale_modifier=1.0, viewmatrix=inp["viewmatrix"].to(dev),
        projmatrix=inp["projmatrix"].to(dev), sh_degree=inp["sh_degree"], campos=inp["campos"].to(dev),
        prefiltered=False, debug=False, antialiasing=False)
    leaves = {k: inp[k].to(dev).requires_grad_(True) for k in ("means3D", "shs", "opacities", "scales", "rotations")}
    means2D = torch.zeros_like(leaves["means3D"], requires_grad=True)
    color, radii, invd = GaussianRasterizer(settings)(
        means3D=leaves["means3D"], means2D=means2D, shs=leaves["shs"], opacities=leaves["opacities"],
        scales=leaves["scales"], rotations=leaves["rotations"])
    torch.autograd.backward([color, invd], [gc.to(dev), gd.to(dev)])
    return [color.detach(), means2D.grad] + [leaves[k].grad for k in sorted(leaves)]


@pytest.mark.parametrize("tag", ["", "_mod"])
def test_cov3d_precomp_from_reference_get_covariance(tag):
    """compute_cov3D_python (gaussian_renderer/__init__.py:86-87): cov3D_precomp made by the reference's own
    GaussianModel.get_covariance (tests/golden/cov3d.npz) through the HIP path equals the f32 oracle on the
    same inputs (integers exactly, colour 1e-5, gradients incl. dL_dcov3D 2e-4), and equals the in-kernel
    covariance from scales + normalised rotations (the reference's two switch positions)."""
    import os

    z = np.load(os.path.join(C.GOLDEN, "cov3d.npz"))
    case = next(c for c in C.SMALL_CASES if c.name == "cov3d_precomp")
    inp = C.build(C.Case(case.name, P=case.P, W=case.W, H=case.H, seed=case.seed))
    mod = float(z["modifier" + tag])
    assert np.allclose(inp["scales"].numpy(), z["scales"])  # the fixture's scene is this case's
    inp_cov = dict(inp, cov3D_precomp=torch.from_numpy(z["cov3D" + tag]), scales=None, rotations=None)
    inp_sr = dict(inp, rotations=torch.from_numpy(z["rotations"]), scale_modifier=mod)
    ref = C.run_oracle(inp_cov)
    fwd = C.run_gpu_forward(inp_cov)
    fwd_sr = C.run_gpu_forward(inp_sr)
    torch.cuda.synchronize()
    assert fwd[0] == ref.num_rendered
    np.testing.assert_array_equal(_to_np(fwd[2]).astype(np.int32), ref.radii)
    np.testing.assert_allclose(_to_np(fwd[1]), ref.color, atol=ATOL_FWD, rtol=0)
    np.testing.assert_allclose(_to_np(fwd_sr[1]), _to_np(fwd[1]), atol=ATOL_FWD, rtol=0)
    gc, gd = C.unit_grads(case.H, case.W)
    out = dict(zip(C.GRAD_NAMES, C.run_gpu_backward(inp_cov, fwd, gc, gd)))
    r = ref.handle.backward(gc, gd)
    for k in ("dL_dmeans3D", "dL_dcov3D", "dL_dopacity", "dL_dsh", "dL_dmeans2D"):
        assert C.rel_err(_to_np(out[k]), r[k]) <= RTOL_BWD, (k, C.rel_err(_to_np(out[k]), r[k]))


@pytest.mark.record_path
def test_autograd_under_save_on_cpu():
    """The saved buffers may travel through saved-tensor hooks (here: to the host and back): the backward
    recovers the binning layout from the buffer's size, so results are bitwise those of a plain run."""
    case = C.SMALL_CASES[-3]
    inp = C.build(case)
    gc, gd = C.unit_grads(case.H, case.W)
    plain = _module_grads(case, inp, gc, gd)
    with torch.autograd.graph.save_on_cpu():
        hooked = _module_grads(case, inp, gc, gd)
    for a, b in zip(plain, hooked):
        assert torch.equal(a, b)


@pytest.mark.parametrize("name", C.RASTER_FIXTURES)
def test_matches_golden_fixture(name):
    """The HIP path against the committed golden vectors (tests/golden/, float64 oracle outputs)."""
    inp, exp, grads = C.load_raster(name)
    nr, color, radii, geom, binning, img, invd = fwd = C.run_gpu_forward(inp)
    torch.cuda.synchronize()
    # integer work is identical to the f32 oracle (the reference's arithmetic type) on the same inputs;
    # the fixture itself holds float64 outputs, where a radius may round the other way
    ref32 = C.run_oracle(inp)
    assert nr == ref32.num_rendered, (name, nr, ref32.num_rendered)
    np.testing.assert_array_equal(_to_np(radii).astype(np.int64), ref32.radii.astype(np.int64))
    from gaussian_splatting_amd import _C as CM
    st = CM.debug_forward_state(fwd, inp["means3D"].shape[0])
    np.testing.assert_array_equal(st["point_list"].numpy(), ref32.handle.binning()["point_list"].astype(np.int64))
    # the committed fixture's own integers: identical (no tolerance)
    assert nr == int(exp["num_rendered"]), (name, nr, int(exp["num_rendered"]))
    np.testing.assert_array_equal(_to_np(radii).astype(np.int64), exp["radii"].astype(np.int64))
    # the full-size rule (tests/test_gpu_fullsize.py): every pixel over 1e-5 against the fixture is
    # explained by a discrete threshold of the reference's blend that rounding flips -- its last
    # contributor differs from the f32 oracle's, or the f32 oracle's walk over it lies within the
    # margin of power = 0, alpha = 1/255 or T = 1e-4
    d = np.maximum(np.abs(_to_np(color) - exp["color"]).max(0), np.abs(_to_np(invd) - exp["invdepth"])[0])
    m = ref32.handle.pixel_margins()
    near = (m["power"] < 1e-5) | (m["alpha"] < 1e-4) | (m["T"] < 1e-4)
    nc_diff = st["n_contrib"].numpy() != ref32.handle.image()["n_contrib"].astype(np.int64)
    unexplained = (d > ATOL_FWD) & ~(near | nc_diff)
    assert not unexplained.any(), (name, int(unexplained.sum()), float(d[unexplained].max()))
    print(f"[{name}] pixels over 1e-5: {int((d > ATOL_FWD).sum())}, all explained; max|diff| elsewhere "
          f"{float(d[~(near | nc_diff)].max()) if (~(near | nc_diff)).any() else 0.0:.2e}")
    if grads is None:
        return
    out = C.run_gpu_backward(inp, fwd, *grads)
    torch.cuda.synchronize()
    for k, got in zip(C.GRAD_NAMES, out):
        assert C.rel_err(_to_np(got), exp[k]) <= RTOL_BWD, (name, k, C.rel_err(_to_np(got), exp[k]))


def _run_pair(inp, gc, gd):
    fwd = C.run_gpu_forward(inp)
    out = C.run_gpu_backward(inp, fwd, gc, gd)
    torch.cuda.synchronize()
    return [fwd[0]] + [_to_np(fwd[i]) for i in (1, 2, 6)] + [_to_np(o) for o in out]


@pytest.mark.parametrize("hint", ["previous", "too_small", "too_large"])
@pytest.mark.record_path
def test_capacity_forward_matches_sync_forward(hint, monkeypatch):
    """gsr_rasterize_forward_ex (no mid-forward host sync, binning sized from a capacity hint) gives bitwise
    the same results as the reference-style synchronising forward, whether the hint fits, is too small (the
    binning stage is redone) or is far too large (heavy sentinel padding in the sort)."""
    from gaussian_splatting_amd import _C as CM

    case = C.SMALL_CASES[-1]
    inp = C.build(case)
    gc, gd = C.unit_grads(case.H, case.W)
    monkeypatch.setenv("GSR_SYNC_FORWARD", "1")
    ref = _run_pair(inp, gc, gd)
    monkeypatch.setenv("GSR_SYNC_FORWARD", "0")
    key = (torch.cuda.current_device(), case.W, case.H)
    CM._capacity[key] = (case.P, {"previous": ref[0], "too_small": 10, "too_large": 40 * ref[0]}[hint])
    rebuilds = CM.forward_rebuilds()
    got = _run_pair(inp, gc, gd)
    assert CM.forward_rebuilds() - rebuilds == (1 if hint == "too_small" else 0)
    assert got[0] == ref[0]
    for a, b in zip(got[1:], ref[1:]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("name", ["sh3_scalerot", "dense_opaque", "lists_1k_2k"])
@pytest.mark.record_path
def test_census_counts_pairs(name):
    """The census render kernels (include/gsr.h "Census") count the (pixel, entry) pairs the blend
    performs: blended pairs in the forward equal the pure-PyTorch fallback's count of kept pairs,
    and the backward's pairs with a gradient term are exactly those pairs; the census kernels'
    outputs are bitwise those of the production kernels."""
    from gaussian_splatting_amd import _lib
    from oracle import torch_fallback as tf

    case = next(c for c in C.SMALL_CASES if c.name == name)
    inp = C.build(case)
    gc, gd = C.unit_grads(case.H, case.W)
    fwd = C.run_gpu_forward(inp)
    out = C.run_gpu_backward(inp, fwd, gc, gd)
    box = {}

    def run():
        box["fwd"] = C.run_gpu_forward(inp)
        box["out"] = C.run_gpu_backward(inp, box["fwd"], gc, gd)
    cz = _lib.census(run)
    fb = tf.rasterize(inp["means3D"], inp["opacities"], inp["viewmatrix"], inp["projmatrix"], inp["campos"],
                      inp["tanfovx"], inp["tanfovy"], inp["H"], inp["W"], bg=inp["bg"], shs=inp["shs"],
                      sh_degree=inp["sh_degree"], colors_precomp=inp["colors_precomp"], scales=inp["scales"],
                      rotations=inp["rotations"], cov3D_precomp=inp["cov3D_precomp"],
                      scale_modifier=inp["scale_modifier"], antialiasing=inp["antialiasing"])
    assert cz["fwd_pairs_blended"] > 0
    assert cz["fwd_pairs_blended"] == fb["pairs_blended"], (cz, fb["pairs_blended"])
    assert cz["bwd_pairs_grad"] == cz["fwd_pairs_blended"], cz
    assert cz["fwd_pairs_alpha"] >= cz["fwd_pairs_blended"]
    assert cz["fwd_quadrant_evals"] * 64 >= cz["fwd_pairs_alpha"]
    assert cz["bwd_entry_reductions"] <= cz["bwd_entries_staged"] <= fwd[0]
    assert torch.equal(box["fwd"][1], fwd[1])
    for a, b in zip(box["out"], out):
        assert torch.equal(a, b)


@pytest.mark.parametrize("name,prefix", [("lists_1k_2k", 64), ("lists_2k_4k", 64), ("lists_4k_8k", 256),
                                         ("lists_over_8k", 1024), ("lists_2k_4k", 1024)])
@pytest.mark.record_path
def test_sort_prefix_and_redo(name, prefix):
    """The reachable-prefix sort (binning.hip K4, "sort_prefix"): lists longer than one wave's sort are
    sorted to `prefix` (+ a bucket's rest) entries only, and a tile whose forward walk passes that is
    sorted whole and rendered again.  Checked: the prefix was applied (sorted_len < list length for
    the long lists), the redo ran where the walk needed it, every list -- prefix as the product left
    it, tail sorted for inspection -- equals the oracle's, and images and gradients are bitwise those
    of whole-list sorting."""
    from gaussian_splatting_amd import _C as CM
    from gaussian_splatting_amd import _lib

    case = next(c for c in C.SMALL_CASES if c.name == name)
    inp = C.build(case)
    ref = C.run_oracle(inp)
    gc, gd = C.unit_grads(case.H, case.W)
    # (near-first binning off: every list is keyed whole, so sorted_len measures the prefix sort alone;
    # test_near_first_binning covers the two together)
    with _lib.options(sort_prefix=0, near_mass=0):
        whole = _run_pair(inp, gc, gd)
    with _lib.options(sort_prefix=prefix, near_mass=0):
        fwd = C.run_gpu_forward(inp)
        out = C.run_gpu_backward(inp, fwd, gc, gd)
        torch.cuda.synchronize()
        st = CM.debug_sort_state(fwd, case.P)
        lists = CM.debug_forward_state(fwd, case.P)
    got = [fwd[0]] + [_to_np(fwd[i]) for i in (1, 2, 6)] + [_to_np(o) for o in out]
    rng = lists["ranges"].numpy()
    n = rng[:, 1] - rng[:, 0]
    sl = st["sorted_len"].numpy()
    long = n > 1024
    assert long.any()
    assert (sl[~long] == n[~long]).all()
    assert (sl[long] >= np.minimum(prefix, n[long])).all() and (sl[long] <= n[long]).all()
    cut = long & (prefix < n)
    print(f"[{name} prefix {prefix}] long lists {int(long.sum())}, prefix-sorted {int((sl < n).sum())} "
          f"(sorted {int(sl[long].sum())} of {int(n[long].sum())} entries), redone tiles {st['redo_count']}")
    if prefix == 64:
        assert st["redo_count"] > 0  # the blend walks past 64 entries in these dense tiles
    assert cut.any()
    np.testing.assert_array_equal(lists["point_list"].numpy(), ref.handle.binning()["point_list"].astype(np.int64))
    assert got[0] == whole[0]
    for a, b in zip(got[1:], whole[1:]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("P,W,H", [(3000, 2304, 2048), (40000, 2304, 2048), (6000, 5120, 2048), (4000, 8400, 64),
                                   (4000, 64, 8400)],
                         ids=["2304x2048_sparse", "2304x2048_dense", "5120x2048_global_cursors", "8400x64_wide",
                              "64x8400_tall"])
def test_large_image(P, W, H):
    """A 2304x2048 frame (18432 tiles: K3's LDS cursors hold 74 KiB), sparse (3000 Gaussians, every
    binning chunk spanning most of the screen) and denser (40000); a 5120x2048 frame (40960 tiles,
    more than K1 / K3 keep in LDS: the binning falls back to global-memory counters and cursors and the
    unfused tile scan); and a frame wider / taller than 8192 px, whose Z-ordered cell square (256 x 256
    cells) exceeds K0's LDS table, so the cells are numbered row-major (binning.hip bin_cells; round 4
    refused it).  Lists identical, the image by the full-size threshold-flip rule, L1-gradient parity
    1e-5."""
    case = C.Case("large_image", P=P, W=W, H=H, focal=1400.0, scale_range=(0.01, 0.08))
    inp = C.build(case)
    ref = C.run_oracle(inp, nthreads=8)
    fwd = C.run_gpu_forward(inp)
    torch.cuda.synchronize()
    assert fwd[0] == ref.num_rendered
    np.testing.assert_array_equal(_to_np(fwd[2]).astype(np.int32), ref.radii)
    from gaussian_splatting_amd import _C as CM
    st = CM.debug_forward_state(fwd, case.P)
    np.testing.assert_array_equal(st["point_list"].numpy(), ref.handle.binning()["point_list"].astype(np.int64))
    # a frame this size has a few pixels at a threshold flip (tests/test_gpu_fullsize.py's rule)
    d = np.maximum(np.abs(_to_np(fwd[1]) - ref.color).max(0), np.abs(_to_np(fwd[6]) - ref.invdepth)[0])
    m = ref.handle.pixel_margins(nthreads=8)
    near = (m["power"] < 1e-5) | (m["alpha"] < 1e-4) | (m["T"] < 1e-4)
    nc_diff = st["n_contrib"].numpy() != ref.handle.image()["n_contrib"].astype(np.int64)
    unexplained = (d > ATOL_FWD) & ~(near | nc_diff)
    assert not unexplained.any(), (int(unexplained.sum()), float(d[unexplained].max()))
    gc, gd = C.l1_grads(case.H, case.W)
    out = C.run_gpu_backward(inp, fwd, gc, gd)
    r = ref.handle.backward(gc, gd, nthreads=8)
    for k, got in zip(C.GRAD_NAMES, out):
        np.testing.assert_allclose(_to_np(got), r[k], atol=1e-5, rtol=0, err_msg=k)
    print(f"[large_image P={P} {W}x{H}] pixels over 1e-5: {int((d > ATOL_FWD).sum())}, all at threshold flips")


@pytest.mark.parametrize("name,mass", [("lists_4k_8k", 1), ("lists_4k_8k", 8), ("lists_over_8k", 2),
                                       ("lists_over_8k", 30), ("lists_2k_4k", 1), ("dense_opaque", 1)])
@pytest.mark.record_path
def test_near_first_binning(name, mass):
    """Near-first binning (binning.hip, "near_mass"): with a capacity hint, only the Gaussians in front of
    the depth at which the frame's screen-averaged opacity mass reaches `mass` get keys and are sorted; a
    tile whose forward walk passes its near entries is filed, its far instances emitted behind them, its
    whole list sorted and rendered again.  Small targets cut early, so many tiles are redone.  It applies
    to frames whose mean list is at least 2048 entries (api.hip kNearMinMeanList).  Checked:
    a cut was made where the frame's mass reaches the target, each tile's near entries are a prefix of
    its list and never longer, every list (near entries as the product sorted them, the far ones filled
    and sorted for inspection) equals the oracle's, num_rendered / radii are the whole lists', and images
    and gradients are bitwise those of the binning without a cut."""
    from gaussian_splatting_amd import _C as CM
    from gaussian_splatting_amd import _lib

    case = next(c for c in C.SMALL_CASES if c.name == name)
    inp = C.build(case)
    ref = C.run_oracle(inp)
    gc, gd = C.unit_grads(case.H, case.W)
    key = (torch.cuda.current_device(), case.W, case.H)
    with _lib.options(near_mass=0):
        whole = _run_pair(inp, gc, gd)
    CM._capacity[key] = (case.P, ref.num_rendered)  # the capacity-hinted (fused) forward takes the cut
    with _lib.options(near_mass=mass):
        fwd = C.run_gpu_forward(inp)
        out = C.run_gpu_backward(inp, fwd, gc, gd)
        torch.cuda.synchronize()
        nst = CM.debug_near_state(fwd, case.P)
        st = CM.debug_sort_state(fwd, case.P)
        lists = CM.debug_forward_state(fwd, case.P)
    CM._capacity.pop(key, None)
    rng = lists["ranges"].numpy()
    n = rng[:, 1] - rng[:, 0]
    near = nst["near_len"].numpy()
    # the screen-averaged mass, as the library forms it (radius > 0: visible)
    g = ref.handle.geom()
    conic, op = g["conic_opacity"][:, :3].astype(np.float64), g["conic_opacity"][:, 3].astype(np.float64)
    det_inv = conic[:, 0] * conic[:, 2] - conic[:, 1] ** 2
    m = np.where((ref.radii > 0) & (det_inv > 0), op * 2 * np.pi / np.sqrt(np.maximum(det_inv, 1e-30)), 0.0)
    total = m.sum() / (case.W * case.H)
    print(f"[{name} near_mass {mass}] frame mass {total:.1f}, cut bin {nst['zcut']}, near entries "
          f"{int(near.sum())} of {int(n.sum())}, redone tiles {st['redo_count']}")
    if total > 1.1 * mass and n.mean() >= 2048:
        assert nst["zcut"] is not None and near.sum() < n.sum()
    if (name, mass) == ("lists_2k_4k", 1):
        # a cut this early leaves tiles whose walk passes their near entries (an f32 replay of the blend over
        # the oracle's lists: all 4 tiles reach past theirs; lists_4k_8k / lists_over_8k stop inside them)
        assert st["redo_count"] > 0
    assert (near <= n).all()
    np.testing.assert_array_equal(lists["point_list"].numpy(), ref.handle.binning()["point_list"].astype(np.int64))
    np.testing.assert_array_equal(_to_np(fwd[2]).astype(np.int32), ref.radii)
    got = [fwd[0]] + [_to_np(fwd[i]) for i in (1, 2, 6)] + [_to_np(o) for o in out]
    assert got[0] == whole[0] == ref.num_rendered
    for a, b in zip(got[1:], whole[1:]):
        np.testing.assert_array_equal(a, b)
