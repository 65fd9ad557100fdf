"""Adaptive density control (include/gsr_densify.h, csrc/densify.hip, gaussian_splatting_amd/densify.py).

Oracle: oracle/densify.py, the numpy float32 restatement of GaussianModel.densify_and_prune
and its helpers (scene/gaussian_model.py:400-654) and of train.py:212-215's statistics.
CPU tests pin the oracle with known answers (every section of the output order, every
prune rule, the NaN-grad rule, the zeroed max_radii2D quirk).  GPU tests run the native
path on a model shaped like GaussianModel (six optimizer groups, SH3) and compare it with
the oracle given the same normal samples: the structure (counts, which rows, their order)
exactly, copied values and Adam moments bitwise, the children's computed xyz and scaling
within 1e-6.
"""
import numpy as np
import pytest
import torch

from oracle import densify as od

WIDTH = {"xyz": (3,), "f_dc": (1, 3), "f_rest": (15, 3), "opacity": (1,), "scaling": (3,), "rotation": (4,)}
ATTR = {"xyz": "_xyz", "f_dc": "_features_dc", "f_rest": "_features_rest", "opacity": "_opacity",
        "scaling": "_scaling", "rotation": "_rotation"}


def _rand_params(P, rng, scale_lo=-6.0, scale_hi=-2.0):
    return {
        "xyz": rng.uniform(-3, 3, (P, 3)).astype(np.float32),
        "f_dc": rng.standard_normal((P, 1, 3)).astype(np.float32),
        "f_rest": (rng.standard_normal((P, 15, 3)) * 0.1).astype(np.float32),
        "opacity": rng.normal(0.0, 3.0, (P, 1)).astype(np.float32),
        "scaling": rng.uniform(scale_lo, scale_hi, (P, 3)).astype(np.float32),
        "rotation": rng.standard_normal((P, 4)).astype(np.float32),
    }


def _rand_moments(P, rng):
    return {k: ((rng.standard_normal((P,) + w) * 1e-3).astype(np.float32),
                (rng.random((P,) + w) * 1e-6).astype(np.float32)) for k, w in WIDTH.items()}


# ---- CPU: the oracle's known answers -------------------------------------------------
def test_oracle_known_answers():
    """Six Gaussians, one per rule; extent 10, percent_dense 0.01 (clone/split boundary at
    scale 0.1), max_grad 0.5, min_opacity 0.005, screen size on (world-space limit 1.0)."""
    P = 6
    p = {"xyz": np.arange(P * 3, dtype=np.float32).reshape(P, 3),
         "f_dc": np.arange(P * 3, dtype=np.float32).reshape(P, 1, 3) + 100,
         "f_rest": np.zeros((P, 15, 3), np.float32),
         "opacity": np.full((P, 1), 2.0, np.float32),
         "scaling": np.log(np.full((P, 3), 0.05, np.float32)),
         "rotation": np.tile(np.array([1, 0, 0, 0], np.float32), (P, 1))}
    accum = np.array([0.0, 1.0, 1.0, 0.0, 0.0, 3.0], np.float32)
    denom = np.array([1.0, 1.0, 1.0, 0.0, 1.0, 2.0], np.float32)
    # 0: kept (grad 0); 1: clone (grad 1, small); 2: split (grad 1, scale 0.5 > 0.1);
    # 3: grad 0/0 = NaN -> 0, low opacity -> pruned; 4: scale 2 > 1 (world-space) -> pruned;
    # 5: split whose children (scale 3/1.6 > 1) are pruned, parent dropped
    p["scaling"][2] = np.log(np.float32(0.5))
    p["opacity"][3] = -10.0
    p["scaling"][4] = np.log(np.float32(2.0))
    p["scaling"][5] = np.log(np.float32(3.0))
    mom = {k: (np.ones_like(v), np.full_like(v, 2.0)) for k, v in p.items()}
    st = od.State(p, mom, accum, denom)
    samples = np.array([[0.1, 0.2, 0.3], [0.4, 0.5, 0.6], [1, 1, 1], [2, 2, 2]], np.float32)  # 2 splits x 2 copies
    od.densify_and_prune(st, 0.5, 0.005, 10.0, 20, 0.01, samples)
    # kept originals 0 and 1, clone of 1, two children of 2 (copy 0, copy 1)
    assert st.P == 5
    np.testing.assert_array_equal(st.params["f_dc"][:, 0, 0], [100, 103, 103, 106, 106])
    np.testing.assert_allclose(st.params["xyz"][3], p["xyz"][2] + samples[0], rtol=0, atol=1e-6)  # identity rotation
    np.testing.assert_allclose(st.params["xyz"][4], p["xyz"][2] + samples[2], rtol=0, atol=1e-6)
    np.testing.assert_allclose(np.exp(st.params["scaling"][3:]), 0.5 / 1.6, rtol=1e-6)
    m, v = st.moments["xyz"]
    np.testing.assert_array_equal(m[:, 0], [1, 1, 0, 0, 0])  # kept rows keep moments, new rows zero
    np.testing.assert_array_equal(v[:, 0], [2, 2, 0, 0, 0])
    assert st.accum.shape == (5, 1) and not st.accum.any() and not st.denom.any() and not st.max_radii2D.any()


def test_oracle_screen_size_off_keeps_big():
    p = _rand_params(8, np.random.default_rng(1), -1.0, 1.0)  # scales up to e
    p["opacity"][:] = 5.0
    st = od.State(p, {}, np.zeros(8), np.ones(8))
    od.densify_and_prune(st, 1.0, 0.005, 1.0, None, 0.01, np.zeros((0, 3)))
    assert st.P == 8  # no world-space prune without max_screen_size, nothing selected


def test_oracle_build_rotation_orthonormal():
    q = np.random.default_rng(2).standard_normal((100, 4)).astype(np.float32)
    R = od.build_rotation(q).astype(np.float64)
    np.testing.assert_allclose(R @ R.transpose(0, 2, 1), np.tile(np.eye(3), (100, 1, 1)), atol=1e-6)


def test_product_path_rejects_cpu_tensors():
    from gaussian_splatting_amd import densify

    with pytest.raises(RuntimeError, match="no CPU implementation"):
        densify.densification_stats(torch.zeros(4, 3), torch.zeros(4, 1), torch.zeros(4, 1), radii=torch.ones(4))


# ---- GPU ------------------------------------------------------------------------------
class _Model:
    """The attributes GaussianModel's densification reads and writes (scene/gaussian_model.py)."""

    def __init__(self, params, moments, accum, denom, dev, percent_dense=0.01):
        from torch import nn

        for k, a in ATTR.items():
            setattr(self, a, nn.Parameter(torch.tensor(params[k], device=dev).requires_grad_(True)))
        groups = [{"params": [getattr(self, ATTR[k])], "lr": 1e-3, "name": k} for k in ATTR]
        self.optimizer = torch.optim.Adam(groups, lr=0.0, eps=1e-15)
        if moments is not None:
            for k, a in ATTR.items():
                prm = getattr(self, a)
                self.optimizer.state[prm] = {"step": torch.tensor(7.0),
                                             "exp_avg": torch.tensor(moments[k][0], device=dev),
                                             "exp_avg_sq": torch.tensor(moments[k][1], device=dev)}
        P = params["xyz"].shape[0]
        self.xyz_gradient_accum = torch.tensor(accum, device=dev).reshape(P, 1).contiguous()
        self.denom = torch.tensor(denom, device=dev).reshape(P, 1).contiguous()
        self.max_radii2D = torch.zeros(P, device=dev)
        self.tmp_radii = None
        self.percent_dense = percent_dense

    @property
    def get_scaling(self):
        return torch.exp(self._scaling)


def _case(P, seed, with_moments=True):
    rng = np.random.default_rng(seed)
    params = _rand_params(P, rng)
    moments = _rand_moments(P, rng) if with_moments else None
    accum = (rng.random(P) * 2e-3).astype(np.float32)
    denom = rng.integers(0, 5, P).astype(np.float32)  # zeros -> NaN grads -> 0
    return params, moments, accum, denom


def _run(params, moments, accum, denom, max_grad, extent, max_screen, seed=5):
    from gaussian_splatting_amd import densify

    dev = torch.device("cuda", 0)
    model = _Model(params, moments, accum, denom, dev)
    gen = torch.Generator(device=dev).manual_seed(seed)
    densify.densify_and_prune(model, max_grad, 0.005, extent, max_screen, torch.ones(len(accum), device=dev),
                              generator=gen)
    torch.cuda.synchronize()
    # the oracle with the same samples: the same draw on the same device
    st = od.State(params, moments or {}, accum, denom)
    with np.errstate(divide="ignore", invalid="ignore"):
        grads = st.accum / st.denom
    grads[np.isnan(grads)] = 0
    st_c = od.State(params, moments or {}, accum, denom)
    od.densify_and_clone(st_c, grads, max_grad, extent, 0.01)
    sel = od.split_mask(st_c, grads, max_grad, extent, 0.01)
    # the split parents are originals (clones get zero grads); std as the native path forms it
    P = len(accum)
    assert not sel[P:].any()
    sel_t = torch.tensor(sel[:P], device=dev)
    stds = torch.exp(torch.tensor(params["scaling"], device=dev)[sel_t]).repeat(2, 1)
    gen2 = torch.Generator(device=dev).manual_seed(seed)
    samples = torch.normal(mean=torch.zeros((stds.size(0), 3), device=dev), std=stds, generator=gen2).cpu().numpy()
    od.densify_and_prune(st, max_grad, 0.005, extent, max_screen, 0.01, samples)
    return model, st


def _compare(model, st, moments):
    P_new = st.P
    assert model._xyz.shape[0] == P_new
    for k, a in ATTR.items():
        got = getattr(model, a).detach().cpu().numpy()
        ref = st.params[k]
        assert got.shape == ref.shape, (k, got.shape, ref.shape)
        if k in ("xyz", "scaling"):
            np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-6, err_msg=k)
        else:
            np.testing.assert_array_equal(got, ref, err_msg=k)
        state = model.optimizer.state.get(getattr(model, a))
        if moments is None:
            assert state is None or "exp_avg" not in state
        else:
            np.testing.assert_array_equal(state["exp_avg"].cpu().numpy(), st.moments[k][0], err_msg=k)
            np.testing.assert_array_equal(state["exp_avg_sq"].cpu().numpy(), st.moments[k][1], err_msg=k)
            assert float(state["step"]) == 7.0  # other state entries move with the parameter
        assert model.optimizer.param_groups[list(ATTR).index(k)]["params"][0] is getattr(model, a)
    assert model.xyz_gradient_accum.shape == (P_new, 1) and not model.xyz_gradient_accum.any()
    assert model.denom.shape == (P_new, 1) and model.max_radii2D.shape == (P_new,)
    assert model.tmp_radii is None


@pytest.mark.gpu
@pytest.mark.parametrize("P,seed,max_grad,extent,max_screen,moments", [
    (20000, 0, 2e-4, 2.0, 20, True),     # clones, splits, opacity and world-space prunes
    (20000, 1, 2e-4, 2.0, None, True),   # no world-space prune
    (777, 2, 2e-4, 2.0, 20, False),      # ragged block, no optimizer state yet
    (5000, 3, 10.0, 2.0, 20, True),      # nothing selected: prune only
    (3000, 4, 0.0, 0.05, 20, True),      # everything selected, most children pruned
])
def test_densify_and_prune_matches_oracle(P, seed, max_grad, extent, max_screen, moments):
    params, mom, accum, denom = _case(P, seed, moments)
    model, st = _run(params, mom, accum, denom, max_grad, extent, max_screen)
    _compare(model, st, mom)


@pytest.mark.gpu
def test_densify_everything_pruned():
    params, mom, accum, denom = _case(300, 6)
    params["opacity"][:] = -20.0
    model, st = _run(params, mom, accum, denom, 2e-4, 2.0, 20)
    assert st.P == 0
    _compare(model, st, mom)


@pytest.mark.gpu
def test_densify_deterministic():
    params, mom, accum, denom = _case(20000, 7)
    m1, _ = _run(params, mom, accum, denom, 2e-4, 2.0, 20)
    m2, _ = _run(params, mom, accum, denom, 2e-4, 2.0, 20)
    for a in ATTR.values():
        assert torch.equal(getattr(m1, a), getattr(m2, a))


@pytest.mark.gpu
@pytest.mark.parametrize("use_index_filter", [False, True])
def test_densification_stats_match_oracle(use_index_filter):
    from gaussian_splatting_amd import densify

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(8)
    P = 10007
    vg = rng.standard_normal((P, 3)).astype(np.float32)
    radii = rng.integers(-2, 30, P).astype(np.int32)
    accum = (rng.random((P, 1)) * 0.1).astype(np.float32)
    denom = rng.integers(0, 9, (P, 1)).astype(np.float32)
    maxr = (rng.random(P) * 20).astype(np.float32)
    model = type("M", (), {})()
    model.xyz_gradient_accum = torch.tensor(accum, device=dev)
    model.denom = torch.tensor(denom, device=dev)
    model.max_radii2D = torch.tensor(maxr, device=dev)
    vpt = torch.tensor(vg, device=dev, requires_grad=True)
    vpt.grad = torch.tensor(vg, device=dev)
    rt = torch.tensor(radii, device=dev)
    filt = (rt > 0).nonzero() if use_index_filter else (rt > 0)
    densify.update_max_radii(model, rt, filt)        # train.py:212-213
    densify.add_densification_stats(model, vpt, filt)  # train.py:215
    torch.cuda.synchronize()
    od.densification_stats(vg, accum, denom, maxr, radii)
    np.testing.assert_array_equal(model.xyz_gradient_accum.cpu().numpy(), accum)
    np.testing.assert_array_equal(model.denom.cpu().numpy(), denom)
    np.testing.assert_array_equal(model.max_radii2D.cpu().numpy(), maxr)


# ---- the reference's own densification code (this container only) ------------------------
REF = "/root/reference"


class _CudaToCpu(__import__("ast").NodeTransformer):
    def visit_Constant(self, node):
        if node.value == "cuda":
            node.value = "cpu"
        return node


def _reference_gaussian_model():
    """GaussianModel (scene/gaussian_model.py) and build_rotation / strip_symmetric / ...
    (utils/general_utils.py) compiled from the reference's source with the literal device
    "cuda" read as "cpu" -- the only change -- so its densification runs on this CPU-only
    host.  (The scene package does not import here: scene/cameras.py needs cv2.)  Skipped
    where the reference is not mounted."""
    import ast
    import os

    if not os.path.isdir(os.path.join(REF, "scene")):
        pytest.skip("reference not mounted")
    from torch import nn

    from gaussian_splatting_amd.ply import BasicPointCloud

    ns = {"torch": torch, "nn": nn, "np": np, "os": os, "BasicPointCloud": BasicPointCloud}
    gu = ast.parse(open(os.path.join(REF, "utils/general_utils.py")).read())
    funcs = [n for n in gu.body if isinstance(n, ast.FunctionDef)]
    exec(compile(_CudaToCpu().visit(ast.Module(body=funcs, type_ignores=[])), "general_utils", "exec"), ns)
    gm = ast.parse(open(os.path.join(REF, "scene/gaussian_model.py")).read())
    cls = [n for n in gm.body if isinstance(n, ast.ClassDef) and n.name == "GaussianModel"]
    exec(compile(_CudaToCpu().visit(ast.Module(body=cls, type_ignores=[])), "gaussian_model", "exec"), ns)
    return ns["GaussianModel"]


@pytest.mark.parametrize("max_screen,moments", [(20, True), (None, True), (20, False)])
def test_oracle_matches_reference_code(max_screen, moments):
    """oracle/densify.py against the reference's own densify_and_prune / add_densification_stats
    on the same inputs and the same normal samples (CPU generator, same seed, same draw)."""
    from torch import nn

    GM = _reference_gaussian_model()
    P = 3000
    params, mom, accum, denom = _case(P, 11, moments)
    m = GM(3)
    for k, a in ATTR.items():
        setattr(m, a, nn.Parameter(torch.tensor(params[k]).requires_grad_(True)))
    m.optimizer = torch.optim.Adam([{"params": [getattr(m, ATTR[k])], "lr": 1e-3, "name": k} for k in ATTR],
                                   lr=0.0, eps=1e-15)
    if mom is not None:
        for k, a in ATTR.items():
            m.optimizer.state[getattr(m, a)] = {"step": torch.tensor(3.0), "exp_avg": torch.tensor(mom[k][0]),
                                                "exp_avg_sq": torch.tensor(mom[k][1])}
    m.percent_dense = 0.01
    # the statistics through the reference's add_densification_stats and train.py:212-213
    rng = np.random.default_rng(12)
    vg = rng.standard_normal((P, 3)).astype(np.float32) * 1e-3
    radii = rng.integers(-1, 9, P).astype(np.int32)
    m.xyz_gradient_accum = torch.tensor(accum).reshape(P, 1).clone()
    m.denom = torch.tensor(denom).reshape(P, 1).clone()
    m.max_radii2D = torch.zeros(P)
    vpt = torch.zeros(P, 3, requires_grad=True)
    vpt.grad = torch.tensor(vg)
    vis = torch.tensor(radii) > 0
    m.max_radii2D[vis] = torch.max(m.max_radii2D[vis], torch.tensor(radii)[vis])
    m.add_densification_stats(vpt, vis)
    acc_o, den_o, maxr_o = accum.reshape(P, 1).copy(), denom.reshape(P, 1).copy(), np.zeros(P, np.float32)
    od.densification_stats(vg, acc_o, den_o, maxr_o, radii)
    np.testing.assert_allclose(m.xyz_gradient_accum.numpy(), acc_o, rtol=1e-6, atol=0)
    np.testing.assert_array_equal(m.denom.numpy(), den_o)
    np.testing.assert_array_equal(m.max_radii2D.numpy(), maxr_o)

    st = od.State(params, mom or {}, m.xyz_gradient_accum.numpy(), m.denom.numpy())
    # the samples the reference will draw: same seed, same stds, same call
    with np.errstate(divide="ignore", invalid="ignore"):
        grads = st.accum / st.denom
    grads[np.isnan(grads)] = 0
    st_c = od.State(params, mom or {}, st.accum, st.denom)
    od.densify_and_clone(st_c, grads, 2e-4, 2.0, 0.01)
    sel = od.split_mask(st_c, grads, 2e-4, 2.0, 0.01)
    stds = torch.exp(torch.tensor(st_c.params["scaling"][sel])).repeat(2, 1)
    torch.manual_seed(123)
    samples = torch.normal(mean=torch.zeros((stds.size(0), 3)), std=stds).numpy()
    torch.manual_seed(123)
    m.densify_and_prune(2e-4, 0.005, 2.0, max_screen, torch.ones(P, dtype=torch.int32))
    od.densify_and_prune(st, 2e-4, 0.005, 2.0, max_screen, 0.01, samples)
    assert m._xyz.shape[0] == st.P
    for k, a in ATTR.items():
        got = getattr(m, a).detach().numpy()
        if k in ("xyz", "scaling"):
            np.testing.assert_allclose(got, st.params[k], rtol=1e-6, atol=1e-6, err_msg=k)
        else:
            np.testing.assert_array_equal(got, st.params[k], err_msg=k)
        state = m.optimizer.state.get(getattr(m, a))
        if mom is not None:
            np.testing.assert_array_equal(state["exp_avg"].numpy(), st.moments[k][0], err_msg=k)
            np.testing.assert_array_equal(state["exp_avg_sq"].numpy(), st.moments[k][1], err_msg=k)
    assert m.tmp_radii is None
