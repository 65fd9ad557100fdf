"""One training iteration composed from this repository's packages, the way the reference's
train.py runs it (train.py:131-256, separate_sh=True / --optimizer_type sparse_adam), on a seeded
synthetic scene -- each stage checked against its CPU oracle:

  1. render   GaussianRasterizer(dc=_features_dc, shs=_features_rest) on the activated parameters
              (gaussian_renderer/__init__.py:55-135), clamped to [0, 1] (:148)
              vs oracle/gsr_oracle.c: radii identical, colour within 1e-5;
  2. loss     (1 - 0.2) L1 + 0.2 (1 - fused_ssim) (train.py:155-162)
              vs numpy L1 + oracle/ssim.py;
  3. backward loss.backward() through the clamp, the rasterizer and the activations
              (sigmoid, exp, normalize) into the six parameters and means2D
              vs the oracle's rasterizer backward fed the oracle loss gradient, chained through the
              same activations by torch autograd on the CPU: 2e-4 of max |ref| and 1e-5 absolute;
  4. stats    max_radii2D / add_densification_stats (train.py:212-215)
              vs oracle/densify.py densification_stats on the same inputs: bitwise;
  5. step     SparseGaussianAdam.step(radii > 0, N) (train.py:240-246)
              vs oracle/adam.py on the same gradients: bitwise, every group;
  6. densify  densify_and_prune with the optimizer state it edits (scene/gaussian_model.py:508-640)
              vs oracle/densify.py with the same normal samples: structure, copies and moments
              bitwise, computed children within 1e-6.

Each stage is fed the GPU's own outputs of the stage before, so a failure names its stage; stage 3
also holds the whole chain (the oracle's forward -> loss -> backward) against the GPU's.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F
from torch import nn

from tests import common as C

pytestmark = pytest.mark.gpu

LAMBDA = 0.2  # lambda_dssim (arguments/__init__.py OptimizationParams)
GROUPS = (("xyz", "_xyz"), ("f_dc", "_features_dc"), ("f_rest", "_features_rest"), ("opacity", "_opacity"),
          ("scaling", "_scaling"), ("rotation", "_rotation"))
LR = {"xyz": 1.6e-4 * 5.0, "f_dc": 0.0025, "f_rest": 0.0025 / 20.0, "opacity": 0.025, "scaling": 0.005,
      "rotation": 0.001}  # GaussianModel.training_setup (gaussian_model.py:235-242) at spatial_lr_scale 5


class _Model:
    """The attributes of GaussianModel the iteration touches (scene/gaussian_model.py:66-77,235-251)."""

    def __init__(self, raw, dev):
        from diff_gaussian_rasterization import SparseGaussianAdam

        for k, a in GROUPS:
            setattr(self, a, nn.Parameter(raw[k].to(dev).clone().requires_grad_(True)))
        self.optimizer = SparseGaussianAdam([{"params": [getattr(self, a)], "lr": LR[k], "name": k}
                                             for k, a in GROUPS], lr=0.0, eps=1e-15)
        P = raw["xyz"].shape[0]
        self.xyz_gradient_accum = torch.zeros((P, 1), device=dev)
        self.denom = torch.zeros((P, 1), device=dev)
        self.max_radii2D = torch.zeros(P, device=dev)
        self.tmp_radii = None
        self.percent_dense = 0.01

    @property
    def get_scaling(self):
        return torch.exp(self._scaling)


def _activate(raw):
    """gaussian_model.py:32-55 activations: exp, sigmoid, F.normalize."""
    return dict(means3D=raw["xyz"], dc=raw["f_dc"], shs=raw["f_rest"], opacities=torch.sigmoid(raw["opacity"]),
                scales=torch.exp(raw["scaling"]), rotations=F.normalize(raw["rotation"]))


def test_training_iteration_matches_oracles():
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from fused_ssim import fused_ssim
    from gaussian_splatting_amd import densify
    from oracle import adam as oadam
    from oracle import densify as od
    from oracle import ssim as ossim

    dev = torch.device("cuda", 0)
    case = C.Case("train_iter", P=3000, W=96, H=80, focal=90.0, scale_range=(0.02, 0.2))
    inp = C.build(case)
    g = torch.Generator().manual_seed(42)
    P, H, W = case.P, case.H, case.W
    raw = {"xyz": inp["means3D"], "f_dc": inp["shs"][:, :1].contiguous(), "f_rest": inp["shs"][:, 1:].contiguous(),
           "opacity": torch.logit(inp["opacities"]), "scaling": torch.log(inp["scales"]),
           "rotation": inp["rotations"] * (0.5 + torch.rand(P, 1, generator=g))}  # un-normalised quaternions
    gt = torch.rand(3, H, W, generator=g)
    model = _Model(raw, dev)

    # 1. render (gaussian_renderer/__init__.py:42,55-69,115-148)
    settings = GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=inp["tanfovx"], tanfovy=inp["tanfovy"], bg=torch.zeros(3, device=dev),
        scale_modifier=1.0, viewmatrix=inp["viewmatrix"].to(dev), projmatrix=inp["projmatrix"].to(dev), sh_degree=3,
        campos=inp["campos"].to(dev), prefiltered=False, debug=False, antialiasing=False)
    screenspace = torch.zeros_like(model._xyz, requires_grad=True)
    act = _activate({k: getattr(model, a) for k, a in GROUPS})
    rendered, radii, _invd = GaussianRasterizer(settings)(
        means3D=act["means3D"], means2D=screenspace, dc=act["dc"], shs=act["shs"], colors_precomp=None,
        opacities=act["opacities"], scales=act["scales"], rotations=act["rotations"], cov3D_precomp=None)
    image = rendered.clamp(0, 1)
    act_cpu = {k: v.detach().cpu() for k, v in act.items()}
    oinp = dict(inp, means3D=act_cpu["means3D"], opacities=act_cpu["opacities"], scales=act_cpu["scales"],
                rotations=act_cpu["rotations"], shs=torch.cat([act_cpu["dc"], act_cpu["shs"]], 1))
    ref = C.run_oracle(oinp)
    np.testing.assert_array_equal(radii.cpu().numpy(), ref.radii)
    np.testing.assert_allclose(rendered.detach().cpu().numpy(), ref.color, atol=1e-5, rtol=0)

    # 2. loss (train.py:155-162)
    Ll1 = torch.abs(image - gt.to(dev)).mean()
    ssim_value = fused_ssim(image.unsqueeze(0), gt.to(dev).unsqueeze(0))
    loss = (1.0 - LAMBDA) * Ll1 + LAMBDA * (1.0 - ssim_value)
    img_ref = np.clip(ref.color, 0.0, 1.0)
    gt_np = gt.numpy().astype(np.float64)
    l1_ref = np.abs(img_ref - gt_np).mean()
    s_ref, ds_ref = ossim.fused_ssim(img_ref[None], gt_np[None])
    loss_ref = (1.0 - LAMBDA) * l1_ref + LAMBDA * (1.0 - s_ref)
    assert abs(float(loss) - loss_ref) <= 1e-5 * abs(loss_ref), (float(loss), loss_ref)

    # 3. backward
    loss.backward()
    dimg = ((1.0 - LAMBDA) * np.sign(img_ref - gt_np) / img_ref.size - LAMBDA * ds_ref[0])
    dimg = dimg * ((ref.color >= 0.0) & (ref.color <= 1.0))  # clamp's gradient
    rg = ref.handle.backward(torch.from_numpy(dimg.astype(np.float32)), torch.zeros(1, H, W))
    leaves = {k: raw[k].double().clone().requires_grad_(True) for k, _ in GROUPS}
    a = _activate(leaves)
    outs = [a["means3D"], a["opacities"], a["scales"], a["rotations"], torch.cat([a["dc"], a["shs"]], 1)]
    ups = [rg["dL_dmeans3D"], rg["dL_dopacity"], rg["dL_dscales"], rg["dL_drotations"], rg["dL_dsh"]]
    torch.autograd.backward(outs, [torch.from_numpy(np.asarray(u, np.float64)).reshape(o.shape) for o, u in
                                   zip(outs, ups)])
    grads = {}
    for k, attr in GROUPS:
        got = getattr(model, attr).grad.detach().cpu().numpy()
        exp = leaves[k].grad.numpy()
        grads[k] = getattr(model, attr).grad.detach().clone()
        assert C.rel_err(got, exp) <= 2e-4, (k, C.rel_err(got, exp))
        assert np.abs(got - exp).max() <= 1e-5, (k, np.abs(got - exp).max())
    assert C.rel_err(screenspace.grad.cpu().numpy(), rg["dL_dmeans2D"]) <= 2e-4

    # 4. densification statistics (train.py:212-215)
    vis = radii > 0
    acc0, den0, mr0 = (t.cpu().numpy().copy() for t in (model.xyz_gradient_accum, model.denom, model.max_radii2D))
    model.max_radii2D[vis] = torch.max(model.max_radii2D[vis], radii[vis].float())
    densify.add_densification_stats(model, screenspace, vis)
    od.densification_stats(screenspace.grad.cpu().numpy(), acc0, den0, mr0, radii.cpu().numpy())
    np.testing.assert_array_equal(model.xyz_gradient_accum.cpu().numpy(), acc0)
    np.testing.assert_array_equal(model.denom.cpu().numpy(), den0)
    np.testing.assert_array_equal(model.max_radii2D.cpu().numpy(), mr0)

    # 5. SparseGaussianAdam.step(visible, N) (train.py:240-246)
    before = {k: getattr(model, a).detach().cpu().numpy().copy() for k, a in GROUPS}
    model.optimizer.step(vis, P)
    model.optimizer.zero_grad(set_to_none=True)
    moments = {}
    for k, attr in GROUPS:
        p = getattr(model, attr)
        M = p.numel() // P
        zeros = np.zeros_like(before[k])
        ep, em, ev = oadam.adam_update(before[k], grads[k].cpu().numpy(), zeros, zeros, vis.cpu().numpy(), LR[k],
                                       0.9, 0.999, 1e-15, P, M)
        st = model.optimizer.state[p]
        np.testing.assert_array_equal(p.detach().cpu().numpy().reshape(-1), ep, err_msg=k)
        np.testing.assert_array_equal(st["exp_avg"].cpu().numpy().reshape(-1), em, err_msg=k)
        np.testing.assert_array_equal(st["exp_avg_sq"].cpu().numpy().reshape(-1), ev, err_msg=k)
        moments[k] = (em.reshape(p.shape), ev.reshape(p.shape))
    assert not np.array_equal(before["xyz"], model._xyz.detach().cpu().numpy())

    # 6. densify_and_prune (train.py:219-224; scene/gaussian_model.py:574-640)
    acc = model.xyz_gradient_accum.cpu().numpy()
    den = model.denom.cpu().numpy()
    with np.errstate(divide="ignore", invalid="ignore"):
        gr = np.nan_to_num(acc / den).reshape(-1)
    max_grad = float(np.quantile(gr[gr > 0], 0.85))  # a tenth or so of the visible Gaussians grow
    extent = 5.0
    params = {k: getattr(model, a).detach().cpu().numpy().copy() for k, a in GROUPS}
    seed = 17
    densify.densify_and_prune(model, max_grad, 0.005, extent, 20, radii,
                              generator=torch.Generator(device=dev).manual_seed(seed))
    torch.cuda.synchronize()
    st = od.State(params, moments, acc, den)
    grads_d = np.nan_to_num(st.accum / np.where(st.denom == 0, np.nan, st.denom))
    st_c = od.State(params, moments, acc, den)
    od.densify_and_clone(st_c, grads_d, max_grad, extent, 0.01)
    sel = od.split_mask(st_c, grads_d, max_grad, extent, 0.01)
    n_clone = st_c.P - P
    sel_t = torch.tensor(sel[:P], device=dev)
    stds = torch.exp(torch.tensor(params["scaling"], device=dev)[sel_t]).repeat(2, 1)
    samples = torch.normal(mean=torch.zeros((stds.size(0), 3), device=dev), std=stds,
                           generator=torch.Generator(device=dev).manual_seed(seed)).cpu().numpy()
    od.densify_and_prune(st, max_grad, 0.005, extent, 20, 0.01, samples)
    assert n_clone > 0 and int(sel.sum()) > 0, (n_clone, int(sel.sum()))  # the iteration clones and splits
    assert model._xyz.shape[0] == st.P
    for k, attr in GROUPS:
        p = getattr(model, attr)
        got, exp = p.detach().cpu().numpy(), st.params[k]
        assert got.shape == exp.shape, (k, got.shape, exp.shape)
        if k in ("xyz", "scaling"):
            np.testing.assert_allclose(got, exp, rtol=1e-6, atol=1e-6, err_msg=k)
        else:
            np.testing.assert_array_equal(got, exp, err_msg=k)
        s = model.optimizer.state[p]
        np.testing.assert_array_equal(s["exp_avg"].cpu().numpy(), st.moments[k][0], err_msg=k)
        np.testing.assert_array_equal(s["exp_avg_sq"].cpu().numpy(), st.moments[k][1], err_msg=k)
        assert model.optimizer.param_groups[[n for n, _ in GROUPS].index(k)]["params"][0] is p
    assert model.xyz_gradient_accum.shape == (st.P, 1) and not model.xyz_gradient_accum.any()
    print(f"[train_iter] P {P} -> {st.P}: {n_clone} clones, {int(sel.sum())} split, loss {float(loss):.6f}")
