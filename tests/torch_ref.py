"""Differentiable float64 restatement of the reference rasterizer FORWARD, in plain torch.

TEST INFRASTRUCTURE ONLY (like oracle/): it is never imported by the product path.
Torch autograd over it gives an independent derivation of the backward, which pins the
hand-written backward of the C oracle (oracle/gsr_oracle.c) -- in particular the part
the reference source does not contain (BACKWARD::render's launcher and the tail of
computeCov2DCUDA).

It follows the reference line by line in meaning, vectorised over Gaussians and pixels:
  in_frustum            CR/auxiliary.h:164-190 (view-space z <= 0.2 culls)
  computeCov3D          CR/forward.cu:149-190  (unnormalised quaternion, Sigma = R S^2 R^T)
  computeCov2D          CR/forward.cu:89-141   (1.3 tan(fov) clamp, J, W from the view matrix)
  preprocessCUDA        CR/forward.cu:222-351  (+0.3 dilation, AA scaling, radius, ndc2Pix, getRect)
  computeColorFromSH    CR/forward.cu:22-80    (+0.5, clamp at 0)
  renderCUDA            CR/forward.cu:367-513  (skip power > 0 and alpha < 1/255, T(1-a) < 1e-4 ends a pixel)
with the reference's backward conventions expressed as autograd-visible choices:
  * alpha = min(0.99, o G) has a straight-through gradient (CR/backward.cu:549, no clamp mask);
  * the skip/termination decisions carry no gradient;
  * dL/dmeans2D is taken w.r.t. a zero leaf added to the NDC position (the screen-space
    leaf trick of gaussian_renderer/__init__.py:31-37), i.e. NDC units;
  * a view-space x or y clamped to 1.3 tan(fov) enters J as a constant (CR/backward.cu:193-194);
  * dL/dscales from the reference omits the scale_modifier factor (CR/backward.cu:356-364
    differentiates w.r.t. the modified scale): grads() divides autograd's value by it.
Known, documented differences from the reference's hand backward that autograd cannot share:
  * antialiasing: the reference evaluates its d(h_scaling)/d(cov2D) formula at the dilated
    covariance (CR/backward.cu:256-270), which is not the derivative of its forward;
  * the reference uses 1/(det^2 + 1e-7) for 1/det^2 in the conic derivative
    (CR/backward.cu:273-283), a relative deviation of ~1e-7/det^2.
"""
from __future__ import annotations

import torch

F64 = torch.float64
SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
SH_C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
         1.445305721320277, -0.5900435899266435]
BLOCK = 16


def eval_sh(deg, sh, d):
    """SH polynomial of CR/forward.cu:22-80 (same as utils/sh_utils.py:57-112); sh [P,M,3], d [P,3] unit."""
    x, y, z = d[:, 0:1], d[:, 1:2], d[:, 2:3]
    res = SH_C0 * sh[:, 0]
    if deg > 0:
        res = res - SH_C1 * y * sh[:, 1] + SH_C1 * z * sh[:, 2] - SH_C1 * x * sh[:, 3]
        if deg > 1:
            xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
            res = (res + SH_C2[0] * xy * sh[:, 4] + SH_C2[1] * yz * sh[:, 5] + SH_C2[2] * (2.0 * zz - xx - yy) * sh[:, 6]
                   + SH_C2[3] * xz * sh[:, 7] + SH_C2[4] * (xx - yy) * sh[:, 8])
            if deg > 2:
                res = (res + SH_C3[0] * y * (3.0 * xx - yy) * sh[:, 9] + SH_C3[1] * xy * z * sh[:, 10]
                       + SH_C3[2] * y * (4.0 * zz - xx - yy) * sh[:, 11]
                       + SH_C3[3] * z * (2.0 * zz - 3.0 * xx - 3.0 * yy) * sh[:, 12]
                       + SH_C3[4] * x * (4.0 * zz - xx - yy) * sh[:, 13] + SH_C3[5] * z * (xx - yy) * sh[:, 14]
                       + SH_C3[6] * x * (xx - 3.0 * yy) * sh[:, 15])
    return res


def cov3d_from_scale_rot(scales, mod, rot):
    """computeCov3D (CR/forward.cu:149-190): R from the *unnormalised* quaternion (r, x, y, z)."""
    r, x, y, z = rot.unbind(1)
    R = torch.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
        2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
        2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], 1).reshape(-1, 3, 3)
    L = R * (mod * scales)[:, None, :]
    S = L @ L.transpose(1, 2)
    return torch.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1], S[:, 1, 2], S[:, 2, 2]], 1)


def _leaf(t):
    return None if t is None else t.detach().to(F64).clone().requires_grad_(True)


def _preprocess(L, V, Pm, campos, tanfovx, tanfovy, W, H, sh_degree, mod, antialiasing, idx):
    """Per-Gaussian quantities for the Gaussians ``idx`` (differentiable)."""
    fx, fy = W / (2.0 * tanfovx), H / (2.0 * tanfovy)
    p = L["means3D"][idx]
    ph = torch.cat([p, torch.ones_like(p[:, :1])], 1)
    p_view = ph @ V[:, :3]                        # transformPoint4x3: column-major 4x4, CR/auxiliary.h:75-84
    p_hom = ph @ Pm                               # transformPoint4x4
    p_w = 1.0 / (p_hom[:, 3:4] + 1e-7)
    p_proj = p_hom[:, :3] * p_w
    ndc = p_proj[:, :2] + L["means2D"][idx, :2]   # the screen-space leaf
    if L["cov3D_precomp"] is not None:
        cov3D = L["cov3D_precomp"][idx]
    else:
        cov3D = cov3d_from_scale_rot(L["scales"][idx], mod, L["rotations"][idx])
    # computeCov2D
    t = p_view
    limx, limy = 1.3 * tanfovx, 1.3 * tanfovy
    tz = t[:, 2]
    # clamp to 1.3 tan(fov); a clamped coordinate is a constant for the backward (the reference's
    # x_grad_mul / y_grad_mul masks, CR/backward.cu:193-194, and its dJ/dtz terms use it as a value)
    txtz, tytz = t[:, 0] / tz, t[:, 1] / tz
    tx = torch.where((txtz < -limx) | (txtz > limx), (torch.clamp(txtz, -limx, limx) * tz).detach(), t[:, 0])
    ty = torch.where((tytz < -limy) | (tytz > limy), (torch.clamp(tytz, -limy, limy) * tz).detach(), t[:, 1])
    zero = torch.zeros_like(tz)
    J = torch.stack([fx / tz, zero, zero, zero, fy / tz, zero, -(fx * tx) / (tz * tz), -(fy * ty) / (tz * tz), zero],
                    1).reshape(-1, 3, 3)          # J_math[r][c] from glm::mat3's column-major fill
    Wm = V[:3, :3]                                # W_math[r][c] = viewmatrix[4r + c]
    T = Wm[None] @ J
    c = cov3D
    Vrk = torch.stack([c[:, 0], c[:, 1], c[:, 2], c[:, 1], c[:, 3], c[:, 4], c[:, 2], c[:, 4], c[:, 5]], 1).reshape(-1, 3, 3)
    cov = T.transpose(1, 2) @ Vrk.transpose(1, 2) @ T
    cxx, cxy, cyy = cov[:, 0, 0], cov[:, 0, 1], cov[:, 1, 1]
    det_cov = cxx * cyy - cxy * cxy
    cxx, cyy = cxx + 0.3, cyy + 0.3
    det = cxx * cyy - cxy * cxy
    h_scale = torch.sqrt(torch.clamp_min(det_cov / det, 0.000025)) if antialiasing else torch.ones_like(det)
    conic = torch.stack([cyy / det, -cxy / det, cxx / det], 1)
    opac = L["opacities"][idx, 0] * h_scale
    xy = ((ndc + 1.0) * torch.tensor([W, H], dtype=F64) - 1.0) * 0.5   # ndc2Pix
    if L["colors_precomp"] is not None:
        rgb = L["colors_precomp"][idx]
    else:
        d = p - campos[None]
        d = d / d.norm(dim=1, keepdim=True)
        rgb = torch.clamp_min(eval_sh(sh_degree, L["shs"][idx], d) + 0.5, 0.0)
    with torch.no_grad():
        mid = 0.5 * (cxx + cyy)
        lam1 = mid + torch.sqrt(torch.clamp_min(mid * mid - det, 0.1))
        lam2 = mid - torch.sqrt(torch.clamp_min(mid * mid - det, 0.1))
        radius = torch.ceil(3.0 * torch.sqrt(torch.maximum(lam1, lam2)))
    return dict(p_view=p_view, cov3D=cov3D, conic=conic, opac=opac, xy=xy, rgb=rgb, radius=radius, det=det)


def _rect(xy, radius, gx, gy):
    """getRect (CR/auxiliary.h:49-59): C float->int truncation toward zero, then clamps."""
    def trunc(v):
        return torch.trunc(v).to(torch.int64)
    xmin = torch.clamp(torch.clamp_min(trunc((xy[:, 0] - radius) / BLOCK), 0), max=gx)
    ymin = torch.clamp(torch.clamp_min(trunc((xy[:, 1] - radius) / BLOCK), 0), max=gy)
    xmax = torch.clamp(torch.clamp_min(trunc((xy[:, 0] + radius + BLOCK - 1) / BLOCK), 0), max=gx)
    ymax = torch.clamp(torch.clamp_min(trunc((xy[:, 1] + radius + BLOCK - 1) / BLOCK), 0), max=gy)
    return xmin, ymin, xmax, ymax


def render(inp, antialiasing=None):
    """Forward pass.  ``inp`` uses tests/common.py's vocabulary.  Returns a dict with the
    outputs (color [3,H,W], invdepth [1,H,W], radii [P] int, n_contrib [H,W]) and the
    autograd leaves/intermediates needed by grads()."""
    aa = inp["antialiasing"] if antialiasing is None else antialiasing
    W, H = inp["W"], inp["H"]
    P = inp["means3D"].shape[0]
    V = inp["viewmatrix"].detach().to(F64)
    Pm = inp["projmatrix"].detach().to(F64)
    campos = inp["campos"].detach().to(F64)
    bg = inp["bg"].detach().to(F64)
    L = {k: _leaf(inp.get(k)) for k in ("means3D", "opacities", "shs", "colors_precomp", "scales", "rotations",
                                        "cov3D_precomp")}
    L["means2D"] = torch.zeros(P, 3, dtype=F64, requires_grad=True)
    gx, gy = (W + BLOCK - 1) // BLOCK, (H + BLOCK - 1) // BLOCK
    mod = float(inp["scale_modifier"])
    tanfovx, tanfovy = float(inp["tanfovx"]), float(inp["tanfovy"])

    # pass 1 (no grad): which Gaussians survive preprocess
    with torch.no_grad():
        allidx = torch.arange(P)
        ph = torch.cat([L["means3D"], torch.ones(P, 1, dtype=F64)], 1)
        in_frustum = (ph @ V[:, :3])[:, 2] > 0.2
        idx = allidx[in_frustum]
        pre = _preprocess(L, V, Pm, campos, tanfovx, tanfovy, W, H, inp["sh_degree"], mod, aa, idx)
        ok = pre["det"] != 0
        xmin, ymin, xmax, ymax = _rect(pre["xy"], pre["radius"], gx, gy)
        ok &= (xmax - xmin) * (ymax - ymin) != 0
        idx = idx[ok]
    # pass 2 (with grad) on the survivors
    pre = _preprocess(L, V, Pm, campos, tanfovx, tanfovy, W, H, inp["sh_degree"], mod, aa, idx)
    if L["colors_precomp"] is None:
        pre["rgb"].retain_grad()
    if L["cov3D_precomp"] is None:
        pre["cov3D"].retain_grad()
    depth = pre["p_view"][:, 2]
    radii = torch.zeros(P, dtype=torch.int64)
    radii[idx] = pre["radius"].to(torch.int64)
    xmin, ymin, xmax, ymax = _rect(pre["xy"].detach(), pre["radius"], gx, gy)

    # depth order, ties by Gaussian index (stable sort of (tile | depth) keys, CR/rasterizer_impl.cu:335-340)
    order = torch.sort(depth.detach(), stable=True).indices
    xy, conic, opac, rgb = pre["xy"][order], pre["conic"][order], pre["opac"][order], pre["rgb"][order]
    invd = 1.0 / depth[order]
    xmin, ymin, xmax, ymax = xmin[order], ymin[order], xmax[order], ymax[order]

    py, px = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    px, py = px.reshape(-1), py.reshape(-1)
    tx, ty = px // BLOCK, py // BLOCK
    member = ((tx[:, None] >= xmin[None]) & (tx[:, None] < xmax[None]) & (ty[:, None] >= ymin[None]) &
              (ty[:, None] < ymax[None]))                       # [N, Pv]: entry of the pixel's tile list
    dx = xy[None, :, 0] - px[:, None].to(F64)
    dy = xy[None, :, 1] - py[:, None].to(F64)
    power = -0.5 * (conic[None, :, 0] * dx * dx + conic[None, :, 2] * dy * dy) - conic[None, :, 1] * dx * dy
    raw = opac[None] * torch.exp(power)
    val = torch.clamp_max(raw, 0.99)
    a_st = raw + (val - raw).detach()                           # straight-through clamp
    with torch.no_grad():
        use = member & (power <= 0) & (val >= 1.0 / 255.0)
        a_d = torch.where(use, val, torch.zeros_like(val))
        # sequential transmittance, first T(1-a) < 1e-4 ends the pixel (that entry not added)
        Tin = torch.cumprod(torch.cat([torch.ones_like(a_d[:, :1]), 1.0 - a_d[:, :-1]], 1), 1)
        term = use & (Tin * (1.0 - a_d) < 0.0001)
        keep = use & (torch.cumsum(term.to(torch.int64), 1) == 0)
        pos = torch.cumsum(member.to(torch.int64), 1)          # 1-based position in the tile list
        n_contrib = torch.where(keep, pos, torch.zeros_like(pos)).max(1).values if keep.shape[1] else \
            torch.zeros(H * W, dtype=torch.int64)
    a = torch.where(keep, a_st, torch.zeros_like(a_st))
    T_incl = torch.cumprod(1.0 - a, 1)
    T_excl = torch.cat([torch.ones_like(a[:, :1]), T_incl[:, :-1]], 1)
    w = a * T_excl
    final_T = T_incl[:, -1] if a.shape[1] else torch.ones(H * W, dtype=F64)
    color = w @ rgb                                             # [N, 3]
    inv = w @ invd
    out = color + final_T[:, None] * bg[None]
    return dict(color=out.t().reshape(3, H, W), invdepth=inv.reshape(1, H, W), radii=radii,
                n_contrib=n_contrib.reshape(H, W), final_T=final_T.reshape(H, W), leaves=L, pre=pre,
                num_rendered=int(((xmax - xmin) * (ymax - ymin)).sum()), idx=idx, mod=mod)


def grads(res, dL_dcolor, dL_dinvdepth=None):
    """Autograd of L = <dL_dcolor, color> + <dL_dinvdepth, invdepth>, returned in the
    reference's 8-tuple conventions (RI/rasterize_points.cu:247) as float64 numpy arrays."""
    L = res["leaves"]
    loss = (res["color"] * dL_dcolor.to(F64)).sum()
    if dL_dinvdepth is not None and dL_dinvdepth.numel():
        loss = loss + (res["invdepth"] * dL_dinvdepth.to(F64)).sum()
    loss.backward()
    P = L["means3D"].shape[0]
    idx = res["idx"]

    def full(src, shape):
        out = torch.zeros(shape, dtype=F64)
        if src is not None:
            out[idx] = src
        return out

    pre = res["pre"]
    if L["colors_precomp"] is not None:
        dcol = L["colors_precomp"].grad
    else:
        dcol = full(pre["rgb"].grad, (P, 3))
    if L["cov3D_precomp"] is not None:
        dcov = L["cov3D_precomp"].grad
    else:
        dcov = full(pre["cov3D"].grad, (P, 6))

    def g(t, shape):
        return torch.zeros(shape, dtype=F64) if (t is None or t.grad is None) else t.grad

    M = 0 if L["shs"] is None else L["shs"].shape[1]
    out = dict(
        dL_dmeans2D=g(L["means2D"], (P, 3)),
        dL_dcolors=dcol if dcol is not None else torch.zeros(P, 3, dtype=F64),
        dL_dopacity=g(L["opacities"], (P, 1)),
        dL_dmeans3D=g(L["means3D"], (P, 3)),
        dL_dcov3D=dcov if dcov is not None else torch.zeros(P, 6, dtype=F64),
        dL_dsh=g(L["shs"], (P, M, 3)),
        dL_dscales=g(L["scales"], (P, 3)) / res["mod"],
        dL_drotations=g(L["rotations"], (P, 4)),
    )
    return {k: v.detach().numpy() for k, v in out.items()}
