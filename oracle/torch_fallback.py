"""Pure-PyTorch fallback rasterizer (CPU, float32): the CPU BASELINE of north_star.

TEST AND BASELINE INFRASTRUCTURE ONLY, like the rest of ``oracle/``: imported by ``tests/``
and by ``bench.py``'s ``cpu_baseline`` leg, never by the product package (whose entry points
raise on CPU tensors).  north_star: "the reference CPU baseline is the pure-PyTorch fallback
rasterizer timed on the host cores"; SURVEY.md section 8d "CPU baseline"; BASELINE.json
configs[0] ("10k random Gaussians, 256x256, SH degree 0, forward-only via PyTorch CPU fallback").

It is the reference's tile algorithm written with torch tensor ops, vectorised over Gaussians,
instances and (tile, pixel, list entry) blocks -- not a translation of the CUDA thread code:
  preprocess   CR/forward.cu:222-351 (+ in_frustum CR/auxiliary.h:164-190, computeCov3D
               :149-190, computeCov2D :89-141, computeColorFromSH :22-80, ndc2Pix / getRect
               CR/auxiliary.h:43-59), in the C oracle's operation order (gsr_oracle.c
               preprocess_one) so the radius / rectangle decisions agree with it;
  binning      duplicateWithKeys + the stable (tile | depth) sort + identifyTileRanges,
               CR/rasterizer_impl.cu:78-164, 335-340: instances generated in Gaussian order
               and ``torch.sort(stable=True)`` on the 64-bit keys give the same lists;
  render       renderCUDA CR/forward.cu:367-513, per block of tiles: alpha for every
               (pixel, entry), the two skip tests, the transmittance by a cumulative product
               along the list and the T < 1e-4 termination (the terminating entry excluded);
  backward     torch autograd of the above, with the reference's conventions expressed as
               autograd choices (straight-through 0.99 clamp CR/backward.cu:549, no gradient
               through skip / termination decisions, dL/dmeans2D in NDC units :509-510, a
               clamped view-space x / y treated as a constant :193-194, dL/dscales without the
               scale_modifier factor :356-364).  The render part runs block by block, each
               block's graph freed after its backward, so memory stays bounded.
Known differences from the reference, all below the tests' tolerances: torch's CPU cumprod
accumulates in double before rounding (the reference multiplies in float), the conic gradient
is the exact derivative (the reference adds 1e-7 to det^2, CR/backward.cu:273-283), and the
antialiasing gradient is autograd's (the reference's AA formula, :256-270, is not the
derivative of its forward).
"""
from __future__ import annotations

from typing import Optional

import torch

F32 = torch.float32
BLOCK = 16
SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = (1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396)
SH_C3 = (-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
         1.445305721320277, -0.5900435899266435)


def _f(x) -> torch.Tensor:
    return torch.as_tensor(x, dtype=F32)


def _xform(p, m, rows):
    """transformPoint4x3 / 4x4 (CR/auxiliary.h:75-95): 16 floats read column-major, summed left to right."""
    x, y, z = p[:, 0], p[:, 1], p[:, 2]
    return [x * m[r] + y * m[4 + r] + z * m[8 + r] + m[12 + r] for r in rows]


def _cov3d(scales, mod, rot):
    """computeCov3D (CR/forward.cu:149-190), the oracle's order (gsr_oracle.c cov3d_fwd)."""
    S = [mod * scales[:, 0], mod * scales[:, 1], mod * scales[:, 2]]
    r, x, y, z = rot[:, 0], rot[:, 1], rot[:, 2], rot[:, 3]
    Rg = [[1.0 - 2.0 * (y * y + z * z), 2.0 * (x * y - r * z), 2.0 * (x * z + r * y)],
          [2.0 * (x * y + r * z), 1.0 - 2.0 * (x * x + z * z), 2.0 * (y * z - r * x)],
          [2.0 * (x * z - r * y), 2.0 * (y * z + r * x), 1.0 - 2.0 * (x * x + y * y)]]
    Mg = [[S[rr] * Rg[c][rr] for rr in range(3)] for c in range(3)]

    def sg(c, rr):
        return Mg[rr][0] * Mg[c][0] + Mg[rr][1] * Mg[c][1] + Mg[rr][2] * Mg[c][2]
    return torch.stack([sg(0, 0), sg(0, 1), sg(0, 2), sg(1, 1), sg(1, 2), sg(2, 2)], 1)


def _eval_sh(deg, sh, d):
    """computeColorFromSH polynomial (CR/forward.cu:22-80), per channel, the oracle's order."""
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


def preprocess(means3D, opacities, viewmatrix, projmatrix, campos, tanfovx, tanfovy, H, W, shs=None, sh_degree=0,
               colors_precomp=None, scales=None, rotations=None, cov3D_precomp=None, scale_modifier=1.0,
               antialiasing=False, means2D_leaf=None):
    """preprocessCUDA over every Gaussian (differentiable in its float inputs).

    Returns a dict of [P] / [P, k] tensors: ``radii`` (int64, 0 = culled), ``rect`` (int64 xmin,
    ymin, xmax, ymax), ``xy`` (pixel units), ``conic`` (a, b, c), ``opac`` (opacity x AA scale),
    ``rgb``, ``invz``, ``depth``, plus ``cov3D`` / ``rgb`` intermediates for gradient reporting."""
    P = means3D.shape[0]
    V = viewmatrix.detach().reshape(-1).to(F32)
    Pm = projmatrix.detach().reshape(-1).to(F32)
    cp = campos.detach().reshape(-1).to(F32)
    gx, gy = (W + BLOCK - 1) // BLOCK, (H + BLOCK - 1) // BLOCK
    # focal = W / (2 tan(fov/2)) in float32, as the reference computes it (CR/rasterizer_impl.cu:256-257;
    # gsr_oracle.c forward): the double quotient rounded once differs by an ulp on some frames, which moved
    # two radii and 6 instances at 1M@1080p
    fx, fy = float(_f(W) / (_f(2.0) * _f(tanfovx))), float(_f(H) / (_f(2.0) * _f(tanfovy)))
    pv = _xform(means3D, V, (0, 1, 2))
    front = pv[2].detach() > 0.2  # in_frustum; culled Gaussians get a harmless depth so autograd stays finite
    pv[2] = torch.where(front, pv[2], torch.ones_like(pv[2]))
    ph = _xform(means3D, Pm, (0, 1, 2, 3))
    p_w = 1.0 / (ph[3] + 0.0000001)
    ndc = [ph[0] * p_w, ph[1] * p_w]
    if means2D_leaf is not None:  # the screen-space leaf of gaussian_renderer/__init__.py:31-37 (NDC units)
        ndc = [ndc[0] + means2D_leaf[:, 0], ndc[1] + means2D_leaf[:, 1]]
    cov3D = cov3D_precomp if cov3D_precomp is not None else _cov3d(scales, float(scale_modifier), rotations)
    # computeCov2D: clamp t.x/t.z, t.y/t.z to 1.3 tan(fov); a clamped coordinate is a constant for autograd
    limx, limy = float(_f(1.3) * _f(tanfovx)), float(_f(1.3) * _f(tanfovy))
    tz = pv[2]
    txtz, tytz = pv[0] / tz, pv[1] / tz
    cx = torch.clamp(txtz, -limx, limx) * tz
    cy = torch.clamp(tytz, -limy, limy) * tz
    tx = torch.where((txtz < -limx) | (txtz > limx), cx.detach(), cx)
    ty = torch.where((tytz < -limy) | (tytz > limy), cy.detach(), cy)
    tz2 = tz * tz
    zero = torch.zeros_like(tz)
    J = [[fx / tz, zero, -(fx * tx) / tz2], [zero, fy / tz, -(fy * ty) / tz2], [zero, zero, zero]]
    Wg = [[V[0], V[4], V[8]], [V[1], V[5], V[9]], [V[2], V[6], V[10]]]
    Tg = [[Wg[0][rr] * J[c][0] + Wg[1][rr] * J[c][1] + Wg[2][rr] * J[c][2] for rr in range(3)] for c in range(3)]
    c3 = cov3D
    Vm = [[c3[:, 0], c3[:, 1], c3[:, 2]], [c3[:, 1], c3[:, 3], c3[:, 4]], [c3[:, 2], c3[:, 4], c3[:, 5]]]
    X = [[Tg[rr][0] * Vm[c][0] + Tg[rr][1] * Vm[c][1] + Tg[rr][2] * Vm[c][2] for rr in range(3)] for c in range(3)]

    def cc(c, rr):
        return X[0][rr] * Tg[c][0] + X[1][rr] * Tg[c][1] + X[2][rr] * Tg[c][2]
    cxx, cxy, cyy = cc(0, 0), cc(0, 1), cc(1, 1)
    det_cov = cxx * cyy - cxy * cxy
    cxx, cyy = cxx + 0.3, cyy + 0.3
    det = cxx * cyy - cxy * cxy
    h_scale = torch.sqrt(torch.clamp_min(det_cov / det, 0.000025)) if antialiasing else None
    det_inv = 1.0 / det
    conic = torch.stack([cyy * det_inv, -cxy * det_inv, cxx * det_inv], 1)
    opac = opacities[:, 0] * h_scale if antialiasing else opacities[:, 0]
    with torch.no_grad():
        mid = 0.5 * (cxx + cyy)
        root = torch.sqrt(torch.clamp_min(mid * mid - det, 0.1))
        radius = torch.ceil(3.0 * torch.sqrt(torch.maximum(mid + root, mid - root)))
    # ndc2Pix (CR/auxiliary.h:43-46) evaluated in double, rounded to float
    x_pix = (((ndc[0].detach().double() + 1.0) * W - 1.0) * 0.5).to(F32)
    y_pix = (((ndc[1].detach().double() + 1.0) * H - 1.0) * 0.5).to(F32)
    # the differentiable pixel position: same value, gradient d(pix)/d(ndc) = S/2
    xy = torch.stack([x_pix + (ndc[0] - ndc[0].detach()) * (0.5 * W), y_pix + (ndc[1] - ndc[1].detach()) * (0.5 * H)], 1)
    with torch.no_grad():
        r = radius
        rect = torch.stack([
            torch.clamp(torch.clamp_min(torch.trunc((x_pix - r) / BLOCK), 0), max=gx),
            torch.clamp(torch.clamp_min(torch.trunc((y_pix - r) / BLOCK), 0), max=gy),
            torch.clamp(torch.clamp_min(torch.trunc((((x_pix + r) + BLOCK) - 1.0) / BLOCK), 0), max=gx),
            torch.clamp(torch.clamp_min(torch.trunc((((y_pix + r) + BLOCK) - 1.0) / BLOCK), 0), max=gy)],
            1).to(torch.int64)
        area = (rect[:, 2] - rect[:, 0]) * (rect[:, 3] - rect[:, 1])
        ok = front & (det != 0) & (area != 0) & torch.isfinite(radius)
        radii = torch.where(ok, radius, torch.zeros_like(radius)).to(torch.int64)
    if colors_precomp is not None:
        rgb = colors_precomp
    else:
        d = means3D - cp[None]
        d = d / torch.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1] + d[:, 2] * d[:, 2])[:, None]
        rgb = torch.clamp_min(_eval_sh(sh_degree, shs, d) + 0.5, 0.0)
    return dict(radii=radii, rect=rect, visible=ok, xy=xy, conic=conic, opac=opac, rgb=rgb, invz=1.0 / tz, depth=tz,
                cov3D=cov3D, P=P, gx=gx, gy=gy)


def binning(pre):
    """duplicateWithKeys + stable radix sort + identifyTileRanges (CR/rasterizer_impl.cu:78-164,335-340).

    Returns (point_list [R] int64 Gaussian ids, tile-major, (depth, index) order inside a tile;
    starts [tiles], counts [tiles])."""
    gx, gy = pre["gx"], pre["gy"]
    vis = torch.nonzero(pre["visible"]).reshape(-1)
    rect = pre["rect"][vis]
    w = rect[:, 2] - rect[:, 0]
    cnt = w * (rect[:, 3] - rect[:, 1])
    R = int(cnt.sum())
    gid = torch.repeat_interleave(vis, cnt)
    first = torch.cumsum(cnt, 0) - cnt
    k = torch.arange(R, dtype=torch.int64) - torch.repeat_interleave(first, cnt)
    wv = torch.repeat_interleave(w, cnt)
    tile = (torch.repeat_interleave(rect[:, 1], cnt) + k // wv) * gx + torch.repeat_interleave(rect[:, 0], cnt) + k % wv
    depth_bits = pre["depth"].detach().contiguous().view(torch.int32).to(torch.int64)
    keys = (tile << 32) | depth_bits[gid]
    order = torch.sort(keys, stable=True).indices
    counts = torch.bincount(tile, minlength=gx * gy)
    starts = torch.cumsum(counts, 0) - counts
    return gid[order], starts, counts


def _tile_blocks(counts, target_elems):
    """Tiles in decreasing list length, cut into blocks of about ``target_elems`` (pixel, entry) pairs."""
    order = torch.argsort(counts, descending=True, stable=True)
    cs = counts[order].tolist()
    blocks, i, n = [], 0, len(cs)
    while i < n and cs[i] > 0:
        L = cs[i]
        b = max(1, min(n - i, target_elems // (BLOCK * BLOCK * L)))
        blocks.append((order[i:i + b], L))
        i += b
    return blocks


ROUND = 256  # list entries per round, the reference's BLOCK_SIZE batches (CR/forward.cu:404-425)


def _render_block(tiles, L, starts, counts, plist, sc, W, H, gx, bg, grads=None, gc=None, gd=None):
    """renderCUDA (CR/forward.cu:367-513) for a block of tiles, vectorised over (tile, pixel, entry).

    The list is walked in rounds of 256 entries, as the reference's batches; the block stops once
    every pixel of every tile in it is done (CR/forward.cu:420-425).  Writes the block's pixels into
    the full-image outputs in ``sc['out']``; with ``grads`` also runs the block's backward and adds
    the per-Gaussian screen-space gradients into ``grads``.  Returns (list entries walked, (pixel, entry) pairs blended)."""
    B = tiles.numel()
    loc = torch.arange(BLOCK * BLOCK, dtype=torch.int64)
    px = (tiles % gx)[:, None] * BLOCK + loc[None] % BLOCK                         # [B, 256]
    py = (tiles // gx)[:, None] * BLOCK + loc[None] // BLOCK
    inside = (px < W) & (py < H)
    pxf, pyf = px.to(F32)[:, :, None], py.to(F32)[:, :, None]
    cnt, st = counts[tiles], starts[tiles]
    T_run = torch.where(inside, 1.0, 0.0)       # product over every used entry: the termination test
    T_keep = torch.ones(B, BLOCK * BLOCK)       # product over the contributing entries (autograd carries it)
    color = torch.zeros(B, BLOCK * BLOCK, 3)
    inv = torch.zeros(B, BLOCK * BLOCK)
    nc = torch.zeros(B, BLOCK * BLOCK, dtype=torch.int64)
    leaves, walked, pairs = [], 0, 0
    with torch.set_grad_enabled(grads is not None):
        for r0 in range(0, L, ROUND):
            if not bool((T_run >= 0.0001).any()):
                break
            C = min(ROUND, L - r0)
            pos = r0 + torch.arange(C, dtype=torch.int64)
            valid = pos[None] < cnt[:, None]                                       # [B, C]
            walked += int(valid.sum())
            gidx = torch.where(valid, plist[(st[:, None] + pos[None]).clamp(max=plist.numel() - 1)],
                               torch.zeros_like(pos[None]))
            ent = {k: sc[k][gidx] for k in ("xy", "conic", "opac", "rgb", "invz")}  # [B, C, ...]
            if grads is not None:
                ent = {k: v.requires_grad_(True) for k, v in ent.items()}
                leaves.append((gidx, valid, ent))
            dx = ent["xy"][:, None, :, 0] - pxf                                    # [B, 256, C]
            dy = ent["xy"][:, None, :, 1] - pyf
            ca, cb, cc = (ent["conic"][:, None, :, i] for i in range(3))
            power = -0.5 * (ca * dx * dx + cc * dy * dy) - cb * dx * dy
            raw = ent["opac"][:, None, :] * torch.exp(power)
            clamped = torch.clamp_max(raw, 0.99)
            with torch.no_grad():
                use = (power <= 0) & (clamped >= 1.0 / 255.0) & valid[:, None, :]
                a0 = torch.where(use, clamped, torch.zeros_like(clamped))
                T_in = T_run[:, :, None] * torch.cumprod(1.0 - a0, 2)               # T after each entry
                keep = use & (T_in >= 0.0001)  # non-increasing: the first T(1-a) < 1e-4 ends the pixel
                pairs += int(keep.sum())
                T_run = T_in[:, :, -1]
                last = torch.where(keep, pos[None, None] + 1, torch.zeros_like(pos[None, None])).amax(2)
                nc = torch.maximum(nc, last)
            a_st = raw + (clamped - raw).detach()                                  # straight-through clamp
            a = torch.where(keep, a_st, torch.zeros_like(a_st))
            T_incl = T_keep[:, :, None] * torch.cumprod(1.0 - a, 2)
            T_excl = torch.cat([T_keep[:, :, None], T_incl[:, :, :-1]], 2)
            wgt = a * T_excl
            color = color + torch.bmm(wgt, ent["rgb"])
            inv = inv + torch.bmm(wgt, ent["invz"][:, :, None])[:, :, 0]
            T_keep = T_incl[:, :, -1]
        out = color + T_keep[:, :, None] * bg[None, None]
    pix = (py * W + px)[inside]
    o = sc["out"]
    with torch.no_grad():
        o["color"][:, pix] = out.detach()[inside].t()
        o["invdepth"][pix] = inv.detach()[inside]
        o["final_T"][pix] = T_keep.detach()[inside]
        o["n_contrib"][pix] = nc[inside]
    if grads is not None and leaves:
        gcol = torch.zeros(B, BLOCK * BLOCK, 3)
        gcol[inside] = gc[:, pix].t()
        terms = [(out, gcol)]
        if gd is not None:
            ginv = torch.zeros(B, BLOCK * BLOCK)
            ginv[inside] = gd[pix]
            terms.append((inv, ginv))
        torch.autograd.backward([t for t, _ in terms], [g for _, g in terms])
        for gidx, valid, ent in leaves:
            flat = gidx[valid]
            for k, v in ent.items():
                if v.grad is not None:
                    grads[k].index_add_(0, flat, v.grad[valid])
    return walked, pairs


def rasterize(means3D, opacities, viewmatrix, projmatrix, campos, tanfovx, tanfovy, image_height, image_width,
              bg=(0.0, 0.0, 0.0), shs=None, sh_degree=0, colors_precomp=None, scales=None, rotations=None,
              cov3D_precomp=None, scale_modifier=1.0, antialiasing=False, dL_dcolor=None, dL_dinvdepth=None,
              tile_fraction: float = 1.0, target_elems: int = 1 << 21):
    """Forward (and, when ``dL_dcolor`` is given, the backward) of the fallback rasterizer.

    Arguments as ``GaussianRasterizer`` / ``_C.rasterize_gaussians`` (CPU tensors).  Returns a dict:
    ``color`` [3,H,W], ``invdepth`` [1,H,W], ``radii`` [P] int32, ``num_rendered``, ``n_contrib``,
    ``final_T``, ``rendered_instances`` (list entries of the rendered tiles), ``walked_instances`` (those
    the rounds reached before every pixel was done), ``pairs_blended`` ((pixel, entry) pairs blended),
    ``timings``, and with gradients
    ``grads`` in the reference's 8-tuple names (RI/rasterize_points.cu:247).

    ``tile_fraction`` < 1 renders only every k-th tile of the length-sorted tile order (a stratified
    sample, for a bounded CPU timing); preprocess, binning and the preprocess backward always run
    in full."""
    import time

    clock = time.perf_counter
    t0 = clock()
    H, W = int(image_height), int(image_width)
    want_grad = dL_dcolor is not None
    P = means3D.shape[0]

    def leaf(t):
        if t is None or t.numel() == 0:
            return None
        t = t.detach().to(F32).contiguous()
        return t.requires_grad_(True) if want_grad else t
    L_ = {k: leaf(v) for k, v in dict(means3D=means3D, opacities=opacities, shs=shs, colors_precomp=colors_precomp,
                                      scales=scales, rotations=rotations, cov3D_precomp=cov3D_precomp).items()}
    m2d = torch.zeros(P, 3, requires_grad=True) if want_grad else None
    with torch.set_grad_enabled(want_grad):
        pre = preprocess(L_["means3D"], L_["opacities"], viewmatrix, projmatrix, campos, tanfovx, tanfovy, H, W,
                         shs=L_["shs"], sh_degree=sh_degree, colors_precomp=L_["colors_precomp"], scales=L_["scales"],
                         rotations=L_["rotations"], cov3D_precomp=L_["cov3D_precomp"], scale_modifier=scale_modifier,
                         antialiasing=antialiasing, means2D_leaf=m2d)
        if want_grad and L_["colors_precomp"] is None:
            pre["rgb"].retain_grad()
        if want_grad and L_["cov3D_precomp"] is None:
            pre["cov3D"].retain_grad()
    t1 = clock()
    plist, starts, counts = binning(pre)
    t2 = clock()
    gx = pre["gx"]
    bgt = torch.as_tensor(bg, dtype=F32).reshape(3)
    N = H * W
    out = dict(color=bgt[:, None].repeat(1, N), invdepth=torch.zeros(N), final_T=torch.ones(N),
               n_contrib=torch.zeros(N, dtype=torch.int64))
    sc = {k: pre[k].detach() for k in ("xy", "conic", "opac", "rgb", "invz")}
    sc["out"] = out
    grads = {k: torch.zeros_like(v) for k, v in sc.items() if k != "out"} if want_grad else None
    gc = dL_dcolor.detach().to(F32).reshape(3, N) if want_grad else None
    gd = (dL_dinvdepth.detach().to(F32).reshape(N) if want_grad and dL_dinvdepth is not None
          and dL_dinvdepth.numel() else None)
    blocks = _tile_blocks(counts, target_elems)
    if tile_fraction <= 0.0:  # preprocess, binning and the preprocess backward only
        blocks = []
    elif tile_fraction < 1.0:  # stratified sample over the length-sorted tiles
        order = torch.argsort(counts, descending=True, stable=True)
        order = order[counts[order] > 0]
        step = max(1, int(round(1.0 / tile_fraction)))
        sample = order[::step]
        blocks = _tile_blocks_from(sample, counts, target_elems)
    visited = walked = pairs = 0
    for tiles, L in blocks:
        w_, p_ = _render_block(tiles, L, starts, counts, plist, sc, W, H, gx, bgt, grads, gc, gd)
        walked += w_
        pairs += p_
        visited += int(counts[tiles].sum())
    t3 = clock()
    res = dict(color=out["color"].reshape(3, H, W), invdepth=out["invdepth"].reshape(1, H, W),
               radii=pre["radii"].to(torch.int32), num_rendered=int(plist.numel()),
               n_contrib=out["n_contrib"].reshape(H, W), final_T=out["final_T"].reshape(H, W),
               rendered_instances=visited, walked_instances=walked, pairs_blended=pairs)
    if want_grad:
        roots = [pre[k] for k in ("xy", "conic", "opac", "rgb", "invz")]
        gr = [grads[k] for k in ("xy", "conic", "opac", "rgb", "invz")]
        live = [(r, g) for r, g in zip(roots, gr) if r.requires_grad]
        torch.autograd.backward([r for r, _ in live], [g for _, g in live])

        def g(t, shape):
            return torch.zeros(shape) if (t is None or t.grad is None) else t.grad.detach()
        M = 0 if L_["shs"] is None else L_["shs"].shape[1]
        vis = pre["visible"][:, None]
        dcol = L_["colors_precomp"].grad if L_["colors_precomp"] is not None else pre["rgb"].grad
        dcov = L_["cov3D_precomp"].grad if L_["cov3D_precomp"] is not None else pre["cov3D"].grad
        res["grads"] = dict(
            dL_dmeans2D=g(m2d, (P, 3)),
            dL_dcolors=torch.where(vis, dcol, 0.0) if dcol is not None else torch.zeros(P, 3),
            dL_dopacity=g(L_["opacities"], (P, 1)),
            dL_dmeans3D=g(L_["means3D"], (P, 3)),
            dL_dcov3D=torch.where(vis, dcov, 0.0) if dcov is not None else torch.zeros(P, 6),
            dL_dsh=g(L_["shs"], (P, M, 3)),
            dL_dscales=g(L_["scales"], (P, 3)) / float(scale_modifier),
            dL_drotations=g(L_["rotations"], (P, 4)),
        )
    res["timings"] = dict(preprocess=t1 - t0, binning=t2 - t1, render=t3 - t2, preprocess_backward=clock() - t3)
    return res


def _tile_blocks_from(tiles, counts, target_elems):
    """_tile_blocks over a given tile subset (already in decreasing length order)."""
    cs = counts[tiles].tolist()
    blocks, i, n = [], 0, len(cs)
    while i < n:
        L = cs[i]
        b = max(1, min(n - i, target_elems // (BLOCK * BLOCK * max(L, 1))))
        blocks.append((tiles[i:i + b], L))
        i += b
    return blocks


def splats_per_second(scene, cam, sh_degree, dL_dcolor=None, dL_dinvdepth=None, tile_fraction=1.0, reps=1):
    """Time the fallback on ``scene`` / ``cam`` (gaussian_splatting_amd.synthetic objects, CPU):
    forward only when ``dL_dcolor`` is None, else forward + backward.  With ``tile_fraction`` < 1 the
    render is timed on that stratified tile sample and scaled to the whole frame by list entries:
    t = t(preprocess) + t(binning) + t(render of the sample) x R / R_sample + t(preprocess backward).
    Returns (splats/s, seconds per frame, the last result dict); the time is the mean over ``reps``."""
    P = scene.means3D.shape[0]
    total = 0.0
    for _ in range(max(1, reps)):
        res = rasterize(scene.means3D, scene.opacities, cam.viewmatrix, cam.projmatrix, cam.campos, cam.tanfovx,
                        cam.tanfovy, cam.height, cam.width, shs=scene.shs, sh_degree=sh_degree, scales=scene.scales,
                        rotations=scene.rotations, dL_dcolor=dL_dcolor, dL_dinvdepth=dL_dinvdepth,
                        tile_fraction=tile_fraction)
        t = res["timings"]
        scale = res["num_rendered"] / max(1, res["rendered_instances"]) if tile_fraction < 1.0 else 1.0
        total += t["preprocess"] + t["binning"] + t["render"] * scale + t["preprocess_backward"]
    t_frame = total / max(1, reps)
    return P / t_frame, t_frame, res
