"""Multi-GPU view exchange (include/gsr.h "Multi-GPU view exchange", distributed.ViewExchange).

The exchange replaces the all-reduce of parameter gradients by an all-gather of per-view
render-gradient sums; every rank then runs the per-Gaussian backward over all views.  On one
GPU the views are rendered one after another, so this checks the arithmetic the ranks do:
* one view through the exchange path equals the single-view backward to float32 rounding
  (the same formulas; the compiler may contract them into FMAs differently in the two
  kernels);
* several views equal the sum of the single-view backwards (different summation order:
  float32 tolerance), for the combined and the separate-SH (dc) layouts;
* a view block's dL/dmeans2D equals the backward's;
* the CPU gloo test checks the in-place all-gather layout of the exchange buffer.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests import common as C

GROUPS = ("dL_dmeans3D", "dL_dsh", "dL_dopacity", "dL_dscales", "dL_drotations")


def _view_inputs(case_kw, yaw, dev):
    case = C.Case("views", yaw=yaw, **case_kw)
    return C.build(case), case


def _single_and_block(inp, case, dev, split):
    """Single-view backward grads, and the same view's block."""
    from gaussian_splatting_amd import _C

    fwd = C.run_gpu_forward(inp, device=dev)
    gc, gd = C.l1_grads(case.H, case.W)
    gc, gd = gc.to(dev), gd.to(dev)
    nr, color, radii, geom, binning, img, invd = fwd
    t = {k: (v.to(dev) if isinstance(v, torch.Tensor) else v) for k, v in inp.items()}
    empty = torch.empty(0, device=dev)
    sh = t["shs"]
    if split:
        dc, rest = sh[:, :1].contiguous(), sh[:, 1:].contiguous()
        args = (t["bg"], t["means3D"], radii, empty, t["opacities"], t["scales"], t["rotations"], t["scale_modifier"],
                empty, t["viewmatrix"], t["projmatrix"], t["tanfovx"], t["tanfovy"], gc, gd, dc, rest, t["sh_degree"],
                t["campos"], geom, nr, binning, img, bool(t["antialiasing"]), False)
    else:
        args = (t["bg"], t["means3D"], radii, empty, t["opacities"], t["scales"], t["rotations"], t["scale_modifier"],
                empty, t["viewmatrix"], t["projmatrix"], t["tanfovx"], t["tanfovy"], gc, gd, sh, t["sh_degree"],
                t["campos"], geom, nr, binning, img, bool(t["antialiasing"]), False)
    out = _C.rasterize_gaussians_backward(*args)
    P = t["means3D"].shape[0]
    block = torch.empty(_C.view_block_floats(P), device=dev)
    _C.rasterize_gaussians_backward_screen(*args, view_block=block)
    if split:
        names = ("dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_ddc", "dL_dsh",
                 "dL_dscales", "dL_drotations")
    else:
        names = ("dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
                 "dL_drotations")
    return dict(zip(names, out)), block, t


def _views_backward(t, blocks, split, dev, flags=None, live=None, out=None):
    from gaussian_splatting_amd import _C

    P = t["means3D"].shape[0]
    sh = t["shs"]
    M = sh.shape[1]
    new = torch.zeros if live is not None else torch.empty  # the live-list form leaves unlisted rows as they are
    given = out is not None  # (the caller's outputs: chunk by chunk into one set)
    if not given:
        out = {"dL_dmeans3D": new(P, 3, device=dev), "dL_dopacity": new(P, 1, device=dev),
               "dL_dscales": new(P, 3, device=dev), "dL_drotations": new(P, 4, device=dev)}
    if split:
        dc, rest = sh[:, :1].contiguous(), sh[:, 1:].contiguous()
        if not given:
            out["dL_ddc"] = new(P, 1, 3, device=dev)
            out["dL_dsh"] = new(P, M - 1, 3, device=dev)
        _C.gauss_backward_views(t["means3D"], dc, rest, t["sh_degree"], t["opacities"], t["scales"], t["rotations"],
                                t["scale_modifier"], blocks, out, flags=flags, live=live)
    else:
        if not given:
            out["dL_dsh"] = new(P, M, 3, device=dev)
        _C.gauss_backward_views(t["means3D"], None, sh, t["sh_degree"], t["opacities"], t["scales"], t["rotations"],
                                t["scale_modifier"], blocks, out, flags=flags, live=live)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("case_kw", [dict(P=300, W=64, H=48), dict(P=250, W=48, H=40, sh_degree=1),
                                     dict(P=300, W=64, H=48, antialiasing=True)])
@pytest.mark.record_path
def test_one_view_equals_single_view(case_kw, split):
    dev = torch.device("cuda", 0)
    inp, case = _view_inputs(case_kw, 0.0, dev)
    single, block, t = _single_and_block(inp, case, dev, split)
    got = _views_backward(t, block.view(1, -1), split, dev)
    torch.cuda.synchronize()
    for k in got:
        err = (got[k] - single[k]).abs().max().item()
        assert err <= 1e-5 * max(single[k].abs().max().item(), 1e-3), (k, err)
    P = t["means3D"].shape[0]
    m2 = block[64 + 4 * P: 64 + 8 * P].view(P, 4)[:, :2]
    assert torch.equal(m2, single["dL_dmeans2D"][:, :2])


@pytest.mark.gpu
@pytest.mark.parametrize("split", [False, True])
@pytest.mark.record_path
def test_views_sum_equals_sum_of_single_views(split):
    dev = torch.device("cuda", 0)
    blocks, sums = [], None
    for v, yaw in enumerate((0.0, 7.0, -12.0, 20.0)):
        inp, case = _view_inputs(dict(P=2000, W=96, H=80), yaw, dev)
        single, block, t = _single_and_block(inp, case, dev, split)
        blocks.append(block)
        sums = {k: single[k].clone() for k in single} if sums is None else {k: sums[k] + single[k] for k in sums}
    got = _views_backward(t, torch.stack(blocks), split, dev)
    torch.cuda.synchronize()
    for k in got:
        ref = sums[k]
        err = (got[k] - ref).abs().max().item()
        scale = ref.abs().max().item()
        assert err <= 2e-6 * max(scale, 1e-3) + 1e-9, (k, err, scale)


@pytest.mark.gpu
@pytest.mark.parametrize("split", [False, True])
def test_screen_block_atomic_matches_record(split):
    """The screen-space backward on the atomic path (the default; gauss_live_views writes the block's sums from
    the accumulator rows) gives the record path's view block (gauss_reduce) to float32 re-association: every
    sum plane within 1e-5 of its max |sum|, the flag words (visible, SH clamp bits) and the camera header
    identical."""
    from gaussian_splatting_amd import _lib

    dev = torch.device("cuda", 0)
    inp, case = _view_inputs(dict(P=2000, W=96, H=80), 7.0, dev)
    blocks = {}
    for mode in (0, 1):
        with _lib.options(bwd_atomic=mode):
            _, blocks[mode], t = _single_and_block(inp, case, dev, split)
    torch.cuda.synchronize()
    P = t["means3D"].shape[0]
    rec, atm = blocks[0], blocks[1]
    assert torch.equal(rec[:41], atm[:41])  # the camera header (floats 41-63 are unused)
    assert torch.equal(rec[64 + 10 * P:64 + 11 * P].view(torch.int32), atm[64 + 10 * P:64 + 11 * P].view(torch.int32))
    for lo, hi in ((0, 4 * P), (4 * P, 8 * P), (8 * P, 10 * P)):
        r, a = rec[64 + lo:64 + hi], atm[64 + lo:64 + hi]
        scale = max(float(r.abs().max()), 1e-30)
        assert float((a - r).abs().max()) <= 1e-5 * scale, (lo, float((a - r).abs().max()), scale)
    assert float(atm[64:64 + 10 * P].abs().max()) > 0


def _live(block, P):
    """Gaussians a packed block keeps: visible (flag bit 0) with a non-zero sum."""
    body = block[64:64 + 11 * P]
    sums = torch.cat([body[:4 * P].view(P, 4), body[4 * P:8 * P].view(P, 4), body[8 * P:10 * P].view(P, 2)], 1)
    flags = body[10 * P:11 * P].view(torch.int32)
    return ((flags & 1) != 0) & (sums != 0).any(1)


@pytest.mark.gpu
@pytest.mark.parametrize("split", [False, True])
def test_sparse_blocks_pack_unpack(split):
    """Packed (sparse) view blocks: the entry count is the number of visible Gaussians with a non-zero
    sum, unpacking restores exactly those rows and clears the others' flag words (their sums are left
    as they were, here NaN, and never read), and the multi-view backward over the unpacked blocks
    equals the one over the dense blocks."""
    from gaussian_splatting_amd import _C

    dev = torch.device("cuda", 0)
    blocks, t = [], None
    for yaw in (0.0, 9.0, -15.0):
        inp, case = _view_inputs(dict(P=3000, W=96, H=80, opacity_std=3.0), yaw, dev)
        _, block, t = _single_and_block(inp, case, dev, split)
        blocks.append(block)
    P = t["means3D"].shape[0]
    dense = torch.stack(blocks)
    packed = torch.zeros(len(blocks), _C.view_pack_floats(P), device=dev)
    scratch = torch.empty(4 * P, dtype=torch.uint8, device=dev)
    count = torch.zeros(1, dtype=torch.int32, device=dev)
    counts = []
    for v, b in enumerate(blocks):
        _C.view_block_pack(b, packed[v], scratch, count, P)
        live = _live(b, P)
        counts.append(int(count.item()))
        assert counts[-1] == int(live.sum()) and 0 < counts[-1] < P, (counts[-1], int(live.sum()))
        assert int(packed[v, 63].view(torch.int32).item()) == counts[-1]
        idx = packed[v, 64:64 + 12 * counts[-1]].view(-1, 12)[:, 0].view(torch.int32).long()
        assert torch.equal(idx, torch.nonzero(live).view(-1))  # Gaussian order
    # a packed size that holds the largest count, as the exchange sizes it
    size = _C.view_pack_floats(max(counts))
    recv = packed[:, :size].contiguous()
    unpacked = torch.full_like(dense, float("nan"))
    _C.view_block_unpack(recv, unpacked, P)
    for v, b in enumerate(blocks):
        live = _live(b, P)
        body_d, body_u = b[64:64 + 11 * P], unpacked[v, 64:64 + 11 * P]
        assert torch.equal(unpacked[v, :41], b[:41])  # the camera header (floats 41-62 are unused)
        cols = [(0, 4), (4, 8), (8, 10)]
        for lo, hi in cols:
            w = hi - lo
            d = body_d[lo * P:hi * P].view(P, w)
            u = body_u[lo * P:hi * P].view(P, w)
            assert torch.equal(u[live], d[live])
            assert bool(u[~live].isnan().all())  # left as they were: never read (flag 0)
        flags_u = body_u[10 * P:].view(torch.int32)
        assert torch.equal(flags_u[live], body_d[10 * P:].view(torch.int32)[live])
        assert bool((flags_u[~live] == 0).all())
    # the NaN sums of the left-out Gaussians must not reach the gradients
    got = _views_backward(t, unpacked, split, dev)
    ref = _views_backward(t, dense, split, dev)
    for k in ref:
        assert torch.equal(got[k], ref[k]), k
    # packed mode: the index (one flag word per Gaussian and view) and the backward over the packed
    # blocks in place give the same result
    flags = torch.full((len(blocks), P), -1, dtype=torch.int32, device=dev)
    _C.view_block_index(recv, flags, P)
    for v, b in enumerate(blocks):
        live = _live(b, P)
        f = flags[v]
        assert bool((f[~live] == 0).all())
        assert torch.equal(f[live] & 15, b[64 + 10 * P: 64 + 11 * P].view(torch.int32)[live] & 15)
        assert torch.equal(f[live] >> 4, torch.arange(int(live.sum()), dtype=torch.int32, device=dev))
    got = _views_backward(t, recv, split, dev, flags=flags)
    for k in ref:
        assert torch.equal(got[k], ref[k]), k
    # live-list form: only Gaussians some view flags are visited (zeroed outputs), the same result
    live = torch.empty(_C.views_live_floats(P), dtype=torch.int32, device=dev)
    _C.views_live_list(flags, live, P)
    any_live = torch.stack([_live(b, P) for b in blocks]).any(0)
    cap = (live.numel() - 64 * 32) // 64
    shard_n = live[64 * cap:].view(64, 32)[:, 0]
    listed = torch.cat([live[s * cap: s * cap + int(shard_n[s])] for s in range(64)]).long()
    assert torch.equal(torch.sort(listed).values, torch.nonzero(any_live).view(-1))
    got = _views_backward(t, recv, split, dev, flags=flags, live=live)
    for k in ref:
        assert torch.equal(got[k], ref[k]), k
    # a packed block smaller than the count: the count is reported whole, cap entries are written
    small = torch.zeros(_C.view_pack_floats(5), device=dev)
    _C.view_block_pack(blocks[0], small, scratch, count, P)
    assert int(count.item()) == counts[0]
    # chunked exchange (ViewExchange(chunks=K)): each Gaussian range packs exactly the whole block's entries
    # of its Gaussians (absolute indices), and index + live list + backward run chunk by chunk over the
    # ranges' blocks write the whole-block result bit for bit (an empty range included)
    bounds = [0, 777, 777, 2100, P]
    out = {k: torch.zeros_like(v) for k, v in ref.items()}
    flags_c = torch.full((len(blocks), P), -1, dtype=torch.int32, device=dev)
    for g0, g1 in zip(bounds[:-1], bounds[1:]):
        pk = torch.zeros(len(blocks), _C.view_pack_floats(max(g1 - g0, 1)), device=dev)
        for v, b in enumerate(blocks):
            _C.view_block_pack(b, pk[v], scratch, count, P, rng=(g0, g1))
            n = int(count.item())
            full = packed[v, 64:64 + 12 * counts[v]].view(-1, 12)
            gi = full[:, 0].view(torch.int32)
            want = full[(gi >= g0) & (gi < g1)]
            assert n == want.shape[0]
            assert torch.equal(pk[v, 64:64 + 12 * n].view(-1, 12), want)
            assert torch.equal(pk[v, :41], packed[v, :41])
        _C.view_block_index(pk, flags_c, P, rng=(g0, g1))
        _C.views_live_list(flags_c, live, P, rng=(g0, g1))
        _views_backward(t, pk, split, dev, flags=flags_c, live=live, out=out)
    assert bool((flags_c != -1).all())  # every range's flags written
    for k in ref:
        assert torch.equal(out[k], ref[k]), k


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        buf = torch.empty(2, 5)  # the exchange buffer's layout, without the library
        buf[rank] = torch.arange(5, dtype=torch.float32) + 10 * rank
        dist.all_gather_into_tensor(buf.view(-1), buf[rank])
        np.save(os.path.join(out, f"g{rank}.npy"), buf.numpy())
    finally:
        dist.destroy_process_group()


def test_exchange_layout_gloo(tmp_path):
    """All-gather in place into [world, block] puts rank r's block at row r on every rank."""
    mp.spawn(_worker, args=(_free_port(), str(tmp_path)), nprocs=2, join=True)
    expect = np.stack([np.arange(5) + 10 * r for r in range(2)]).astype(np.float32)
    for r in range(2):
        np.testing.assert_array_equal(np.load(tmp_path / f"g{r}.npy"), expect)
