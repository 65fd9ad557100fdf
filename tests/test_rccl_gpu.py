"""RCCL on the hardware: every exchange of distributed.py through an nccl process group of one (SURVEY.md
section 8e).  The 8-GPU run is the driver's; this runs the same collectives -- the arena all-reduce, the
count MAX all-reduce and the all-gathers of the sparse, dense and chunked (async) view-block exchanges -- on
cuda:0 in a fresh child process (spawned before anything touches the GPU), so RCCL's stream semantics are
exercised: ``work.wait()`` makes the compute stream wait, the pinned-host count copies are ordered after the
collectives, the side-stream zero fill.

What is checked, in the child, with the deterministic record backward (``bwd_atomic=0``) so the comparisons
can be bitwise:
  * ``GradArena.all_reduce`` over the group leaves the single-view backward's gradients bit for bit (a SUM
    over one rank);
  * the ``views`` (sparse), ``dense`` and ``chunked`` (K = 4, async all-gathers) exchanges -- the chunked one
    also without ``zero=`` -- and a forced capacity resync give bit for bit what ``gauss_backward_views``
    gives over the local view block with no process group at all;
  * those equal the single-view backward (``rasterize_gaussians_backward``) to float32 rounding (the two
    kernels contract FMAs differently, test_view_exchange.py): max |diff| <= 1e-5 max |ref| per tensor;
  * ``dist.get_backend()`` is ``nccl``; each exchange's wall time at N = 1 is printed.
"""
import json
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from tests import common as C

pytestmark = pytest.mark.gpu

CASE = C.Case("rccl1", P=3000, W=96, H=80, focal=90.0, yaw=5.0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _child(rank, port, outdir):
    import time

    import torch.distributed as dist

    from gaussian_splatting_amd import _C, _lib
    from gaussian_splatting_amd.distributed import GradArena, ViewExchange

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    inp = C.build(CASE)
    gc, gd = C.unit_grads(CASE.H, CASE.W, seed=2)
    P, M = CASE.P, inp["shs"].shape[1]
    d = lambda k: inp[k].to(dev)  # noqa: E731
    res = {}
    with _lib.options(bwd_atomic=0):
        fwd = C.run_gpu_forward(inp, device=dev)
        nr, color, radii, geom, binning, img, invd = fwd
        bwd = (d("bg"), d("means3D"), radii, torch.Tensor([]), d("opacities"), d("scales"), d("rotations"), 1.0,
               torch.Tensor([]), d("viewmatrix"), d("projmatrix"), inp["tanfovx"], inp["tanfovy"], gc.to(dev),
               gd.to(dev), d("shs"), inp["sh_degree"], d("campos"), geom, nr, binning, img, False, False)
        single = GradArena(P, M, dev)
        _C.rasterize_gaussians_backward(*bwd, out=single.views())
        block = torch.empty(_C.view_block_floats(P), device=dev)
        _C.rasterize_gaussians_backward_screen(*bwd, view_block=block)
        # the multi-view backward over the local block, no process group anywhere
        local = GradArena(P, M, dev)
        _C.gauss_backward_views(d("means3D"), None, d("shs"), inp["sh_degree"], d("opacities"), d("scales"),
                                d("rotations"), 1.0, block.view(1, -1), local.views())
        torch.cuda.synchronize()

        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
        try:
            res["backend"] = dist.get_backend()
            timing = {}
            # 1. the arena all-reduce: the backward writes the arena, one RCCL all-reduce over the group
            arena = GradArena(P, M, dev)
            _C.rasterize_gaussians_backward(*bwd, out=arena.views())
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            arena.all_reduce()
            torch.cuda.synchronize()
            timing["allreduce"] = (time.perf_counter() - t0) * 1e3
            res["allreduce_bitwise_single"] = bool(torch.equal(arena.flat, single.flat))
            # 2. the view exchanges
            runs = {}
            for mode, sparse, chunks, zero in (("views", True, 1, True), ("dense", False, 1, False),
                                               ("chunked", True, 4, True), ("chunked_nozero", True, 4, False)):
                ex = ViewExchange(P, dev, sparse=sparse, chunks=chunks)
                assert ex.collective and ex.world == 1
                out = GradArena(P, M, dev)
                steps = []
                for step in range(3):  # step 0 waits for the counts; later steps gather at the capacity hint
                    ex.local_block().copy_(block)
                    out.flat.fill_(float("nan"))
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    ex.exchange(zero=out.flat if zero else None)
                    ex.views_backward(d("means3D"), None, d("shs"), inp["sh_degree"], d("opacities"), d("scales"),
                                      d("rotations"), 1.0, out=out.views())
                    torch.cuda.synchronize()
                    steps.append((time.perf_counter() - t0) * 1e3)
                    runs[(mode, step)] = out.flat.clone()
                timing[mode] = min(steps[1:])
                if sparse:
                    res[f"{mode}_hinted"] = (ex.capacity_hint() > 0 if chunks == 1 else
                                             min(ex.chunk_hint(k) for k in range(chunks)) > 0)
                    # a hint below the count: detected after the backward is queued, the exchange redone
                    ex.capacity_hint = lambda: 8  # noqa: E731
                    ex.chunk_hint = lambda k: 8  # noqa: E731
                    ex.local_block().copy_(block)
                    out.flat.fill_(float("nan"))
                    ex.exchange(zero=out.flat if zero else None)
                    ex.views_backward(d("means3D"), None, d("shs"), inp["sh_degree"], d("opacities"), d("scales"),
                                      d("rotations"), 1.0, out=out.views())
                    torch.cuda.synchronize()
                    runs[(mode, "resync")] = out.flat.clone()
                    res[f"{mode}_resyncs"] = ex.resyncs
            for key, flat in runs.items():
                res[f"bitwise_{key[0]}_{key[1]}"] = bool(torch.equal(flat, local.flat))
            worst = 0.0
            for k, v in single.views().items():
                ref = v.abs().max().item()
                got = GradArena(P, M, dev)
                got.flat.copy_(runs[("views", 0)])
                worst = max(worst, (got.views()[k] - v).abs().max().item() / max(ref, 1e-30))
            res["views_vs_single_rel"] = worst
            res["exchange_ms_n1"] = timing
            dist.barrier()
        finally:
            dist.destroy_process_group()
    with open(os.path.join(outdir, "res.json"), "w") as f:
        json.dump(res, f)


@pytest.mark.timeout(300)
def test_exchanges_through_rccl_group_of_one():
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_child, args=(_free_port(), d), nprocs=1, join=True, start_method="spawn")
        with open(os.path.join(d, "res.json")) as f:
            res = json.load(f)
    print(f"[rccl group of one] backend {res['backend']}; exchange wall ms at N=1: "
          + ", ".join(f"{k} {v:.3f}" for k, v in res["exchange_ms_n1"].items())
          + f"; views vs single-view backward rel {res['views_vs_single_rel']:.2e}")
    assert res["backend"] == "nccl"
    assert res["allreduce_bitwise_single"]
    bad = [k for k, v in res.items() if k.startswith("bitwise_") and not v]
    assert not bad, bad
    for mode in ("views", "chunked", "chunked_nozero"):
        assert res[f"{mode}_hinted"], mode
        assert res[f"{mode}_resyncs"] == 1, (mode, res[f"{mode}_resyncs"])
    assert res["views_vs_single_rel"] <= 1e-5
    assert np.isfinite(list(res["exchange_ms_n1"].values())).all()
