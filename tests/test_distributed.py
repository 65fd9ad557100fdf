"""View-sharded data parallelism on CPU with the gloo backend, world size 2.

Each rank renders its own view (camera yawed 5 degrees per rank, as bench.py does), writes
the parameter gradients into its GradArena -- here computed by the oracle, since there is no
GPU in this test -- and the arena is reduced with ONE all_reduce.  The result must equal the
sum of the per-view gradients computed in a single process, and the densification statistics
must reduce as train.py:212-215 needs (SUM of norms and counts, MAX of radii).
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests import common as C

WORLD = 2
CASE = C.Case("dist", P=150, W=48, H=40)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def view_grads(rank):
    """Gradients of view `rank` for the five parameter groups, as the backward writes them."""
    case = C.Case(CASE.name, P=CASE.P, W=CASE.W, H=CASE.H, yaw=5.0 * rank)
    inp = C.build(case)
    r = C.run_oracle(inp, precision="f32")
    gc, gd = C.l1_grads(case.H, case.W, seed=1 + rank)
    g = r.handle.backward(gc.numpy(), gd.numpy())
    return g, r.radii


def _worker(rank, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        from gaussian_splatting_amd.distributed import GradArena, reduce_densification_stats

        g, radii = view_grads(rank)
        arena = GradArena(CASE.P, 16, "cpu")
        v = arena.views()
        for k in v:
            v[k].copy_(torch.from_numpy(g[k]).reshape(v[k].shape))
        arena.all_reduce()
        np.save(os.path.join(outdir, f"arena{rank}.npy"), arena.flat.numpy())
        # densification statistics (gaussian_model.py:643-654): norm of the screen-space grad, count, max radius
        norm = torch.from_numpy(np.linalg.norm(g["dL_dmeans2D"][:, :2], axis=1, keepdims=True))
        visible = torch.from_numpy((radii > 0).astype(np.float32)).reshape(-1, 1)
        maxr = torch.from_numpy(radii.astype(np.float32))
        reduce_densification_stats(norm, visible, maxr)
        np.save(os.path.join(outdir, f"stats{rank}.npy"), np.concatenate([norm.numpy().ravel(),
                                                                         visible.numpy().ravel(), maxr.numpy()]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_view_sharded_allreduce_equals_sum_of_views():
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(_free_port(), d), nprocs=WORLD, join=True, start_method="spawn")
        arenas = [np.load(os.path.join(d, f"arena{r}.npy")) for r in range(WORLD)]
        stats = [np.load(os.path.join(d, f"stats{r}.npy")) for r in range(WORLD)]
    # replicas identical after the collective
    np.testing.assert_array_equal(arenas[0], arenas[1])
    from gaussian_splatting_amd.distributed import GradArena

    ref = GradArena(CASE.P, 16, "cpu")
    ref.flat.zero_()
    per_view = [view_grads(r) for r in range(WORLD)]
    for g, _ in per_view:
        for k, t in ref.views().items():
            t.add_(torch.from_numpy(g[k]).reshape(t.shape))
    np.testing.assert_allclose(arenas[0], ref.flat.numpy(), rtol=1e-6, atol=1e-12)
    # the views differ, so the reduction is not trivially 2x one view
    assert not np.allclose(per_view[0][0]["dL_dmeans3D"], per_view[1][0]["dL_dmeans3D"])
    P = CASE.P
    norms = sum(np.linalg.norm(g["dL_dmeans2D"][:, :2], axis=1) for g, _ in per_view)
    counts = sum((r > 0).astype(np.float32) for _, r in per_view)
    maxr = np.maximum(per_view[0][1], per_view[1][1]).astype(np.float32)
    for s in stats:
        np.testing.assert_allclose(s[:P], norms, rtol=1e-5)
        np.testing.assert_array_equal(s[P:2 * P], counts)
        np.testing.assert_array_equal(s[2 * P:], maxr)


def _accumulator_worker(rank, port, outdir, steps):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        from gaussian_splatting_amd.distributed import reduce_densification_stats

        accum, denom, maxr = _local_accumulators(rank, steps)
        reduce_densification_stats(accum, denom, maxr)  # once, right before densify_and_prune
        np.save(os.path.join(outdir, f"acc{rank}.npy"), torch.cat([accum.ravel(), denom.ravel(), maxr]).numpy())
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _local_accumulators(rank, steps, P=64):
    """train.py's running accumulators over `steps` iterations of this rank's views
    (add_densification_stats, gaussian_model.py:643-654, and the max_radii2D update of train.py:212-213)."""
    g = torch.Generator().manual_seed(100 + rank)
    accum = torch.zeros(P, 1)
    denom = torch.zeros(P, 1)
    maxr = torch.zeros(P)
    for _ in range(steps):
        visible = torch.rand(P, generator=g) < 0.7
        norm = torch.rand(P, 1, generator=g)
        radii = torch.randint(0, 20, (P,), generator=g).float() * visible
        accum[visible] += norm[visible]
        denom[visible] += 1
        maxr[visible] = torch.max(maxr[visible], radii[visible])
    return accum, denom, maxr


def test_densification_stats_reduced_once_per_interval():
    """The way train.py would use it: each rank accumulates every iteration, then ONE reduction before
    densify_and_prune gives every rank the statistics of all ranks' views over the whole interval."""
    steps = 100
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_accumulator_worker, args=(_free_port(), d, steps), nprocs=WORLD, join=True,
                           start_method="spawn")
        got = [np.load(os.path.join(d, f"acc{r}.npy")) for r in range(WORLD)]
    np.testing.assert_array_equal(got[0], got[1])
    loc = [_local_accumulators(r, steps) for r in range(WORLD)]
    P = 64
    np.testing.assert_allclose(got[0][:P], sum(a.ravel() for a, _, _ in loc).numpy(), rtol=1e-6)
    np.testing.assert_array_equal(got[0][P:2 * P], sum(b.ravel() for _, b, _ in loc).numpy())
    np.testing.assert_array_equal(got[0][2 * P:], torch.max(loc[0][2], loc[1][2]).numpy())
    assert got[0][P:2 * P].max() <= WORLD * steps  # counts stay bounded by the number of views seen


def test_separate_sh_arena_is_gaussian_model_groups():
    """The separate-SH arena holds GaussianModel's six parameter groups back to back, in training_setup's order
    (gaussian_model.py:235-242), each one contiguous -- the 3DGS-accel backward writes them in place."""
    from gaussian_splatting_amd.distributed import GradArena

    P = 10
    a = GradArena(P, 16, "cpu", separate_sh=True)
    assert a.floats_per_gaussian == 59
    g = a.param_grads()
    assert list(g) == ["xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"] or \
        sorted(g) == sorted(["xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"])
    shapes = {"xyz": (P, 3), "f_dc": (P, 1, 3), "f_rest": (P, 15, 3), "opacity": (P, 1), "scaling": (P, 3),
              "rotation": (P, 4)}
    off = 0
    for name in ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"):
        t = g[name]
        assert tuple(t.shape) == shapes[name] and t.is_contiguous()
        assert t.data_ptr() == a.flat.data_ptr() + 4 * off, name
        off += t.numel()
    assert off == a.flat.numel()
    dc, rest = a.split_features()
    assert dc.data_ptr() == g["f_dc"].data_ptr() and rest.data_ptr() == g["f_rest"].data_ptr()
