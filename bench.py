#!/usr/bin/env python3
"""Benchmark: Gaussian-splats/sec, forward + backward, 1M Gaussians @ 1920x1080, SH degree 3.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 1m_1080p_sh3]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

One step = ``_C.rasterize_gaussians`` + ``_C.rasterize_gaussians_backward`` for one
view, on synthetic inputs already resident in HBM.  When N > 1
the step also makes every rank's gradients the sum over all N views, by one of two
exchanges over RCCL: the all-gather of the sparse per-view
render-gradient blocks followed by the multi-view backward (``views``), or the
all-reduce of the flat 59-float-per-Gaussian parameter-gradient arena (``allreduce``).
``--exchange auto`` (the default) times both during the warm-up on this fabric, with the
same collective count on every rank, and keeps the faster; the line's ``multi_gpu``
object carries both timings and the pick.  Rank r renders view r (camera yawed by 5*r
degrees), so per-GPU work is fixed as N grows ("weak" scaling) and value = N * P * K /
(max over ranks of the K-step time).

Rank 0 prints one JSON line.  It carries the roofline of the dominant kernel (its
algorithmic bytes per launch / its mean duration from HIP events on the launch
stream), the host side of every step (``host``: forward call, the forward's wait for
the instance count, backward enqueue, exchange), and the CPU baseline: the
pure-PyTorch fallback rasterizer (oracle/torch_fallback.py) timed on one full frame
on this host's cores, with the C restatement (oracle/) beside it.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from gaussian_splatting_amd import _C, _lib  # noqa: E402
from gaussian_splatting_amd import synthetic as syn  # noqa: E402
from gaussian_splatting_amd.distributed import GradArena, ViewExchange  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# HBM bytes per launch measured with rocprofv3 PMC passes (scripts/pmc_session.sh -> tools/pmc_summary.py);
# reported as roofline.traffic for the dominant kernel when the profile has it.
PMC_PROFILE = os.path.join(ROOT, "profiles", "pmc_latest.json")


def algorithmic_bytes(stage: str, P: int, I: int, W: int, H: int, K: int) -> float:
    """Algorithmic HBM bytes of one launch of each stage (DESIGN.md "Roofline"; SURVEY.md section 8d itemisation)."""
    N = W * H
    table = {
        # reads means 12, scale 12, rot 16, opacity 4, SH 12K; writes radii 4, means2D 8, depth 4, conic+opacity 16,
        # rgb 12, tiles_touched 4
        "preprocess": (44 + 12 * K + 48) * P,
        # binning.hip: K1+K2 read rect 8 + tiles_touched 4 per Gaussian; K3 reads rect, tiles_touched, depth 16 and
        # writes record starts 4 per Gaussian plus an 8 B key per instance; K4 reads the keys, writes 4 B ids
        "bin_count": 12 * P,
        "bin_scatter": 20 * P + 8 * I,
        "tile_sort": 12 * I,
        # gather 44 B per instance (xy 8, conic+opacity 16, rgb 12, depth 4, index 4); write 24 B per pixel
        "render_fwd": 44 * I + 24 * N,
        # gather 44 B per instance; read 24 B per pixel; write the per-Gaussian accumulators (10 floats)
        "render_bwd": 44 * I + 24 * N + 40 * P,
        # read accumulators 40 + preprocess inputs 48 + 12K; write grads 56 + 12K
        "gauss_reduce": 40 * I + 40 * P,
        "gauss_bwd": (40 + 48 + 12 * K + 56 + 12 * K) * P,
    }
    return float(table.get(stage, 0))


def step_algorithmic_bytes(P, I, W, H, K):
    """B_alg of SURVEY.md section 8d for one forward + backward."""
    return (304 + 36 * K) * P + 132 * I + 48 * W * H


def cpu_threads():
    """Threads for the CPU baselines: the process's real CPU set (``os.sched_getaffinity``), capped by the
    box's OMP_NUM_THREADS share when one is set (a GPU lease's worker-pool share; the affinity mask may
    still show the whole machine).  Returns (threads, facts for the bench line)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:  # not Linux
        aff = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    share = int(omp) if omp and omp.isdigit() and int(omp) > 0 else None
    threads = max(1, min(aff, share) if share else aff)
    policy = ("the lease's OMP_NUM_THREADS share: the GPU pool gives one GPU's job a 16-CPU share of the host and "
              "asks worker pools to stay within it (the affinity mask still lists the whole machine), so the "
              "whole affinity set is not used (DESIGN.md section 8)" if share and share < aff else
              "the process's whole CPU set (os.sched_getaffinity)")
    return threads, {"affinity_cpus": aff, "omp_num_threads": share, "host_cpus": os.cpu_count(),
                     "threads_policy": policy}


def cpu_baseline(cfg_name: str, P: int, W: int, H: int, forward_only: bool = False, gpu_num_rendered=None):
    """north_star's CPU baseline: the pure-PyTorch fallback rasterizer (oracle/torch_fallback.py, fp32)
    on this host's cores, forward + autograd backward on the same frame as the GPU -- one FULL frame
    (every tile rendered; SURVEY.md section 8d: 1 rep at configs 2/3, 5 forward reps at config 1),
    after an untimed warm-up on a small tile sample."""
    from oracle import torch_fallback as tf

    threads, cpus = cpu_threads()
    torch.set_num_threads(threads)
    scene, cam = syn.config_scene(cfg_name, seed=0, P=P)
    gc, gd = (None, None) if forward_only else syn.upstream_grads(H, W)
    reps = 5 if P <= 100_000 else 1
    tf.splats_per_second(scene, cam, scene.sh_degree, gc, gd, tile_fraction=0.02)  # untimed warm-up
    t0 = time.perf_counter()
    value, t_frame, res = tf.splats_per_second(scene, cam, scene.sh_degree, gc, gd, tile_fraction=1.0, reps=reps)
    wall = time.perf_counter() - t0
    what = "forward" if forward_only else "forward + autograd backward"
    t = res["timings"]
    # the same workload as the GPU's: its instance count (tests/test_torch_fallback.py pins the integers)
    same = {} if gpu_num_rendered is None else {
        "num_rendered_gpu": int(gpu_num_rendered),
        "num_rendered_diff": int(res["num_rendered"]) - int(gpu_num_rendered)}
    return {"value": value, "unit": "Gaussian-splats/s", "cores": torch.get_num_threads(), **cpus,
            "num_rendered": int(res["num_rendered"]), **same,
            "kind": "port", "impl": "pure-PyTorch fallback rasterizer (oracle/torch_fallback.py, fp32)",
            "sample": f"{cfg_name} ({P} Gaussians, {W}x{H}) {what}: {reps} full frame(s), every tile rendered "
                      f"({res['num_rendered']} list entries); {t_frame:.2f} s per frame (preprocess "
                      f"{t['preprocess']:.2f}, binning {t['binning']:.2f}, render {t['render']:.2f}, preprocess "
                      f"backward {t['preprocess_backward']:.2f} s), {wall:.1f} s timed on {torch.get_num_threads()} torch "
                      f"threads: the process's CPU set ({cpus['affinity_cpus']} CPUs, os.sched_getaffinity), capped "
                      f"by the box's OMP_NUM_THREADS share ({cpus['omp_num_threads']}); os.cpu_count() = "
                      f"{cpus['host_cpus']}"}


def cpu_baseline_c(cfg_name: str, P: int, W: int, H: int, threads: int, min_seconds: float = 8.0):
    """Second CPU figure: the C restatement (oracle/gsr_oracle.c, OpenMP) forward + backward on the
    same frame, repeated until at least ``min_seconds`` of CPU work."""
    from oracle import oracle

    scene, cam = syn.config_scene(cfg_name, seed=0, P=P)
    gc, gd = syn.upstream_grads(H, W)
    reps, total = 0, 0.0
    while total < min_seconds and reps < 50:
        t0 = time.perf_counter()
        r = oracle.forward(scene.means3D, scene.opacities, cam.viewmatrix, cam.projmatrix, cam.campos, cam.tanfovx,
                           cam.tanfovy, H, W, shs=scene.shs, sh_degree=scene.sh_degree, scales=scene.scales,
                           rotations=scene.rotations, nthreads=threads)
        r.handle.backward(gc, gd, nthreads=threads)
        total += time.perf_counter() - t0
        reps += 1
        del r
    return {"value": reps * P / total, "unit": "Gaussian-splats/s", "cores": threads, **cpu_threads()[1],
            "kind": "port",
            "impl": "C restatement (oracle/gsr_oracle.c, float32, OpenMP)",
            "sample": f"{reps} full {cfg_name} frames ({P} Gaussians, {W}x{H}), forward+backward, "
                      f"{total:.1f} s on {threads} OpenMP threads"}


def cpu_only(cfg_name: str) -> None:
    """BASELINE.json configs[0] ("forward-only via PyTorch CPU fallback, plumbing, no GPU"): the
    fallback alone, one JSON line, no HIP device touched."""
    cfg = syn.CONFIGS[cfg_name]
    base = cpu_baseline(cfg_name, cfg["P"], cfg["width"], cfg["height"], forward_only=True)
    print(json.dumps({"metric": "Gaussian-splats/sec forward, CPU fallback", "value": base["value"],
                      "unit": "Gaussian-splats/s", "n_gpus": 0, "higher_is_better": True, "dtype": "fp32",
                      "data": "synthetic (frustum-uniform Gaussians, SURVEY.md 8d; seed 0)",
                      "config": {"workload": cfg_name, "gaussians": cfg["P"], "width": cfg["width"],
                                 "height": cfg["height"], "sh_degree": cfg["sh_degree"], "pass": "forward"},
                      "cpu_baseline": base}), flush=True)


def _time_exchange(kind, E, arena, dev, reps=5):
    """One exchange alone (no render): ``reps`` passes, every rank the same collective count; the max over
    ranks of the mean wall time per pass (ms)."""
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        if kind in ("views", "chunked"):
            E.exchange()
            if kind == "chunked":  # the chunks' gathers are waited for by the backward; here by hand
                for w in E._cworks or []:
                    if w is not None:
                        w.wait()
                E._cworks = None
            E.finish()
        else:
            arena.all_reduce()
    torch.cuda.synchronize()
    ms = torch.tensor([(time.perf_counter() - t0) / reps * 1e3], dtype=torch.float64, device=dev)
    dist.all_reduce(ms, op=dist.ReduceOp.MAX)
    return float(ms.item())


def multi_rank_diagnostics(args, world, exchange, ex, exc, arena, per_rank, cand_ms, cand_spread, dev):
    """With a process group: which exchange ran and why (the interleaved warm-up timings of the candidates
    when ``auto``: median and spread), every candidate exchange's time alone (untimed passes after the
    timed region, every rank running the same collective count), the bytes each rank receives, and every
    rank's own ms/step -- so a straggler or a wrong pick shows in the record."""
    E = exc if exchange == "chunked" else ex
    alone = {"allreduce": _time_exchange("allreduce", None, arena, dev)}
    if ex is not None:
        alone["views" if ex.sparse else "dense"] = _time_exchange("views", ex, arena, dev)
    if exc is not None:
        alone["chunked"] = _time_exchange("chunked", exc, arena, dev)
    ms = alone["dense" if exchange == "views" and not ex.sparse else exchange]
    if exchange in ("views", "chunked"):
        recv = E.received_bytes()
        what = ("all-gather of sparse view blocks (48 B per Gaussian with a non-zero render gradient; "
                f"{E.last_entries} entries gathered per rank at the capacity hint; "
                f"{E.resyncs} re-gathers after a hint below the count)" if E.sparse and E.last_entries else
                "all-gather of dense 44-B/Gaussian view blocks") + " + the multi-view backward on every rank"
        if exchange == "chunked":
            what = (f"{E.chunks} Gaussian-range chunks, each an async " + what +
                    "; chunk k+1's all-gather runs during chunk k's backward")
    else:
        recv = int(2 * (world - 1) / world * arena.flat.numel() * 4)
        what = "RCCL all-reduce of the 59-float/Gaussian parameter-gradient arena"
    if args.exchange == "auto":
        why = ("--exchange auto: the candidates timed in the warm-up on this fabric in interleaved rounds (whole "
               f"steps, max over ranks, {args.auto_steps} steps per candidate and round), median over "
               f"{max(3, args.auto_rounds)} rounds: " + ", ".join(f"{k} {v:.4f} ms/step" for k, v in cand_ms.items())
               + f"; the fastest is {exchange}")
    else:
        why = f"--exchange {args.exchange}"
    return {"exchange": exchange, "what": what, "why": why, "candidates_ms_per_step": cand_ms or None,
            "candidates_spread_ms": cand_spread or None,
            "exchange_ms": ms, "exchange_ms_alone": alone, "received_bytes_per_rank": recv,
            "exchange_GBs_per_rank": recv / (ms * 1e-3) / 1e9 if ms > 0 else None,
            "per_rank_ms_per_step": [round(e / args.steps * 1e3, 4) for e in per_rank],
            "backend": dist.get_backend(), "world_size": world, "group_of_one": world == 1}


class HostClock:
    """Host-side timings of the timed steps (per step: the forward call, which includes its wait for
    the instance count; forward return -> backward call; the backward call; the exchange), so every
    run carries the evidence for a GPU that waits on the host."""

    KEYS = ("forward_call", "fwd_return_to_bwd_call", "backward_call", "exchange", "step_wall")

    def __init__(self):
        self.t = {k: [] for k in self.KEYS}
        self.gc_runs = 0
        self.on = False

    def add(self, k, dt):
        if self.on:
            self.t[k].append(dt * 1e3)

    def summary(self, lib):
        import statistics

        out = {}
        for k, v in self.t.items():
            if v:
                out[k + "_ms"] = {"mean": round(statistics.fmean(v), 4), "median": round(statistics.median(v), 4),
                                  "max": round(max(v), 4)}
        # inside the library (include/gsr.h gsr_host_stats): the count wait, and the whole forward /
        # backward calls -- the Python side of a call is its call time minus these
        for k, st in lib.items():
            out[f"lib_{k}_ms"] = {"mean": round(st["total_ms"] / st["calls"], 4) if st["calls"] else None,
                                  "max": round(st["max_ms"], 4), "calls": st["calls"]}
        out["python_gc_collections"] = self.gc_runs
        # the steps whose wall time is well above the median (a host stall leaves the GPU idle): step
        # index, step wall / forward call / backward call (ms), so a slow run carries which step and call
        walls = self.t["step_wall"]
        if walls:
            med = statistics.median(walls)
            slow = [i for i, w in enumerate(walls) if w > 1.3 * med]
            out["slow_steps"] = [[i, round(walls[i], 3), round(self.t["forward_call"][i], 3),
                                  round(self.t["backward_call"][i], 3)] for i in slow[:8]]
        return out


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_command(n: int, argv, port: int) -> list:
    """The command that runs this bench as ``n`` ranks, one process per GPU (the driver's own form:
    ``torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1``)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def maybe_launch(args, argv) -> int | None:
    """``--gpus N`` with N > 1 and no torch.distributed environment: start the N ranks as a CHILD
    process (torch.distributed.run) and return its exit code -- the caller exits with it.  Runs before
    anything touches the GPU (the library loads lazily; torch.cuda is not called), so this process holds
    no HIP context.  Returns None when this process is itself a rank (or N == 1).  Inside a rank, a
    WORLD_SIZE different from --gpus is an error (exit 2), never a silent one-rank run."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus > 1:
            cmd = launch_command(args.gpus, argv, _free_port())
            print(f"[bench] --gpus {args.gpus}: launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr,
                  flush=True)
            env = dict(os.environ)
            env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
            return subprocess.run(cmd, env=env).returncode
        return None
    if int(env_world) != args.gpus:
        print(f"[bench] error: WORLD_SIZE={env_world} but --gpus {args.gpus}: the rank count the launcher "
              f"started differs from the one requested", file=sys.stderr, flush=True)
        return 2
    return None


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="1m_1080p_sh3", choices=sorted(syn.CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-census", action="store_true",
                    help="skip the census pass (profiler runs: keeps its kernel instantiations out of the trace)")
    ap.add_argument("--exchange", choices=("auto", "views", "chunked", "dense", "allreduce"), default="auto",
                    help="N > 1: all-gather the sparse view blocks (views), the same in Gaussian-range chunks whose "
                         "all-gathers overlap the multi-view backward of the earlier chunks (chunked), the dense "
                         "view blocks (dense), or all-reduce the parameter gradients (allreduce); auto times views, "
                         "chunked and allreduce in the warm-up and keeps the fastest (DESIGN.md section 7)")
    ap.add_argument("--exchange-chunks", type=int, default=4, help="Gaussian-range chunks of --exchange chunked")
    ap.add_argument("--auto-steps", type=int, default=3,
                    help="timed steps per candidate and round of --exchange auto")
    ap.add_argument("--auto-rounds", type=int, default=3,
                    help="--exchange auto: interleaved rounds (views, chunked, allreduce, then again); the pick is "
                         "the lowest median over the rounds (at least 3)")
    ap.add_argument("--nccl-group", action="store_true",
                    help="N = 1 inside an nccl (RCCL) process group of one: the step runs the --exchange path "
                         "with every collective issued, so the line's multi_gpu object carries RCCL times at N = 1")
    ap.add_argument("--separate-sh", action="store_true",
                    help="SH as train.py's separate_sh path passes it: dc [P,1,3] + rest [P,M-1,3] (3DGS-accel surface)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="threads of the C-restatement figure (default: the process's CPU set, capped by OMP_NUM_THREADS)")
    ap.add_argument("--cpu-only", action="store_true",
                    help="no GPU: time the pure-PyTorch fallback forward on --config (BASELINE configs[0] plumbing)")
    ap.add_argument("--roofline-every", type=int, default=4,
                    help="time the dominant kernel with a HIP event pair on every E-th timed step (each pair "
                         "leaves the GPU idle for a few us; 1 = every step)")
    ap.add_argument("--ramp-seconds", type=float, default=0.3,
                    help="untimed steps before the warmup, until the GPU clock has ramped up (DVFS)")
    return ap.parse_args(argv)


def main():
    argv = sys.argv[1:]
    args = parse_args(argv)
    if args.gpus < 1:
        print("[bench] error: --gpus must be >= 1", file=sys.stderr)
        sys.exit(2)
    if not args.cpu_only:
        rc = maybe_launch(args, argv)
        if rc is not None:
            sys.exit(rc)
    if args.cpu_only:
        cpu_only(args.config)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # GSR_BENCH_SHARE_GPU=1 (rehearsal on a one-GPU box only): every rank on cuda:0, gloo
    # collectives -- exercises the N > 1 code path, not its speed
    rehearse = os.environ.get("GSR_BENCH_SHARE_GPU", "0") == "1"
    gpu = 0 if rehearse else local_rank
    ndev = torch.cuda.device_count()  # counts devices without initialising HIP on this image
    if gpu >= ndev:
        print(f"[bench] error: rank {rank} (local rank {local_rank}) needs cuda:{gpu} but {ndev} device(s) are "
              "visible", file=sys.stderr, flush=True)
        sys.exit(2)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    ranks_seen = 1
    # a process group whenever N > 1, or at N = 1 with --nccl-group (RCCL exercised by a group of one)
    grouped = world > 1 or args.nccl_group
    if grouped:
        if rehearse:
            dist.init_process_group("gloo")
        elif world == 1 and "MASTER_ADDR" not in os.environ:
            dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                                    device_id=dev)
        else:
            dist.init_process_group("nccl", device_id=dev)
        # the rank count the collective backend really connects: a SUM of ones over the group
        one = torch.ones(1, dtype=torch.int64, device=dev)
        dist.all_reduce(one)
        ranks_seen = int(one.item())
        if ranks_seen != world or dist.get_world_size() != world:
            print(f"[bench] error: {dist.get_backend()} saw {ranks_seen} ranks (world size "
                  f"{dist.get_world_size()}), expected {world}", file=sys.stderr, flush=True)
            sys.exit(2)
        dev_ids = torch.tensor([gpu], dtype=torch.int64, device=dev)
        all_ids = [torch.zeros_like(dev_ids) for _ in range(world)]
        dist.all_gather(all_ids, dev_ids)
        rank_devices = [int(t.item()) for t in all_ids]
        if not rehearse and len(set(rank_devices)) != world:
            print(f"[bench] error: ranks share devices {rank_devices}", file=sys.stderr, flush=True)
            sys.exit(2)

    cfg = syn.CONFIGS[args.config]
    P, W, H, Kdeg = cfg["P"], cfg["width"], cfg["height"], cfg["sh_degree"]
    K = (Kdeg + 1) ** 2
    scene, cam = syn.config_scene(args.config, seed=0, yaw_deg=5.0 * rank)
    scene, cam = scene.to(dev), cam.to(dev)
    gc, gd = syn.upstream_grads(H, W, seed=1 + rank)
    gc, gd = gc.to(dev), gd.to(dev)
    bg = torch.zeros(3, device=dev)
    empty = torch.empty(0, device=dev)
    # SH layout: one [P,M,3] tensor (the vendored rasterizer), or dc + rest as train.py's separate_sh path
    # hands them over (gaussian_renderer/__init__.py:106-125)
    if args.separate_sh:
        sh_dc, sh_rest = scene.shs[:, :1].contiguous(), scene.shs[:, 1:].contiguous()
        sh_in = (sh_dc, sh_rest)
    else:
        sh_dc, sh_rest = None, scene.shs
        sh_in = (scene.shs,)
    arena = GradArena(P, scene.shs.shape[1], dev, separate_sh=args.separate_sh)
    uses_views = grouped and args.exchange in ("auto", "views", "dense")
    ex = ViewExchange(P, dev, sparse=args.exchange != "dense") if uses_views else None
    exc = (ViewExchange(P, dev, chunks=args.exchange_chunks)
           if grouped and args.exchange in ("auto", "chunked") else None)
    # the exchange the steps run: fixed by --exchange, or (auto) picked by timing in the warm-up below
    exchange = "none" if not grouped else ("allreduce" if args.exchange == "allreduce" else
                                           "chunked" if args.exchange == "chunked" else "views")
    clock = HostClock()
    pc = time.perf_counter

    def step(collective=True):
        t0 = pc()
        fwd = _C.rasterize_gaussians(bg, scene.means3D, empty, scene.opacities, scene.scales, scene.rotations, 1.0,
                                     empty, cam.viewmatrix, cam.projmatrix, cam.tanfovx, cam.tanfovy, H, W, *sh_in,
                                     Kdeg, cam.campos, False, False, False)
        t1 = pc()
        nr, color, radii, geom, binning, img, invd = fwd
        bwd = (bg, scene.means3D, radii, empty, scene.opacities, scene.scales, scene.rotations, 1.0, empty,
               cam.viewmatrix, cam.projmatrix, cam.tanfovx, cam.tanfovy, gc, gd, *sh_in, Kdeg, cam.campos, geom, nr,
               binning, img, False, False)
        t2 = pc()
        if exchange in ("views", "chunked") and collective:  # view blocks, every rank sums all views' gradients
            E = exc if exchange == "chunked" else ex
            _C.rasterize_gaussians_backward_screen(*bwd, view_block=E.local_block())
            t3 = pc()
            E.exchange(zero=arena.flat)  # the outputs zeroed beside the exchange; a live-list backward
            E.views_backward(scene.means3D, sh_dc, sh_rest, Kdeg, scene.opacities, scene.scales, scene.rotations,
                             1.0, out=arena.views())
        else:
            _C.rasterize_gaussians_backward(*bwd, out=arena.views())
            t3 = pc()
            if grouped and collective:
                arena.all_reduce()
        t4 = pc()
        clock.add("forward_call", t1 - t0)
        clock.add("fwd_return_to_bwd_call", t2 - t1)
        clock.add("backward_call", t3 - t2)
        if grouped and collective:
            clock.add("exchange", t4 - t3)
        return nr

    # Untimed clock ramp: the GPU lowers its clock when idle and takes ~0.1 s of load to come back
    # (measured: 1.225 ms/step after 3 warm-up steps vs 1.200 after 300).  Then the W warm-up steps.
    # The ramp runs a time-bounded number of steps, which differs between ranks, so it runs
    # without collectives (a mismatched collective count would hang the job).
    t_ramp = time.perf_counter()
    while time.perf_counter() - t_ramp < args.ramp_seconds:
        step(collective=False)
        torch.cuda.synchronize()
    if grouped:
        dist.barrier()
    for _ in range(args.warmup):
        nr = step()
    torch.cuda.synchronize()
    # --exchange auto with a group: time whole steps with each exchange on this fabric, in interleaved rounds
    # (views, chunked, allreduce, then again: a one-off stall hits one sample, not one candidate), the same
    # number of steps and collectives on every rank, the max over ranks; keep the lowest median
    cand_ms, cand_spread = {}, {}
    if grouped and args.exchange == "auto":
        import statistics

        samples = {c: [] for c in ("views", "chunked", "allreduce")}
        for _ in range(max(3, args.auto_rounds)):
            for cand in samples:
                exchange = cand
                step()  # one untimed step after the switch
                torch.cuda.synchronize()
                dist.barrier()
                t0 = time.perf_counter()
                for _ in range(args.auto_steps):
                    step()
                torch.cuda.synchronize()
                tt = torch.tensor([(time.perf_counter() - t0) / args.auto_steps * 1e3], dtype=torch.float64,
                                  device=dev)
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                samples[cand].append(float(tt.item()))
        cand_ms = {c: statistics.median(v) for c, v in samples.items()}
        cand_spread = {c: {"min": min(v), "max": max(v), "rounds": [round(x, 4) for x in v]}
                       for c, v in samples.items()}
        exchange = min(cand_ms, key=cand_ms.get)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
    # Per-stage breakdown in a separate, untimed pass: every timed stage adds an event pair
    # (~10 us of idle GPU each), so the timed region below records events only around the
    # dominant kernel.
    _lib.profile_reset()
    _lib.profile_enable(True)
    for _ in range(max(3, min(args.steps, 10))):
        step()
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    stages = _lib.profile_collect()
    per_stage = {k: (v[0] / v[1] if v[1] else 0.0) for k, v in stages.items()}
    dom = max(per_stage, key=per_stage.get)
    # Work census (untimed, census kernel instantiations): how many (pixel, splat) pairs the render
    # kernels blend -- their cost follows these pairs, not the per-instance bytes of the roofline.
    census = None if args.no_census else _lib.census(lambda: step(collective=False), dev)

    _lib.profile_reset()
    every = max(1, args.roofline_every)
    if grouped:
        dist.barrier()
    torch.cuda.synchronize()
    import gc as _gc

    def _gc_cb(phase, info):
        if phase == "start" and clock.on:
            clock.gc_runs += 1
    _gc.callbacks.append(_gc_cb)
    _lib.host_stats(reset=True)
    clock.on = True
    t0 = time.perf_counter()
    for i in range(args.steps):
        ts = pc()
        # the dominant kernel's launches are timed live, on its own stream, on every `every`-th step
        if i % every == 0:
            _lib.profile_enable(True, stages=[dom])
        elif i % every == 1:
            _lib.profile_enable(False)
        nr = step()
        clock.add("step_wall", pc() - ts)
    torch.cuda.synchronize()
    if grouped:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    clock.on = False
    _gc.callbacks.remove(_gc_cb)
    host = clock.summary(_lib.host_stats())
    _lib.profile_enable(False)
    dom_total, dom_calls = _lib.profile_collect()[dom]
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    per_rank = [elapsed]
    if grouped:
        gathered = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(gathered, t)
        per_rank = [float(g.item()) for g in gathered]
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    multi = (multi_rank_diagnostics(args, world, exchange, ex, exc, arena, per_rank, cand_ms, cand_spread, dev)
             if grouped else None)
    if multi is not None:
        multi.update({"ranks_seen_by_backend": ranks_seen, "rank_devices": rank_devices,
                      "visible_devices_per_rank": ndev, "shared_gpu_rehearsal": rehearse})

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = world * P * args.steps / elapsed
        dom_ms = dom_total / dom_calls if dom_calls else 0.0  # HIP events on the launch stream, timed region
        # SURVEY.md 8d's algorithmic bytes of the kernel's own work (render_bwd: 44 I + 24 W H + 40 P); the
        # contract excludes zero-init memsets, so the fill that rides in the launch is reported beside it
        alg = algorithmic_bytes(dom, P, nr, W, H, K)
        # zero_fill = 3 (the default): the zero fill of the backward's dense outputs rides in render_bwd's
        # launch (api.hip): 4 B x (means2D 3, opacity 1, colour 3, inverse depth 1, means3D 3, cov3D 6, SH 3K,
        # scale 3, rotation 4) per Gaussian -- NOT algorithmic bytes, its own field and rate
        fill_bytes = 4.0 * P * (24 + 3 * K) if dom == "render_bwd" and _lib.option_get("zero_fill") == 3 else 0.0
        traffic, traffic_src, kk, traffic_detail = None, None, {}, None
        if os.path.exists(PMC_PROFILE):
            prof = json.load(open(PMC_PROFILE))
            entry = prof.get("configs", {}).get(args.config) or (prof if args.config == "1m_1080p_sh3" else {})
            kk = entry.get("kernels", {}).get(dom) or {}
            if kk:
                traffic = kk["hbm_read_bytes"] + kk["hbm_write_bytes"]
                traffic_src = entry.get("source")
                # the raw counters beside the corrected figure: FETCH_SIZE x 1024 B and WRITE_SIZE x 1024 B per
                # launch, and the read factor applied (tools/pmc_summary.py; calibrated per access shape by
                # tools/fetch_calib.hip where the kernel's reads are not wide coalesced streams)
                rf = kk.get("read_factor", 2.0)
                traffic_detail = {"fetch_size_bytes_raw": kk.get("fetch_size_bytes", kk["hbm_read_bytes"] / rf),
                                  "write_size_bytes_raw": kk.get("write_size_bytes", kk["hbm_write_bytes"]),
                                  "read_factor": rf, "read_factor_basis": kk.get("read_factor_basis",
                                                                                 "x2: MI355X_MICROARCH.md 'HBM'"),
                                  "read_bytes": kk["hbm_read_bytes"], "write_bytes": kk["hbm_write_bytes"],
                                  "write_bytes_less_fill": kk["hbm_write_bytes"] - fill_bytes}
        achieved = alg / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
        traffic_frac = traffic / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if traffic is not None and dom_ms > 0 else None
        # the kernel's own counter bytes: the fill's writes taken out, as from the model
        own_traffic = traffic - fill_bytes if traffic is not None else None
        own_frac = own_traffic / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if own_traffic is not None and dom_ms > 0 else None
        # 5M@4K: the 8d byte model bills 44 B for every instance, but the render walks ~7% of each 3,540-entry
        # list, so there the counter-based fraction (fill excluded) is the headline and the
        # model's beside it
        counter_headline = args.config == "5m_4k_sh3" and own_frac is not None
        valu_frac = None
        if traffic is not None and kk.get("valu_insts"):
            # wave64 VALU issues in 2 cycles on a 32-wide SIMD; 1024 SIMDs at 2.4 GHz (MI355X_MICROARCH.md)
            valu_frac = kk["valu_insts"] * 2.0 / (dom_ms * 1e-3 * 2.4e9 * 1024)
        work = dict(census or {})
        for k, stage in (("fwd", "render_fwd"), ("bwd", "render_bwd")) if census else ():
            t_ms = per_stage.get(stage, 0.0)
            pairs = census["fwd_pairs_blended" if k == "fwd" else "bwd_pairs_grad"]
            work[f"{stage}_pairs_per_s"] = pairs / (t_ms * 1e-3) if t_ms > 0 else None
        if census:
            work["pairs_per_instance"] = census["fwd_pairs_blended"] / nr if nr else None
        # BASELINE.json's metric names the headline workload; another --config says its own
        metric = ("Gaussian-splats/sec fwd+bwd @1080p, 1M Gaussians" if args.config == "1m_1080p_sh3" else
                  f"Gaussian-splats/sec fwd+bwd @{W}x{H}, {P} Gaussians ({args.config}; not the headline metric)")
        par = f"view-sharded x{world}"
        if grouped:
            # the backend that really ran (gloo in the one-GPU rehearsal, nccl = RCCL on ROCm)
            be = "RCCL" if multi["backend"] == "nccl" else multi["backend"]
            par += {"views": f" + {be} all-gather of " + ("sparse " if ex is not None and ex.sparse else "dense ")
                    + "view blocks",
                    "chunked": f" + {be} all-gathers of sparse view blocks in {args.exchange_chunks} Gaussian-range "
                               "chunks, overlapped with the multi-view backward",
                    "allreduce": f" + {be} all-reduce of the gradient arena"}[exchange]
        line = {
            "metric": metric,
            "value": value,
            "unit": "Gaussian-splats/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "clock_ramp_s": args.ramp_seconds,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (frustum-uniform Gaussians, SURVEY.md 8d; seed 0)",
            "config": {"workload": args.config, "gaussians": P, "width": W, "height": H, "sh_degree": Kdeg,
                       "num_rendered": nr, "views": "one per GPU, yaw 5 deg x rank", "parallelism": par,
                       "sh_layout": "dc + rest (separate_sh)" if args.separate_sh else "one [P,M,3] tensor"},
            "roofline": {"kernel": dom, "bound": "hbm",
                         "achieved": own_traffic / (dom_ms * 1e-3) / 1e9 if counter_headline else achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": own_frac if counter_headline else achieved / HBM_PEAK_GBS,
                         "frac_basis": ("PMC counter bytes per launch less the fused zero fill (the 8d model "
                                        "overstates this frame)" if counter_headline
                                        else "SURVEY.md 8d algorithmic bytes per launch"),
                         "model_frac": achieved / HBM_PEAK_GBS, "model_GBs": achieved,
                         "traffic": traffic, "traffic_source": traffic_src, "traffic_counters": traffic_detail,
                         # counter bytes per launch over the launch time: the HBM rate the kernel really moves
                         "traffic_frac": traffic_frac,
                         "traffic_frac_less_fill": own_frac,
                         "algorithmic_bytes_per_launch": alg,
                         # the zero fill riding in the launch: its bytes and their rate over the launch time,
                         # excluded from frac (SURVEY.md 8d "zero-init memsets")
                         "fused_zero_fill_bytes": fill_bytes,
                         "fused_zero_fill_GBs": fill_bytes / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0,
                         "mean_launch_ms": dom_ms, "timed_launches": int(dom_calls), "timed_every": every,
                         # what actually limits the render kernels: "hbm" above is the
                         # contract's roofline axis, not the limiter
                         "limiter": ("VALU issue + latency (per (pixel, splat) pair work)"
                                     if dom.startswith("render") else "hbm"),
                         "valu_issue_frac": valu_frac},
            "work": work,
            "stage_ms": {k: round(v, 4) for k, v in per_stage.items()},  # untimed breakdown pass
            "host": host,
            "step_algorithmic_GBs": step_algorithmic_bytes(P, nr, W, H, K) / (ms_per_step * 1e-3) / 1e9,
        }
        if multi is not None:
            line["multi_gpu"] = multi
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.config, P, W, H, gpu_num_rendered=nr)
            line["cpu_baseline_c"] = cpu_baseline_c(args.config, P, W, H, args.cpu_threads or cpu_threads()[0])
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    if grouped:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
