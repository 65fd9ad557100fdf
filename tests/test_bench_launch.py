"""bench.py's multi-GPU launcher: ``--gpus N`` starts N ranks as a child
``torch.distributed.run``, and a rank whose WORLD_SIZE differs from --gpus exits non-zero.
CPU only: the launch itself is captured, and the mismatch exits before any HIP call."""
from __future__ import annotations

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_launch_command_shape():
    cmd = bench.launch_command(8, ["--gpus", "8", "--steps", "5"], 29517)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29517" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "5"]


def test_maybe_launch_spawns_child_and_relays_rc(monkeypatch):
    seen = {}

    class R:
        returncode = 7

    def fake_run(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return R()

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    args = bench.parse_args(["--gpus", "4", "--steps", "3"])
    assert bench.maybe_launch(args, ["--gpus", "4", "--steps", "3"]) == 7
    assert "--nproc-per-node=4" in seen["cmd"]
    assert seen["cmd"][-4:] == ["--gpus", "4", "--steps", "3"]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_maybe_launch_single_and_inside_rank(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.maybe_launch(bench.parse_args([]), []) is None
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.maybe_launch(bench.parse_args(["--gpus", "2"]), []) is None
    assert bench.maybe_launch(bench.parse_args(["--gpus", "1"]), []) == 2
    assert bench.maybe_launch(bench.parse_args(["--gpus", "8"]), []) == 2


@pytest.mark.parametrize("gpus,world", [("1", "2"), ("8", "4")])
def test_world_size_mismatch_exits_nonzero(gpus, world):
    env = dict(os.environ, WORLD_SIZE=world, RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", gpus, "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, r.stderr
    assert f"WORLD_SIZE={world} but --gpus {gpus}" in r.stderr
    assert r.stdout.strip() == ""  # no bench line from a wrong-sized job


def test_cpu_threads_affinity(monkeypatch):
    aff = len(os.sched_getaffinity(0))
    monkeypatch.delenv("OMP_NUM_THREADS", raising=False)
    n, facts = bench.cpu_threads()
    assert n == aff and facts["affinity_cpus"] == aff and facts["omp_num_threads"] is None
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    n, facts = bench.cpu_threads()
    assert n == 1 and facts["omp_num_threads"] == 1
