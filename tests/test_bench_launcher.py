"""CPU: bench.py's multi-GPU launcher and rank checks (no GPU needed, nothing is computed).

`python bench.py --gpus N` (N > 1) must run N ranks, not one process on GPU 0: without an outer
torch.distributed.run it starts them as ONE child process (never an exec) before anything touches
the GPU, and every rank refuses to run unless the process group is exactly the N ranks asked for,
each with a GPU of its own under RCCL.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_rank_launch_cmd():
    cmd = bench.rank_launch_cmd(["--gpus", "8", "--steps", "20", "--warmup", "5"], 8, 29500)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert "--master-port=29500" in cmd
    i = cmd.index(os.path.abspath(bench.__file__))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "20", "--warmup", "5"]


def test_launch_ranks_runs_one_child(monkeypatch):
    seen = []

    def fake_call(cmd, env):
        seen.append((cmd, env))
        return 3

    assert bench.launch_ranks(["--gpus", "2"], 2, call=fake_call) == 3      # the child's exit code
    (cmd, env), = seen
    assert "--nproc-per-node=2" in cmd and cmd[-2:] == ["--gpus", "2"]
    assert env.get("HSA_ENABLE_IPC_MODE_LEGACY") == "0"


def test_main_launches_without_world(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    calls = []
    monkeypatch.setattr(bench, "launch_ranks", lambda argv, n: calls.append((list(argv), n)) or 0)
    assert bench.main(["--gpus", "4", "--steps", "3"]) == 0
    assert calls == [(["--gpus", "4", "--steps", "3"], 4)]


def test_main_single_gpu_does_not_launch(monkeypatch):
    """--gpus 1 is the plain single-process run (it goes on to need a GPU, so stop it at the
    first torch call)."""
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "launch_ranks", lambda *a: pytest.fail("launched ranks for --gpus 1"))
    monkeypatch.setattr(bench, "world_error", lambda *a: "stop here")
    assert bench.main(["--gpus", "1"]) == 2


@pytest.mark.parametrize("gpus,world,backend,local,ndev,ok", [
    (1, 1, "nccl", 1, 1, True),
    (8, 8, "nccl", 8, 8, True),
    (2, 1, "nccl", 1, 1, False),       # the driver asked for 2, the group has 1
    (2, 4, "nccl", 4, 8, False),
    (2, 2, "nccl", 2, 1, False),       # RCCL: one GPU per local rank
    (2, 2, "gloo", 2, 1, True),        # the gloo rehearsal shares the GPU on purpose
    (1, 1, "nccl", 1, 0, True),        # single rank: the engine reports a missing GPU itself
])
def test_world_error(gpus, world, backend, local, ndev, ok):
    assert (bench.world_error(gpus, world, backend, local, ndev) is None) == ok


def test_rank_refuses_mismatched_world(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("LOCAL_RANK", "0")
    assert bench.main(["--gpus", "4"]) == 2


def test_launched_ranks_fail_fast_without_gpus():
    """End to end on this GPU-less container: `bench.py --gpus 2` starts two RCCL ranks through
    torch.distributed.run; both see no GPU, refuse, and the launcher exits non-zero quickly."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("EDC_DIST_BACKEND", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode != 0
    assert "GPU(s) visible" in r.stderr
    assert r.stdout.strip() == ""        # no JSON line from a refused run


def test_default_inflight_by_shard_size():
    """batches in flight per GPU by signatures per GPU: the N = 1 headline (2^20) and the 2-, 4-
    and 8-rank strong shards (2^19, 2^18, 2^17; small shards keep 16, beside RCCL too)"""
    assert bench.default_inflight(1 << 21, 12) == 6
    assert bench.default_inflight(1 << 20, 16) == 6
    assert bench.default_inflight(1 << 19, 12) == 7
    assert bench.default_inflight((1 << 19) + 5, 16) == 7
    assert bench.default_inflight(1 << 18, 12) == 12
    assert bench.default_inflight(1 << 17, 16) == 16
