"""bench.py --gpus N: the rank launch.

`python bench.py --gpus N` started by hand (no WORLD_SIZE) must start N ranks itself
through torch.distributed.run; under the driver's own torch.distributed.run each rank
checks that WORLD_SIZE equals --gpus.  The CPU tests cover the launch plan, the mismatch
guard, and a real two-rank rendezvous over gloo (--launch-check: no GPU work); the GPU
test runs the full bench with two ranks sharing the box's GPU.
"""
import json
import os
import subprocess
import sys

import pytest

from snapcheck import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402

BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def test_launch_plan_single_gpu_runs_in_process():
    args = bench.parse_args(["--gpus", "1"])
    assert bench.launch_plan(args, {}, ["--gpus", "1"]) is None


def test_launch_plan_spawns_torchrun_with_same_args():
    argv = ["--gpus", "4", "--config", "c2", "--steps", "3"]
    args = bench.parse_args(argv)
    cmd = bench.launch_plan(args, {}, argv)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-len(argv) - 1:] == [os.path.abspath(BENCH)] + argv


def test_launch_plan_rank_of_matching_world():
    args = bench.parse_args(["--gpus", "8"])
    assert bench.launch_plan(args, {"WORLD_SIZE": "8"}, []) is None


@pytest.mark.parametrize("gpus,world", [(2, "1"), (1, "2"), (8, "4")])
def test_launch_plan_world_mismatch_is_an_error(gpus, world):
    args = bench.parse_args(["--gpus", str(gpus)])
    with pytest.raises(SystemExit) as e:
        bench.launch_plan(args, {"WORLD_SIZE": world}, [])
    assert e.value.code not in (0, None)


def test_mismatch_exits_nonzero_before_any_work():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], env=_env(WORLD_SIZE="1", RANK="0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr and r.stdout == ""


def test_two_rank_launch_by_hand():
    """`bench.py --gpus 2` with no WORLD_SIZE: two ranks rendezvous, rank 0 prints one line."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["rank_sum"] == 1 and d["gpus_arg"] == 2


@pytest.mark.gpu
def test_two_rank_bench_by_hand_shared_device():
    """The whole bench with two ranks on the box's one GPU (gloo collective): the line is the
    2-GPU line of the 2^20 batch, and its parity holds against the oracle fixture."""
    r = subprocess.run([sys.executable, "-u", BENCH, "--gpus", "2", "--shared-device", "--dist-backend", "gloo",
                        "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-collect", "--no-fresh"],
                       env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    assert d["config"]["instances_per_gpu"] == 524288 and d["config"]["instances_total"] == 1 << 20
    assert d["parity"] is True
    assert d["value"] > 0
