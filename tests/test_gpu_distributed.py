"""The sharded bench path with two ranks on the GPU box: each
rank extracts and matches its own block of the synthetic sequence and the
per-frame keypoint counts are all-gathered once per step.  The box has one GPU,
so both ranks are pinned to it (ORB_BENCH_DEVICE) and the collective runs on
gloo (RCCL does not take two ranks on one device); the 8-GPU RCCL run is the
driver's scaling bench."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_ranks_shard_and_gather(gpu):
    env = dict(os.environ, ORB_BENCH_DEVICE="0", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
           "--dist-backend", "gloo", "--frames", "512", "--steps", "2", "--warmup", "1",
           "--no-cpu", "--no-secondary", "--no-dropin", "--threads", "4"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 2 and res["scaling"] == "weak"
    assert res["config"]["frames_per_gpu_per_step"] == 512
    assert res["config"]["count_gather_verified"] is True
    # whole-job value = frames of both ranks / the slowest rank's time
    assert abs(res["value"] - 2 * 512 * res["steps"] / (res["ms_per_step"] * 1e-3 * res["steps"])) \
        < 1e-6 * res["value"]


def test_bench_gpus_flag_launches_ranks(gpu):
    """`bench.py --gpus 2` from a plain shell (no WORLD_SIZE) starts two ranks
    itself (a torch.distributed.run child) and the job line reports both."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
                        "TORCHELASTIC_RUN_ID")}
    env.update(ORB_BENCH_DEVICE="0", OMP_NUM_THREADS="4")
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--frames", "512", "--steps", "2", "--warmup", "1", "--no-cpu", "--no-secondary", "--no-dropin",
           "--threads", "4", "--host-frames", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert res["n_gpus"] == 2
    assert res["config"]["count_gather_verified"] is True


def test_rccl_gather_single_rank_torchrun(gpu):
    """The RCCL path itself: bench.py under torchrun with one rank initialises
    the nccl (= RCCL) process group, all-gathers each step's per-frame counts
    with all_gather_into_tensor on the matcher stream and verifies them against
    the untimed pass; the host-input leg runs through the same pipeline."""
    env = dict(os.environ, OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
           "--frames", "1024", "--steps", "2", "--warmup", "1", "--no-cpu", "--no-secondary", "--no-dropin",
           "--threads", "4", "--host-frames", "1024", "--host-passes", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert res["n_gpus"] == 1
    assert "RCCL" in res["config"]["parallelism"]
    assert res["config"]["count_gather_verified"] is True
    h = res["host_input"]
    assert h["frames"] == 1024 and h["frames_per_s"] > 0 and h["h2d_GBps"] > 0
