"""bench.py's multi-GPU plumbing (frame sharding, keypoint-count all-gather,
max-over-ranks timing) on world_size 2 with the gloo backend on CPU."""
import os
import socket

import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B = 4
    frames = bench.shard_frames(rank, B)
    counts = torch.tensor([1000 + f for f in frames], dtype=torch.int32)
    out = torch.zeros(world * B, dtype=torch.int32)
    bench.gather_counts(dist, counts, out)
    t = bench.max_over_ranks(dist, 1.0 + rank, "cpu")
    q.put((rank, frames, out.tolist(), t))
    dist.destroy_process_group()


def test_bench_distributed_plumbing_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    all_frames = res[0][1] + res[1][1]
    assert sorted(all_frames) == list(range(8))  # disjoint, complete shards
    for _, _, gathered, t in res:
        assert gathered == [1000 + f for f in range(8)]
        assert t == 2.0  # slowest rank's time


def test_bench_gpus_flag_world_resolution():
    """`--gpus` against the launcher's env: a mismatch with WORLD_SIZE fails
    loudly; --gpus > 1 from a plain shell asks for child ranks."""
    import bench

    assert bench.resolve_world(None, {}) == (1, False)
    assert bench.resolve_world(1, {}) == (1, False)
    assert bench.resolve_world(8, {}) == (8, True)
    assert bench.resolve_world(None, {"WORLD_SIZE": "4"}) == (4, False)
    assert bench.resolve_world(4, {"WORLD_SIZE": "4"}) == (4, False)
    with pytest.raises(SystemExit):
        bench.resolve_world(8, {"WORLD_SIZE": "1"})
    with pytest.raises(SystemExit):
        bench.resolve_world(0, {})


def test_bench_gpus_mismatch_exits_nonzero():
    """A rank whose WORLD_SIZE differs from --gpus exits non-zero before it
    touches a device (it never measures one GPU under an N-GPU label)."""
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
