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
