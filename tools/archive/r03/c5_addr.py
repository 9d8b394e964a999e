#!/usr/bin/env python3
"""Probe: C5 rate vs allocation history -- a torch pad buffer of P MiB is held
across each proj_workload call (shifting where its buffers land), then freed."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[3]))
import torch  # noqa: E402

import bench  # noqa: E402

orb = bench.load_package()
dev = torch.device("cuda:0")
for pad in (0, 0, 2, 4, 6, 8, 32, 64, 0, 1024, 0):
    p = torch.empty(pad << 20, dtype=torch.uint8, device=dev) if pad else None
    r, _ = bench.proj_workload(orb, torch, dev, 16, 1920, 1080, 4000, 50000, 16, bench.C5_SEED,
                               steps=200, warmup=10)
    print(f"pad {pad} MiB: {r['value']:.0f} problems/s; torch reserved "
          f"{torch.cuda.memory_reserved(dev) >> 20} MiB", flush=True)
    del p
