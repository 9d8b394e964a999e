#!/usr/bin/env python3
"""Probe: C5 (bench.proj_workload) rate by call order and timed-step count in one process."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[3]))
import torch  # noqa: E402

import bench  # noqa: E402

orb = bench.load_package()
dev = torch.device("cuda:0")
for steps, warm in ((20, 3), (20, 3), (200, 10), (200, 10), (20, 3)):
    r, _ = bench.proj_workload(orb, torch, dev, 16, 1920, 1080, 4000, 50000, 16, bench.C5_SEED,
                               steps=steps, warmup=warm)
    print(f"C5 steps {steps} warmup {warm}: {r['value']:.0f} problems/s, match alone "
          f"{r['match_only_problems_per_s']:.0f}", flush=True)
