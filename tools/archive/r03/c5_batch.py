#!/usr/bin/env python3
"""Probe: C5 rate (bench.proj_workload) vs problems per launch."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[3]))
import torch  # noqa: E402

import bench  # noqa: E402

orb = bench.load_package()
dev = torch.device("cuda:0")
for B in (16, 32, 64, 128):
    steps = max(50, 3200 // B)
    r, _ = bench.proj_workload(orb, torch, dev, 16, 1920, 1080, 4000, 50000, B, bench.C5_SEED,
                               steps=steps, warmup=5)
    print(f"B={B}: {r['value']:.0f} problems/s ({r['ms_per_step']:.3f} ms/step), match alone "
          f"{r['match_only_problems_per_s']:.0f} ({r['match_only_frac_of_8TBps']:.3f} of 8 TB/s)",
          flush=True)
