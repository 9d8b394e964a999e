#!/usr/bin/env python3
"""Probe: does the number of live streams in the process (other extractor /
matcher handles, torch streams) change the C5 rate (bench.proj_workload)?"""
import gc
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[3]))
import torch  # noqa: E402

import bench  # noqa: E402

orb = bench.load_package()
dev = torch.device("cuda:0")


def c5(tag):
    r, _ = bench.proj_workload(orb, torch, dev, 16, 1920, 1080, 4000, 50000, 16, bench.C5_SEED,
                               steps=200, warmup=10)
    print(f"{tag}: {r['value']:.0f} problems/s, match alone {r['match_only_problems_per_s']:.0f}",
          flush=True)


c5("fresh process")
c5("again")
extra = [orb.ORBextractor(1000, 1.2, 8, 20, 7, device=0) for _ in range(3)]
extra += [orb.ORBmatcher(0.8, device=0) for _ in range(2)]
ts = [torch.cuda.Stream(dev) for _ in range(4)]
for s in ts:  # make sure each torch stream exists on the device
    with torch.cuda.stream(s):
        torch.zeros(1, device=dev).add_(1)
torch.cuda.synchronize()
c5("with 3 extractors + 2 matchers + 4 torch streams alive")
del extra
gc.collect()
c5("extractors / matchers freed (torch streams stay)")
c3, _ = bench.c3_workload(orb, torch, dev, 16, steps=40, warmup=5)
print(f"C3 {c3['value']:.0f}", flush=True)
gc.collect()
c5("after C3")
