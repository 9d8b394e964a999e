#!/usr/bin/env python3
"""Probe: which stage slows down in C5's slow placement mode (tools/probe/c5_addr.py)?
Stage profiler on for the extractor and the matcher inside proj_workload."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[3]))
import torch  # noqa: E402

import bench  # noqa: E402

orb = bench.load_package()
dev = torch.device("cuda:0")
made = []


def capture(cls):
    class C(cls):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            self.profile(True)
            made.append(self)
    return C


orb.ORBextractor = capture(orb.ORBextractor)
orb.ORBmatcher = capture(orb.ORBmatcher)
for pad in (0, 0, 8, 0):
    p = torch.empty(pad << 20, dtype=torch.uint8, device=dev) if pad else None
    made.clear()
    r, st = bench.proj_workload(orb, torch, dev, 16, 1920, 1080, 4000, 50000, 16, bench.C5_SEED,
                                steps=200, warmup=10)
    ext, mt = made[0], made[1]
    parts = []
    for h, n in ((ext, 7), (mt, 3)):
        for i in range(n):
            name, ms, cnt = h.profile_read(i)
            if cnt:
                parts.append(f"{name} {ms / cnt:.3f}x{cnt}")
    print(f"pad {pad}: {r['value']:.0f} problems/s; set0 k {st['set0']['k'].data_ptr():#x} "
          f"de {st['set0']['de'].data_ptr():#x}; " + "; ".join(parts), flush=True)
    del p, st
