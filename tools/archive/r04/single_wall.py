#!/usr/bin/env python3
"""Wall time of one ORBextractor::operator() call through the host API
(pinned H2D, the hipGraph replay, D2H), 1241x376, 1000 features: median of 500
calls after 20 warm-up, frames 0..15 of the bench stream in turn."""
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import numpy as np  # noqa: E402

import bench  # noqa: E402

orb = bench.load_package()
imgs = bench.synth_images(orb, 0x4B495454, list(range(16)), 1241, 376, 16)
ext = orb.ORBextractor(1000, 1.2, 8, 20, 7)
for i in range(20):
    ext(imgs[i % 16])
ts = []
for i in range(500):
    t0 = time.perf_counter()
    ext(imgs[i % 16])
    ts.append(time.perf_counter() - t0)
knobs = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("ORB_"))
print(f"[{knobs}] single-frame extract wall: median {np.median(ts) * 1e3:.4f} ms, "
      f"p10 {np.percentile(ts, 10) * 1e3:.4f}, p90 {np.percentile(ts, 90) * 1e3:.4f}", flush=True)
