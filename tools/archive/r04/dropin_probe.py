#!/usr/bin/env python3
"""bench.py's `dropin` leg alone: 16 frames of the bench stream extracted on the
GPU, their 5,000-point local maps, then the harness's per-frame timings."""
import json
import sys
from argparse import Namespace
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import numpy as np  # noqa: E402

import bench  # noqa: E402

orb = bench.load_package()
W, H, NF, M = 1241, 376, 1000, 5000
args = Namespace(width=W, height=H, features=NF, mappoints=M, seed=0x4B495454)
imgs = bench.synth_images(orb, args.seed, list(range(16)), W, H, 16)
ext = orb.ORBextractor(NF, 1.2, 8, 20, 7)
scale = np.float32(ext.GetScaleFactors())
maps = []
for i in range(16):
    k, d = ext(imgs[i])
    maps.append(orb.synth_local_map(args.seed + i, k, d, M, W, H))
print(json.dumps(bench.dropin_leg(orb, imgs, maps, scale, args, 16)), flush=True)
