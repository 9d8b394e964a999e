#!/usr/bin/env python3
"""Extraction stages alone (no matcher stream): per-stage HIP-event times of
extract_batch over B-frame batches of the C4 stream, and the whole call.
Usage (GPU box): python tools/probe/stage_times.py [--batch 512] [--calls 20]"""
import argparse
import importlib
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
orb = importlib.import_module("orb_slam2-chinese-annotation_amd")

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=512)
ap.add_argument("--calls", type=int, default=20)
ap.add_argument("--width", type=int, default=1241)
ap.add_argument("--height", type=int, default=376)
ap.add_argument("--features", type=int, default=1000)
a = ap.parse_args()
W, H, B = a.width, a.height, a.batch
imgs = np.stack([orb.synth_image(7, f, W, H) for f in range(16)])
imgs = np.concatenate([imgs] * ((B + 15) // 16))[:B]
ext = orb.ORBextractor(a.features, 1.2, 8, 20, 7)
cap = ext.capacity(W, H)
d_img = torch.from_numpy(imgs).cuda()
d_kps = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
d_desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
d_cnt = torch.zeros(B, dtype=torch.int32, device="cuda")


def call():
    ext.extract_batch(d_img.data_ptr(), B, W, H, W, W * H, d_kps.data_ptr(), d_desc.data_ptr(), cap,
                      d_cnt.data_ptr())


for _ in range(3):
    call()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(a.calls):
    call()
torch.cuda.synchronize()
wall = (time.perf_counter() - t) / a.calls * 1e3
ext.profile(True)
for _ in range(a.calls):
    call()
torch.cuda.synchronize()
parts = []
for st in range(7):
    name, ms, n = ext.profile_read(st)
    if n:
        parts.append(f"{name} {ms / a.calls:.3f}")
ext.profile(False)
print(f"B={B}: wall {wall:.3f} ms/call ({B / wall * 1e3:.0f} frames/s); " + "; ".join(parts), flush=True)
