#!/usr/bin/env python3
"""Extraction stages timed alone (profile mode 2: every stage after the
previous one on one stream, FAST as one launch over all levels) over B frames
of the C4 stream; prints ms per call of each stage.  Run once per library
variant (ORB_AMD_LIB) by tools/r04/fast_attr.sh."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

B = int(os.environ.get("ATTR_BATCH", "1024"))
CALLS = int(os.environ.get("ATTR_CALLS", "10"))
orb = bench.load_package()
W, H = 1241, 376
imgs = bench.synth_images(orb, 0x4B495454, list(range(B)), W, H, 16)
ext = orb.ORBextractor(1000, 1.2, 8, 20, 7, device=0)
cap = ext.capacity(W, H)
d = torch.from_numpy(imgs).cuda()
k = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
de = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
n = torch.zeros(B, dtype=torch.int32, device="cuda")
s = torch.cuda.Stream()


def call():
    ext.extract_batch(d.data_ptr(), B, W, H, W, W * H, k.data_ptr(), de.data_ptr(), cap, n.data_ptr(),
                      s.cuda_stream)


ext.profile(2)
for _ in range(3):
    call()
torch.cuda.synchronize()
ext.profile(2)
for _ in range(CALLS):
    call()
torch.cuda.synchronize()
parts = {}
for st in range(7):
    name, ms, cnt = ext.profile_read(st)
    if cnt:
        parts[name] = ms / CALLS
ext.profile(False)
lib = os.environ.get("ORB_AMD_LIB", "default")
print(f"{Path(lib).stem} B={B}: " + "; ".join(f"{a} {b:.4f}" for a, b in parts.items()), flush=True)
