#!/usr/bin/env python3
"""Probe (needs a stamp build of extractor_kernels.hip): per-phase cycle
counts of k_fast_band workgroups of image 0 (s_memtime by thread 0)."""
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT)]
import bench  # noqa: E402

orb = bench.load_package()
W, H, B = 1241, 376, 512
imgs = np.stack([orb.synth_image(0x4B495454, f, W, H) for f in range(B)])
d_img = torch.from_numpy(imgs).cuda()
ext = orb.ORBextractor(1000, 1.2, 8, 20, 7)
cap = ext.capacity(W, H)
kps = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for _ in range(3):
    ext.extract_batch(d_img.data_ptr(), B, W, H, W, W * H, kps.data_ptr(), desc.data_ptr(), cap,
                      cnt.data_ptr(), s)
torch.cuda.synchronize()
st = np.zeros((4096, 8), np.uint64)
L = orb.lib()
L.orb_k_fast_stamps.argtypes = [ctypes.c_void_p]
assert L.orb_k_fast_stamps(st.ctypes.data) == 0
nb = int((st[:, 0] > 0).sum())
st = st[:nb].astype(np.int64)
done_a = st[:, 6] > 0  # returned after phase A
end = np.where(done_a, st[:, 6], st[:, 7])
names = ["staging", "init", "fastA", "nmsA", "compactA"]
for i, n in enumerate(names):
    d = st[:, i + 1] - st[:, i]
    print(f"{n:9s} mean {d.mean():8.0f} median {np.median(d):8.0f}")
pb = ~done_a
print(f"bands {nb}, phase B in {pb.sum()}")
if pb.any():
    d = (st[pb, 7] - st[pb, 5])
    print(f"phaseB    mean {d.mean():8.0f} (bands with fallback)")
tot = end - st[:, 0]
print(f"total     mean {tot.mean():8.0f} median {np.median(tot):8.0f}  (s_memtime ticks)")
