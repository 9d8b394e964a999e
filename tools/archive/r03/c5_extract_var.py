#!/usr/bin/env python3
"""Probe: C5's extraction (16 frames of 1920x1080, 4000 features) alone, one
fresh handle + fresh input copy per trial; wall time per call and per-stage
HIP-event times, with the buffer addresses, to find which stage varies."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[3]))
import torch  # noqa: E402

import bench  # noqa: E402

orb = bench.load_package()
dev = torch.device("cuda:0")
W, H, B, NF = 1920, 1080, 16, 4000
host = bench.synth_images(orb, bench.C5_SEED, list(range(B)), W, H, 16)
keep = []
for trial in range(8):
    ext = orb.ORBextractor(NF, 1.2, 8, 20, 7, device=0)
    cap = ext.capacity(W, H)
    d = torch.from_numpy(host).to(dev)
    k = torch.zeros((B, cap, 7), dtype=torch.int32, device=dev)
    de = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
    n = torch.zeros(B, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(dev)

    def call():
        ext.extract_batch(d.data_ptr(), B, W, H, W, W * H, k.data_ptr(), de.data_ptr(), cap,
                          n.data_ptr(), s.cuda_stream)

    for _ in range(10):
        call()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(200):
        call()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) / 200 * 1e3
    ext.profile(True)
    for _ in range(100):
        call()
    torch.cuda.synchronize()
    st = []
    for i in range(7):
        name, ms, cnt = ext.profile_read(i)
        if cnt:
            st.append(f"{name} {ms / 100:.3f}")
    ext.profile(False)
    print(f"trial {trial}: wall {wall:.3f} ms/call; d % 2MiB = {d.data_ptr() % (2 << 20)}; "
          + "; ".join(st), flush=True)
    if trial % 2:
        keep.append((ext, d, k, de, n))  # keep every other trial's buffers alive
