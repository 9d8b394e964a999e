#!/usr/bin/env python3
"""Probe: SearchByProjection(F, localMap) stage times at C5 (1920x1080, 4000 feat,
50,000 map points), B problems per call, each stage alone (matcher profile
events on one stream).  Usage: c5_stages.py [B ...]"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

orb = bench.load_package()
dev = torch.device("cuda:0")
W, H, NF, M = 1920, 1080, 4000, 50000
for B in [int(a) for a in sys.argv[1:]] or [16, 128]:
    r, st = bench.proj_workload(orb, torch, dev, 16, W, H, NF, M, B, bench.C5_SEED, steps=20,
                                warmup=3)
    s0 = st["set0"]
    cap = s0["k"].shape[1]
    d_mps = torch.from_numpy(st["mps"].view(np.uint8).reshape(B, -1)).to(dev)
    d_mpd = torch.from_numpy(st["mpd"]).to(dev)
    d_lk = torch.from_numpy(st["lk"]).to(dev)
    d_nm = torch.full((B,), M, dtype=torch.int32, device=dev)
    km = torch.zeros((B, cap), dtype=torch.int32, device=dev)
    nm = torch.zeros(B, dtype=torch.int32, device=dev)
    mt = orb.ORBmatcher(0.8, device=0)
    s = torch.cuda.Stream(dev)

    def call():
        mt.search_by_projection_batch(B, s0["k"].data_ptr(), s0["de"].data_ptr(), s0["n"].data_ptr(),
                                      d_lk.data_ptr(), cap, d_mps.data_ptr(), d_mpd.data_ptr(),
                                      d_nm.data_ptr(), M, W, H, st["scale"], 1.0, km.data_ptr(),
                                      nm.data_ptr(), s.cuda_stream)

    for _ in range(5):
        call()
    torch.cuda.synchronize()
    mt.profile(True)
    n = 50
    for _ in range(n):
        call()
    torch.cuda.synchronize()
    parts = []
    for stg in range(4):
        name, ms, cnt = mt.profile_read(stg)
        parts.append(f"{name} {ms / n:.4f}")
    mt.profile(False)
    import os
    knobs = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith(("ORB_PROJ", "ORB_RESOLVE", "ORB_JACOBI")))
    print(f"[{knobs}] C5 B={B}: pipelined {r['value']:.0f} problems/s, match alone "
          f"{r['match_only_problems_per_s']:.0f}; stages ms/call: " + "; ".join(parts), flush=True)
