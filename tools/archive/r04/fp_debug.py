#!/usr/bin/env python3
"""Per-window rounds and s_memtime clock deltas of k_proj_resolve_fp for problem 0
of the C5 workload (B = 16), from the FP_DEBUG variant build
(ORB_AMD_LIB=.../variants/fpdbg.so)."""
import ctypes
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

orb = bench.load_package()
dev = torch.device("cuda:0")
W, H, NF, M, B = 1920, 1080, 4000, 50000, 16
r, st = bench.proj_workload(orb, torch, dev, 16, W, H, NF, M, B, bench.C5_SEED, steps=5, warmup=2)
torch.cuda.synchronize()
lib = ctypes.CDLL(os.environ["ORB_AMD_LIB"])
buf = (ctypes.c_ulonglong * 514)()
assert lib.orb_k_fp_debug(buf, 514) == 0
a = np.array(buf[:], dtype=np.uint64).astype(np.int64)
nw = int(a[0])
rounds = a[2:2 + 2 * nw:2]
t = np.concatenate([[a[1]], a[3:3 + 2 * nw:2]])
dt = np.diff(t)
dr = np.diff(np.concatenate([[0], rounds]))
print(f"windows {nw}; rounds per window mean {dr.mean():.2f} max {dr.max()}; "
      f"memtime ticks per window mean {dt.mean():.0f} (min {dt.min()}, max {dt.max()}); "
      f"ticks per round {dt.sum() / dr.sum():.0f}; total {t[-1] - t[0]}")
print("rounds:", dr.tolist())
print("ticks:", dt.tolist())
