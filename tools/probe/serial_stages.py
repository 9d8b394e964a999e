"""Extraction stages one after another on one stream (profile mode 2: no side
stream), B frames of the C4 stream per call, for a kernel trace:
  rocprofv3 --kernel-trace -- python3 tools/probe/serial_stages.py --batch 1024
then tools/trace_summary.py splits the launches by grid shape (one row per
pyramid level for k_pyr_resize)."""
import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "tests"))
from conftest import load_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--calls", type=int, default=10)
    a = ap.parse_args()
    import torch
    orb = load_pkg()
    W, H, B = 1241, 376, a.batch
    imgs = np.stack([orb.synth_image(0x4B495454, f, W, H) for f in range(min(B, 64))])
    imgs = np.concatenate([imgs] * ((B + 63) // 64))[:B]
    ext = orb.ORBextractor(1000, 1.2, 8, 20, 7)
    cap = ext.capacity(W, H)
    d = torch.from_numpy(imgs).cuda()
    k = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
    de = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(B, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    ext.profile(2)
    for _ in range(a.calls):
        ext.extract_batch(d.data_ptr(), B, W, H, W, W * H, k.data_ptr(), de.data_ptr(), cap,
                          n.data_ptr(), s.cuda_stream)
    s.synchronize()
    for st in range(7):
        name, ms, cnt = ext.profile_read(st)
        if cnt:
            print(f"{name}: {ms / a.calls:.4f} ms per call", flush=True)


if __name__ == "__main__":
    main()
