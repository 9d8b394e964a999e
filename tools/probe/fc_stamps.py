#!/usr/bin/env python3
"""Per-phase clock counts of k_fast_cells (needs the FC_STAMPS build:
tools/attribution/build.sh fcst -DFC_STAMPS, run with ORB_AMD_LIB=.../fcst.so).
Image 0's cells of the last B-frame batch call, s_memtime by lane 0 of each
cell's wave: stage (staging, strength clear, next loads issued, setup), fastA
(pretest, queue, scoring at iniThFAST), nmsA (NMS and key emit), phaseB
(minThFAST rescan, cells with no corner at iniThFAST), and the gap to the
wave's next cell."""
import ctypes
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "tests"))
from conftest import load_pkg  # noqa: E402


def main():
    import torch
    orb = load_pkg()
    W, H, B = 1241, 376, int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    imgs = np.stack([orb.synth_image(0x4B495454, f, W, H) for f in range(min(B, 64))])
    imgs = np.concatenate([imgs] * ((B + 63) // 64))[:B]
    ext = orb.ORBextractor(1000, 1.2, 8, 20, 7)
    cap = ext.capacity(W, H)
    d = torch.from_numpy(imgs).cuda()
    k = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
    de = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(B, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    for _ in range(3):
        ext.extract_batch(d.data_ptr(), B, W, H, W, W * H, k.data_ptr(), de.data_ptr(), cap,
                          n.data_ptr(), s.cuda_stream)
    s.synchronize()
    st = np.zeros((8192, 8), np.uint64)
    L = orb.lib()
    L.orb_k_fc_stamps.argtypes = [ctypes.c_void_p]
    assert L.orb_k_fc_stamps(st.ctypes.data) == 0
    st = st.astype(np.int64)
    ok = (st[:, 0] > 0) & (st[:, 1] >= st[:, 0]) & (st[:, 2] >= st[:, 1]) & (st[:, 3] >= st[:, 2]) & \
         (st[:, 4] >= st[:, 3])
    c = st[ok]
    tot = c[:, 4] - c[:, 0]
    print(f"cells stamped: {ok.sum()}  (B = {B})")
    names = ["stage", "fastA", "nmsA", "phaseB"]
    for i, nm in enumerate(names):
        dd = c[:, i + 1] - c[:, i]
        print(f"{nm:7s} mean {dd.mean():9.0f} median {np.median(dd):9.0f}  share {dd.sum() / tot.sum():.3f}")
    jc = c[:, 5]
    for j in range(int(jc.max()) + 1):
        m = jc == j
        if m.any():
            print(f"  cell {j} of its wave: n {m.sum():5d} stage {np.mean(c[m, 1] - c[m, 0]):8.0f} "
                  f"fastA {np.mean(c[m, 2] - c[m, 1]):8.0f} total {np.mean(c[m, 4] - c[m, 0]):8.0f}")
    pb = (c[:, 4] - c[:, 3]) > 2 * np.median(c[:, 4] - c[:, 3]) + 200
    print(f"cells running phase B (by time): {pb.mean():.3f}")
    print(f"cell total mean {tot.mean():.0f} median {np.median(tot):.0f} clocks")


if __name__ == "__main__":
    main()
