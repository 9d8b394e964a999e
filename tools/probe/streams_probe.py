#!/usr/bin/env python3
"""Probe: does splitting the C4 step's batch over S independent extractor /
matcher handles on S HIP streams overlap kernels usefully?  Prints ms/step
for S in 1, 2, 4 (same 512 frames, same work)."""
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT)]
import bench  # noqa: E402

orb = bench.load_package()
W, H, B, NF, M = 1241, 376, 512, 1000, 5000
imgs = np.stack([orb.synth_image(0x4B495454, f, W, H) for f in range(B)])
dev = torch.device("cuda:0")
d_img = torch.from_numpy(imgs).to(dev)
ext0 = orb.ORBextractor(NF, 1.2, 8, 20, 7)
cap = ext0.capacity(W, H)
scale = np.float32(ext0.GetScaleFactors())
d_kps = torch.zeros((B, cap, 7), dtype=torch.int32, device=dev)
d_desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
d_cnt = torch.zeros(B, dtype=torch.int32, device=dev)
ext0.extract_batch(d_img.data_ptr(), B, W, H, W, W * H, d_kps.data_ptr(), d_desc.data_ptr(), cap,
                   d_cnt.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
kh = d_kps.cpu().numpy().view(orb.KEYPOINT_DTYPE).reshape(B, cap)
dh = d_desc.cpu().numpy()
ch = d_cnt.cpu().numpy()
mps_all = np.zeros((B, M), orb.MP_TRACK_DTYPE)
mpd_all = np.zeros((B, M, 32), np.uint8)
lock_all = np.zeros((B, cap), np.uint8)
for i in range(B):
    n = int(ch[i])
    a, b, c = orb.synth_local_map(0x4B495454 + i, kh[i, :n], dh[i, :n], M, W, H)
    mps_all[i], mpd_all[i], lock_all[i, :n] = a, b, c
d_mps = torch.from_numpy(mps_all.view(np.uint8).reshape(B, -1)).to(dev)
d_mpd = torch.from_numpy(mpd_all).to(dev)
d_lock = torch.from_numpy(lock_all).to(dev)
d_nmps = torch.full((B,), M, dtype=torch.int32, device=dev)
d_match = torch.zeros((B, cap), dtype=torch.int32, device=dev)
d_nm = torch.zeros(B, dtype=torch.int32, device=dev)
ref_match = None

for S in (1, 2, 4):
    exts = [orb.ORBextractor(NF, 1.2, 8, 20, 7) for _ in range(S)]
    mts = [orb.ORBmatcher(0.8) for _ in range(S)]
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    b = B // S
    main = torch.cuda.current_stream()

    def step():
        ev = torch.cuda.Event()
        ev.record(main)
        for s in range(S):
            st = streams[s]
            st.wait_event(ev)
            o = s * b
            sp = st.cuda_stream
            exts[s].extract_batch(d_img.data_ptr() + o * W * H, b, W, H, W, W * H,
                                  d_kps[o].data_ptr(), d_desc[o].data_ptr(), cap,
                                  d_cnt[o:].data_ptr(), sp)
            mts[s].search_by_projection_batch(b, d_kps[o].data_ptr(), d_desc[o].data_ptr(),
                                              d_cnt[o:].data_ptr(), d_lock[o].data_ptr(), cap,
                                              d_mps[o].data_ptr(), d_mpd[o].data_ptr(),
                                              d_nmps[o:].data_ptr(), M, W, H, scale, 1.0,
                                              d_match[o].data_ptr(), d_nm[o:].data_ptr(), sp)
        for s in range(S):
            e2 = torch.cuda.Event()
            e2.record(streams[s])
            main.wait_event(e2)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 20 * 1e3
    m = d_match.cpu().numpy()
    same = ref_match is None or np.array_equal(m, ref_match)
    ref_match = m if ref_match is None else ref_match
    print(f"streams {S}: {ms:.3f} ms/step  {B / ms * 1e3:.0f} frames/s  same={same}", flush=True)
