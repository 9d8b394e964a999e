#!/usr/bin/env python3
"""Probe: overlap step k's SearchByProjection (matcher stream) with step k+1's
extraction (extract stream), two buffer sets.  Prints ms/step serial vs
pipelined (same 512 frames per step, same work)."""
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
ext = orb.ORBextractor(NF, 1.2, 8, 20, 7)
cap = ext.capacity(W, H)
scale = np.float32(ext.GetScaleFactors())
sets = []
for _ in range(2):
    sets.append(dict(kps=torch.zeros((B, cap, 7), dtype=torch.int32, device=dev),
                     desc=torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev),
                     cnt=torch.zeros(B, dtype=torch.int32, device=dev),
                     match=torch.zeros((B, cap), dtype=torch.int32, device=dev),
                     nm=torch.zeros(B, dtype=torch.int32, device=dev)))
s0 = sets[0]
ext.extract_batch(d_img.data_ptr(), B, W, H, W, W * H, s0["kps"].data_ptr(), s0["desc"].data_ptr(),
                  cap, s0["cnt"].data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
kh = s0["kps"].cpu().numpy().view(orb.KEYPOINT_DTYPE).reshape(B, cap)
dh = s0["desc"].cpu().numpy()
ch = s0["cnt"].cpu().numpy()
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
mt = orb.ORBmatcher(0.8)
se = torch.cuda.Stream(dev)
sm = torch.cuda.Stream(dev)


def run(k, pipelined):
    st = sets[k % 2] if pipelined else sets[0]
    es = se if pipelined else torch.cuda.current_stream()
    ms = sm if pipelined else torch.cuda.current_stream()
    if pipelined and k >= 2:  # buffer set reuse: wait for its previous matcher
        es.wait_event(done[k % 2])
    ext.extract_batch(d_img.data_ptr(), B, W, H, W, W * H, st["kps"].data_ptr(),
                      st["desc"].data_ptr(), cap, st["cnt"].data_ptr(), es.cuda_stream)
    if pipelined:
        ev = torch.cuda.Event()
        ev.record(es)
        ms.wait_event(ev)
    mt.search_by_projection_batch(B, st["kps"].data_ptr(), st["desc"].data_ptr(),
                                  st["cnt"].data_ptr(), d_lock.data_ptr(), cap, d_mps.data_ptr(),
                                  d_mpd.data_ptr(), d_nmps.data_ptr(), M, W, H, scale, 1.0,
                                  st["match"].data_ptr(), st["nm"].data_ptr(), ms.cuda_stream)
    if pipelined:
        done[k % 2].record(ms)


done = [torch.cuda.Event(), torch.cuda.Event()]
for pipelined in (False, True, False, True):
    for k in range(3):
        run(k, pipelined)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(20):
        run(k, pipelined)
    torch.cuda.synchronize()
    ms_ = (time.perf_counter() - t0) / 20 * 1e3
    same = all(np.array_equal(sets[0]["match"].cpu().numpy(), s["match"].cpu().numpy()) for s in sets)
    print(f"pipelined={pipelined}: {ms_:.3f} ms/step {B / ms_ * 1e3:.0f} frames/s same={same}",
          flush=True)
