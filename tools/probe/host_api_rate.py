#!/usr/bin/env python3
"""Probe: frames/s of the host-buffer drop-in path (ORBextractor.__call__ ->
orb_extractor_extract: image H2D, extraction, keypoints + descriptors D2H,
one frame per call, as Frame::ExtractORB uses it) at 1241x376, 1000 features,
and of ORBmatcher.SearchByProjection on host buffers (5,000 map points).
PCIe-inclusive rates quoted in DESIGN.md §5; never the bench metric."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT)]
import bench  # noqa: E402

orb = bench.load_package()
W, H, N = 1241, 376, 300
imgs = [orb.synth_image(0x4B495454, f, W, H) for f in range(16)]
ext = orb.ORBextractor(1000, 1.2, 8, 20, 7, device=0)
for i in range(20):
    k, d = ext(imgs[i % 16])
t0 = time.perf_counter()
for i in range(N):
    k, d = ext(imgs[i % 16])
t1 = time.perf_counter()
print(f"extract (host buffers, 1 frame/call): {N / (t1 - t0):.0f} frames/s, "
      f"{1e3 * (t1 - t0) / N:.3f} ms/frame")
scale = np.float32(ext.GetScaleFactors())
mps, mpd, locked = orb.synth_local_map(1, k, d, 5000, W, H)
m = orb.ORBmatcher(0.8)
fr = orb.Frame(k, d, scale, W, H)
for _ in range(10):
    m.SearchByProjection(fr, mps, mpd, 1.0, locked)
t0 = time.perf_counter()
for _ in range(N):
    m.SearchByProjection(fr, mps, mpd, 1.0, locked)
t1 = time.perf_counter()
print(f"SearchByProjection (host buffers, 5000 MPs): {N / (t1 - t0):.0f} calls/s, "
      f"{1e3 * (t1 - t0) / N:.3f} ms/call")
# Frame::ComputeStereoMatches on host buffers (both 8-level pyramids uploaded per call)
el, er = orb.ORBextractor(2000, 1.2, 8, 20, 7), orb.ORBextractor(2000, 1.2, 8, 20, 7)
kl, dl = el(orb.synth_image(1, 0, W, H, 0))
kr, dr = er(orb.synth_image(1, 0, W, H, 1))
lp, rp = el.mvImagePyramid, er.mvImagePyramid
inv = el.GetInverseScaleFactors()
F2 = orb.Frame(kl, dl, np.float32(el.GetScaleFactors()), W, H)
for _ in range(5):
    m.ComputeStereoMatches(F2, kr, dr, lp, rp, inv, 386.1448, 718.856)
t0 = time.perf_counter()
for _ in range(100):
    m.ComputeStereoMatches(F2, kr, dr, lp, rp, inv, 386.1448, 718.856)
t1 = time.perf_counter()
print(f"ComputeStereoMatches (host buffers, 2000 + 2000 kps, pyramids uploaded): "
      f"{100 / (t1 - t0):.0f} pairs/s, {1e3 * (t1 - t0) / 100:.3f} ms/pair")
