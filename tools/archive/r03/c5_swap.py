#!/usr/bin/env python3
"""Probe: which buffer's placement decides C5's slow / fast mode?  One C5
state; between timed runs, move one group of buffers to a new allocation
(a 6 MiB pad held in between shifts it) or recreate one handle."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[3]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

orb = bench.load_package()
dev = torch.device("cuda:0")
W, H, NF, M, B, seed = 1920, 1080, 4000, 50000, 16, bench.C5_SEED
S = {}
S["ext"] = orb.ORBextractor(NF, 1.2, 8, 20, 7, device=0)
scale = np.float32(S["ext"].GetScaleFactors())
cap = S["ext"].capacity(W, H)
host = bench.synth_images(orb, seed, list(range(B)), W, H, 16)
S["d"] = torch.from_numpy(host).to(dev)
z = lambda *sh, dt=torch.int32: torch.zeros(sh, dtype=dt, device=dev)
S["sets"] = [dict(k=z(B, cap, 7), de=z(B, cap, 32, dt=torch.uint8), n=z(B), km=z(B, cap), nm=z(B))
             for _ in range(2)]
s0 = torch.cuda.Stream(dev)
st = S["sets"][0]
S["ext"].extract_batch(S["d"].data_ptr(), B, W, H, W, W * H, st["k"].data_ptr(), st["de"].data_ptr(),
                       cap, st["n"].data_ptr(), s0.cuda_stream)
torch.cuda.synchronize()
kh = st["k"].cpu().numpy().view(orb.KEYPOINT_DTYPE).reshape(B, cap)
dh, nh = st["de"].cpu().numpy(), st["n"].cpu().numpy()
maps = [orb.synth_local_map(seed + i, kh[i, :nh[i]], dh[i, :nh[i]], M, W, H) for i in range(B)]
mps = np.stack([m[0] for m in maps])
mpd = np.stack([m[1] for m in maps])
lk = np.zeros((B, cap), np.uint8)
for i in range(B):
    lk[i, :nh[i]] = maps[i][2]
S["mps"] = torch.from_numpy(mps.view(np.uint8).reshape(B, -1)).to(dev)
S["mpd"] = torch.from_numpy(mpd).to(dev)
S["lk"] = torch.from_numpy(lk).to(dev)
S["nm"] = torch.full((B,), M, dtype=torch.int32, device=dev)
S["mt"] = orb.ORBmatcher(0.8, device=0)


def extract(j, s):
    st = S["sets"][j]
    S["ext"].extract_batch(S["d"].data_ptr(), B, W, H, W, W * H, st["k"].data_ptr(),
                           st["de"].data_ptr(), cap, st["n"].data_ptr(), s)


def match(j, s):
    st = S["sets"][j]
    S["mt"].search_by_projection_batch(B, st["k"].data_ptr(), st["de"].data_ptr(), st["n"].data_ptr(),
                                       S["lk"].data_ptr(), cap, S["mps"].data_ptr(),
                                       S["mpd"].data_ptr(), S["nm"].data_ptr(), M, W, H, scale, 1.0,
                                       st["km"].data_ptr(), st["nm"].data_ptr(), s)


def run(tag):
    sec = bench.pipelined(torch, dev, extract, match, 2, 200, 10, lanes=1)
    print(f"{tag}: {B / sec:.0f} problems/s", flush=True)


def move(keys, pad_mib=6):
    pad = torch.empty(pad_mib << 20, dtype=torch.uint8, device=dev)
    for k in keys:
        if k == "sets":
            S["sets"] = [{a: b.clone() for a, b in s.items()} for s in S["sets"]]
        else:
            S[k] = S[k].clone()
    torch.cuda.synchronize()
    return pad


if "--repeat" in sys.argv:
    for i in range(6):
        run(f"run {i}")
    sys.exit(0)
run("initial")
run("initial again")
pads = []
for keys in (["d"], ["sets"], ["mps", "mpd"], ["lk", "nm"], ["d"], ["sets"], ["mps", "mpd"]):
    pads.append(move(keys))
    run("moved " + "+".join(keys))
S["ext"] = orb.ORBextractor(NF, 1.2, 8, 20, 7, device=0)
run("new extractor handle")
S["mt"] = orb.ORBmatcher(0.8, device=0)
run("new matcher handle")
S["ext"] = orb.ORBextractor(NF, 1.2, 8, 20, 7, device=0)
run("new extractor handle")
S["mt"] = orb.ORBmatcher(0.8, device=0)
run("new matcher handle")
