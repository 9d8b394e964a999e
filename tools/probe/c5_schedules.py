"""C5 SearchByProjection alone (16 problems, 1920x1080, 4000 features, 50,000-point
maps, one stream, one call at a time) under each resolve schedule, with the
matcher's stage times.  Prints one JSON line per schedule."""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "tests"))


def main():
    import torch
    from conftest import load_pkg
    orb = load_pkg()
    W, H, NF, M, B, seed = 1920, 1080, 4000, 50000, 16, 5
    ext = orb.ORBextractor(NF, 1.2, 8, 20, 7)
    scale = np.float32(ext.GetScaleFactors())
    cap = ext.capacity(W, H)
    imgs = np.stack([orb.synth_image(seed, f, W, H) for f in range(B)])
    d = torch.from_numpy(imgs).cuda()
    k = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
    de = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(B, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    ext.extract_batch(d.data_ptr(), B, W, H, W, W * H, k.data_ptr(), de.data_ptr(), cap, n.data_ptr(),
                      s.cuda_stream)
    s.synchronize()
    kh = k.cpu().numpy().view(orb.KEYPOINT_DTYPE).reshape(B, cap)
    dh, nh = de.cpu().numpy(), n.cpu().numpy()
    maps = [orb.synth_local_map(seed + i, kh[i, :nh[i]], dh[i, :nh[i]], M, W, H) for i in range(B)]
    lk = np.zeros((B, cap), np.uint8)
    for i in range(B):
        lk[i, :nh[i]] = maps[i][2]
    d_mps = torch.from_numpy(np.stack([m[0] for m in maps]).view(np.uint8).reshape(B, -1)).cuda()
    d_mpd = torch.from_numpy(np.stack([m[1] for m in maps])).cuda()
    d_lk = torch.from_numpy(lk).cuda()
    d_nm = torch.full((B,), M, dtype=torch.int32, device="cuda")
    km = torch.zeros((B, cap), dtype=torch.int32, device="cuda")
    nm = torch.zeros(B, dtype=torch.int32, device="cuda")
    for sched, rounds in ((0, 6), (2, 6), (3, 4), (3, 6), (3, 10)):
        mt = orb.ORBmatcher(0.8)
        mt.set_resolve(sched, rounds)

        def match():
            mt.search_by_projection_batch(B, k.data_ptr(), de.data_ptr(), n.data_ptr(), d_lk.data_ptr(),
                                          cap, d_mps.data_ptr(), d_mpd.data_ptr(), d_nm.data_ptr(), M,
                                          W, H, scale, 1.0, km.data_ptr(), nm.data_ptr(), s.cuda_stream)
        for _ in range(10):
            match()
        s.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            match()
        s.synchronize()
        dt = (time.perf_counter() - t0) / 200
        mt.profile(True)
        for _ in range(50):
            match()
        s.synchronize()
        st = {}
        for i in range(4):
            name, ms, cnt = mt.profile_read(i)
            if cnt:
                st[name] = round(ms / 50, 4)
        mt.profile(False)
        print(json.dumps({"schedule": sched, "jacobi_rounds": rounds, "ms_per_call": round(dt * 1e3, 4),
                          "problems_per_s": round(B / dt), "stage_ms": st,
                          "mean_matches": float(nm.float().mean().item())}), flush=True)


if __name__ == "__main__":
    main()
