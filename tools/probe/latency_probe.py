"""One-frame latency of the batch entry points (SURVEY §8(d) C4's per-GPU shape).

Device-resident 1241x376 frame, 1000 features, SearchByProjection against a
5,000-point map; each call synchronized before the next, median over --calls.
Prints one JSON line: extraction alone, matcher alone, both, and the host
single-frame API (ORBextractor.__call__, H2D + graph + D2H).  ORB_AMD_LIB
selects a library variant.
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "tests"))
from conftest import load_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=300)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--tag", default="")
    ap.add_argument("--resolve", type=int, default=0, help="matcher resolve schedule (ORB_RESOLVE_*)")
    ap.add_argument("--timeline", type=int, default=0,
                    help="only N extract+match calls 1 ms apart (for a kernel-trace timeline)")
    a = ap.parse_args()
    import torch
    orb = load_pkg()
    W, H, NF, M, B = 1241, 376, 1000, 5000, a.batch
    ext = orb.ORBextractor(NF, 1.2, 8, 20, 7)
    scale = np.float32(ext.GetScaleFactors())
    cap = ext.capacity(W, H)
    imgs = np.stack([orb.synth_image(0x4B495454, f, W, H) for f in range(B)])
    d = torch.from_numpy(imgs).cuda()
    k = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
    de = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(B, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    ext.extract_batch(d.data_ptr(), B, W, H, W, W * H, k.data_ptr(), de.data_ptr(), cap,
                      n.data_ptr(), s.cuda_stream)
    s.synchronize()
    kh = k.cpu().numpy().view(orb.KEYPOINT_DTYPE).reshape(B, cap)
    dh, nh = de.cpu().numpy(), n.cpu().numpy()
    maps = [orb.synth_local_map(0x4B495454 + i, kh[i, :nh[i]], dh[i, :nh[i]], M, W, H)
            for i in range(B)]
    lk = np.zeros((B, cap), np.uint8)
    for i in range(B):
        lk[i, :nh[i]] = maps[i][2]
    d_mps = torch.from_numpy(np.stack([m[0] for m in maps]).view(np.uint8).reshape(B, -1)).cuda()
    d_mpd = torch.from_numpy(np.stack([m[1] for m in maps])).cuda()
    d_lk = torch.from_numpy(lk).cuda()
    d_nm = torch.full((B,), M, dtype=torch.int32, device="cuda")
    km = torch.zeros((B, cap), dtype=torch.int32, device="cuda")
    nm = torch.zeros(B, dtype=torch.int32, device="cuda")
    mt = orb.ORBmatcher(0.8)
    mt.set_resolve(a.resolve)

    def extract():
        ext.extract_batch(d.data_ptr(), B, W, H, W, W * H, k.data_ptr(), de.data_ptr(), cap,
                          n.data_ptr(), s.cuda_stream)

    def match():
        mt.search_by_projection_batch(B, k.data_ptr(), de.data_ptr(), n.data_ptr(), d_lk.data_ptr(),
                                      cap, d_mps.data_ptr(), d_mpd.data_ptr(), d_nm.data_ptr(), M,
                                      W, H, scale, 1.0, km.data_ptr(), nm.data_ptr(), s.cuda_stream)

    if a.timeline:
        for _ in range(a.timeline):
            extract()
            match()
            s.synchronize()
            time.sleep(0.001)
        return

    def med(fn):
        ts = []
        for i in range(a.calls + 10):
            t0 = time.perf_counter()
            fn()
            s.synchronize()
            if i >= 10:
                ts.append(time.perf_counter() - t0)
        return float(np.median(ts)) * 1e3

    out = {"tag": a.tag, "batch": B, "resolve": a.resolve, "extract_ms": med(extract), "match_ms": med(match),
           "both_ms": med(lambda: (extract(), match()))}
    # per-stage GPU time by the libraries' stage events (profile mode 1: the
    # call's own launch shape; events add a little per stage)
    ext.profile(1)
    mt.profile(True)
    for _ in range(100):
        extract()
        match()
        s.synchronize()
    stages = {}
    for st in range(7):
        name, ms, cnt = ext.profile_read(st)
        if cnt:
            stages[name] = ms / 100
    for st in range(4):
        name, ms, cnt = mt.profile_read(st)
        if cnt:
            stages[name] = ms / 100
    ext.profile(0)
    mt.profile(False)
    out["stage_ms"] = stages
    host = orb.ORBextractor(NF, 1.2, 8, 20, 7)
    img0 = imgs[0]
    ts = []
    for i in range(a.calls + 10):
        t0 = time.perf_counter()
        host(img0)
        if i >= 10:
            ts.append(time.perf_counter() - t0)
    out["host_api_extract_ms"] = float(np.median(ts)) * 1e3
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
