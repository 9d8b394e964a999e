#!/usr/bin/env python3
"""Secondary measurements for BASELINE.json's other configs (C1, C2, C3, C5).

bench.py is the driver contract and measures the headline C4 workload; this
script reports the remaining configs, one JSON line each, for BASELINE.md's
results table:

  C1  CPU oracle only: 1241x376, 1000 features, 100-frame synthetic sequence,
      extraction; 1 thread and all host cores (frames/s)
  C2  640x480, 1000 features, GPU extraction only (frames/s) + bit-exact check
  C3  1241x376 stereo pairs, 2000 features per image, both extractions +
      ComputeStereoMatches on the GPU (pairs/s) + bit-exact check
  C5  1920x1080, 4000 features, SearchByProjection against a 50,000-point
      local map (th 1, nnratio 0.8), 16 problems per launch (problems/s for
      extract+match, and the matcher alone with its HBM roofline)
  C4M the headline's matcher alone: 1241x376, 1000 features, 5,000-point local
      maps, 512 problems per launch (same keys as C5)
  F1  SURVEY §8(f): SearchForInitialization, 640x480 frames from the 2000-feature
      initial extractor, window 100, ORBmatcher(0.9, true), 64 pairs per launch
      (pairs/s) + CPU oracle rate + exact check
  F2  SURVEY §8(f): Frame::ComputeBoW (DBoW2 transform, levelsup 4) on an
      ORBvoc-shaped synthetic vocabulary (k 10, L 6, 10^6 words, TF-IDF, L1),
      1000 extracted descriptors per frame, 512 frames per launch (frames/s)
      + CPU oracle rate + exact check
  F3  SURVEY §8(f): ComputeDistinctiveDescriptors over 100,000 map points with
      1..20 observations (points/s) + CPU oracle rate + exact check

Usage: python tools/bench_configs.py [--configs C1,C2,C3,C5,F1,F3] [--steps K]
The oracle (CPU restatement) is used only for the CPU rows and parity checks.
"""
import argparse
import json
import os
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tests")]

import bench  # noqa: E402

SEED = 0x4B495454


def timed(fn, steps, warmup, torch):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def cpu_rate(fn, items, seconds, threads=1):
    """items/s of fn(i) over a bounded sample, on `threads` host threads (the
    oracle's ctypes calls release the GIL)."""
    done = [0]
    lock = threading.Lock()
    stop = time.perf_counter() + seconds

    def worker(t):
        i = t
        while time.perf_counter() < stop:
            fn(i % items)
            with lock:
                done[0] += 1
            i += threads

    t0 = time.perf_counter()
    ths = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    return done[0] / (time.perf_counter() - t0)


def c1(args, orb, oracle):
    W, H = 1241, 376
    imgs = [oracle.synth_image(SEED, f, W, H) for f in range(100)]
    one = cpu_rate(lambda i: oracle.extract(imgs[i], 1000), 100, args.cpu_seconds, 1)
    nthr = int(os.environ.get("OMP_NUM_THREADS", 0)) or os.cpu_count() or 1  # the box grants 16
    allc = cpu_rate(lambda i: oracle.extract(imgs[i], 1000), 100, args.cpu_seconds, nthr)
    return {"config": "C1", "workload": "1241x376 synthetic 100-frame sequence, 1000 feat, CPU "
            "oracle ORBextractor only", "unit": "frames/s", "cpu_1_thread": one,
            "cpu_all_cores": allc, "cores": nthr, "ms_per_frame_1_thread": 1e3 / one}


def c2(args, orb, oracle, torch):
    W, H, B = 640, 480, args.batch
    imgs = np.stack([orb.synth_image(1 + (f % 3), 0 if f < 3 else f, W, H) for f in range(B)])
    ext = orb.ORBextractor(1000, 1.2, 8, 20, 7)
    cap = ext.capacity(W, H)
    d = torch.from_numpy(imgs).cuda()
    k = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
    de = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(B, dtype=torch.int32, device="cuda")
    # an explicit stream: a NULL stream would mean the handle's own stream
    s = torch.cuda.Stream().cuda_stream

    def step():
        ext.extract_batch(d.data_ptr(), B, W, H, W, W * H, k.data_ptr(), de.data_ptr(), cap,
                          n.data_ptr(), s)

    sec = timed(step, args.steps, 2, torch)
    exact = True
    for i in range(3):  # seeds 1..3, frame 0
        kr, dr, _ = oracle.extract(imgs[i], 1000)
        ni = int(n[i].item())
        kg = k[i, :ni].cpu().numpy().view(orb.KEYPOINT_DTYPE).reshape(-1)
        exact &= ni == len(kr) and kg.tobytes() == kr.tobytes() and \
            de[i, :ni].cpu().numpy().tobytes() == dr.tobytes()
    cpu = cpu_rate(lambda i: oracle.extract(imgs[i], 1000), 3, args.cpu_seconds, 1)
    return {"config": "C2", "workload": f"640x480 synthetic, 1000 feat, GPU extraction, batch {B}",
            "unit": "frames/s", "value": B / sec, "ms_per_step": sec * 1e3,
            "bit_exact_seeds_1_3": bool(exact), "cpu_1_thread": cpu}


def c3(args, orb, oracle, torch):
    """bench.c3_workload (the driver line's C3 key, same inputs and schedule)
    plus the oracle check of pair 0 and the oracle's CPU rate."""
    import scenarios

    dev = torch.device("cuda:0")
    r, st = bench.c3_workload(orb, torch, dev, 16, steps=max(args.steps, 40), warmup=5,
                              pairs=args.batch // 2)
    il, ir, s0 = st["il"], st["ir"], st["set0"]
    W, H, NF = 1241, 376, 2000
    p = oracle.params(NF)
    klh, dlh, _ = oracle.extract(il[0], NF)
    krh, drh, _ = oracle.extract(ir[0], NF)
    ur_ref, dp_ref = oracle.stereo_match(klh, dlh, p["scale"], krh, drh, oracle.pyramid(il[0]),
                                         oracle.pyramid(ir[0]), p["inv_scale"], scenarios.BF,
                                         scenarios.FX, W, H)
    n0 = int(s0["nl"][0].item())
    exact = n0 == len(klh) and s0["ur"][0, :n0].cpu().numpy().tobytes() == ur_ref.tobytes() and \
        s0["dp"][0, :n0].cpu().numpy().tobytes() == dp_ref.tobytes()

    def cpu_pair(i):
        a, da, _ = oracle.extract(il[i], NF)
        b, db, _ = oracle.extract(ir[i], NF)
        oracle.stereo_match(a, da, p["scale"], b, db, oracle.pyramid(il[i]), oracle.pyramid(ir[i]),
                            p["inv_scale"], scenarios.BF, scenarios.FX, W, H)

    cpu = cpu_rate(cpu_pair, 4, args.cpu_seconds, 1)
    return dict(config="C3", bit_exact_pair_0=bool(exact), cpu_1_thread=cpu, **r)


def c5(args, orb, oracle, torch):
    return proj_config(args, orb, oracle, torch, "C5", 1920, 1080, 4000, 50000, 16, bench.C5_SEED)


def c4m(args, orb, oracle, torch):
    """the headline's matcher by itself: 512 KITTI-shaped frames, 5,000-point maps"""
    return proj_config(args, orb, oracle, torch, "C4M", 1241, 376, 1000, 5000, 512, 7)


def proj_config(args, orb, oracle, torch, name, W, H, NF, M, B, seed):
    """bench.proj_workload (the driver line's C5 key for C5) plus the oracle
    check of problem 0."""
    dev = torch.device("cuda:0")
    # ~0.1 s timed regions (bench.secondary_configs): short ones are noisy
    steps = max(args.steps, 200 if B <= 64 else 40)
    r, st = bench.proj_workload(orb, torch, dev, 16, W, H, NF, M, B, seed, steps=steps, warmup=10)
    n0 = int(st["nh"][0])
    s0 = st["set0"]
    nr, kmr = oracle.match_projection_local(st["kh"][0, :n0], st["dh"][0, :n0], st["scale"], W, H,
                                            st["mps"][0], st["mpd"][0], 1.0, 0.8, st["lk"][0, :n0])
    exact = int(s0["nm"][0].item()) == nr and np.array_equal(s0["km"][0, :n0].cpu().numpy(), kmr)
    return dict(config=name, bit_exact_problem_0=bool(exact), **r)


def f1(args, orb, oracle, torch):
    import scenarios
    W, H, P, U = 640, 480, 64, 16
    pairs = [scenarios.init_pair(oracle, 100 + i, 1 + i % 3, w=W, h=H, nf=2000) for i in range(U)]
    stride = max(max(len(s["k1"]), len(s["k2"])) for s in pairs)
    K1 = np.zeros((P, stride), orb.KEYPOINT_DTYPE)
    K2 = np.zeros((P, stride), orb.KEYPOINT_DTYPE)
    D1 = np.zeros((P, stride, 32), np.uint8)
    D2 = np.zeros((P, stride, 32), np.uint8)
    PR = np.zeros((P, stride, 2), np.float32)
    n1 = np.zeros(P, np.int32)
    n2 = np.zeros(P, np.int32)
    for i in range(P):
        s = pairs[i % U]
        n1[i], n2[i] = len(s["k1"]), len(s["k2"])
        K1[i, :n1[i]], D1[i, :n1[i]], PR[i, :n1[i]] = s["k1"], s["d1"], s["prev"]
        K2[i, :n2[i]], D2[i, :n2[i]] = s["k2"], s["d2"]
    t = {k: torch.from_numpy(np.ascontiguousarray(v).view(np.uint8)).cuda()
         for k, v in dict(K1=K1, K2=K2, D1=D1, D2=D2, n1=n1, n2=n2).items()}
    pr0 = torch.from_numpy(PR).cuda()
    pr = pr0.clone()
    m12 = torch.zeros((P, stride), dtype=torch.int32, device="cuda")
    nm = torch.zeros(P, dtype=torch.int32, device="cuda")
    mt = orb.ORBmatcher(0.9, True)
    # a real stream shared with torch: the prev-position reset must be ordered
    # before the kernels (handle 0 would select the matcher's own stream)
    ts = torch.cuda.Stream()
    s_ = ts.cuda_stream

    def step():
        with torch.cuda.stream(ts):
            pr.copy_(pr0)  # vbPrevMatched is in/out: restore the initial positions
        mt.search_for_initialization_batch(P, t["K1"].data_ptr(), t["D1"].data_ptr(),
                                           t["n1"].data_ptr(), t["K2"].data_ptr(),
                                           t["D2"].data_ptr(), t["n2"].data_ptr(), stride, 0.0,
                                           float(W), 0.0, float(H), 100, pr.data_ptr(),
                                           m12.data_ptr(), nm.data_ptr(), s_)

    sec = timed(step, args.steps, 2, torch)
    exact = True
    for i in range(U):
        s = pairs[i]
        rn, rm, rp = oracle.search_for_initialization(s["k1"], s["d1"], s["k2"], s["d2"], W, H,
                                                      s["prev"], 100, 0.9, True)
        exact &= int(nm[i].item()) == rn and np.array_equal(m12[i, :n1[i]].cpu().numpy(), rm)
    cpu = cpu_rate(lambda i: oracle.search_for_initialization(
        pairs[i]["k1"], pairs[i]["d1"], pairs[i]["k2"], pairs[i]["d2"], W, H, pairs[i]["prev"],
        100, 0.9, True), U, args.cpu_seconds, 1)
    return {"config": "F1", "workload": f"SearchForInitialization 640x480, 2000-feature initial "
            f"extractor, window 100, {P} pairs per launch", "unit": "pairs/s", "value": P / sec,
            "ms_per_step": sec * 1e3, "cpu_oracle_1_thread": cpu,
            "mean_level0_keypoints": float(np.mean([(s["k1"]["octave"] == 0).sum() for s in pairs])),
            "bit_exact": bool(exact)}


def f3(args, orb, oracle, torch):
    import scenarios
    M = 100000
    rng = np.random.default_rng(9)
    counts = rng.integers(1, 21, M)
    offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    base = rng.integers(0, 256, (M, 32), dtype=np.uint8)
    rows = np.repeat(base, counts, axis=0)
    bits = np.unpackbits(rows, axis=1)
    bits ^= (rng.random(bits.shape) < 0.1).astype(np.uint8)
    desc = np.packbits(bits, axis=1)
    d_offs = torch.from_numpy(offs).cuda()
    d_desc = torch.from_numpy(desc).cuda()
    d_best = torch.zeros(M, dtype=torch.int32, device="cuda")
    d_out = torch.zeros((M, 32), dtype=torch.uint8, device="cuda")
    mt = orb.ORBmatcher()
    s_ = torch.cuda.current_stream().cuda_stream

    def step():
        mt.distinctive_descriptors_batch(M, d_offs.data_ptr(), d_desc.data_ptr(),
                                         d_best.data_ptr(), d_out.data_ptr(), s_)

    sec = timed(step, args.steps, 2, torch)
    ref = oracle.distinctive_descriptors(offs, desc)
    exact = np.array_equal(d_best.cpu().numpy(), ref)
    chunk = 1000
    cpu = cpu_rate(lambda i: oracle.distinctive_descriptors(
        offs[i * chunk:(i + 1) * chunk + 1] - offs[i * chunk],
        desc[offs[i * chunk]:offs[(i + 1) * chunk]]), M // chunk, args.cpu_seconds, 1) * chunk
    alg_bytes = offs[-1] * 32 + (M + 1) * 4 + M * 36
    return {"config": "F3", "workload": "ComputeDistinctiveDescriptors, 100,000 map points, "
            "1..20 observations each", "unit": "points/s", "value": M / sec,
            "ms_per_step": sec * 1e3, "cpu_oracle_1_thread": cpu,
            "alg_GBps": alg_bytes / sec / 1e9, "bit_exact": bool(exact)}


def f2(args, orb, oracle, torch):
    import scenarios
    W, H, NF = 1241, 376, 1000
    voc = scenarios.vocabulary(rng_seed=11, k=10, L=6)
    V = orb.ORBVocabulary(voc["k"], voc["L"], voc["parent"], voc["leaf"], voc["desc"],
                          voc["weight"])
    B = args.batch
    ext = orb.ORBextractor(NF, 1.2, 8, 20, 7)
    frames = []
    for f in range(32):
        _, d = ext(orb.synth_image(SEED, f, W, H))
        frames.append(d[:NF])
    stride = NF + 8
    counts = np.array([len(frames[f % 32]) for f in range(B)], np.int32)
    desc = np.zeros((B, stride, 32), np.uint8)
    for f in range(B):
        desc[f, :counts[f]] = frames[f % 32]
    dev = torch.device("cuda:0")
    d_counts = torch.from_numpy(counts).to(dev)
    d_desc = torch.from_numpy(desc).to(dev)
    n = B * stride
    i32 = lambda m: torch.zeros(m, dtype=torch.int32, device=dev)
    f64 = lambda m: torch.zeros(m, dtype=torch.float64, device=dev)
    fw, fwt, fn, bw, bv, nw = i32(n), f64(n), i32(n), i32(n), f64(n), i32(B)
    fvn, fvo, fvf, nfv = i32(n), i32(B * (stride + 1)), i32(n), i32(B)
    s_ = torch.cuda.current_stream().cuda_stream

    def step():
        V.transform_batch(B, d_counts.data_ptr(), d_desc.data_ptr(), stride, 4, fw.data_ptr(),
                          fwt.data_ptr(), fn.data_ptr(), bw.data_ptr(), bv.data_ptr(),
                          nw.data_ptr(), fvn.data_ptr(), fvo.data_ptr(), fvf.data_ptr(),
                          nfv.data_ptr(), s_)

    sec = timed(step, args.steps, 2, torch)
    exact = True
    h = lambda t: t.cpu().numpy()
    bw_, bv_, nw_, fvn_, fvf_ = h(bw).view(np.uint32), h(bv), h(nw), h(fvn).view(np.uint32), h(fvf)
    for f in range(4):
        r = oracle.vocab_transform(voc, frames[f], 4)
        o = f * stride
        exact &= (np.array_equal(bw_[o:o + nw_[f]], r[0]) and
                  np.array_equal(bv_[o:o + nw_[f]].view(np.uint64), r[1].view(np.uint64)) and
                  np.array_equal(fvn_[o:o + len(r[2])], r[2]) and
                  np.array_equal(fvf_[o:o + len(r[4])].view(np.uint32), r[4]))
    cpu_frames = 8
    cpu_sec = oracle.vocab_time(voc, np.concatenate(frames[:cpu_frames]), cpu_frames, NF, 4)
    feats = int(counts.sum())
    tree_bytes = len(voc["parent"]) * (32 + 8 + 4 + 8 + 4)
    alg_bytes = tree_bytes + feats * (32 + 4 + 8 + 4 + 4 + 8 + 4 + 4 + 4)
    return {"config": "F2", "workload": "Frame::ComputeBoW, ORBvoc-shaped synthetic vocabulary "
            "(k 10, L 6, 10^6 words), 1000 descriptors/frame, levelsup 4", "unit": "frames/s",
            "value": B / sec, "ms_per_step": sec * 1e3, "frames_per_launch": B,
            "features_per_s": feats / sec, "cpu_oracle_1_thread": cpu_frames / cpu_sec,
            "alg_GBps": alg_bytes / sec / 1e9, "bit_exact": bool(exact)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C1,C2,C3,C5")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--cpu-seconds", type=float, default=6.0)
    args = ap.parse_args()
    import torch
    import oracle

    orb = bench.load_package()
    for c in args.configs.split(","):
        if c == "C1":
            r = c1(args, orb, oracle)
        elif c == "C2":
            r = c2(args, orb, oracle, torch)
        elif c == "C3":
            r = c3(args, orb, oracle, torch)
        elif c == "C5":
            r = c5(args, orb, oracle, torch)
        elif c == "C4M":
            r = c4m(args, orb, oracle, torch)
        elif c == "F1":
            r = f1(args, orb, oracle, torch)
        elif c == "F2":
            r = f2(args, orb, oracle, torch)
        elif c == "F3":
            r = f3(args, orb, oracle, torch)
        else:
            raise SystemExit(f"unknown config {c}")
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
