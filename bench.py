#!/usr/bin/env python3
"""bench.py -- frames/s of ORB extract + match (BASELINE.json metric) on N MI355X GPUs.

One step = one batch of B synthetic KITTI-shaped 1241x376 frames per GPU through
the whole hot path, resident in HBM: ORBextractor (1000 features, 8 levels,
FAST 20/7) + SearchByProjection(F, local map) against a 5,000-point synthetic
local map per frame (the headline workload).  Frames shard
one batch per rank (weak scaling); the only collective is an RCCL all-gather of
the per-frame keypoint counts each step and of the per-rank times at the end.
Steps are pipelined over two HIP streams and two buffer sets: step k's matcher
overlaps step k+1's extraction (every step still does all of its work; the
timed region ends with a device synchronize).

Prints ONE JSON line on rank 0 (driver contract) with `roofline` (dominant
kernel, HIP-event timed over the timed region) and `cpu_baseline` (the C++ CPU
oracle, single thread, on a bounded sample of the same workload).
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
PKG_DIR = ROOT / "orb_slam2-chinese-annotation_amd"
METRIC = "frames/sec (extract+match) at 1241×376, 1000 feat/frame; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, MI355X_MICROARCH.md "Chip-level parameters"


def load_package():
    if "orb_amd" in sys.modules:
        return sys.modules["orb_amd"]
    spec = importlib.util.spec_from_file_location(
        "orb_amd", PKG_DIR / "__init__.py", submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["orb_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def level_sizes(w, h, scale, nlevels):
    inv = [np.float32(1.0) / np.float32(s) for s in scale]
    out = []
    for l in range(nlevels):
        if l == 0:
            out.append((w, h))
        else:
            out.append((int(np.rint(np.float32(w) * inv[l])), int(np.rint(np.float32(h) * inv[l]))))
    return out


def algorithmic_bytes(w, h, scale, nlevels, n_kp, n_mp):
    """Per-frame algorithmic HBM bytes of each kernel."""
    sizes = level_sizes(w, h, scale, nlevels)
    P = [a * b for a, b in sizes]
    pyr = sum(P[l - 1] + P[l] for l in range(1, nlevels))  # read level l-1, write level l
    fast = sum(P)                                          # read every level once
    desc = 60 * n_kp                                       # 28 B keypoint + 32 B descriptor
    match = 60 * n_mp + 48 * n_kp + 24576                  # SURVEY §8(d) B_lm
    octree = 8 * n_kp                                      # selected keys in, out (4 B each)
    blur = 2 * sum(P)                                      # read + write every level
    return {"k_pyr_resize": pyr, "k_blur_levels": blur, "k_fast_band": fast, "k_octree": octree,
            "k_orient_desc": desc, "k_proj_candidates": match, "k_proj_resolve": 24 * n_mp,
            "k_grid_build": 32 * n_kp,
            "frame_total_survey": (2 * sum(P) - P[0]) + 60 * n_kp + match}


def shard_frames(rank, batch):
    """Frame ids this rank processes in each step: a contiguous block of the
    synthetic sequence per rank (weak scaling, no data-path collective)."""
    return [rank * batch + i for i in range(batch)]


def gather_counts(dist, counts, out):
    """RCCL all-gather of every frame's keypoint count (int32 per frame)."""
    dist.all_gather_into_tensor(out, counts)
    return out


def max_over_ranks(dist, elapsed, device):
    """The job's time = the slowest rank's time."""
    import torch

    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def measured_traffic(kernel, batch):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/rNN_hbm_traffic.json, tools/pmc_summary.py), scaled to this batch."""
    files = sorted((ROOT / "profiles").glob("r*_hbm_traffic.json"))
    if not files:
        return None, None
    t = json.loads(files[-1].read_text())
    k = t["kernels"].get(kernel)
    if k is None:
        return None, files[-1].name
    return k["traffic_bytes"] * batch / t["batch"], files[-1].name


# VALU issue time per wave-instruction per SIMD on gfx950, measured by
# tools/probe/valu_rates.hip (profiles/r01_valu_rates.txt): plain 32-bit
# integer / f32 ops ~1.0 ns, packed, 3-input and 24/32-bit multiply ops ~1.8 ns.
VALU_NS_FAST, VALU_NS_SLOW, N_SIMD = 1.0, 1.8, 1024


def valu_issue(kernel, batch, ms_per_launch):
    """Lower/upper bound on the time the SIMDs need just to issue `kernel`'s
    VALU instructions (SQ_INSTS_VALU from the newest profiles/rNN_pmc.json,
    scaled to this batch), as a fraction of its measured launch time."""
    files = sorted((ROOT / "profiles").glob("r*_pmc.json"))
    if not files:
        return None
    t = json.loads(files[-1].read_text())
    k = t["kernels"].get(kernel)
    if k is None or "SQ_INSTS_VALU" not in k:
        return None
    n = k["SQ_INSTS_VALU"] * batch / t["batch"]
    lo, hi = (n / N_SIMD * ns * 1e-6 for ns in (VALU_NS_FAST, VALU_NS_SLOW))
    return {"valu_instr_per_launch": n, "issue_ms_range": [lo, hi],
            "frac_range": [lo / ms_per_launch, hi / ms_per_launch],
            "source": f"profiles/{files[-1].name} SQ_INSTS_VALU x "
                      f"{VALU_NS_FAST}-{VALU_NS_SLOW} ns per wave-instruction per SIMD "
                      "(profiles/r01_valu_rates.txt)"}


def cpu_baseline(imgs_host, maps, args, scale):
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle  # CPU oracle: checker / baseline only

    t0 = time.perf_counter()
    n = 0
    while True:
        i = n % len(imgs_host)
        k, d, _ = oracle.extract(imgs_host[i], args.features, 1.2, 8, 20, 7)
        mps, mpd, locked = maps[i]
        oracle.match_projection_local(k, d, scale, args.width, args.height, mps, mpd, 1.0, 0.8,
                                      locked[: len(k)])
        n += 1
        el = time.perf_counter() - t0
        if (el >= args.cpu_seconds and n >= 3) or n >= args.cpu_max_frames:
            break
    return {"value": n / el, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"{n} frames {args.width}x{args.height}: oracle ORBextractor "
                      f"({args.features} feat) + SearchByProjection vs {args.mappoints} map "
                      f"points, C++ -O3 scalar, 1 thread, {el:.1f} s"}


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=512, help="frames per GPU per step")
    ap.add_argument("--width", type=int, default=1241)
    ap.add_argument("--height", type=int, default=376)
    ap.add_argument("--features", type=int, default=1000)
    ap.add_argument("--mappoints", type=int, default=5000)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-max-frames", type=int, default=400)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--seed", type=int, default=0x4B495454)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    orb = load_package()
    W, H, B, NF, M = args.width, args.height, args.batch, args.features, args.mappoints

    # ---------------- inputs: this rank's shard of the synthetic sequence, in HBM
    frames = shard_frames(rank, B)
    imgs = np.stack([orb.synth_image(args.seed, f, W, H) for f in frames])
    ext = orb.ORBextractor(NF, 1.2, 8, 20, 7, device=local)
    scale = np.float32(ext.GetScaleFactors())
    cap = ext.capacity(W, H)
    dev = torch.device("cuda", local)
    # Two streams, two buffer sets: step k's SearchByProjection (matcher
    # stream) overlaps step k+1's extraction (extract stream).  Step k's
    # extraction writes buffer set k % 2 once the matcher of step k - 2 (the
    # set's previous reader) has finished; its matcher starts once it is done.
    ext_stream = torch.cuda.Stream(dev)
    match_stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(ext_stream)
    d_img = torch.from_numpy(imgs).to(dev)
    sets = [dict(kps=torch.zeros((B, cap, 7), dtype=torch.int32, device=dev),
                 desc=torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev),
                 cnt=torch.zeros(B, dtype=torch.int32, device=dev),
                 match=torch.zeros((B, cap), dtype=torch.int32, device=dev),
                 nmatch=torch.zeros(B, dtype=torch.int32, device=dev),
                 gathered=torch.zeros(world * B, dtype=torch.int32, device=dev) if world > 1 else None)
            for _ in range(2)]
    extracted = [torch.cuda.Event(), torch.cuda.Event()]
    matched = [torch.cuda.Event(), torch.cuda.Event()]

    def extract(st, stream):
        ext.extract_batch(d_img.data_ptr(), B, W, H, W, W * H, st["kps"].data_ptr(),
                          st["desc"].data_ptr(), cap, st["cnt"].data_ptr(), stream.cuda_stream)

    extract(sets[0], ext_stream)  # untimed: derive each frame's local map from its own keypoints
    torch.cuda.synchronize()
    kps_h = sets[0]["kps"].cpu().numpy().view(orb.KEYPOINT_DTYPE).reshape(B, cap)
    desc_h = sets[0]["desc"].cpu().numpy()
    cnt_h = sets[0]["cnt"].cpu().numpy()
    mps_all = np.zeros((B, M), orb.MP_TRACK_DTYPE)
    mpd_all = np.zeros((B, M, 32), np.uint8)
    lock_all = np.zeros((B, cap), np.uint8)
    maps = []
    for i in range(B):
        n = int(cnt_h[i])
        mps, mpd, lk = orb.synth_local_map(args.seed + frames[i], kps_h[i, :n], desc_h[i, :n], M, W, H)
        mps_all[i], mpd_all[i], lock_all[i, :n] = mps, mpd, lk
        maps.append((mps, mpd, lk))
    d_mps = torch.from_numpy(mps_all.view(np.uint8).reshape(B, -1)).to(dev)
    d_mpd = torch.from_numpy(mpd_all).to(dev)
    d_lock = torch.from_numpy(lock_all).to(dev)
    d_nmps = torch.full((B,), M, dtype=torch.int32, device=dev)
    matcher = orb.ORBmatcher(0.8, device=local)
    torch.cuda.synchronize()

    def step(k):
        j = k % 2
        st = sets[j]
        if k >= 2:
            ext_stream.wait_event(matched[j])
        extract(st, ext_stream)
        extracted[j].record(ext_stream)
        match_stream.wait_event(extracted[j])
        matcher.search_by_projection_batch(B, st["kps"].data_ptr(), st["desc"].data_ptr(),
                                           st["cnt"].data_ptr(), d_lock.data_ptr(), cap,
                                           d_mps.data_ptr(), d_mpd.data_ptr(), d_nmps.data_ptr(),
                                           M, W, H, scale, 1.0, st["match"].data_ptr(),
                                           st["nmatch"].data_ptr(), match_stream.cuda_stream)
        if dist is not None:  # RCCL: gather every frame's keypoint count
            with torch.cuda.stream(match_stream):
                gather_counts(dist, st["cnt"], st["gathered"])
        matched[j].record(match_stream)

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    ext.profile(True)
    matcher.profile(True)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist is not None:
        dist.barrier()
    elapsed = t1 - t0
    if dist is not None:
        elapsed = max_over_ranks(dist, elapsed, dev)

    # per-kernel HIP-event times over the timed region, each on its own stream.
    # The extract stream is the critical path (the matcher stream runs in its
    # shadow, so matcher kernel times include time-sharing with the next
    # step's extraction): the roofline kernel is the longest extraction kernel.
    kern, ext_kern = {}, []
    for st in range(5):
        name, ms, n = ext.profile_read(st)
        kern[name] = (ms, n)
        ext_kern.append(name)
    for st in range(3):
        name, ms, n = matcher.profile_read(st)
        kern[name] = (ms, n)
    ext.profile(False)
    matcher.profile(False)
    n_kp = float(sets[0]["cnt"].float().mean().item())
    nmatch = float(sets[0]["nmatch"].float().mean().item())
    alg = algorithmic_bytes(W, H, scale, 8, n_kp, M)
    dom = max(ext_kern, key=lambda k: kern[k][0])
    dom_ms_per_launch = kern[dom][0] / max(kern[dom][1], 1)
    # bytes one launch of the dominant kernel processes
    launches_per_step = kern[dom][1] / args.steps
    dom_bytes = alg[dom] * B / launches_per_step
    achieved = dom_bytes / (dom_ms_per_launch * 1e-3) / 1e9

    traffic, traffic_src = measured_traffic(dom, B)
    total_frames = B * args.steps * world
    result = {
        "metric": METRIC,
        "value": total_frames / elapsed,
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {
            "workload": f"C4: {W}x{H} KITTI-shaped synthetic stream, {NF} feat/frame, "
                        f"SearchByProjection vs {M}-point local map per frame",
            "frames_per_gpu_per_step": B,
            "parallelism": f"frames sharded over {world} rank(s), RCCL all-gather of counts",
            "mean_keypoints_per_frame": n_kp,
            "mean_matches_per_frame": nmatch,
        },
        "roofline": {
            "kernel": dom,
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": f"profiles/{traffic_src} (rocprofv3 FETCH_SIZE+WRITE_SIZE, "
                              "separate passes, raw KiB x 1024)" if traffic_src else None,
            "bytes_per_launch": dom_bytes,
            "ms_per_launch": dom_ms_per_launch,
            "valu_issue": valu_issue(dom, B, dom_ms_per_launch),
        },
        "kernels_ms_per_step": {k: v[0] / args.steps for k, v in kern.items()},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(imgs, maps, args, scale)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
