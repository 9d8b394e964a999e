#!/usr/bin/env python3
"""bench.py -- frames/s of ORB extract + match (BASELINE.json metric) on N MI355X GPUs.

Each GPU holds a resident sequence of D distinct synthetic KITTI-shaped
1241x376 frames (default 8192) in HBM; one step = one pass of the whole hot
path over all D frames, in launches of B = 1024: ORBextractor (1000 features,
8 levels, FAST 20/7) + SearchByProjection(F, local map) against each frame's
own 5,000-point synthetic local map (the headline
workload).  Frames shard per rank (weak scaling); the only collectives are one
RCCL all-gather of the step's per-frame keypoint counts per step and a MAX of
the per-rank times at the end.  Launches alternate between two extraction
lanes (extractor handles on streams of their own, so one launch's
latency-bound resize chain and octree overlap the other's FAST and
descriptors) and a match stream, over four buffer sets: launch g's matcher
overlaps the next launches' extraction (every launch does all of its work; the
timed region ends with a device synchronize).

Prints ONE JSON line on rank 0 (driver contract) with `roofline` (dominant
kernel, HIP-event timed alone after the timed region, and pipelined in a
profiled pass of the same launches after it -- no event sits inside the timed
region; HBM bytes per SURVEY §8(d) as
the primary fraction, VALU issue beside it), `host_input` (the same pipeline
fed from pinned host memory: H2D of every frame and D2H of every result, the
drop-in's PCIe-inclusive rate, never `value`), `parity_sample` (64 frames of
the timed pipeline's own output buffers re-computed by the CPU oracle, bit for
bit; a mismatch exits non-zero) and `cpu_baseline` (the C++ CPU oracle, single
thread, on a bounded sample of the same workload).
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


def algorithmic_bytes(w, h, scale, nlevels, n_kp, n_mp, resize_launches=None):
    """Per-frame algorithmic HBM bytes of each kernel.
    resize_launches: launches per call of the pyramid stage; when the planner
    paired the levels (k_pyr_resize2 builds l and l + 1 from l - 1, pairs from
    level 1), level l of a pair is written and never read back."""
    sizes = level_sizes(w, h, scale, nlevels)
    P = [a * b for a, b in sizes]
    pyr = sum(P[l - 1] + P[l] for l in range(1, nlevels))  # read level l-1, write level l
    pairs = [(l, l + 1 < nlevels) for l in range(1, nlevels, 2)]
    if resize_launches is not None and resize_launches == len(pairs) < nlevels - 1:
        pyr = sum(P[l - 1] + P[l] + (P[l + 1] if two else 0) for l, two in pairs)
    fast = sum(P)                                          # read every level once
    desc = 60 * n_kp                                       # 28 B keypoint + 32 B descriptor
    match = 60 * n_mp + 48 * n_kp + 24576                  # SURVEY §8(d) B_lm
    octree = 8 * n_kp                                      # selected keys in, out (4 B each)
    blur = 2 * sum(P)                                      # read + write every level
    return {"k_pyr_resize": pyr, "k_blur_levels": blur, "k_fast_band": fast, "k_fast_cells": fast,
            "k_octree": octree,
            "k_orient_desc": desc, "k_proj_candidates": match, "k_proj_resolve": 24 * n_mp,
            "k_grid_build": 32 * n_kp,
            "frame_total_survey": (2 * sum(P) - P[0]) + 60 * n_kp + match}


def shard_frames(rank, frames):
    """Frame ids this rank processes in each step: a contiguous block of the
    synthetic sequence per rank (weak scaling, no data-path collective)."""
    return [rank * frames + i for i in range(frames)]


def gather_counts(dist, counts, out):
    """RCCL all-gather of the step's per-frame keypoint counts (int32 per frame,
    one collective per step).  With the gloo backend (the multi-process test on
    one GPU) through host copies."""
    if dist.get_backend() == "gloo":
        parts = [c.cpu() for c in out.chunk(dist.get_world_size())]
        dist.all_gather(parts, counts.cpu())
        out.copy_(__import__("torch").cat(parts))
        return out
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


# VALU issue peak (MI355X_MICROARCH.md "Wave scheduling"): 1,024 SIMDs, one
# wave64 VALU instruction per 2 cycles each, at the 2.4 GHz maximum clock =
# 1,229 G wave-instructions/s.  tools/probe/valu_rates.hip measured ~1.0 ns per
# plain and ~1.8 ns per packed / 3-input / multiply wave-instruction per SIMD
# under load (profiles/r01_valu_rates.txt): the range of the issue-time bound.
N_SIMD, CLOCK_GHZ, VALU_CYCLES = 1024, 2.4, 2
VALU_PEAK_G = N_SIMD * CLOCK_GHZ / VALU_CYCLES
VALU_NS_FAST, VALU_NS_SLOW = 1.0, 1.8


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


def parallel_map(fn, items, threads):
    """fn over items on host threads (the library's ctypes calls release the GIL)."""
    from concurrent.futures import ThreadPoolExecutor

    with ThreadPoolExecutor(max_workers=threads) as ex:
        return list(ex.map(fn, items))


def synth_images(orb, seed, frame_ids, W, H, threads, view=0):
    """(len(frame_ids), H, W) synthetic frames, rendered straight into one array."""
    imgs = np.empty((len(frame_ids), H, W), np.uint8)
    lib = orb.lib()

    def one(i):
        lib.orb_synth_image(seed, frame_ids[i], view, W, H, imgs[i].ctypes.data, W)

    parallel_map(one, range(len(frame_ids)), threads)
    return imgs


def host_cpu():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return model, os.cpu_count()


def snapshot_sample(sets, g_end, n_sets, n_batches, B, orb, per_set=16):
    """Host copies of `per_set` frames of each buffer set as the timed region
    left it: set j holds launch gg's outputs for the last n_sets launches gg
    (batch gg % n_batches).  Returns [(frame index, keypoints, descriptors,
    kp_match, nmatches)]."""
    out = []
    for gg in range(max(0, g_end - n_sets), g_end):  # (a short run may not have used every set)
        st, b = sets[gg % n_sets], gg % n_batches
        for q in range(per_set):
            i = (gg * 389 + q * (B // per_set) + 7) % B
            n = int(st["cnt"][i].item())
            k = st["kps"][i, :max(n, 0)].cpu().numpy().view(orb.KEYPOINT_DTYPE).reshape(-1)
            out.append((b * B + i, k, st["desc"][i, :max(n, 0)].cpu().numpy(),
                        st["match"][i, :max(n, 0)].cpu().numpy(), int(st["nmatch"][i].item())))
    return out


def cpu_leg(imgs, maps, sample, args, scale, timed):
    """The CPU leg: the oracle (checker) recomputes the sampled frames of the
    timed pipeline (extraction + SearchByProjection against the same local map)
    and compares them bit for bit; then, when `timed`, the CPU baseline."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle  # CPU oracle: checker / baseline only

    def check(smp):
        f, k, d, km, nm = smp
        kr, dr, _ = oracle.extract(imgs[f], args.features, 1.2, 8, 20, 7)
        mps, mpd, locked = maps[f]
        n_ref, km_ref = oracle.match_projection_local(kr, dr, scale, args.width, args.height, mps,
                                                      mpd, 1.0, 0.8, locked[: len(kr)])
        ok = (k.tobytes() == kr.tobytes() and d.tobytes() == dr.tobytes() and nm == n_ref
              and np.array_equal(km, km_ref))
        if ok:
            return None
        return {"frame": int(f), "n": int(len(k)), "n_ref": int(len(kr)),
                "keys": k.tobytes() == kr.tobytes(), "desc": d.tobytes() == dr.tobytes(),
                "nmatch": int(nm), "nmatch_ref": int(n_ref),
                "kp_match_diff": int(np.sum(km != km_ref)) if len(km) == len(km_ref) else -1}

    bad = [r for r in parallel_map(check, sample, args.threads) if r is not None]
    if bad:
        print("bench.py parity_sample mismatch:", json.dumps(bad), file=sys.stderr, flush=True)
    par = {"frames": [int(s[0]) for s in sample], "bit_exact": not bad, "mismatched": bad,
           "checked": "keypoints (28 B records, order), descriptors, SearchByProjection "
                      "kp_match and nmatches of frames taken from the timed pipeline's own "
                      "buffers after the timed region, against the CPU oracle"}
    return (cpu_baseline(imgs[:64], maps[:64], args, scale) if timed else None), par


def cpu_baseline(imgs_host, maps, args, scale):
    """The CPU oracle (same C++ restatement the parity tests use; the reference
    itself cannot be built here) on a bounded sample of the same workload: one
    thread pinned to one core, each frame timed alone (extract + match), the
    median frame time reported as frames/s (SURVEY §8(d) method)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle  # CPU oracle: checker / baseline only

    aff = os.sched_getaffinity(0) if hasattr(os, "sched_getaffinity") else None
    core = min(aff) if aff else None
    if core is not None:
        os.sched_setaffinity(0, {core})
    try:
        times = []
        t_start = time.perf_counter()
        n = 0
        while True:
            i = n % len(imgs_host)
            t0 = time.perf_counter()
            k, d, _ = oracle.extract(imgs_host[i], args.features, 1.2, 8, 20, 7)
            mps, mpd, locked = maps[i]
            oracle.match_projection_local(k, d, scale, args.width, args.height, mps, mpd, 1.0, 0.8,
                                          locked[: len(k)])
            t1 = time.perf_counter()
            n += 1
            if n > 3:  # 3 warm-up frames
                times.append(t1 - t0)
            el = t1 - t_start
            if (el >= args.cpu_seconds and len(times) >= 20) or len(times) >= args.cpu_max_frames:
                break
    finally:
        if aff is not None:
            os.sched_setaffinity(0, aff)
    med = float(np.median(times))
    model, ncpu = host_cpu()
    allc = cpu_all_cores(imgs_host, maps, args, scale, oracle) if args.cpu_all_seconds > 0 else None
    return {"value": 1.0 / med, "unit": "frames/s", "cores": 1, "kind": "port",
            "all_cores": allc,
            "sample": f"{len(times)} timed frames (after 3 warm-up) of the same {args.width}x"
                      f"{args.height} stream: oracle ORBextractor ({args.features} feat) + "
                      f"SearchByProjection vs {args.mappoints} map points, C++ -O3 "
                      f"-march=x86-64-v3 -ffp-contract=off, scalar, 1 thread pinned to core "
                      f"{core}; median {med * 1e3:.2f} ms/frame (mean "
                      f"{np.mean(times) * 1e3:.2f}), {el:.1f} s",
            "host_cpu": model, "host_nproc": ncpu}


def cpu_threads():
    """Host threads this process may use: its CPU affinity, capped by
    OMP_NUM_THREADS where the box sets it (the GPU box grants 16 cores and
    sets it to 16; nproc there counts the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(n, omp) if omp > 0 else n)


def cpu_all_cores(imgs_host, maps, args, scale, oracle):
    """The same oracle extract + match on every host thread this process may
    use (one frame per thread at a time, as a CPU deployment would shard the
    sequence), frames/s over a bounded wall-clock sample."""
    import threading

    nthr = cpu_threads()
    done = [0] * nthr
    stop = [False]

    def worker(t):
        i = t
        while not stop[0]:
            f = i % len(imgs_host)
            k, d, _ = oracle.extract(imgs_host[f], args.features, 1.2, 8, 20, 7)
            mps, mpd, locked = maps[f]
            oracle.match_projection_local(k, d, scale, args.width, args.height, mps, mpd, 1.0, 0.8,
                                          locked[: len(k)])
            done[t] += 1
            i += nthr

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(nthr)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    time.sleep(args.cpu_all_seconds)
    n0, t1 = sum(done), time.perf_counter()
    stop[0] = True
    for th in ths:
        th.join()
    return {"value": n0 / (t1 - t0), "unit": "frames/s", "cores": nthr,
            "sample": f"{n0} frames completed in {t1 - t0:.1f} s on {nthr} threads (oracle "
                      "extract + SearchByProjection, one frame per thread at a time; the "
                      "ctypes calls release the GIL)"}


_HIP = None
_STREAMS = {}
# HIP backs streams by a few HSA queues per priority level (GPU_MAX_HW_QUEUES,
# 4 here), and two streams on one queue run in submission order.  The
# library's own streams are least priority and its side stream has an HSA
# queue of its own (a CU-masked stream); the extraction and match streams are
# normal priority, the copy streams high priority (tools/archive/r03/c5_swap.py,
# profiles/r03_streams.txt).  The match streams at the greatest priority ran
# the headline at 315-321k frames/s against 333-334k at normal once the stage
# events left the timed region (the events had been pacing the match stream),
# and C5's two-stream pipeline at 47-48k problems/s against 56-57k with its
# second match stream at normal too (profiles/r05_markers.txt)
_STREAM_PRIO = {"extract": "normal", "match": "normal", "h2d": "greatest", "d2h": "greatest"}
_STREAM_PRIO.update({f"extract{i}": "normal" for i in range(1, 4)})
_STREAM_PRIO.update({f"match{i}": "normal" for i in range(1, 4)})


def _hip(torch):
    global _HIP
    import ctypes
    if _HIP is None:  # torch's own HIP runtime (one runtime per process)
        _HIP = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    return _HIP


def new_stream(torch, dev, key):
    """The bench's stream for `key` (created once per process): a HIP stream of
    the priority _STREAM_PRIO names, or (ORB_BENCH_STREAMS=torch) a torch pool
    stream."""
    import ctypes
    mode = os.environ.get("ORB_BENCH_STREAMS", "prio")
    if mode == "torch":
        return torch.cuda.Stream(dev)
    if key in _STREAMS:
        return _STREAMS[key]
    hip = _hip(torch)
    h = ctypes.c_void_p()
    with torch.cuda.device(dev):
        least, greatest = ctypes.c_int(), ctypes.c_int()
        hip.hipDeviceGetStreamPriorityRange(ctypes.byref(least), ctypes.byref(greatest))
        name = os.environ.get("ORB_BENCH_PRIO_" + key.upper(), _STREAM_PRIO[key])
        prio = {"normal": 0, "least": least.value, "greatest": greatest.value}[name]
        ncu = int(os.environ.get("ORB_BENCH_CUS_" + key.upper(), "0"))  # A/B: a CU-masked stream
        if ncu > 0:
            total = torch.cuda.get_device_properties(dev).multi_processor_count
            step = max(1, total // ncu)
            words = [0] * ((total + 31) // 32)
            for c in range(0, total, step):
                words[c >> 5] |= 1 << (c & 31)
            arr = (ctypes.c_uint32 * len(words))(*words)
            rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(len(words)), arr)
        else:
            rc = hip.hipStreamCreateWithPriority(ctypes.byref(h), ctypes.c_uint(1), ctypes.c_int(prio))
    if rc != 0:
        raise RuntimeError(f"HIP stream creation failed ({rc})")
    _STREAMS[key] = torch.cuda.ExternalStream(h.value, device=dev)  # kept for the process's lifetime
    return _STREAMS[key]


def pipelined(torch, dev, extract, match, n_sets, steps, warmup, lanes=None, match_lanes=1):
    """Seconds per step of `extract(j, stream)` then `match(j, stream)` over
    buffer set j = step % n_sets, pipelined: set j's extraction runs on lane
    j % lanes (a stream of its own; each set has its own extractor handles),
    its match on match stream j % match_lanes, so step k's match overlaps the
    next steps' extraction (and, with two match streams, the next set's match);
    a set is rewritten only after its previous match has finished (events).
    Every step does all of its work."""
    if lanes is None:
        lanes = min(n_sets, max(1, int(os.environ.get("ORB_BENCH_LANES", "2"))))
    ess = [new_stream(torch, dev, "extract" if i == 0 else f"extract{i}") for i in range(lanes)]
    mss = [new_stream(torch, dev, "match" if i == 0 else f"match{i}") for i in range(match_lanes)]
    ext_done = [torch.cuda.Event() for _ in range(n_sets)]
    match_done = [torch.cuda.Event() for _ in range(n_sets)]

    def one(g):
        j = g % n_sets
        es = ess[j % lanes]
        ms = mss[j % match_lanes]
        if g >= n_sets:
            es.wait_event(match_done[j])
        extract(j, es.cuda_stream)
        ext_done[j].record(es)
        ms.wait_event(ext_done[j])
        match(j, ms.cuda_stream)
        match_done[j].record(ms)

    for g in range(warmup):
        one(g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for g in range(warmup, warmup + steps):
        one(g)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


C3_SEED, C5_SEED = 0x4B495454 ^ 3, 5
# buffer sets the C3 / C5 pipelines rotate (each with its own extractor and
# matcher handles): a set is rewritten only after its previous match
_SEC_SETS = int(os.environ.get("ORB_BENCH_SEC_SETS", "4"))


def c3_workload(orb, torch, dev, threads, steps=20, warmup=3, pairs=256):
    """C3: 1241x376 stereo pairs (frames 0..pairs-1 of the C3_SEED sequence,
    left and right views), 2000 features per image, both extractions +
    ComputeStereoMatches, pipelined as `pipelined` (two handle pairs, since
    the stereo match reads both handles' pyramids).  Returns (result, state);
    state holds the inputs and set 0's outputs for parity checks."""
    W, H, P, NF = 1241, 376, pairs, 2000
    bf, fx = 386.1448, 718.856
    ids = list(range(P))
    il = synth_images(orb, C3_SEED, ids, W, H, threads, 0)
    ir = synth_images(orb, C3_SEED, ids, W, H, threads, 1)
    dl, dr = torch.from_numpy(il).to(dev), torch.from_numpy(ir).to(dev)
    z = lambda *sh, dt=torch.int32: torch.zeros(sh, dtype=dt, device=dev)
    sets = []
    for _ in range(_SEC_SETS):
        L = orb.ORBextractor(NF, 1.2, 8, 20, 7, device=dev.index)
        R = orb.ORBextractor(NF, 1.2, 8, 20, 7, device=dev.index)
        cap = L.capacity(W, H)
        sets.append(dict(L=L, R=R, cap=cap, kl=z(P, cap, 7), dl=z(P, cap, 32, dt=torch.uint8),
                         nl=z(P), kr=z(P, cap, 7), dr=z(P, cap, 32, dt=torch.uint8), nr=z(P),
                         ur=z(P, cap, dt=torch.float32), dp=z(P, cap, dt=torch.float32),
                         sad=z(P, cap)))
    # a matcher handle per set: a handle's stereo scratch serves one call at a time
    mts = [orb.ORBmatcher(device=dev.index) for _ in range(len(sets))]

    def extract(j, s):
        st = sets[j]
        st["L"].extract_batch(dl.data_ptr(), P, W, H, W, W * H, st["kl"].data_ptr(),
                              st["dl"].data_ptr(), st["cap"], st["nl"].data_ptr(), s)
        st["R"].extract_batch(dr.data_ptr(), P, W, H, W, W * H, st["kr"].data_ptr(),
                              st["dr"].data_ptr(), st["cap"], st["nr"].data_ptr(), s)

    def match(j, s):
        st = sets[j]
        mts[j].stereo_match_batch(P, st["L"], st["R"], st["kl"].data_ptr(), st["dl"].data_ptr(),
                             st["nl"].data_ptr(), st["kr"].data_ptr(), st["dr"].data_ptr(),
                             st["nr"].data_ptr(), st["cap"], bf, fx, st["ur"].data_ptr(),
                             st["dp"].data_ptr(), st["sad"].data_ptr(), s)

    sec = pipelined(torch, dev, extract, match, _SEC_SETS, steps, warmup,
                    match_lanes=int(os.environ.get("ORB_BENCH_C3_MATCH_LANES", "1")))
    if min(int(torch.minimum(st["nl"], st["nr"]).min().item()) for st in sets) < 0:
        raise RuntimeError("C3: an extraction reported failure (negative count)")
    # the two stages alone, one after another on one stream (set 0)
    s0 = torch.cuda.Stream(dev)
    with torch.cuda.stream(s0):
        esec = timed_loop(lambda: extract(0, s0.cuda_stream), max(5, steps // 4), 2, torch)
        msec = timed_loop(lambda: match(0, s0.cuda_stream), max(5, steps // 4), 2, torch)
    res = {"value": P / sec, "unit": "pairs/s", "pairs_per_step": P, "ms_per_step": sec * 1e3,
           "extraction_only_ms_per_step": esec * 1e3, "stereo_match_only_ms_per_step": msec * 1e3,
           "workload": f"1241x376 stereo pairs (frames 0..{P - 1} of seed {C3_SEED:#x}, left and "
                       "right views), 2000 feat/img, extraction x2 + ComputeStereoMatches, "
                       "pipelined over two extraction lanes and a match stream"}
    return res, dict(il=il, ir=ir, set0=sets[0], bf=bf, fx=fx)


def proj_workload(orb, torch, dev, threads, W, H, NF, M, B, seed, steps=20, warmup=3,
                  serial_calls=0, match_streams2=False):
    """extract + SearchByProjection(F, localMap) against M-point synthetic maps
    (orb_synth_local_map(seed + i, ...)), B problems (frames 0..B-1 of `seed`)
    per launch, pipelined as `pipelined`; also the matcher alone, serial on
    one stream.  Returns (result, state) with set 0's outputs for parity."""
    nsets = _SEC_SETS
    ext = orb.ORBextractor(NF, 1.2, 8, 20, 7, device=dev.index)
    exts = [ext] + [orb.ORBextractor(NF, 1.2, 8, 20, 7, device=dev.index)
                    for _ in range(nsets - 1)]  # one per set
    scale = np.float32(ext.GetScaleFactors())
    cap = ext.capacity(W, H)
    d = torch.from_numpy(synth_images(orb, seed, list(range(B)), W, H, threads)).to(dev)
    z = lambda *sh, dt=torch.int32: torch.zeros(sh, dtype=dt, device=dev)
    sets = [dict(k=z(B, cap, 7), de=z(B, cap, 32, dt=torch.uint8), n=z(B), km=z(B, cap),
                 nm=z(B)) for _ in range(nsets)]
    s0 = torch.cuda.Stream(dev)
    ext.extract_batch(d.data_ptr(), B, W, H, W, W * H, sets[0]["k"].data_ptr(),
                      sets[0]["de"].data_ptr(), cap, sets[0]["n"].data_ptr(), s0.cuda_stream)
    torch.cuda.synchronize()
    kh = sets[0]["k"].cpu().numpy().view(orb.KEYPOINT_DTYPE).reshape(B, cap)
    dh, nh = sets[0]["de"].cpu().numpy(), sets[0]["n"].cpu().numpy()
    maps = parallel_map(lambda i: orb.synth_local_map(seed + i, kh[i, :nh[i]], dh[i, :nh[i]], M,
                                                      W, H), range(B), threads)
    mps = np.stack([mm[0] for mm in maps])
    mpd = np.stack([mm[1] for mm in maps])
    lk = np.zeros((B, cap), np.uint8)
    for i in range(B):
        lk[i, :nh[i]] = maps[i][2]
    d_mps = torch.from_numpy(mps.view(np.uint8).reshape(B, -1)).to(dev)
    d_mpd = torch.from_numpy(mpd).to(dev)
    d_lk = torch.from_numpy(lk).to(dev)
    d_nm = torch.full((B,), M, dtype=torch.int32, device=dev)
    # one matcher handle per buffer set: a handle's scratch serves one call at a
    # time, and two sets' matches may run at once on two streams
    mts = [orb.ORBmatcher(0.8, device=dev.index) for _ in range(nsets)]

    def extract(j, s):
        st = sets[j]
        exts[j].extract_batch(d.data_ptr(), B, W, H, W, W * H, st["k"].data_ptr(),
                              st["de"].data_ptr(), cap, st["n"].data_ptr(), s)

    def match(j, s):
        st = sets[j]
        mts[j].search_by_projection_batch(B, st["k"].data_ptr(), st["de"].data_ptr(),
                                          st["n"].data_ptr(), d_lk.data_ptr(), cap, d_mps.data_ptr(),
                                          d_mpd.data_ptr(), d_nm.data_ptr(), M, W, H, scale, 1.0,
                                          st["km"].data_ptr(), st["nm"].data_ptr(), s)

    sec = pipelined(torch, dev, extract, match, nsets, steps, warmup)
    sec2 = pipelined(torch, dev, extract, match, nsets, steps, warmup, match_lanes=2) \
        if match_streams2 else None
    if min(int(st["n"].min().item()) for st in sets) < 0:
        raise RuntimeError("extract + match: an extraction reported failure (negative count)")
    with torch.cuda.stream(s0):
        msec = timed_loop(lambda: match(0, s0.cuda_stream), steps, warmup, torch)
    msec2 = None
    if match_streams2:
        # the matcher alone with two sets in flight on two streams (set j's
        # resolve, which holds one workgroup per problem, beside set j+1's
        # chip-wide candidate scan)
        s1 = new_stream(torch, dev, "match1")
        ss = [s0.cuda_stream, s1.cuda_stream]
        it = [0]

        def two():
            match(it[0] % 2, ss[it[0] % 2])
            it[0] += 1
        msec2 = timed_loop(two, steps, warmup, torch)
    serial = None
    if serial_calls:
        # latency shape: one call (extraction + match of the B frames) at a time,
        # each waited for before the next is issued; median over the calls
        ts = []
        for i in range(serial_calls + 5):
            t0 = time.perf_counter()
            extract(0, s0.cuda_stream)
            match(0, s0.cuda_stream)
            s0.synchronize()
            if i >= 5:
                ts.append(time.perf_counter() - t0)
        serial = float(np.median(ts))
    n_kp = float(sets[0]["n"].float().mean().item())
    b_lm = 60 * M + 48 * n_kp + 24576  # SURVEY §8(d) B_lm
    # with match_streams2 (C5) the reported schedule is the two-match-stream
    # one: independent problems, a matcher handle per buffer set, each set's
    # SearchByProjection on one of two match streams, so one set's 16-CU
    # resolve runs beside the next set's chip-wide candidate scan
    # (profiles/r05_secsets.txt); the one-stream figures stay beside it
    best, mbest = (sec2, msec2) if match_streams2 else (sec, msec)
    res = {"value": B / best, "unit": "problems/s", "problems_per_step": B, "ms_per_step": best * 1e3,
           "match_only_problems_per_s": B / mbest, "match_only_alg_GBps": b_lm * B / mbest / 1e9,
           "match_only_frac_of_8TBps": b_lm * B / mbest / 8e12, "mean_keypoints": n_kp,
           **({"one_match_stream": {
               "problems_per_s": B / sec, "match_only_problems_per_s": B / msec,
               "note": "every set's SearchByProjection on one match stream (one call at a time)"}}
              if match_streams2 else {}),
           "mean_matches": float(sets[0]["nm"].float().mean().item()),
           **({"serial_ms_per_call": serial * 1e3, "serial_frames_per_s": B / serial,
               "serial_calls": serial_calls} if serial else {}),
           "workload": f"{W}x{H}, {NF} feat, extraction + SearchByProjection vs {M:,} map points "
                       f"(frames 0..{B - 1} of seed {seed}), {B} problems per launch, {nsets} buffer "
                       "sets pipelined over two extraction lanes and "
                       + ("two match streams (a matcher handle per set)" if match_streams2
                          else "a match stream")}
    return res, dict(scale=scale, kh=kh, dh=dh, nh=nh, mps=mps, mpd=mpd, lk=lk, set0=sets[0])


def secondary_configs(orb, torch, args, dev, threads):
    """C3 (stereo pairs/s) and C5 (problems/s at M = 50k), GPU rates only (their
    parity is tests/test_gpu_matchers_more.py and tests/test_gpu_matcher.py;
    tools/bench_configs.py runs the same workloads with an oracle check)."""
    # timed regions of ~0.1 s each: C5's 16-problem steps take ~0.45 ms, and
    # 20 of them measured anywhere from 26k to 34k problems/s on one box
    # (profiles/r03_configs.txt); 200 steps repeat within 0.3 %
    c3, _ = c3_workload(orb, torch, dev, threads, steps=40, warmup=5)
    c5, _ = proj_workload(orb, torch, dev, threads, 1920, 1080, 4000, 50000, 16, C5_SEED,
                          steps=200, warmup=10, match_streams2=True)
    # C4's latency shape (1 frame per GPU per step, batches of 8 over
    # 8 GPUs): one device-resident 1241x376 frame per call, extraction +
    # SearchByProjection vs 5,000 map points, each call waited for; and the
    # 8-frame batch on one GPU the same way
    lat = {}
    for b in (1, 8):
        r, _ = proj_workload(orb, torch, dev, threads, 1241, 376, 1000, 5000, b, 0x4B495454,
                             steps=50, warmup=5, serial_calls=200)
        lat[f"frames_per_call_{b}"] = {k: r[k] for k in ("serial_ms_per_call", "serial_frames_per_s",
                                                          "serial_calls", "mean_keypoints")}
    lat["workload"] = ("1241x376, 1000 feat, extraction + SearchByProjection vs 5,000 map points, "
                       "device-resident, one call at a time (synchronized), median of 200 calls")
    return {"C3_stereo_pairs_per_s": c3, "C5_problems_per_s": c5, "C4_latency": lat}


def host_input_leg(orb, torch, ext, matcher, imgs, args, dev, sets, d_mps, d_mpd, d_lock,
                   d_nmps, scale, cap, dist, rank):
    """The same extract + match pipeline fed from pinned host memory, as a
    drop-in caller pays it (src/Frame.cc:278-285 hands ORBextractor a host
    cv::Mat): each launch's B frames go H2D on a copy stream into one of two
    device slots, double-buffered against the extraction, and every result
    (keypoints, descriptors, counts, match assignments) comes back D2H on a
    second copy stream.  The local maps stay resident.  Frames cycle through
    --host-frames pinned host frames.  Returns rates; never the headline."""
    W, H, B, M = args.width, args.height, args.batch, args.mappoints
    NB = args.frames // B
    nh = min(args.host_frames, len(imgs)) // B * B
    if nh < B:
        return None
    h_img = torch.from_numpy(imgs[:nh]).pin_memory()
    slots = [torch.empty((B, H, W), dtype=torch.uint8, device=dev) for _ in range(2)]
    outs = [dict(kps=torch.empty((B, cap, 7), dtype=torch.int32).pin_memory(),
                 desc=torch.empty((B, cap, 32), dtype=torch.uint8).pin_memory(),
                 cnt=torch.empty(B, dtype=torch.int32).pin_memory(),
                 match=torch.empty((B, cap), dtype=torch.int32).pin_memory()) for _ in range(2)]
    cnts = [torch.zeros(B, dtype=torch.int32, device=dev) for _ in range(2)]
    h2d, d2h = new_stream(torch, dev, "h2d"), new_stream(torch, dev, "d2h")
    es, ms = new_stream(torch, dev, "extract"), new_stream(torch, dev, "match")
    ev = {k: [torch.cuda.Event() for _ in range(2)] for k in ("in", "ext", "match", "out")}
    fb = W * H

    def launch(g):
        j, b, hb = g % 2, g % NB, g % (nh // B)
        st, o = sets[j], outs[j]
        if g >= 2:
            h2d.wait_event(ev["ext"][j])  # slot j's previous frames are extracted
        with torch.cuda.stream(h2d):
            slots[j].copy_(h_img[hb * B:(hb + 1) * B], non_blocking=True)
        ev["in"][j].record(h2d)
        es.wait_event(ev["in"][j])
        if g >= 2:
            es.wait_event(ev["out"][j])  # result set j has been copied out
        ext.extract_batch(slots[j].data_ptr(), B, W, H, W, fb, st["kps"].data_ptr(),
                          st["desc"].data_ptr(), cap, cnts[j].data_ptr(), es.cuda_stream)
        ev["ext"][j].record(es)
        ms.wait_event(ev["ext"][j])
        matcher.search_by_projection_batch(B, st["kps"].data_ptr(), st["desc"].data_ptr(),
                                           cnts[j].data_ptr(), d_lock[b * B].data_ptr(), cap,
                                           d_mps[b * B].data_ptr(), d_mpd[b * B].data_ptr(),
                                           d_nmps.data_ptr(), M, W, H, scale, 1.0,
                                           st["match"].data_ptr(), st["nmatch"].data_ptr(),
                                           ms.cuda_stream)
        ev["match"][j].record(ms)
        d2h.wait_event(ev["match"][j])
        with torch.cuda.stream(d2h):
            o["kps"].copy_(st["kps"], non_blocking=True)
            o["desc"].copy_(st["desc"], non_blocking=True)
            o["cnt"].copy_(cnts[j], non_blocking=True)
            o["match"].copy_(st["match"], non_blocking=True)
        ev["out"][j].record(d2h)

    g = 0
    for _ in range(4):
        launch(g)
        g += 1
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    n = args.host_passes * NB
    t0 = time.perf_counter()
    for _ in range(n):
        launch(g)
        g += 1
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
        el = max_over_ranks(dist, el, dev if args.dist_backend == "nccl" else "cpu")
    if min(int(o["cnt"].min().item()) for o in outs) < 0:
        raise RuntimeError("host-input leg: an extraction reported a failed frame")
    frames = n * B * (dist.get_world_size() if dist is not None else 1)
    out_b = cap * (28 + 32 + 4) + 4
    return {"frames_per_s": frames / el, "unit": "frames/s", "frames": frames, "seconds": el,
            "h2d_GBps": frames * fb / el / 1e9, "d2h_GBps": frames * out_b / el / 1e9,
            "bytes_per_frame": {"h2d": fb, "d2h": out_b},
            "note": "pinned host frames -> H2D (copy stream, two device slots) -> extract -> "
                    "SearchByProjection -> D2H of keypoints, descriptors, counts and matches "
                    "(second copy stream); local maps resident; PCIe-inclusive drop-in rate"}


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """`bench.py --gpus N` from a plain shell: start one rank per GPU as a child
    `torch.distributed.run` (never exec: this process has made no GPU call and
    makes none), relay its output and return its exit code.  The ranks shard
    the frame sequence as the driver loop of Examples/Monocular/mono_kitti.cc:73-119
    would if each GPU took every N-th block of frames."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
           str(n), "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           str(Path(__file__).resolve()), *sys.argv[1:]]
    env = dict(os.environ, ORB_BENCH_LAUNCHED_BY="bench.py --gpus")
    sys.stdout.flush()
    return subprocess.run(cmd, env=env).returncode


def resolve_world(gpus, environ):
    """(world size, launch-children?) for `--gpus` against the launcher's env.
    WORLD_SIZE set: the ranks already exist and must match --gpus (a mismatch is
    an error, not a silent single-GPU run).  Unset and --gpus > 1: start them."""
    ws = environ.get("WORLD_SIZE")
    if ws is not None:
        world = int(ws)
        if gpus is not None and gpus != world:
            raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}; launch one "
                             "rank per GPU (or drop --gpus / WORLD_SIZE)")
        return world, False
    n = 1 if gpus is None else gpus
    if n < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    return n, n > 1


def isolated_kernels(ext, matcher, launch, stream, nb, n, torch):
    """Per-stage HIP-event times with every kernel alone: profile mode 2 runs
    the extraction's stages one after another on the caller's stream (no side
    stream), and the matcher follows on the same stream.  Returns
    ({name: (total ms, launches)}, calls)."""
    torch.cuda.synchronize()
    ext.profile(2)
    matcher.profile(True)
    for i in range(n):
        launch(i % nb, stream)
    torch.cuda.synchronize()
    out = {}
    for st in range(6):
        name, ms, cnt = ext.profile_read(st)
        if cnt:
            out[name] = (ms, cnt)
    for st in range(3):
        name, ms, cnt = matcher.profile_read(st)
        if cnt:
            out[name] = (ms, cnt)
    ext.profile(False)
    matcher.profile(False)
    return out, n


def kernel_table(iso, calls, pipelined_kern, n_prof, alg, batch):
    """Every extraction and match kernel: SURVEY §8(d) algorithmic bytes per
    launch, time per launch alone and pipelined, and the HBM fraction alone."""
    table = {}
    for name, (ms, n) in iso.items():
        per_call = n / calls
        ms_l = ms / n
        b = alg.get(name, 0.0) * batch / per_call
        row = {"launches_per_call": per_call, "ms_per_launch_isolated": ms_l,
               "ms_per_call_isolated": ms / calls, "alg_bytes_per_launch": b,
               "alg_GBps_isolated": b / (ms_l * 1e-3) / 1e9,
               "frac_hbm_isolated": b / (ms_l * 1e-3) / 1e9 / HBM_PEAK_GBS}
        if name in pipelined_kern:
            pm, pn = pipelined_kern[name]
            row["ms_per_call_pipelined"] = pm / n_prof if name.startswith("k_fast") or \
                name in ("k_pyr_resize", "k_octree", "k_orient_desc") else pm / max(pn, 1)
            row["ms_per_launch_pipelined"] = row["ms_per_call_pipelined"] / per_call
        table[name] = row
    return table


HARNESS_DIR = ROOT / "tests" / "integration_run"


def dropin_prepare(args, d, nfr=16, iters=500):
    """The drop-in leg's inputs (child process `bench.py --dropin-prepare DIR`):
    frames 0..nfr-1 of the bench stream (and their right views), each frame's
    5,000-point local map built from its own keypoints exactly as the main
    workload builds it (one-frame extraction, bit-identical to the batch's)."""
    orb = load_package()
    W, H, M = args.width, args.height, args.mappoints
    d = Path(d)
    ids = list(range(nfr))
    imgs = synth_images(orb, args.seed, ids, W, H, 1)
    right = synth_images(orb, args.seed, ids, W, H, 1, view=1)
    ext = orb.ORBextractor(args.features, 1.2, 8, 20, 7)
    tracks, descs = [], []
    for f in ids:
        k, dsc = ext(imgs[f])
        mps, mpd, _ = orb.synth_local_map(args.seed + f, k, dsc, M, W, H)
        tracks.append(np.ascontiguousarray(mps).view(np.uint8).reshape(-1))
        descs.append(np.ascontiguousarray(mpd).reshape(-1))
    imgs.tofile(d / "imgs.bin")
    right.tofile(d / "imgsR.bin")
    np.concatenate(tracks).tofile(d / "tracks.bin")
    np.concatenate(descs).tofile(d / "mpdesc.bin")
    np.asarray(ext.GetScaleFactors(), np.float32).tofile(d / "scale.bin")
    (d / "meta.txt").write_text(f"{W} {H} {args.features} {M} {nfr} {iters} 386.1448 718.856")
    ext.close()


def dropin_leg(args, nfr=16, iters=500):
    """The reference-typed drop-ins (integration/*.cc, linked to the library by
    tests/integration_run) timed at ORB-SLAM2's own granularity, one frame per
    call: mono = ORBextractor::operator() + SearchByProjection(F, vpMapPoints)
    over 5,000 MapPoint objects (Frame::ExtractORB, Tracking::SearchLocalPoints);
    stereo = both extractions on two threads + Frame::ComputeStereoMatches.
    Both harness builds: ORB_AMD_GPU_STEREO (the recommended integration:
    nothing reads mvImagePyramid on the host) and the default (mvImagePyramid
    mirrored to the host every call).  Median wall ms per frame / pair.
    Run first, before this process touches the GPU: the inputs are made by a
    child process, and the harness runs on an otherwise idle GPU, as
    ORB-SLAM2's tracking thread would (after the batch workloads, the same
    binary measured 0.30-0.33 ms per mono frame against 0.28-0.29 alone,
    profiles/r06_dropin.txt)."""
    import subprocess
    import tempfile

    out = {}
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run([sys.executable, str(Path(__file__).resolve()), "--dropin-prepare", d,
                            "--seed", str(args.seed), "--width", str(args.width), "--height",
                            str(args.height), "--features", str(args.features), "--mappoints",
                            str(args.mappoints)], capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            raise RuntimeError(f"dropin inputs: {r.stderr[-1000:]}")
        for key, exe in (("gpu_stereo_build", "dropin_harness_gpustereo"),
                         ("host_pyramid_build", "dropin_harness")):
            path = HARNESS_DIR / exe
            if not path.exists():
                out[key] = f"{path.name} not built (make -C tests/integration_run)"
                continue
            r = subprocess.run([str(path), "time", d], capture_output=True, text=True,
                               timeout=240)
            if r.returncode != 0:
                raise RuntimeError(f"{exe} time: {r.stderr[-1000:]}")
            out[key] = json.loads((Path(d) / "time.json").read_text())
    out["note"] = ("integration/ORBextractor.cc + ORBmatcher.cc (+ FrameStereo.cc) run by "
                   "tests/integration_run/harness.cc with stand-in cv::Mat / Frame / MapPoint, "
                   f"{args.width}x{args.height} frames 0..{nfr - 1} of the bench stream (right "
                   f"views for stereo), {args.features} feat mono / {2 * args.features} per image "
                   f"stereo, SearchByProjection vs {args.mappoints} MapPoint objects per frame, "
                   f"th 1, nnratio 0.8; median of {iters} calls after 3 warm-up; PCIe-inclusive "
                   "(host images in, host keypoints / descriptors / matches out); run before the "
                   "bench's workloads, on an idle GPU")
    return out


def timed_loop(fn, steps, warmup, torch):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks, one per GPU); > 1 without WORLD_SIZE starts the ranks "
                         "with torch.distributed.run (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=60,
                    help="timed steps; one step = one pass over the --frames resident frames")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--frames", type=int, default=8192,
                    help="distinct resident frames per GPU (a step processes each once)")
    ap.add_argument("--batch", type=int, default=1024,
                    help="frames per extraction launch (capped at --frames)")
    ap.add_argument("--width", type=int, default=1241)
    ap.add_argument("--height", type=int, default=376)
    ap.add_argument("--features", type=int, default=1000)
    ap.add_argument("--mappoints", type=int, default=5000)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-max-frames", type=int, default=400)
    ap.add_argument("--iso-launches", type=int, default=8,
                    help="extract + match calls timed with every kernel alone (kernel table)")
    ap.add_argument("--bounded", action="store_true",
                    help="the host queues a buffer set's next launch only once its previous one is "
                         "matched (at most one launch per set in flight)")
    ap.add_argument("--timed-events", choices=("off", "ext", "match", "both"), default="off",
                    help="record the per-stage HIP events inside the timed region (A/B; default: "
                         "in a profiled pipelined pass after it)")
    ap.add_argument("--cpu-all-seconds", type=float, default=8.0,
                    help="wall-clock sample of the all-cores oracle rate (0: skip)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="skip the C3 / C5 extra keys")
    ap.add_argument("--dropin-prepare", metavar="DIR", help=argparse.SUPPRESS)
    ap.add_argument("--no-dropin", action="store_true",
                    help="skip the per-frame drop-in timing (tests/integration_run harness)")
    ap.add_argument("--threads", type=int, default=16, help="host threads for input synthesis")
    ap.add_argument("--seed", type=int, default=0x4B495454)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL, the measured path); gloo only for the multi-rank test "
                         "on one GPU (ORB_BENCH_DEVICE pins every rank to one device)")
    ap.add_argument("--host-frames", type=int, default=2048,
                    help="pinned host frames the host-input leg cycles through (0: skip the leg)")
    ap.add_argument("--host-passes", type=int, default=4,
                    help="timed passes of the host-input leg over --frames frames")
    ap.add_argument("--lanes", type=int, default=int(os.environ.get("ORB_BENCH_LANES", "2")),
                    help="extraction lanes: extractor handles on streams of their own, "
                         "taking launches round-robin (1 / 2 / 3 / 4 lanes: 307k / 315k / "
                         "305k / 296k frames/s, profiles/r03_lanes.txt)")
    ap.add_argument("--match-streams", type=int,
                    default=int(os.environ.get("ORB_BENCH_MATCH_STREAMS", "1")),
                    help="match streams (each with a matcher handle of its own) taking the "
                         "launches' SearchByProjection round-robin")
    ap.add_argument("--lane-match", default=os.environ.get("ORB_BENCH_LANE_MATCH", "stream"),
                    choices=["stream", "inlane"],
                    help="matcher on one match stream, or on each lane's own stream after "
                         "its extraction")
    args = ap.parse_args()

    if args.dropin_prepare:  # child of dropin_leg
        dropin_prepare(args, args.dropin_prepare)
        return
    world, spawn = resolve_world(args.gpus, os.environ)
    if spawn:  # before any torch / HIP call in this process
        raise SystemExit(launch_ranks(world))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dropin = None
    if rank == 0 and world == 1 and not args.no_dropin and local == 0 \
            and os.environ.get("ORB_BENCH_DEVICE") is None:
        dropin = dropin_leg(args)  # first: before this process touches the GPU
    import torch

    if os.environ.get("ORB_BENCH_DEVICE") is not None:
        local = int(os.environ["ORB_BENCH_DEVICE"])
    torch.cuda.set_device(local)
    dist = None
    # a torchrun launch initialises the process group even at world size 1, so
    # the RCCL gather runs (and is verified) on a single GPU too
    if world > 1 or "TORCHELASTIC_RUN_ID" in os.environ or "MASTER_ADDR" in os.environ:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    orb = load_package()
    D = args.frames
    args.batch = min(args.batch, D)
    W, H, B, NF, M = args.width, args.height, args.batch, args.features, args.mappoints
    if D % B:
        raise SystemExit("--frames must be a multiple of --batch")
    NB = D // B

    # ---------------- inputs: this rank's shard of the synthetic sequence, in HBM
    frames = shard_frames(rank, D)
    imgs = synth_images(orb, args.seed, frames, W, H, args.threads)
    ext = orb.ORBextractor(NF, 1.2, 8, 20, 7, device=local)
    scale = np.float32(ext.GetScaleFactors())
    cap = ext.capacity(W, H)
    dev = torch.device("cuda", local)
    # Two streams, two buffer sets: launch g's SearchByProjection (matcher
    # stream) overlaps launch g+1's extraction (extract stream).  Launch g
    # writes buffer set g % 2 once the matcher of launch g - 2 (the set's
    # previous reader) has finished; its matcher starts once it is done.
    L = max(1, args.lanes)
    ext_streams = [new_stream(torch, dev, "extract" if i == 0 else f"extract{i}") for i in range(L)]
    ext_stream = ext_streams[0]
    match_stream = new_stream(torch, dev, "match")
    MSN = max(1, args.match_streams)
    # every stream the run uses, created up front in one order (HIP maps a new
    # stream onto the least-used HSA queue of its priority, so the mapping
    # depends on creation order; profiles/r05_secsets.txt)
    for key in ("match1", "h2d", "d2h"):
        new_stream(torch, dev, key)
    exts = [ext] + [orb.ORBextractor(NF, 1.2, 8, 20, 7, device=local) for _ in range(L - 1)]
    match_streams = [match_stream] + [new_stream(torch, dev, f"match{i}") for i in range(1, MSN)]
    torch.cuda.set_stream(ext_stream)
    d_img = torch.from_numpy(imgs).to(dev)
    NS = 2 * L  # buffer sets: launch g writes set g % NS
    sets = [dict(kps=torch.zeros((B, cap, 7), dtype=torch.int32, device=dev),
                 desc=torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev),
                 cnt=torch.zeros(B, dtype=torch.int32, device=dev),
                 match=torch.zeros((B, cap), dtype=torch.int32, device=dev),
                 nmatch=torch.zeros(B, dtype=torch.int32, device=dev))
            for _ in range(NS)]
    # every frame's keypoint count of a step, double-buffered over steps (the
    # step's one all-gather reads buffer k % 2 while step k + 1 writes the other)
    step_counts = [torch.zeros(D, dtype=torch.int32, device=dev) for _ in range(2)]
    gathered = [torch.zeros(world * D, dtype=torch.int32, device=dev) for _ in range(2)]
    extracted = [torch.cuda.Event() for _ in range(NS)]
    matched = [torch.cuda.Event() for _ in range(NS)]
    frame_bytes = W * H

    def extract(st, batch, stream):
        ext.extract_batch(d_img.data_ptr() + batch * B * frame_bytes, B, W, H, W, frame_bytes,
                          st["kps"].data_ptr(), st["desc"].data_ptr(), cap, st["cnt"].data_ptr(),
                          stream.cuda_stream)

    # untimed pass: every frame's local map is derived from its own keypoints
    kps_h = np.zeros((D, cap), orb.KEYPOINT_DTYPE)
    desc_h = np.zeros((D, cap, 32), np.uint8)
    cnt_h = np.zeros(D, np.int32)
    for b in range(NB):
        extract(sets[0], b, ext_stream)
        torch.cuda.synchronize()
        kps_h[b * B:(b + 1) * B] = sets[0]["kps"].cpu().numpy().view(orb.KEYPOINT_DTYPE).reshape(B, cap)
        desc_h[b * B:(b + 1) * B] = sets[0]["desc"].cpu().numpy()
        cnt_h[b * B:(b + 1) * B] = sets[0]["cnt"].cpu().numpy()
    if cnt_h.min() < 0:  # the extractor marks an image it could not finish with a negative count
        raise RuntimeError(f"extraction failed on {int((cnt_h < 0).sum())} frame(s)")
    maps = parallel_map(lambda i: orb.synth_local_map(args.seed + frames[i], kps_h[i, :cnt_h[i]],
                                                      desc_h[i, :cnt_h[i]], M, W, H),
                        range(D), args.threads)
    mps_all = np.stack([mm[0] for mm in maps])
    mpd_all = np.stack([mm[1] for mm in maps])
    lock_all = np.zeros((D, cap), np.uint8)
    for i in range(D):
        lock_all[i, :cnt_h[i]] = maps[i][2]
    d_mps = torch.from_numpy(mps_all.view(np.uint8).reshape(D, -1)).to(dev)
    d_mpd = torch.from_numpy(mpd_all).to(dev)
    d_lock = torch.from_numpy(lock_all).to(dev)
    d_nmps = torch.full((B,), M, dtype=torch.int32, device=dev)
    del mpd_all, lock_all
    matcher = orb.ORBmatcher(0.8, device=local)
    inlane = args.lane_match == "inlane"
    matchers = [matcher] + [orb.ORBmatcher(0.8, device=local)
                            for _ in range(L - 1 if inlane else MSN - 1)]
    torch.cuda.synchronize()

    def launch(g):
        j, b, ln = g % NS, g % NB, g % L
        st = sets[j]
        es = ext_streams[ln]
        ms = es if inlane else match_streams[g % MSN]
        mt = matchers[ln] if inlane else matchers[g % MSN]
        cnt = step_counts[(g // NB) % 2][b * B:(b + 1) * B]
        st["cnt"] = cnt
        if g >= NS and args.bounded:
            # the host waits for set j's previous launch (g - NS) to be matched
            # before it queues the next use of the set: at most NS launches in flight
            matched[j].synchronize()
        if g >= NS and not inlane:
            es.wait_event(matched[j])
        exts[ln].extract_batch(d_img.data_ptr() + b * B * frame_bytes, B, W, H, W, frame_bytes,
                               st["kps"].data_ptr(), st["desc"].data_ptr(), cap, cnt.data_ptr(),
                               es.cuda_stream)
        if not inlane:
            extracted[j].record(es)
            ms.wait_event(extracted[j])
        mt.search_by_projection_batch(B, st["kps"].data_ptr(), st["desc"].data_ptr(),
                                      cnt.data_ptr(), d_lock[b * B].data_ptr(), cap,
                                      d_mps[b * B].data_ptr(), d_mpd[b * B].data_ptr(),
                                      d_nmps.data_ptr(), M, W, H, scale, 1.0,
                                      st["match"].data_ptr(), st["nmatch"].data_ptr(),
                                      ms.cuda_stream)
        if dist is not None and b == NB - 1:  # one RCCL all-gather of the step's counts
            k = (g // NB) % 2
            # every lane's launches of the step are done before the gather
            for o in range(1, L if inlane else 1):
                matched[(j - o) % NS].record(ext_streams[(ln - o) % L])
                ms.wait_event(matched[(j - o) % NS])
            for o in range(1, 1 if inlane else MSN):  # the other match streams' last launches
                ms.wait_event(matched[(j - o) % NS])
            with torch.cuda.stream(ms):
                gather_counts(dist, step_counts[k], gathered[k])
        matched[j].record(ms)

    g = 0
    for k in range(args.warmup):
        for _ in range(NB):
            launch(g)
            g += 1
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    # stage events (the pipelined kernel table) go in a profiled pass after the
    # timed region, so no event record sits between the timed kernels
    # (--timed-events: inside it, the round-4 / round-5 layout)
    if args.timed_events in ("ext", "both"):
        ext.profile(True)
    if args.timed_events in ("match", "both"):
        matcher.profile(True)
    # diagnostic (ORB_BENCH_STEP_EVENTS=1, never in the driver's run): one
    # timing event per step on the stream of its last match, and the host's
    # clock when it has queued each step
    step_diag = os.environ.get("ORB_BENCH_STEP_EVENTS") == "1"
    step_ev, host_q = [], []
    t0 = time.perf_counter()
    g_first = g
    for k in range(args.steps):
        for _ in range(NB):
            launch(g)
            g += 1
        if step_diag:
            e = torch.cuda.Event(enable_timing=True)
            e.record(ext_streams[(g - 1) % L] if inlane else match_streams[(g - 1) % MSN])
            step_ev.append(e)
            host_q.append(time.perf_counter())
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist is not None:
        dist.barrier()
    elapsed = t1 - t0
    if dist is not None:
        elapsed = max_over_ranks(dist, elapsed, dev if args.dist_backend == "nccl" else "cpu")
    if min(int(c.min().item()) for c in step_counts) < 0:
        raise RuntimeError("extraction reported a failed frame (negative count)")
    # every lane's last-step keypoint counts equal the untimed pass's
    last_k = ((g - 1) // NB) % 2
    counts_ok = bool(torch.equal(step_counts[last_k].cpu(), torch.from_numpy(cnt_h)))
    if not counts_ok:
        raise RuntimeError("timed-step keypoint counts differ from the untimed pass")
    # the timed pipeline's own outputs for 64 sampled frames of its last launches
    # (keypoints, descriptors, matches), checked against the oracle in the CPU leg
    sample = snapshot_sample(sets, g, NS, NB, B, orb)
    gather_ok = None
    if dist is not None:  # the gathered counts of the last step hold this rank's own
        k = ((g - 1) // NB) % 2
        mine = gathered[k][rank * D:(rank + 1) * D]
        gather_ok = bool(torch.equal(mine, step_counts[k])) and bool(
            torch.equal(step_counts[k].cpu(), torch.from_numpy(cnt_h)))
        ok = torch.tensor([1 if gather_ok else 0], dtype=torch.int32)
        if args.dist_backend == "nccl":
            ok = ok.to(dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        gather_ok = bool(ok.item())

    if args.timed_events != "both":
        # the profiled pipelined pass: the same launches, stage events on
        prof_steps = max(2, min(args.steps, 6))
        ext.profile(False)  # (drops whatever the timed region recorded)
        matcher.profile(False)
        ext.profile(True)
        matcher.profile(True)
        g_first = g
        for k in range(prof_steps):
            for _ in range(NB):
                launch(g)
                g += 1
        torch.cuda.synchronize()
    # per-kernel HIP-event times over the timed region (or the profiled pass
    # after it), each on its own stream.
    # The extract stream is the critical path (the matcher stream runs in its
    # shadow, so matcher kernel times include time-sharing with the next
    # launch's extraction): the roofline kernel is the longest extraction kernel.
    # the profiled handle is lane 0's: it ran every L-th launch of the region
    n_prof = max(1, sum(1 for gg in range(g_first, g) if gg % L == 0))
    kern, ext_kern = {}, []
    for st in range(6):
        name, ms, n = ext.profile_read(st)
        if n == 0:
            continue  # stage not run (k_blur_levels: split A/B mode only)
        kern[name] = (ms, n)
        ext_kern.append(name)
    # FAST of level 0 and levels 1-2 runs as launches of its own on the side
    # stream (beside the resize chain): one pass of the kernel = all its launches
    # (summed durations, counted once per call)
    side_ms = {}
    for name in [k for k in ext_kern if k.endswith("_side")]:
        ms0, _ = kern.pop(name)
        ext_kern.remove(name)
        side_ms[name] = ms0 / n_prof
        base = name[:-5]
        if base in kern:
            ms1, n1 = kern[base]
            kern[base] = (ms0 + ms1, n1)
    _, call_ms, call_n = ext.profile_read(6)  # whole extraction call, start to join
    for st in range(3):
        name, ms, n = matcher.profile_read(st)
        kern[name] = (ms, n)
    ext.profile(False)
    matcher.profile(False)
    n_kp = float(cnt_h.mean())
    nmatch = float(sets[0]["nmatch"].float().mean().item())
    rl = kern.get("k_pyr_resize", (0, 0))[1] / max(n_prof, 1)
    alg = algorithmic_bytes(W, H, scale, 8, n_kp, M, resize_launches=round(rl) if rl else None)
    # every kernel alone (one stream, every stage after the previous one, no
    # side stream): kernel-only launch times for the roofline and the per-kernel
    # table; the pipelined HIP-event times above stay beside them
    def launch_iso(b, stream):
        st = sets[0]
        ext.extract_batch(d_img.data_ptr() + b * B * frame_bytes, B, W, H, W, frame_bytes,
                          st["kps"].data_ptr(), st["desc"].data_ptr(), cap, st["cnt"].data_ptr(),
                          stream.cuda_stream)
        matcher.search_by_projection_batch(B, st["kps"].data_ptr(), st["desc"].data_ptr(),
                                           st["cnt"].data_ptr(), d_lock[b * B].data_ptr(), cap,
                                           d_mps[b * B].data_ptr(), d_mpd[b * B].data_ptr(),
                                           d_nmps.data_ptr(), M, W, H, scale, 1.0,
                                           st["match"].data_ptr(), st["nmatch"].data_ptr(),
                                           stream.cuda_stream)

    iso, iso_calls = isolated_kernels(ext, matcher, launch_iso, ext_stream, NB, args.iso_launches,
                                      torch)
    table = kernel_table(iso, iso_calls, kern, n_prof, alg, B)
    # the roofline kernel: the longest kernel per call when each runs alone,
    # among the kernels SURVEY §8(d) assigns algorithmic bytes
    dom = max((k for k in table if table[k]["alg_bytes_per_launch"] > 0),
              key=lambda k: table[k]["ms_per_call_isolated"])
    # (and the longest kernel of all, with the kernels left out for having no
    # §8(d) bytes, so a byte-less bottleneck cannot drop out silently)
    longest = max(table, key=lambda k: table[k]["ms_per_call_isolated"])
    no_bytes = {k: table[k]["ms_per_call_isolated"] for k in table
                if not table[k]["alg_bytes_per_launch"] > 0}
    t = table[dom]
    dom_ms_per_launch = t["ms_per_launch_isolated"]
    dom_bytes = t["alg_bytes_per_launch"]
    hbm_gbs = t["alg_GBps_isolated"]
    traffic, traffic_src = measured_traffic(dom, B)
    valu = valu_issue(dom, B, dom_ms_per_launch)
    total_frames = D * args.steps * world
    # the HBM roofline of the dominant kernel is the primary
    # fraction (algorithmic bytes per launch / its launch time alone); its VALU
    # issue rate against the guide's peak sits beside it (the integer kernels of
    # this path are instruction-bound, not bandwidth-bound: DESIGN.md §4)
    roof = {"kernel": dom, "bound": "hbm", "achieved": hbm_gbs, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": hbm_gbs / HBM_PEAK_GBS, "bytes_per_launch": dom_bytes,
            "bytes_note": f"SURVEY §8(d) algorithmic bytes of {dom} ({alg[dom]:.0f} B/frame) x "
                          f"{B} frames / {t['launches_per_call']:g} launch(es) per call",
            "timing": f"HIP events around each launch, kernels run one after another on one "
                      f"stream ({iso_calls} calls after the timed region); "
                      "`ms_per_launch_pipelined` is the same kernel in a profiled pass of the timed pipeline's "
                      "launches after the timed region "
                      "(time-shared with the other lane and the matcher)"}
    if valu is not None:
        rate = valu["valu_instr_per_launch"] / (dom_ms_per_launch * 1e-3) / 1e9
        roof["valu"] = {"achieved": rate, "peak": VALU_PEAK_G, "unit": "G wave-instructions/s",
                        "frac": rate / VALU_PEAK_G,
                        "note": f"peak = {N_SIMD} SIMDs x {CLOCK_GHZ} GHz / {VALU_CYCLES} cycles per "
                                "wave64 VALU instruction (MI355X_MICROARCH.md); SQ_INSTS_VALU per "
                                "launch from " + valu["source"].split(" ")[0],
                        "issue_bound": valu}
    roof.update({
        "traffic": traffic,
        "traffic_source": f"profiles/{traffic_src} (rocprofv3 FETCH_SIZE x 2 (gfx950 "
                          "calibration, profiles/r02_fetch_calib.txt) + WRITE_SIZE, separate "
                          "passes)" if traffic_src else None,
        "ms_per_launch": dom_ms_per_launch,
        "ms_per_launch_pipelined": t.get("ms_per_launch_pipelined"),
        # the same bytes over the kernel's time inside the pipeline (profiled pass)
        # (time-shared with the other lane and the matcher)
        "frac_pipelined": (dom_bytes / (t["ms_per_launch_pipelined"] * 1e-3) / 1e9 / HBM_PEAK_GBS
                           if t.get("ms_per_launch_pipelined") else None),
        # `bound` names the roofline the contract prices against (HBM: no MFMA
        # work on this path); `limiter` is what holds the kernel below it
        "limiter": "latency",
        "binding_limit": "memory latency per wave, not HBM bandwidth: the kernel moves ~1.07x its "
                         "algorithmic bytes at `frac` of the HBM roof and issues VALU at "
                         "`valu.frac` of peak (DESIGN.md §4)",
        "longest_kernel_isolated": {"kernel": longest,
                                    "ms_per_call": table[longest]["ms_per_call_isolated"]},
        "kernels_without_alg_bytes": no_bytes,
    })
    host = None
    if args.host_frames > 0:
        del d_img
        host = host_input_leg(orb, torch, ext, matcher, imgs, args, dev, sets, d_mps, d_mpd,
                              d_lock, d_nmps, scale, cap, dist, rank)
    if dist is None:
        par = "single rank; no collective (one process, one GPU)"
    else:
        par = (f"frames sharded over {world} rank(s); one "
               f"{'RCCL' if args.dist_backend == 'nccl' else 'gloo'} all-gather of the step's "
               f"per-frame keypoint counts per step")
    if step_diag:
        gpu_ms = [step_ev[i - 1].elapsed_time(step_ev[i]) for i in range(1, len(step_ev))]
        host_ms = [(host_q[i] - t0) * 1e3 for i in range(len(host_q))]
        print(json.dumps({"step_diag": {"gpu_step_ms": [round(v, 3) for v in gpu_ms],
                                        "host_queued_ms": [round(v, 2) for v in host_ms]}}),
              file=sys.stderr)
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
            "frames_per_gpu_per_step": D,
            "distinct_frames_per_gpu": D,
            "frames_per_launch": B,
            "extraction_lanes": f"{L} extractor handle(s) on {L} stream(s), launches "
                                "round-robin; SearchByProjection on " +
                                ("one match stream" if MSN == 1 else
                                 f"{MSN} match streams (a matcher handle each), launches round-robin"),
            "timed_region_s": elapsed,
            "inputs": "frames resident in HBM before the timed region (device-resident rate; "
                      "the PCIe-inclusive drop-in rate is `host_input`)",
            "parallelism": par,
            "count_gather_verified": gather_ok,
            "mean_keypoints_per_frame": n_kp,
            "mean_matches_per_frame": nmatch,
        },
        "roofline": roof,
        "kernels_ms_per_launch": {k: v[0] / max(v[1], 1) for k, v in kern.items()},
        "kernels": table,
        "extraction_kernels_ms_per_launch": sum(kern[k][0] for k in ext_kern) / n_prof,
        "extraction_call_ms_per_launch": call_ms / max(call_n, 1),
        "fast_side_stream_ms_per_launch": side_ms,
        "host_input": host,
    }
    if rank == 0 and world == 1 and not args.no_secondary:
        if args.host_frames <= 0:
            del d_img
        result.update(secondary_configs(orb, torch, args, dev, args.threads))
    if dropin is not None:
        result["dropin"] = dropin
    parity_ok = True
    if rank == 0:
        cpu_b, par = cpu_leg(imgs, maps, sample, args, scale, world == 1 and not args.no_cpu)
        result["parity_sample"] = par
        parity_ok = par["bit_exact"]
        if cpu_b is not None:
            result["cpu_baseline"] = cpu_b
            if isinstance(result.get("dropin"), dict):
                result["dropin"]["cpu_oracle_frame_ms"] = 1e3 / cpu_b["value"]
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    if not parity_ok:
        raise SystemExit("bench.py: the timed pipeline's sampled outputs differ from the oracle")


if __name__ == "__main__":
    main()
