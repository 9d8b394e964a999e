"""GPU timeline of the mono drop-in (integration/ORBextractor.cc +
ORBmatcher.cc through tests/integration_run/harness.cc `time`), per frame:
which part of the wall time is DMA, kernels, or neither (host work and
launch / wake-up latency).

  prepare DIR [--frames 16 --iters 100]   inputs for `harness time DIR`
                                          (touches the GPU: run it as its
                                          own process, before the profiler)
  analyze ROCPROF_DIR                     kernel + memory-copy (+ HIP API)
                                          traces of rocprofv3 --kernel-trace
                                          --memory-copy-trace [--hip-trace]
                                          --output-format csv

A frame = the image's DMA in (the op before the first pyramid kernel of an
extraction) up to the next frame's; the mono loop's frames only (--iters).
"""
import argparse
import csv
import glob
import statistics
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "tests"))


def prepare(a):
    from conftest import load_pkg
    orb = load_pkg()
    W, H, NF, M = 1241, 376, 1000, 5000
    d = Path(a.dir)
    d.mkdir(parents=True, exist_ok=True)
    ext = orb.ORBextractor(NF, 1.2, 8, 20, 7)
    imgs = np.stack([orb.synth_image(a.seed, f, W, H) for f in range(a.frames)])
    right = np.stack([orb.synth_image(a.seed, f, W, H, view=1) for f in range(a.frames)])
    tracks, descs = [], []
    for f in range(a.frames):
        k, dsc = ext(imgs[f])
        mps, mpd, _ = orb.synth_local_map(a.seed + f, k, dsc, M, W, H)
        tracks.append(np.ascontiguousarray(mps).view(np.uint8).reshape(-1))
        descs.append(np.ascontiguousarray(mpd).reshape(-1))
    imgs.tofile(d / "imgs.bin")
    right.tofile(d / "imgsR.bin")
    np.concatenate(tracks).tofile(d / "tracks.bin")
    np.concatenate(descs).tofile(d / "mpdesc.bin")
    np.asarray(ext.GetScaleFactors(), np.float32).tofile(d / "scale.bin")
    (d / "meta.txt").write_text(f"{W} {H} {NF} {M} {a.frames} {a.iters} 386.1448 718.856")
    print(f"prepared {a.frames} frames, {a.iters} iterations in {d}")


def rows_of(pattern):
    out = []
    for p in glob.glob(pattern, recursive=True):
        out += list(csv.DictReader(open(p)))
    return out


def analyze(a):
    ks = rows_of(f"{a.dir}/**/*kernel_trace.csv")
    cs = rows_of(f"{a.dir}/**/*memory_copy_trace.csv")
    ev = []
    for r in ks:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   r["Kernel_Name"].split("(")[0].split("<")[0][:28]))
    for r in cs:
        kind = r.get("Direction") or r.get("Operation") or r.get("Kind") or "copy"
        size = int(r.get("Size") or r.get("Bytes") or 0)
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   f"{'H2D' if 'HOST_TO_DEVICE' in kind.upper() or 'H2D' in kind.upper() else 'D2H' if 'DEVICE_TO_HOST' in kind.upper() or 'D2H' in kind.upper() else kind}:{size}"))
    ev.sort()
    # a frame opens with the image's DMA in: the op just before the first
    # pyramid kernel of each extraction
    starts = []
    for i, e in enumerate(ev):
        if "k_pyr_resize" in e[2] and i > 0 and "k_pyr_resize" not in ev[i - 1][2]:
            starts.append(i - 1)
    frames = []
    for j, i0 in enumerate(starts[:a.iters + 3]):  # the mono loop: warm-up + iters frames
        i1 = starts[j + 1] if j + 1 < len(starts) else len(ev)
        frames.append(ev[i0:i1])
    frames = frames[3:]  # warm-up
    if not frames:
        print("no frames found")
        return
    names = [e[2] for e in frames[len(frames) // 2]]
    print(f"{len(frames)} frames; sequence of the median frame: {names}")
    per = {}
    for g in frames:
        t0 = g[0][0]
        pe = t0
        busy = 0
        for k, (s, e, n) in enumerate(g):
            key = f"{k:02d} {n}"
            per.setdefault(key, {"dur": [], "gap": [], "off": []})
            per[key]["dur"].append((e - s) / 1e3)
            per[key]["gap"].append((s - pe) / 1e3)
            per[key]["off"].append((s - t0) / 1e3)
            busy += max(0, e - max(s, pe))
            pe = max(pe, e)
        per.setdefault("_span", []).append((pe - t0) / 1e3)
        per.setdefault("_busy", []).append(busy / 1e3)
    print("step                              start   dur   gap-before  (us, median over frames)")
    for key in sorted(k for k in per if not k.startswith("_")):
        v = per[key]
        if len(v["dur"]) < len(frames) // 2:
            continue
        print(f"{key:32s} {statistics.median(v['off']):7.1f} {statistics.median(v['dur']):6.1f} "
              f"{statistics.median(v['gap']):7.1f}")
    print(f"GPU span first..last op {statistics.median(per['_span']):.1f} us, "
          f"busy {statistics.median(per['_busy']):.1f} us")
    # frame period = start-to-start (the harness runs frames back to back)
    period = [(frames[i + 1][0][0] - frames[i][0][0]) / 1e3 for i in range(len(frames) - 1)]
    if period:
        print(f"frame period (start to start) median {statistics.median(period):.1f} us")
    # host API calls (rocprofv3 --hip-trace) beside the GPU work of one frame
    api = rows_of(f"{a.dir}/**/*hip_api_trace.csv")
    if api and len(frames) > 2:
        k = len(frames) // 2
        t0, t1 = frames[k][0][0], frames[k + 1][0][0]
        win = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "api " + r["Function"])
               for r in api if t0 - 20_000 <= int(r["Start_Timestamp"]) < t1]
        win += [(s, e, "gpu " + n) for s, e, n in frames[k]]
        print(f"-- frame {k}: host API calls and GPU work, us from its first GPU op")
        for s, e, n in sorted(win):
            print(f"  {(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {n}")


def main():
    ap = argparse.ArgumentParser()
    sp = ap.add_subparsers(dest="cmd", required=True)
    p = sp.add_parser("prepare")
    p.add_argument("dir")
    p.add_argument("--frames", type=int, default=16)
    p.add_argument("--iters", type=int, default=100)
    p.add_argument("--seed", type=int, default=5)
    z = sp.add_parser("analyze")
    z.add_argument("dir")
    z.add_argument("--iters", type=int, default=100, help="the mono loop's iterations (meta.txt)")
    a = ap.parse_args()
    prepare(a) if a.cmd == "prepare" else analyze(a)


if __name__ == "__main__":
    main()
