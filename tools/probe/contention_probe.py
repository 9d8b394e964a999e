"""Batch extraction rate while caller streams are kept busy (queue-sharing probe).

One configuration per process (ORB_AMD_LIB selects a library variant):
  python tools/probe/contention_probe.py --busy 8 --busy-prio normal --prio high
prints one JSON line: idle rate, rate with `--busy` caller threads each keeping
one stream of `--busy-prio` priority busy with ~2 ms one-thread spin kernels.
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "tests"))
from conftest import load_pkg  # noqa: E402

PRIO = {"high": -1, "normal": 0}


def pre_calls(orb, mode):
    """Single-frame extractions before the measurement (two: three handles, two
    threads, as test_two_extractors_in_parallel_threads)."""
    imgs = [orb.synth_image(30, f, 1241, 376) for f in range(6)]
    if mode == "two":
        hs = [orb.ORBextractor(2000, 1.2, 8, 20, 7) for _ in range(3)]
        for im in imgs:
            hs[0](im)
        ts = [threading.Thread(target=lambda h=h: [h(im) for im in imgs]) for h in hs[1:]]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    elif mode == "twoseq":
        hs = [orb.ORBextractor(2000, 1.2, 8, 20, 7) for _ in range(3)]
        for h in hs:
            for im in imgs:
                h(im)
    elif mode == "one":
        h = orb.ORBextractor(2000, 1.2, 8, 20, 7)
        for im in imgs:
            h(im)
    elif mode in ("raw3", "raw3keep", "raw3idle"):
        # three HIP streams of the process's own (normal priority), each given a
        # kernel unless idle, destroyed unless keep: is it the library or any stream?
        import torch
        hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
        x = torch.zeros(1 << 16, device="cuda")
        hs = []
        for _ in range(3):
            h = ctypes.c_void_p()
            assert hip.hipStreamCreateWithFlags(ctypes.byref(h), ctypes.c_uint(1)) == 0
            hs.append(h)
            if mode != "raw3idle":
                with torch.cuda.stream(torch.cuda.ExternalStream(h.value)):
                    x.add_(1.0)
        torch.cuda.synchronize()
        if mode != "raw3keep":
            for h in hs:
                hip.hipStreamDestroy(h)
        pre_calls.keep = hs
    elif mode == "handles":
        hs = [orb.ORBextractor(2000, 1.2, 8, 20, 7) for _ in range(3)]
        del hs
    elif mode:
        raise SystemExit(f"unknown --pre {mode}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--busy", type=int, default=8)
    ap.add_argument("--busy-prio", default="normal")
    ap.add_argument("--prio", default="high", help="priority of the extraction stream")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--spin-ms", type=float, default=2.0)
    ap.add_argument("--tag", default="")
    ap.add_argument("--pre", default="", help="two | twoseq | one | handles: work before the run")
    ap.add_argument("--workload", default="extract", help="extract | torch (elementwise loop)")
    ap.add_argument("--torch-first", action="store_true",
                    help="create torch's stream pools before the first extractor handle")
    a = ap.parse_args()
    import torch
    if a.torch_first:
        torch.cuda.Stream()
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    lo, hi = ctypes.c_int(), ctypes.c_int()
    hip.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi))
    orb = load_pkg()
    pre_calls(orb, a.pre)
    W, H, B = 1241, 376, a.batch
    imgs = np.stack([orb.synth_image(41, f, W, H) for f in range(B)])
    d = torch.from_numpy(imgs).cuda()
    ext = orb.ORBextractor(1000, 1.2, 8, 20, 7)
    cap = ext.capacity(W, H)
    k = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
    de = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(B, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream(priority=PRIO[a.prio])
    xa = torch.randn(2048, 2048, device="cuda")

    def call():
        if a.workload == "torch":
            with torch.cuda.stream(s):
                for _ in range(4):
                    xa.mul_(1.0001)
        else:
            ext.extract_batch(d.data_ptr(), B, W, H, W, W * H, k.data_ptr(), de.data_ptr(), cap,
                              n.data_ptr(), s.cuda_stream)

    def rate():
        for _ in range(3):
            call()
        s.synchronize()
        best = 0.0
        for _ in range(5):
            t0 = time.perf_counter()
            for _ in range(10):
                call()
            s.synchronize()
            best = max(best, 10 * B / (time.perf_counter() - t0))
        return best

    r0 = rate()
    probe = torch.cuda.Stream()
    cycles = 1 << 20
    with torch.cuda.stream(probe):
        torch.cuda._sleep(cycles)
        probe.synchronize()
        t0 = time.perf_counter()
        torch.cuda._sleep(cycles)
        probe.synchronize()
    cycles = max(1 << 12, int(cycles * a.spin_ms * 1e-3 / max(time.perf_counter() - t0, 1e-6)))
    extra = [torch.cuda.Stream(priority=PRIO[a.busy_prio]) for _ in range(a.busy)]
    stop = threading.Event()

    def busy(i):
        with torch.cuda.stream(extra[i]):
            while not stop.is_set():
                torch.cuda._sleep(cycles)
                torch.cuda._sleep(cycles)
                extra[i].synchronize()

    ths = [threading.Thread(target=busy, args=(i,)) for i in range(a.busy)]
    for t in ths:
        t.start()
    try:
        time.sleep(0.05)
        r1 = rate()
    finally:
        stop.set()
        for t in ths:
            t.join(timeout=60)
    torch.cuda.synchronize()
    print(json.dumps({"tag": a.tag, "busy": a.busy, "busy_prio": a.busy_prio, "prio": a.prio,
                      "batch": B, "prio_range": [lo.value, hi.value], "pre": a.pre,
                      "workload": a.workload, "torch_first": a.torch_first, "idle": r0,
                      "busy_rate": r1, "ratio": r1 / r0}), flush=True)


if __name__ == "__main__":
    main()
