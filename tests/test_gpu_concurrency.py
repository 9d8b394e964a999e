"""Thread-safety of the drop-in boundary (include/orb_abi.h: handles are
independent; a handle serialises its own calls).  The reference runs two
ORBextractor instances concurrently for every stereo frame (src/Frame.cc:81-84)
and builds ORBmatcher objects on the Tracking, LocalMapping and LoopClosing
threads at once.  ctypes releases the GIL inside every call, so these threads
really do overlap on the device."""
import threading

import numpy as np
import pytest

import scenarios

pytestmark = pytest.mark.gpu


def _run_threads(fns):
    errors = []

    def wrap(fn):
        try:
            fn()
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(e)

    ts = [threading.Thread(target=wrap, args=(f,)) for f in fns]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errors, errors


def test_two_extractors_in_parallel_threads(gpu):
    # Frame's stereo constructor: left and right extractors on two threads
    left = [gpu.synth_image(30, f, 1241, 376) for f in range(6)]
    right = [gpu.synth_image(30, f, 1241, 376, view=1) for f in range(6)]
    ref_ext = gpu.ORBextractor(2000, 1.2, 8, 20, 7)
    ref = {("L", i): ref_ext(im) for i, im in enumerate(left)}
    ref.update({("R", i): ref_ext(im) for i, im in enumerate(right)})
    got = {}
    exL, exR = gpu.ORBextractor(2000, 1.2, 8, 20, 7), gpu.ORBextractor(2000, 1.2, 8, 20, 7)

    def run(ext, side, imgs):
        def f():
            for i, im in enumerate(imgs):
                got[(side, i)] = ext(im)
        return f

    _run_threads([run(exL, "L", left), run(exR, "R", right)])
    for key, (k, d) in ref.items():
        assert got[key][0].tobytes() == k.tobytes() and got[key][1].tobytes() == d.tobytes(), key


def test_shared_matcher_handle_from_many_threads(gpu):
    # one handle, four threads (its mutex serialises the calls)
    w, h = 1241, 376
    img = gpu.synth_image(5, 0, w, h)
    ext = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    k, d = ext(img)
    scale = np.float32(ext.GetScaleFactors())
    mps, mpd, locked = gpu.synth_local_map(5, k, d, 3000, w, h)
    m = gpu.ORBmatcher(0.8)
    F = gpu.Frame(k, d, scale, w, h)
    ref = m.SearchByProjection(F, mps, mpd, 1.0, locked)
    out = [None] * 4

    def job(i):
        def f():
            for _ in range(5):
                out[i] = m.SearchByProjection(F, mps, mpd, 1.0, locked)
        return f

    _run_threads([job(i) for i in range(4)])
    for o in out:
        assert o[0] == ref[0] and np.array_equal(o[1], ref[1])


def test_vocabulary_handle_from_many_threads(gpu, oracle):
    v = scenarios.vocabulary(rng_seed=3, k=10, L=4)
    voc = gpu.ORBVocabulary(v["k"], v["L"], v["parent"], v["leaf"], v["desc"], v["weight"])
    feats = [scenarios.vocab_features(v, 1000, rng_seed=i) for i in range(4)]
    refs = [oracle.vocab_transform(v, f, 4) for f in feats]
    got = [None] * 4

    def job(i):
        def f():
            for _ in range(5):
                got[i] = voc.transform(feats[i], 4)
        return f

    _run_threads([job(i) for i in range(4)])
    for g, r in zip(got, refs):
        assert np.array_equal(g[0], r[0]) and np.array_equal(g[1].view(np.uint64), r[1].view(np.uint64))
        assert all(np.array_equal(a, b) for a, b in zip(g[2], r[2:5]))


def test_graph_capture_beside_another_handle(gpu):
    """extract_batch is graph-capturable (include/orb_abi.h) while another
    handle on the same device keeps running batches on another thread: the
    captured handle forks its side work onto a stream of its own during the
    capture, so the other handle's side-stream launches never join the graph,
    and both give the same results as uncaptured calls."""
    import torch
    W, H, B = 1241, 376, 8
    imgs = np.stack([gpu.synth_image(40, f, W, H) for f in range(B)])
    d = torch.from_numpy(imgs).cuda()
    ha, hb = gpu.ORBextractor(1000, 1.2, 8, 20, 7), gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    cap = ha.capacity(W, H)

    def bufs():
        return (torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda"),
                torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda"),
                torch.zeros(B, dtype=torch.int32, device="cuda"))

    a, b = bufs(), bufs()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()

    def call(h, o, s):
        h.extract_batch(d.data_ptr(), B, W, H, W, W * H, o[0].data_ptr(), o[1].data_ptr(), cap,
                        o[2].data_ptr(), s.cuda_stream)

    call(ha, a, sa)
    call(hb, b, sb)
    torch.cuda.synchronize()
    ref = [t.clone() for t in a]
    assert int(ref[2].min()) > 0
    stop = threading.Event()
    errors = []

    def other():
        try:
            while not stop.is_set():
                call(hb, b, sb)
                sb.synchronize()
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(e)

    t = threading.Thread(target=other)
    t.start()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, stream=sa, capture_error_mode="relaxed"):
            call(ha, a, sa)
    finally:
        stop.set()
        t.join(timeout=60)
    assert not errors, errors
    for x in a:
        x.zero_()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    for x, r in zip(a, ref):
        assert torch.equal(x, r)
    for x, r in zip(b, ref):
        assert torch.equal(x, r)


_CONTENTION_CHILD = r"""
import sys, threading, time, json
import numpy as np, torch
sys.path.insert(0, ROOT); sys.path.insert(0, ROOT + '/tests')
from conftest import load_pkg
orb = load_pkg()
# the caller's start-up, as ORB-SLAM2's: extractors used from two threads
# (Frame's stereo constructor) and a matcher, before any stream of its own
pre = [orb.ORBextractor(2000, 1.2, 8, 20, 7) for _ in range(3)]
m = orb.ORBmatcher(0.8)
imgs0 = [orb.synth_image(30, f, 1241, 376) for f in range(4)]
for im in imgs0:
    pre[0](im)
ts = [threading.Thread(target=lambda h=h: [h(im) for im in imgs0]) for h in pre[1:]]
for t in ts: t.start()
for t in ts: t.join()
W, H, B = 1241, 376, 128
imgs = np.stack([orb.synth_image(41, f, W, H) for f in range(B)])
d = torch.from_numpy(imgs).cuda()
ext = orb.ORBextractor(1000, 1.2, 8, 20, 7)
cap = ext.capacity(W, H)
k = torch.zeros((B, cap, 7), dtype=torch.int32, device='cuda')
de = torch.zeros((B, cap, 32), dtype=torch.uint8, device='cuda')
n = torch.zeros(B, dtype=torch.int32, device='cuda')
s = torch.cuda.Stream(priority=-1)  # the caller's extraction stream: high priority
def rate():
    for _ in range(3):
        ext.extract_batch(d.data_ptr(), B, W, H, W, W * H, k.data_ptr(), de.data_ptr(), cap, n.data_ptr(), s.cuda_stream)
    s.synchronize()
    best = 0.0
    for _ in range(5):
        t0 = time.perf_counter()
        for _ in range(10):
            ext.extract_batch(d.data_ptr(), B, W, H, W, W * H, k.data_ptr(), de.data_ptr(), cap, n.data_ptr(), s.cuda_stream)
        s.synchronize()
        best = max(best, 10 * B / (time.perf_counter() - t0))
    return best
r0 = rate()
ref = n.clone()
probe = torch.cuda.Stream()
cycles = 1 << 20
with torch.cuda.stream(probe):
    torch.cuda._sleep(cycles); probe.synchronize()
    t0 = time.perf_counter(); torch.cuda._sleep(cycles); probe.synchronize()
cycles = max(1 << 16, int(cycles * 2e-3 / max(time.perf_counter() - t0, 1e-6)))
extra = [torch.cuda.Stream() for _ in range(8)]  # normal priority, as a caller's
stop = threading.Event()
spins = [0] * len(extra)
def busy(i):
    with torch.cuda.stream(extra[i]):
        while not stop.is_set():
            torch.cuda._sleep(cycles); torch.cuda._sleep(cycles)
            spins[i] += 2
            extra[i].synchronize()
ths = [threading.Thread(target=busy, args=(i,)) for i in range(len(extra))]
for t in ths: t.start()
try:
    time.sleep(0.05)
    r1 = rate()
finally:
    stop.set()
    for t in ths: t.join(timeout=60)
torch.cuda.synchronize()
print(json.dumps({"idle": r0, "busy": r1, "spins": min(spins), "same": bool(torch.equal(n, ref)),
                  "cycles": cycles}))
"""


def test_batch_rate_with_extra_caller_streams(gpu):
    """A caller that keeps many streams of its own busy (ORB-SLAM2 runs
    extractors and matchers on three threads) must not push the batch
    extraction into a slow mode.  HIP backs a process's streams by a few HSA
    queues per priority level (GPU_MAX_HW_QUEUES, 4) and maps a new stream
    onto the least-used queue of its level; two streams on one queue run in
    submission order.  The batch path forks level 0's FAST (then levels 1-2)
    onto the device's shared side stream, and every handle's own stream is
    created at the least priority too, so no library stream takes a queue from
    the caller's normal- or high-priority pools (runtime.cpp create_own_stream:
    three normal-priority streams created at start-up, by any code, halved a
    later high-priority stream's rate beside busy normal streams,
    profiles/r05_contention.txt).  In a fresh process (the queue mapping
    depends on every stream the process ever created): extractors used from
    two threads and a matcher at start-up, then a 128-frame batch on a
    high-priority caller stream, idle and while 8 caller threads keep 8
    normal-priority streams busy with 2 ms one-thread spin kernels
    (torch.cuda._sleep: a queue they share is blocked, the chip is not).  The
    busy rate must stay within 15 % of the idle rate: a library stream on a
    caller's queue would wait ~2 ms behind a spin kernel per call (a call of
    128 frames takes ~0.5 ms)."""
    import json
    import os
    import subprocess
    import sys
    from pathlib import Path
    root = str(Path(__file__).resolve().parents[1])
    r = subprocess.run([sys.executable, "-c", f"ROOT = {root!r}\n" + _CONTENTION_CHILD],
                       capture_output=True, text=True, timeout=150, env=dict(os.environ))
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["spins"] > 0 and out["same"], out  # every caller stream ran; results unchanged
    assert out["busy"] > 0.85 * out["idle"], out


_EXIT_CHILD = r"""
import sys
import numpy as np, torch
sys.path.insert(0, ROOT); sys.path.insert(0, ROOT + '/tests')
from conftest import load_pkg
orb = load_pkg()
W, H, B = 640, 480, 8   # B >= 4: the batch forks level 0's FAST onto the side stream
imgs = np.stack([orb.synth_image(5, f, W, H) for f in range(B)])
d = torch.from_numpy(imgs).cuda()
ext = orb.ORBextractor(500, 1.2, 8, 20, 7)
cap = ext.capacity(W, H)
k = torch.zeros((B, cap, 7), dtype=torch.int32, device='cuda')
de = torch.zeros((B, cap, 32), dtype=torch.uint8, device='cuda')
n = torch.zeros(B, dtype=torch.int32, device='cuda')
ext.extract_batch(d.data_ptr(), B, W, H, W, W * H, k.data_ptr(), de.data_ptr(), cap, n.data_ptr())
torch.cuda.synchronize()
assert int(n.min()) > 0
print('child done', flush=True)
"""


def test_clean_exit_under_kernel_trace(gpu, tmp_path):
    """The shared side stream is a CU-masked stream; left to the HIP runtime's
    own teardown it crashed the process at exit under rocprofv3 --kernel-trace
    (SIGSEGV in __cxa_finalize, profiles/r05_exit_crash.txt).  The library now
    releases it from an exit handler: a child that runs a side-stream batch
    and exits under the kernel tracer must exit 0."""
    import os
    import shutil
    import subprocess
    import sys
    from pathlib import Path
    prof = shutil.which("rocprofv3")
    if prof is None:
        pytest.skip("rocprofv3 not on PATH")
    root = str(Path(__file__).resolve().parents[1])
    env = dict(os.environ, TMPDIR="/tmp")
    r = subprocess.run([prof, "--kernel-trace", "-d", str(tmp_path / "trace"), "-o", "run",
                        "--output-format", "csv", "--", sys.executable, "-c",
                        f"ROOT = {root!r}\n" + _EXIT_CHILD],
                       capture_output=True, text=True, timeout=150, env=env, cwd="/tmp")
    assert "child done" in r.stdout, r.stderr[-2000:]
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
