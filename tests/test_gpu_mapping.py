"""GPU SearchForInitialization and ComputeDistinctiveDescriptors
against the CPU oracle: assignments index-exact, vbPrevMatched bit-exact."""
import numpy as np
import pytest

import scenarios

pytestmark = pytest.mark.gpu


def _init_both(gpu, oracle, s, window, nnratio=0.9, check=True):
    ref = oracle.search_for_initialization(s["k1"], s["d1"], s["k2"], s["d2"], s["w"], s["h"],
                                           s["prev"], window, nnratio, check)
    m = gpu.ORBmatcher(nnratio, check)
    F1 = gpu.Frame(s["k1"], s["d1"], np.ones(8, np.float32), s["w"], s["h"])
    F2 = gpu.Frame(s["k2"], s["d2"], np.ones(8, np.float32), s["w"], s["h"])
    got = m.SearchForInitialization(F1, F2, s["prev"], window)
    return ref, got


@pytest.mark.parametrize("seed,frame2,w,h", [(0, 1, 640, 480), (4, 2, 640, 480),
                                             (2, 1, 1241, 376), (9, 3, 1241, 376)])
def test_search_for_initialization(gpu, oracle, seed, frame2, w, h):
    s = scenarios.init_pair(oracle, seed, frame2, w=w, h=h, nf=2000)
    (rn, rm, rp), (n, m12, prev) = _init_both(gpu, oracle, s, 100)
    assert rn > 20
    assert n == rn
    assert np.array_equal(m12, rm), np.nonzero(m12 != rm)[0][:10]
    assert prev.tobytes() == rp.tobytes()


@pytest.mark.parametrize("window,check", [(10, True), (50, False), (400, True), (2000, False)])
def test_search_for_initialization_windows(gpu, oracle, window, check):
    # window 2000 covers the frame: every level-0 keypoint is a candidate
    # (> INIT_LIST of them -> the whole-window rescan path)
    s = scenarios.init_pair(oracle, 6, 1, w=640, h=480, nf=2000)
    (rn, rm, rp), (n, m12, prev) = _init_both(gpu, oracle, s, window, 0.9, check)
    assert n == rn and np.array_equal(m12, rm) and prev.tobytes() == rp.tobytes()


def test_search_for_initialization_collisions(gpu, oracle):
    # few distinct descriptors in a small area: steals, vMatchedDistance skips,
    # batch conflicts and exhausted top-K lists on almost every query
    rng = np.random.default_rng(11)
    n1, n2 = 700, 500
    k1 = np.zeros(n1, oracle.KEYPOINT_DTYPE)
    k2 = np.zeros(n2, oracle.KEYPOINT_DTYPE)
    for k, n in ((k1, n1), (k2, n2)):
        k["x"] = rng.uniform(200, 260, n)
        k["y"] = rng.uniform(200, 260, n)
        k["angle"] = rng.uniform(0, 360, n)
        k["octave"] = np.where(rng.random(n) < 0.8, 0, 1)
    base = rng.integers(0, 256, (12, 32), dtype=np.uint8)
    d1 = base[rng.integers(0, 12, n1)].copy()
    d2 = base[rng.integers(0, 12, n2)].copy()
    for d in (d1, d2):
        bits = np.unpackbits(d, axis=1)
        bits ^= (rng.random(bits.shape) < rng.uniform(0, 0.12, (len(d), 1))).astype(np.uint8)
        d[:] = np.packbits(bits, axis=1)
    prev = np.stack([k1["x"], k1["y"]], 1) + rng.uniform(-5, 5, (n1, 2)).astype(np.float32)
    s = dict(k1=k1, d1=d1, k2=k2, d2=d2, prev=prev.astype(np.float32), w=640, h=480)
    for window, check in ((20, True), (40, False), (100, True)):
        (rn, rm, rp), (n, m12, p) = _init_both(gpu, oracle, s, window, 0.9, check)
        assert rn > 5
        assert n == rn and np.array_equal(m12, rm) and p.tobytes() == rp.tobytes()


def test_search_for_initialization_unstaged(gpu, oracle):
    # more level-0 F2 keypoints than the LDS stage holds: global grid scan path
    rng = np.random.default_rng(12)
    n = 2600
    k1 = np.zeros(n, oracle.KEYPOINT_DTYPE)
    k2 = np.zeros(n, oracle.KEYPOINT_DTYPE)
    for k in (k1, k2):
        k["x"] = rng.uniform(0, 640, n)
        k["y"] = rng.uniform(0, 480, n)
        k["angle"] = rng.uniform(0, 360, n)
    base = rng.integers(0, 256, (40, 32), dtype=np.uint8)
    d1 = base[rng.integers(0, 40, n)].copy()
    d2 = base[rng.integers(0, 40, n)].copy()
    for d in (d1, d2):
        bits = np.unpackbits(d, axis=1)
        bits ^= (rng.random(bits.shape) < 0.05).astype(np.uint8)
        d[:] = np.packbits(bits, axis=1)
    s = dict(k1=k1, d1=d1, k2=k2, d2=d2, prev=np.stack([k1["x"], k1["y"]], 1), w=640, h=480)
    (rn, rm, rp), (got_n, m12, p) = _init_both(gpu, oracle, s, 30, 0.9, True)
    assert rn > 10
    assert got_n == rn and np.array_equal(m12, rm) and p.tobytes() == rp.tobytes()


def test_search_for_initialization_empty(gpu, oracle):
    m = gpu.ORBmatcher(0.9, True)
    s = scenarios.init_pair(oracle, 1, 1, w=640, h=480, nf=500)
    F1 = gpu.Frame(s["k1"], s["d1"], np.ones(8, np.float32), 640, 480)
    F0 = gpu.Frame(s["k1"][:0], s["d1"][:0], np.ones(8, np.float32), 640, 480)
    n, m12, prev = m.SearchForInitialization(F1, F0, s["prev"], 100)
    assert n == 0 and (m12 == -1).all() and prev.tobytes() == s["prev"].tobytes()
    n, m12, prev = m.SearchForInitialization(F0, F1, s["prev"][:0], 100)
    assert n == 0 and len(m12) == 0


def test_search_for_initialization_batch(gpu, oracle):
    torch = pytest.importorskip("torch")
    pairs = [scenarios.init_pair(oracle, 20 + i, 1 + i % 3, w=640, h=480, nf=2000)
             for i in range(5)]
    stride = max(max(len(s["k1"]), len(s["k2"])) for s in pairs)
    P = len(pairs)
    K1 = np.zeros((P, stride), oracle.KEYPOINT_DTYPE)
    K2 = np.zeros((P, stride), oracle.KEYPOINT_DTYPE)
    D1 = np.zeros((P, stride, 32), np.uint8)
    D2 = np.zeros((P, stride, 32), np.uint8)
    PR = np.zeros((P, stride, 2), np.float32)
    n1 = np.array([len(s["k1"]) for s in pairs], np.int32)
    n2 = np.array([len(s["k2"]) for s in pairs], np.int32)
    for i, s in enumerate(pairs):
        K1[i, :n1[i]], D1[i, :n1[i]], PR[i, :n1[i]] = s["k1"], s["d1"], s["prev"]
        K2[i, :n2[i]], D2[i, :n2[i]] = s["k2"], s["d2"]
    dev = "cuda"
    t = {k: torch.from_numpy(np.ascontiguousarray(v).view(np.uint8)).to(dev)
         for k, v in dict(K1=K1, K2=K2, D1=D1, D2=D2, PR=PR, n1=n1, n2=n2).items()}
    m12 = torch.full((P, stride), -7, dtype=torch.int32, device=dev)
    nm = torch.zeros(P, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    gpu.ORBmatcher(0.9, True).search_for_initialization_batch(
        P, t["K1"].data_ptr(), t["D1"].data_ptr(), t["n1"].data_ptr(), t["K2"].data_ptr(),
        t["D2"].data_ptr(), t["n2"].data_ptr(), stride, 0.0, 640.0, 0.0, 480.0, 100,
        t["PR"].data_ptr(), m12.data_ptr(), nm.data_ptr())
    torch.cuda.synchronize()
    prev = t["PR"].cpu().numpy().view(np.float32).reshape(P, stride, 2)
    m12, nm = m12.cpu().numpy(), nm.cpu().numpy()
    for i, s in enumerate(pairs):
        rn, rm, rp = oracle.search_for_initialization(s["k1"], s["d1"], s["k2"], s["d2"], 640,
                                                      480, s["prev"], 100, 0.9, True)
        assert nm[i] == rn
        assert np.array_equal(m12[i, :n1[i]], rm)
        assert prev[i, :n1[i]].tobytes() == rp.tobytes()


def test_distinctive_descriptors(gpu, oracle):
    rng = np.random.default_rng(3)
    offs, desc = scenarios.observation_sets(rng, 2000)
    ref = oracle.distinctive_descriptors(offs, desc)
    init = rng.integers(0, 256, (2000, 32), dtype=np.uint8)
    best, out = gpu.ORBmatcher().ComputeDistinctiveDescriptors(offs, desc, init)
    assert np.array_equal(best, ref)
    has = np.diff(offs) > 0
    assert (np.diff(offs) > 64).any()  # long lists take the chunked path
    assert np.array_equal(out[has], desc[offs[:-1][has] + ref[has]])
    assert np.array_equal(out[~has], init[~has])  # empty lists: untouched


def test_distinctive_descriptors_batch(gpu, oracle):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(5)
    offs, desc = scenarios.observation_sets(rng, 5000, max_obs=12)
    ref = oracle.distinctive_descriptors(offs, desc)
    dev = "cuda"
    d_offs = torch.from_numpy(offs).to(dev)
    d_desc = torch.from_numpy(desc).to(dev)
    d_best = torch.full((5000,), -7, dtype=torch.int32, device=dev)
    d_out = torch.zeros((5000, 32), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    gpu.ORBmatcher().distinctive_descriptors_batch(5000, d_offs.data_ptr(), d_desc.data_ptr(),
                                                   d_best.data_ptr(), d_out.data_ptr())
    torch.cuda.synchronize()
    best = d_best.cpu().numpy()
    assert np.array_equal(best, ref)
    has = ref >= 0
    assert np.array_equal(d_out.cpu().numpy()[has], desc[offs[:-1][has] + ref[has]])
