"""GPU Hamming matcher parity against the CPU oracle (exact integers / indices)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frame(gpu, oracle, w, h, nf, seed):
    img = gpu.synth_image(seed, 0, w, h)
    k, d, _ = oracle.extract(img, nf)
    scale = oracle.params(nf)["scale"]
    return k, d, scale


def test_hamming_batch(gpu):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(0)
    n = 100_003
    a = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    b = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    b[0] = a[0]
    b[1] = ~a[1]
    b[2] = a[2] ^ np.eye(1, 32, 5, dtype=np.uint8)[0]
    ref = np.unpackbits(a ^ b, axis=1).sum(1).astype(np.int32)
    m = gpu.ORBmatcher()
    da, db = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    m.hamming_batch(da.data_ptr(), db.data_ptr(), n, out.data_ptr())
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert got[0] == 0 and got[1] == 256 and got[2] == 1
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("w,h,nf,M,th,seed", [
    (1241, 376, 1000, 5000, 1.0, 0),   # headline workload (C4)
    (640, 480, 1000, 3000, 3.0, 1),
    (640, 480, 1000, 3000, 5.0, 2),
    (1920, 1080, 4000, 50000, 1.0, 5),  # C5
])
def test_search_by_projection_local(gpu, oracle, w, h, nf, M, th, seed):
    k, d, scale = _frame(gpu, oracle, w, h, nf, seed)
    mps, mpd, locked = oracle.synth_local_map(seed, k, d, M, w, h)
    n_ref, km_ref = oracle.match_projection_local(k, d, scale, w, h, mps, mpd, th, 0.8, locked)
    F = gpu.Frame(k, d, scale, w, h)
    n_gpu, km_gpu = gpu.ORBmatcher(0.8).SearchByProjection(F, mps, mpd, th, locked)
    assert n_gpu == n_ref
    assert np.array_equal(km_gpu, km_ref), np.nonzero(km_gpu != km_ref)[0][:10]
    assert n_ref > 0


@pytest.mark.parametrize("M,nsrc", [(4000, 40), (24000, 120)])
def test_search_by_projection_conflicts_and_flags(gpu, oracle, M, nsrc):
    """Many map points on few keypoints (deep first-come chains, top-K overflow),
    points without observations (claims that do not lock), bad / out-of-view
    points, stereo gating through mvuRight.  24,000 points take the
    fixed-point resolve (local maps of 20,000 points and more), 4,000 the
    256-point prefix windows."""
    w, h = 640, 480
    k, d, scale = _frame(gpu, oracle, w, h, 1000, 3)
    rng = np.random.default_rng(7)
    mps = np.zeros(M, oracle.MP_TRACK_DTYPE)
    src = rng.integers(0, nsrc, M)  # M points onto nsrc keypoints
    mps["proj_x"] = k["x"][src] + rng.uniform(-2, 2, M).astype(np.float32)
    mps["proj_y"] = k["y"][src] + rng.uniform(-2, 2, M).astype(np.float32)
    mps["proj_xr"] = mps["proj_x"] - rng.uniform(5, 40, M).astype(np.float32)
    mps["level"] = np.minimum(k["octave"][src] + rng.integers(0, 2, M), 7)
    mps["view_cos"] = np.where(rng.random(M) < 0.5, 0.999, 0.9).astype(np.float32)
    mps["in_view"] = rng.random(M) < 0.97
    mps["bad"] = rng.random(M) < 0.02
    mps["has_obs"] = rng.random(M) < 0.8
    mpd = d[src].copy()
    flips = rng.random((M, 256)) < 0.1
    mpd ^= np.packbits(flips, axis=1, bitorder="little")
    ur = np.where(rng.random(len(k)) < 0.5, k["x"] - rng.uniform(5, 40, len(k)), -1).astype(np.float32)
    locked = (rng.random(len(k)) < 0.1).astype(np.uint8)
    for th in (1.0, 3.0):
        n_ref, km_ref = oracle.match_projection_local(k, d, scale, w, h, mps, mpd, th, 0.8, locked, ur)
        F = gpu.Frame(k, d, scale, w, h, u_right=ur)
        n_gpu, km_gpu = gpu.ORBmatcher(0.8).SearchByProjection(F, mps, mpd, th, locked)
        assert n_gpu == n_ref
        assert np.array_equal(km_gpu, km_ref)


def test_search_by_projection_large_frame(gpu, oracle):
    """More than 8,192 keypoints: the one-wave grid build, the candidate scan
    over the global grid (no LDS staging past 4,096 keypoints) and, with
    20,000+ map points, the 512-point prefix resolve (the fixed-point kernel's
    claim buffers would exceed 64 KiB of LDS)."""
    w, h = 1920, 1080
    rng = np.random.default_rng(1080)
    img = rng.integers(0, 256, (h, w), dtype=np.uint8)
    k, d, _ = oracle.extract(img, 12000, 1.2, 8, 20, 7)
    assert len(k) > 8192
    scale = oracle.params(12000)["scale"]
    mps, mpd, locked = oracle.synth_local_map(11, k, d, 20000, w, h)
    n_ref, km_ref = oracle.match_projection_local(k, d, scale, w, h, mps, mpd, 1.0, 0.8, locked)
    F = gpu.Frame(k, d, scale, w, h)
    n_gpu, km_gpu = gpu.ORBmatcher(0.8).SearchByProjection(F, mps, mpd, 1.0, locked)
    assert n_ref > 0
    assert n_gpu == n_ref
    assert np.array_equal(km_gpu, km_ref)


def test_search_by_projection_empty(gpu, oracle):
    w, h = 640, 480
    k, d, scale = _frame(gpu, oracle, w, h, 1000, 1)
    F = gpu.Frame(k, d, scale, w, h)
    n, km = gpu.ORBmatcher(0.8).SearchByProjection(F, np.zeros(0, oracle.MP_TRACK_DTYPE),
                                                   np.zeros((0, 32), np.uint8), 1.0)
    assert n == 0 and (km == -1).all()
    F0 = gpu.Frame(k[:0], d[:0], scale, w, h)
    mps, mpd, _ = oracle.synth_local_map(1, k, d, 100, w, h)
    n, km = gpu.ORBmatcher(0.8).SearchByProjection(F0, mps, mpd, 1.0)
    assert n == 0 and len(km) == 0
