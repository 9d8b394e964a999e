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
    points, stereo gating through mvuRight.  One problem per call, so the
    default schedule takes the fixed-point resolve at both sizes; the prefix
    kernels are held to the same maps in
    test_search_by_projection_resolve_schedules and test_gpu_headline.py."""
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
    """More than 13,568 keypoints: the four-wave grid build, the candidate scan
    over the global grid (no LDS staging past 4,096 keypoints) and, with
    20,000+ map points, the 512-thread prefix resolve k_proj_resolve<8> (the
    fixed-point kernel's claim buffers, 12 B per keypoint, would exceed the
    160 KB of LDS)."""
    w, h = 1920, 1080
    rng = np.random.default_rng(1080)
    img = rng.integers(0, 256, (h, w), dtype=np.uint8)
    k, d, _ = oracle.extract(img, 15000, 1.2, 8, 20, 7)
    assert len(k) * 12 > 160 * 1024 - 1024
    scale = oracle.params(15000)["scale"]
    mps, mpd, locked = oracle.synth_local_map(11, k, d, 20000, w, h)
    n_ref, km_ref = oracle.match_projection_local(k, d, scale, w, h, mps, mpd, 1.0, 0.8, locked)
    F = gpu.Frame(k, d, scale, w, h)
    m = gpu.ORBmatcher(0.8)
    assert m.resolve_kernel(1, len(k), len(mps)) == "k_proj_resolve<8>"
    n_gpu, km_gpu = m.SearchByProjection(F, mps, mpd, 1.0, locked)
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


def _conflict_map(oracle, k, d, M, nsrc, seed=7):
    rng = np.random.default_rng(seed)
    mps = np.zeros(M, oracle.MP_TRACK_DTYPE)
    src = rng.integers(0, nsrc, M)
    mps["proj_x"] = k["x"][src] + rng.uniform(-2, 2, M).astype(np.float32)
    mps["proj_y"] = k["y"][src] + rng.uniform(-2, 2, M).astype(np.float32)
    mps["proj_xr"] = -1.0
    mps["level"] = np.minimum(k["octave"][src] + rng.integers(0, 2, M), 7)
    mps["view_cos"] = np.where(rng.random(M) < 0.5, 0.999, 0.9).astype(np.float32)
    mps["in_view"] = rng.random(M) < 0.97
    mps["bad"] = rng.random(M) < 0.02
    mps["has_obs"] = rng.random(M) < 0.8
    mpd = d[src].copy()
    mpd ^= np.packbits(rng.random((M, 256)) < 0.1, axis=1, bitorder="little")
    locked = (rng.random(len(k)) < 0.1).astype(np.uint8)
    return mps, mpd, locked


def test_search_by_projection_batch_large_maps(gpu, oracle):
    """Device batch of large local maps with different sizes (30,000 / 50,000 /
    24,000 points in a 50,000-point stride), under the default schedule (the
    fixed-point windows) and then the Jacobi schedule (chip-wide rounds and,
    for the problem with deep first-come chains, the windowed fallback)."""
    torch = pytest.importorskip("torch")
    w, h, nf = 1920, 1080, 4000
    k, d, scale = _frame(gpu, oracle, w, h, nf, 5)
    maps = [oracle.synth_local_map(5, k, d, 30000, w, h), oracle.synth_local_map(6, k, d, 50000, w, h),
            _conflict_map(oracle, k, d, 24000, 200)]
    P, S = len(maps), 50000
    ext = gpu.ORBextractor(nf, 1.2, 8, 20, 7)
    cap = ext.capacity(w, h)
    kk = np.zeros((P, cap), oracle.KEYPOINT_DTYPE)
    dd = np.zeros((P, cap, 32), np.uint8)
    lk = np.zeros((P, cap), np.uint8)
    mp = np.zeros((P, S), oracle.MP_TRACK_DTYPE)
    md = np.zeros((P, S, 32), np.uint8)
    for i, (a, b, c) in enumerate(maps):
        kk[i, :len(k)], dd[i, :len(k)], lk[i, :len(k)] = k, d, c
        mp[i, :len(a)], md[i, :len(a)] = a, b
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.uint8)).cuda()
    dk, dde, dl, dm, dmd = t(kk), t(dd), t(lk), t(mp), t(md)
    dn = torch.full((P,), len(k), dtype=torch.int32, device="cuda")
    dnm = torch.tensor([len(a) for a, _, _ in maps], dtype=torch.int32, device="cuda")
    km = torch.zeros((P, cap), dtype=torch.int32, device="cuda")
    nm = torch.zeros(P, dtype=torch.int32, device="cuda")
    m = gpu.ORBmatcher(0.8)
    for it in range(3):  # the second call reuses the scratch of the first
        if it == 2:
            m.set_resolve(m.RESOLVE_JACOBI, 4)
            km.fill_(-7)
        m.search_by_projection_batch(P, dk.data_ptr(), dde.data_ptr(), dn.data_ptr(), dl.data_ptr(),
                                     cap, dm.data_ptr(), dmd.data_ptr(), dnm.data_ptr(), S, w, h,
                                     scale, 1.0, km.data_ptr(), nm.data_ptr())
        torch.cuda.synchronize()
        for i, (a, b, c) in enumerate(maps):
            n_ref, km_ref = oracle.match_projection_local(k, d, scale, w, h, a, b, 1.0, 0.8, c)
            assert int(nm[i]) == n_ref, i
            assert np.array_equal(km[i, :len(k)].cpu().numpy(), km_ref), i


_SCHEDULES = [("auto", 0, 6), ("prefix", 1, 6), ("fixed_point", 2, 6), ("jacobi_r1", 3, 1),
              ("jacobi_r6", 3, 6), ("jacobi_r48", 3, 48)]


@pytest.mark.parametrize("name,schedule,rounds", _SCHEDULES, ids=[s[0] for s in _SCHEDULES])
def test_search_by_projection_resolve_schedules(gpu, oracle, name, schedule, rounds):
    """Every resolve schedule (orb_matcher_set_resolve) on one handle, in
    process: C5's 50,000-point map and a 24,000-point deep-conflict map (points
    that run out of top-4 candidates take the exact re-scan) on a 4,000-feature
    1920x1080 frame, and C4's 5,000-point map plus a 5,000-point conflict map on
    a 1241x376 frame.  Under the prefix schedule these single problems take
    k_proj_resolve<8> (20,000+ points) and k_proj_resolve<4>."""
    m = gpu.ORBmatcher(0.8)
    m.set_resolve(schedule, rounds)
    for (w, h, nf, seed, M) in ((1920, 1080, 4000, 5, 50000), (1241, 376, 1000, 0, 5000)):
        k, d, scale = _frame(gpu, oracle, w, h, nf, seed)
        cases = [oracle.synth_local_map(seed, k, d, M, w, h),
                 _conflict_map(oracle, k, d, 24000 if M > 20000 else M, 120 if M > 20000 else 40)]
        F = gpu.Frame(k, d, scale, w, h)
        for i, (a, b, c) in enumerate(cases):
            want = {"prefix": "k_proj_resolve<8>" if len(a) >= 20000 else "k_proj_resolve<4>",
                    "fixed_point": "k_proj_resolve_fp<1024>", "auto": "k_proj_resolve_fp<1024>"}
            got_kernel = m.resolve_kernel(1, len(k), len(a))
            assert got_kernel == want.get(name, "k_proj_jacobi+k_proj_resolve_fp"), got_kernel
            n_ref, km_ref = oracle.match_projection_local(k, d, scale, w, h, a, b, 1.0, 0.8, c)
            n, km = m.SearchByProjection(F, a, b, 1.0, c)
            assert n == n_ref, (w, i)
            assert np.array_equal(km, km_ref), (w, i, np.nonzero(km != km_ref)[0][:10])


def _cluster_problem(oracle, seed, n_keys=900, M=6000):
    """Keypoints on a 3-px lattice in a few clusters (windows of 5-16 keypoints at
    level 0-1, dozens at level 5-7) and map points over them whose descriptors are
    near-copies: claims with observations lock keypoints fast, so many points run
    out of their top-4 and need the exact re-scan -- from their candidate list
    (<= 16 candidates) or from the grid (more)."""
    rng = np.random.default_rng(seed)
    w, h = 640, 480
    scale = oracle.params(1000)["scale"]
    k = np.zeros(n_keys, oracle.KEYPOINT_DTYPE)
    cx = rng.uniform(60, w - 60, 6)
    cy = rng.uniform(60, h - 60, 6)
    c = rng.integers(0, 6, n_keys)
    k["x"] = (cx[c] + 3.0 * rng.integers(-7, 8, n_keys)).astype(np.float32)
    k["y"] = (cy[c] + 3.0 * rng.integers(-7, 8, n_keys)).astype(np.float32)
    k["octave"] = rng.choice([0, 0, 0, 1, 1, 5, 6, 7], n_keys)
    k["size"] = 31.0
    k["class_id"] = -1
    d = rng.integers(0, 256, (n_keys, 32), dtype=np.uint8)
    mps = np.zeros(M, oracle.MP_TRACK_DTYPE)
    src = rng.integers(0, n_keys, M)
    mps["proj_x"] = k["x"][src] + rng.uniform(-1.5, 1.5, M).astype(np.float32)
    mps["proj_y"] = k["y"][src] + rng.uniform(-1.5, 1.5, M).astype(np.float32)
    mps["proj_xr"] = -1.0
    mps["level"] = np.minimum(k["octave"][src] + rng.integers(0, 2, M), 7)
    mps["view_cos"] = np.where(rng.random(M) < 0.5, 0.999, 0.9).astype(np.float32)
    mps["in_view"] = 1
    mps["has_obs"] = rng.random(M) < 0.9
    mpd = d[src].copy()
    mpd ^= np.packbits(rng.random((M, 256)) < 0.06, axis=1, bitorder="little")
    locked = (rng.random(n_keys) < 0.05).astype(np.uint8)
    return k, d, scale, w, h, mps, mpd, locked


@pytest.mark.parametrize("schedule", [0, 1, 2, 3])
def test_search_by_projection_rescan_lists(gpu, oracle, schedule):
    """The resolves' exact re-scan (a point's top-4 ran dry) through the candidate
    lists k_proj_candidates writes for points with 5-16 candidates, and through the
    grid walk for points with more, under every schedule, as one problem and as a
    device batch of 8 problems; index-exact against the oracle.  The clusters make
    both kinds of point common (checked on the oracle's side)."""
    torch = pytest.importorskip("torch")
    probs = [_cluster_problem(oracle, 40 + i) for i in range(8)]
    m = gpu.ORBmatcher(0.8)
    m.set_resolve(schedule, 6)
    refs = []
    for (k, d, scale, w, h, mps, mpd, lk) in probs:
        refs.append(oracle.match_projection_local(k, d, scale, w, h, mps, mpd, 1.0, 0.8, lk))
        n, km = m.SearchByProjection(gpu.Frame(k, d, scale, w, h), mps, mpd, 1.0, lk)
        assert n == refs[-1][0] and np.array_equal(km, refs[-1][1])
    # the same problems as one device batch
    k0 = probs[0][0]
    P, cap, M = len(probs), len(k0), len(probs[0][5])
    kk = np.stack([p[0] for p in probs])
    dd = np.stack([p[1] for p in probs])
    lk = np.stack([p[7] for p in probs])
    mp = np.stack([p[5] for p in probs])
    md = np.stack([p[6] for p in probs])
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.uint8)).cuda()
    dk, dde, dl, dm, dmd = t(kk), t(dd), t(lk), t(mp), t(md)
    dn = torch.full((P,), cap, dtype=torch.int32, device="cuda")
    dnm = torch.full((P,), M, dtype=torch.int32, device="cuda")
    dkm = torch.zeros((P, cap), dtype=torch.int32, device="cuda")
    dnmt = torch.zeros(P, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    w, h, scale = probs[0][3], probs[0][4], probs[0][2]
    m.search_by_projection_batch(P, dk.data_ptr(), dde.data_ptr(), dn.data_ptr(), dl.data_ptr(), cap,
                                 dm.data_ptr(), dmd.data_ptr(), dnm.data_ptr(), M, w, h, scale, 1.0,
                                 dkm.data_ptr(), dnmt.data_ptr())
    torch.cuda.synchronize()
    km = dkm.cpu().numpy()
    nm = dnmt.cpu().numpy()
    for i, (n_ref, km_ref) in enumerate(refs):
        assert nm[i] == n_ref and np.array_equal(km[i], km_ref), i


@pytest.mark.parametrize("stereo,locked", [(False, True), (True, True), (False, False)])
def test_search_by_projection_staged(gpu, oracle, stereo, locked):
    """The zero-copy pair orb_match_projection_local_stage / _staged (inputs
    written into the handle's pinned block, as integration/ORBmatcher.cc does;
    with and without _begin sending the frame's part and building the grid
    before the map is written) gives the reference's assignments, mono and
    stereo, with and without pre-locked keypoints; interleaved with the copying
    form on one handle.  Misuse is refused: _staged without _stage, _begin
    with other stereo / locked flags than _staged, a second _begin."""
    w, h = 1241, 376
    k, d, scale = _frame(gpu, oracle, w, h, 1000, 3)
    mps, mpd, lk = oracle.synth_local_map(3, k, d, 5000, w, h)
    ur = None
    if stereo:
        rng = np.random.default_rng(4)
        ur = np.where(rng.random(len(k)) < 0.6, k["x"] - rng.uniform(5, 60, len(k)), -1.0).astype(np.float32)
        mps["proj_xr"] = np.where(rng.random(len(mps)) < 0.7, mps["proj_x"] - rng.uniform(4, 62, len(mps)),
                                  -1.0).astype(np.float32)
    lk = lk if locked else None
    F = gpu.Frame(k, d, scale, w, h, u_right=ur)
    m = gpu.ORBmatcher(0.8)
    n_ref, km_ref = oracle.match_projection_local(k, d, scale, w, h, mps, mpd, 1.0, 0.8, lk, u_right=ur)
    for begin in (True, False, True):  # with and without _begin, copying form between
        n1, km1 = m.SearchByProjectionStaged(F, mps, mpd, 1.0, lk, begin=begin)
        n2, km2 = m.SearchByProjection(F, mps, mpd, 1.0, lk)
        assert n1 == n_ref and np.array_equal(km1, km_ref)
        assert n2 == n_ref and np.array_equal(km2, km_ref)
    # _staged without a matching _stage (fresh handle, or a second call) is refused
    import ctypes
    nm = ctypes.c_int32(0)
    out = np.zeros(F.N, np.int32)
    f = F._c()
    for h in (gpu.ORBmatcher(0.8).handle, m.handle):
        with pytest.raises(gpu.OrbError):
            gpu._check(gpu.lib().orb_match_projection_local_staged(
                h, ctypes.byref(f), len(mps), 0, 0, 1.0, 0.8, out.ctypes.data, ctypes.byref(nm)),
                "staged without stage")
    L = gpu.lib()
    st = gpu._LocalStage()
    gpu._check(L.orb_match_projection_local_stage(m.handle, F.N, len(mps), ctypes.byref(st)), "stage")
    gpu._check(L.orb_match_projection_local_begin(m.handle, ctypes.byref(f), int(stereo), 1), "begin")
    with pytest.raises(gpu.OrbError):  # second _begin
        gpu._check(L.orb_match_projection_local_begin(m.handle, ctypes.byref(f), int(stereo), 1), "begin")
    with pytest.raises(gpu.OrbError):  # flags differ from _begin's
        gpu._check(L.orb_match_projection_local_staged(
            m.handle, ctypes.byref(f), len(mps), int(not stereo), 1, 1.0, 0.8, out.ctypes.data,
            ctypes.byref(nm)), "staged")
    # a fresh stage after the abandoned _begin, then a normal call: exact again
    n3, km3 = m.SearchByProjectionStaged(F, mps, mpd, 1.0, lk)
    assert n3 == n_ref and np.array_equal(km3, km_ref)


@pytest.mark.parametrize("schedule", [0, 1, 2, 3])
def test_search_by_projection_batch_empty_map_stride(gpu, oracle, schedule):
    """mp_stride = 0 (no map point in any problem) under every schedule: no
    match, every keypoint -1 (the Jacobi rounds' grid is clamped to one
    workgroup per problem instead of an invalid x = 0)."""
    torch = pytest.importorskip("torch")
    w, h = 640, 480
    k, d, scale = _frame(gpu, oracle, w, h, 1000, 2)
    P, cap = 3, len(k)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.uint8)).cuda()
    dk = t(np.stack([k] * P))
    dd = t(np.stack([d] * P))
    dn = torch.full((P,), len(k), dtype=torch.int32, device="cuda")
    dnm = torch.zeros(P, dtype=torch.int32, device="cuda")
    dummy = torch.zeros(64, dtype=torch.uint8, device="cuda")
    km = torch.full((P, cap), -7, dtype=torch.int32, device="cuda")
    nm = torch.full((P,), -7, dtype=torch.int32, device="cuda")
    m = gpu.ORBmatcher(0.8)
    m.set_resolve(schedule, 6)
    m.search_by_projection_batch(P, dk.data_ptr(), dd.data_ptr(), dn.data_ptr(), 0, cap,
                                 dummy.data_ptr(), dummy.data_ptr(), dnm.data_ptr(), 0, w, h,
                                 scale, 1.0, km.data_ptr(), nm.data_ptr())
    torch.cuda.synchronize()
    assert (nm.cpu().numpy() == 0).all()
    assert (km.cpu().numpy() == -1).all()


def test_resolve_schedule_rejects_bad_values(gpu):
    m = gpu.ORBmatcher(0.8)
    for sched, r in ((4, 6), (-1, 6), (3, 0), (3, 49)):
        with pytest.raises(gpu.OrbError):
            m.set_resolve(sched, r)
