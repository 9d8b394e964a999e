"""The headline bench's own path against the CPU oracle, at its launch shapes.

bench.py times extract_batch over 1241x376 KITTI-shaped frames (1000
features) followed by one search_by_projection_batch call against each frame's
own 5,000-point local map.  At the bench's 1024 frames
per launch the batch takes the register-free octree (k_octree<false,false>,
more than 16 images) and the one-wave prefix resolve k_proj_resolve<1> (128+
problems); 9-127 problems take k_proj_resolve<4>.  Every frame's keypoints and
descriptors and every problem's assignments are compared with the oracle
(src/ORBextractor.cc:1091-1169; src/ORBmatcher.cc:47-133 with
src/Frame.cc:368-424), index-exact, including first-come claiming
(src/ORBmatcher.cc:90-93,127) on conflict-heavy maps inside the batch.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, NF, M = 1241, 376, 1000, 5000
SEED = 0x4B495454  # bench.py --seed


def _pool(fn, items):
    # the oracle's ctypes calls release the GIL
    with ThreadPoolExecutor(max_workers=16) as ex:
        return list(ex.map(fn, items))


def _conflict_map(oracle, k, d, m, nsrc, seed):
    """m map points projected onto nsrc keypoints (deep first-come chains)."""
    rng = np.random.default_rng(seed)
    mps = np.zeros(m, oracle.MP_TRACK_DTYPE)
    src = rng.integers(0, nsrc, m)
    mps["proj_x"] = k["x"][src] + rng.uniform(-2, 2, m).astype(np.float32)
    mps["proj_y"] = k["y"][src] + rng.uniform(-2, 2, m).astype(np.float32)
    mps["proj_xr"] = -1.0
    mps["level"] = np.minimum(k["octave"][src] + rng.integers(0, 2, m), 7)
    mps["view_cos"] = np.where(rng.random(m) < 0.5, 0.999, 0.9).astype(np.float32)
    mps["in_view"] = rng.random(m) < 0.97
    mps["bad"] = rng.random(m) < 0.02
    mps["has_obs"] = rng.random(m) < 0.8
    mpd = d[src].copy()
    mpd ^= np.packbits(rng.random((m, 256)) < 0.1, axis=1, bitorder="little")
    locked = (rng.random(len(k)) < 0.1).astype(np.uint8)
    return mps, mpd, locked


@pytest.mark.parametrize("B,kernel", [(256, "k_proj_resolve<1>"), (32, "k_proj_resolve<4>")])
def test_headline_batch_extract_and_match(gpu, oracle, B, kernel):
    torch = pytest.importorskip("torch")
    imgs = np.stack([gpu.synth_image(SEED, f, W, H) for f in range(B)])
    ext = gpu.ORBextractor(NF, 1.2, 8, 20, 7)
    scale = np.float32(ext.GetScaleFactors())
    cap = ext.capacity(W, H)
    d_img = torch.from_numpy(imgs).cuda()
    d_kps = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
    d_desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    d_cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ext.extract_batch(d_img.data_ptr(), B, W, H, W, W * H, d_kps.data_ptr(), d_desc.data_ptr(),
                      cap, d_cnt.data_ptr())
    torch.cuda.synchronize()
    kps = d_kps.cpu().numpy().view(gpu.KEYPOINT_DTYPE).reshape(B, cap)
    desc = d_desc.cpu().numpy()
    cnt = d_cnt.cpu().numpy()

    # extraction: every frame bit-exact (all 7 keypoint fields, order, descriptors)
    ref = _pool(lambda f: oracle.extract(imgs[f], NF, 1.2, 8, 20, 7)[:2], range(B))
    for f, (kr, dr) in enumerate(ref):
        assert cnt[f] == len(kr), (f, cnt[f], len(kr))
        assert kps[f, :cnt[f]].tobytes() == kr.tobytes(), f
        assert desc[f, :cnt[f]].tobytes() == dr.tobytes(), f

    # local maps as bench.py builds them, two of them conflict-heavy
    maps = [gpu.synth_local_map(SEED + f, kps[f, :cnt[f]], desc[f, :cnt[f]], M, W, H)
            for f in range(B)]
    for f, nsrc in ((1, 40), (B - 1, 12)):
        maps[f] = _conflict_map(oracle, kps[f, :cnt[f]], desc[f, :cnt[f]], M, nsrc, 100 + f)
    mps = np.stack([mm[0] for mm in maps])
    mpd = np.stack([mm[1] for mm in maps])
    lk = np.zeros((B, cap), np.uint8)
    for f in range(B):
        lk[f, :cnt[f]] = maps[f][2]
    d_mps = torch.from_numpy(mps.view(np.uint8).reshape(B, -1)).cuda()
    d_mpd = torch.from_numpy(mpd).cuda()
    d_lk = torch.from_numpy(lk).cuda()
    d_nm = torch.full((B,), M, dtype=torch.int32, device="cuda")
    km = torch.zeros((B, cap), dtype=torch.int32, device="cuda")
    nm = torch.zeros(B, dtype=torch.int32, device="cuda")

    want = _pool(lambda f: oracle.match_projection_local(
        kps[f, :cnt[f]], desc[f, :cnt[f]], scale, W, H, maps[f][0], maps[f][1], 1.0, 0.8,
        maps[f][2]), range(B))
    m = gpu.ORBmatcher(0.8)
    assert m.resolve_kernel(B, cap, M) == kernel
    for sched in (m.RESOLVE_AUTO, m.RESOLVE_FIXED_POINT, m.RESOLVE_JACOBI):
        m.set_resolve(sched, 6)
        km.fill_(-7)
        nm.fill_(-7)
        m.search_by_projection_batch(B, d_kps.data_ptr(), d_desc.data_ptr(), d_cnt.data_ptr(),
                                     d_lk.data_ptr(), cap, d_mps.data_ptr(), d_mpd.data_ptr(),
                                     d_nm.data_ptr(), M, W, H, scale, 1.0, km.data_ptr(),
                                     nm.data_ptr())
        torch.cuda.synchronize()
        got_km, got_n = km.cpu().numpy(), nm.cpu().numpy()
        for f, (n_ref, km_ref) in enumerate(want):
            assert got_n[f] == n_ref, (sched, f, got_n[f], n_ref)
            assert np.array_equal(got_km[f, :cnt[f]], km_ref), \
                (sched, f, np.nonzero(got_km[f, :cnt[f]] != km_ref)[0][:10])
    assert sum(n for n, _ in want) > 500 * B  # the maps really match (bench: ~796 per frame)
