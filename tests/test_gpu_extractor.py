"""GPU extractor parity: the HIP ORBextractor must reproduce the CPU oracle
bit-for-bit (keypoints: all 7 cv::KeyPoint fields and their order;
descriptors: all 256 bits) -- SURVEY.md §8(d) C2/C3/C5 shapes."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CONFIGS = [
    # (width, height, nfeatures, seed)  -- C2 TUM-shaped, C1/C4 KITTI-shaped, C3, C5
    (640, 480, 1000, 1),
    (640, 480, 1000, 2),
    (640, 480, 1000, 3),
    (1241, 376, 1000, 0),
    (1241, 376, 2000, 7),
    (1920, 1080, 4000, 5),
]


def _diff_report(k_gpu, d_gpu, k_ref, d_ref):
    lines = [f"n gpu={len(k_gpu)} ref={len(k_ref)}"]
    for lvl in range(8):
        g = k_gpu[k_gpu["octave"] == lvl]
        r = k_ref[k_ref["octave"] == lvl]
        same = len(g) == len(r) and (g.tobytes() == r.tobytes())
        if not same:
            gs = set(zip(g["x"].tolist(), g["y"].tolist()))
            rs = set(zip(r["x"].tolist(), r["y"].tolist()))
            lines.append(f" level {lvl}: gpu {len(g)} ref {len(r)} only_gpu {len(gs - rs)} only_ref {len(rs - gs)}")
            n = min(len(g), len(r))
            for f in ("x", "y", "response", "angle", "size"):
                bad = np.nonzero(g[f][:n] != r[f][:n])[0]
                if len(bad):
                    i = bad[0]
                    lines.append(f"   field {f}: {len(bad)} diffs, first at {i}: gpu {g[i]} ref {r[i]}")
    n = min(len(d_gpu), len(d_ref))
    bad = np.nonzero((d_gpu[:n] != d_ref[:n]).any(1))[0]
    lines.append(f" descriptor rows differing: {len(bad)}")
    return "\n".join(lines)


@pytest.mark.parametrize("w,h,nf,seed", CONFIGS)
def test_extract_bit_exact(gpu, oracle, w, h, nf, seed):
    img = gpu.synth_image(seed, 0, w, h)
    ext = gpu.ORBextractor(nf, 1.2, 8, 20, 7)
    k_gpu, d_gpu = ext(img)
    k_ref, d_ref, _ = oracle.extract(img, nf, 1.2, 8, 20, 7)
    ok = len(k_gpu) == len(k_ref) and k_gpu.tobytes() == k_ref.tobytes() and \
        d_gpu.tobytes() == d_ref.tobytes()
    assert ok, _diff_report(k_gpu, d_gpu, k_ref, d_ref)


@pytest.mark.parametrize("w,h", [(640, 480), (1241, 376), (1920, 1080)])
def test_pyramid_bit_exact(gpu, oracle, w, h):
    img = gpu.synth_image(11, 0, w, h)
    ext = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    ext(img)
    pyr = ext.mvImagePyramid
    ref = oracle.pyramid(img)
    for l, (a, b) in enumerate(zip(pyr, ref)):
        assert a.shape == b.shape, (l, a.shape, b.shape)
        assert np.array_equal(a, b), f"level {l}: {(a != b).sum()} pixels differ"


@pytest.mark.parametrize("w,h,sf,nl,launches", [
    (1241, 376, 1.2, 8, 4),    # pairs 1+2, 3+4, 5+6, then 7: k_pyr_resize2 x 3 + k_pyr_resize
    (640, 480, 1.2, 9, 4),     # 1+2, 3+4, 5+6, 7+8
    (1920, 1080, 1.1, 12, 6),  # narrow downscales, 11 levels in 6 launches
    (1241, 376, 1.5, 7, 6),    # wide tiles (downscale > 1.25): one launch per level (8 levels would leave 22 rows)
    (997, 613, 1.2, 7, 3),     # odd sizes: 1+2, 3+4, 5+6
    (1003, 333, 1.22, 8, 4),   # odd sizes, a non-ORB-SLAM2 scale factor
    (997, 613, 1.25, 6, 5)])   # downscales just past 1.25 (levels 1-4 wide, one launch each), 5
def test_pyramid_level_pairs_batch(gpu, oracle, w, h, sf, nl, launches):
    """The batch path's pyramid through the paired-level resize (k_pyr_resize2:
    level l + 1 from a level-l region the workgroup builds in LDS, each level-l
    pixel stored by exactly one workgroup; src/ORBextractor.cc:1172-1207) is
    bit-identical to the oracle's level-by-level resize, for every image of a
    batch; the stage's launch count pins which levels were paired."""
    torch = pytest.importorskip("torch")
    B = 5
    imgs = np.stack([gpu.synth_image(21, f, w, h) for f in range(B)])
    ext = gpu.ORBextractor(1000, sf, nl, 20, 7)
    cap = ext.capacity(w, h)
    d_img = torch.from_numpy(imgs).cuda()
    d_k = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
    d_d = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    d_n = torch.zeros(B, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ext.profile(True)
    ext.extract_batch(d_img.data_ptr(), B, w, h, w, w * h, d_k.data_ptr(), d_d.data_ptr(), cap,
                      d_n.data_ptr())
    torch.cuda.synchronize()
    name, _, n = ext.profile_read(0)
    ext.profile(False)
    assert name == "k_pyr_resize" and n == launches, (name, n)
    for i in (0, B - 1):
        ref = oracle.pyramid(imgs[i], sf, nl)
        for l in range(1, nl):
            got = ext.batch_level(i, l)
            assert got.shape == ref[l].shape, (i, l)
            assert np.array_equal(got, ref[l]), f"image {i} level {l}: {(got != ref[l]).sum()} px differ"


@pytest.mark.parametrize("w,h,sf,nl", [(1241, 376, 1.2, 8), (1920, 1080, 1.2, 8), (997, 613, 1.2, 7)])
def test_pyramid_unpaired_batch(gpu, oracle, w, h, sf, nl):
    """Batches of more than PYR_PAIR_MAX_IMAGES (8) images build the pyramid one
    launch per level (k_pyr_resize; the level pairs cost batches throughput,
    runtime.cpp): nl - 1 launches, every level bit-identical to the oracle."""
    torch = pytest.importorskip("torch")
    B = 9
    imgs = np.stack([gpu.synth_image(23, f, w, h) for f in range(B)])
    ext = gpu.ORBextractor(1000, sf, nl, 20, 7)
    cap = ext.capacity(w, h)
    d_img = torch.from_numpy(imgs).cuda()
    d_k = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
    d_d = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    d_n = torch.zeros(B, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ext.profile(True)
    ext.extract_batch(d_img.data_ptr(), B, w, h, w, w * h, d_k.data_ptr(), d_d.data_ptr(), cap,
                      d_n.data_ptr())
    torch.cuda.synchronize()
    name, _, n = ext.profile_read(0)
    ext.profile(False)
    assert name == "k_pyr_resize" and n == nl - 1, (name, n)
    for i in (0, B - 1):
        ref = oracle.pyramid(imgs[i], sf, nl)
        for l in range(1, nl):
            got = ext.batch_level(i, l)
            assert np.array_equal(got, ref[l]), f"image {i} level {l}: {(got != ref[l]).sum()} px differ"


@pytest.mark.parametrize("w,h", [(640, 480), (1241, 376), (1920, 1080), (403, 301)])
def test_blurred_levels_bit_exact(gpu, oracle, w, h):
    """GaussianBlur(7x7, sigma 2, REFLECT_101) of every level (src/ORBextractor.cc:1143-1145)."""
    img = gpu.synth_image(12, 0, w, h)
    ext = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    ext(img)
    for l, (a, lv) in enumerate(zip(ext.blurred_levels(), oracle.pyramid(img))):
        b = oracle.blur7(lv)
        assert a.shape == b.shape
        bad = np.argwhere(a != b)
        assert len(bad) == 0, f"level {l}: {len(bad)} px differ, first {bad[:5].tolist()}"


def test_accessors_match_reference_tables(gpu, oracle):
    ext = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    p = oracle.params(1000, 1.2, 8)
    assert ext.GetLevels() == 8
    assert np.float32(ext.GetScaleFactor()) == np.float32(1.2)
    assert np.array_equal(np.float32(ext.GetScaleFactors()), p["scale"])
    assert np.array_equal(np.float32(ext.GetInverseScaleFactors()), p["inv_scale"])
    assert np.array_equal(np.float32(ext.GetScaleSigmaSquares()), p["sigma2"])
    assert np.array_equal(np.float32(ext.GetInverseScaleSigmaSquares()), p["inv_sigma2"])
    assert ext.features_per_level() == p["quota"].tolist()


def test_empty_and_invalid(gpu):
    ext = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    assert ext(np.zeros((0, 0), np.uint8)) == (None, None)  # src/ORBextractor.cc:1095-1096
    with pytest.raises(gpu.OrbError):
        ext(np.zeros((480, 640), np.float32))  # non-8UC1: reference asserts (:1100)
    with pytest.raises(gpu.OrbError):
        ext(np.zeros((30, 30), np.uint8))  # too small for an 8-level ORB pyramid


def test_flat_image_has_no_keypoints(gpu, oracle):
    img = np.full((480, 640), 128, np.uint8)
    k, d = gpu.ORBextractor(1000, 1.2, 8, 20, 7)(img)
    kr, dr, _ = oracle.extract(img)
    assert len(k) == 0 and len(kr) == 0 and d.shape == (0, 32)


def test_noise_image_heavy_candidates(gpu, oracle):
    """Uniform noise: every cell is dense with FAST corners, exercising the
    octree's global-memory key path and the deepest final-phase splits."""
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (480, 640), dtype=np.uint8)
    k_gpu, d_gpu = gpu.ORBextractor(1000, 1.2, 8, 20, 7)(img)
    k_ref, d_ref, _ = oracle.extract(img)
    assert k_gpu.tobytes() == k_ref.tobytes(), _diff_report(k_gpu, d_gpu, k_ref, d_ref)
    assert d_gpu.tobytes() == d_ref.tobytes()


def test_low_contrast_fallback_threshold(gpu, oracle):
    """Low-contrast image: most cells find nothing at iniThFAST=20 and fall back
    to minThFAST=7 (src/ORBextractor.cc:846-850)."""
    rng = np.random.default_rng(4)
    base = gpu.synth_image(9, 0, 640, 480).astype(np.int32)
    img = (128 + (base - 128) // 12 + rng.integers(-3, 4, base.shape)).clip(0, 255).astype(np.uint8)
    k_gpu, d_gpu = gpu.ORBextractor(1000, 1.2, 8, 20, 7)(img)
    k_ref, d_ref, _ = oracle.extract(img)
    assert k_gpu.tobytes() == k_ref.tobytes(), _diff_report(k_gpu, d_gpu, k_ref, d_ref)
    assert d_gpu.tobytes() == d_ref.tobytes()


def test_strided_input(gpu):
    img = gpu.synth_image(2, 0, 640, 480)
    wide = np.zeros((480, 704), np.uint8)
    wide[:, :640] = img
    ext = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    k1, d1 = ext(img)
    k2, d2 = ext(wide[:, :640])
    assert k1.tobytes() == k2.tobytes() and d1.tobytes() == d2.tobytes()


def test_batch_matches_single(gpu):
    torch = pytest.importorskip("torch")
    w, h, nf, B = 1241, 376, 1000, 5
    ext = gpu.ORBextractor(nf, 1.2, 8, 20, 7)
    imgs = np.stack([gpu.synth_image(20, f, w, h) for f in range(B)])
    cap = ext.capacity(w, h)
    d_img = torch.from_numpy(imgs).cuda()
    d_kps = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
    d_desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    d_cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ext.extract_batch(d_img.data_ptr(), B, w, h, w, w * h, d_kps.data_ptr(), d_desc.data_ptr(),
                      cap, d_cnt.data_ptr())
    torch.cuda.synchronize()
    kps = d_kps.cpu().numpy().view(gpu.KEYPOINT_DTYPE).reshape(B, cap)
    desc = d_desc.cpu().numpy()
    cnt = d_cnt.cpu().numpy()
    for f in range(B):
        k1, d1 = ext(imgs[f])
        assert cnt[f] == len(k1)
        assert kps[f, : cnt[f]].tobytes() == k1.tobytes()
        assert desc[f, : cnt[f]].tobytes() == d1.tobytes()


@pytest.mark.parametrize("w,h,nf,sf,nl", [
    (640, 480, 1000, 1.2, 1),      # single level
    (1241, 376, 1500, 1.2, 12),    # deep pyramid (level 11: 167 x 51)
    (640, 480, 800, 1.1, 8),       # finer scale steps
    (1920, 1080, 2000, 1.5, 6),    # wide resize variant (downscale > 1.25)
    (1241, 376, 1000, 1.9, 4),     # widest staged downscale
    (1241, 376, 1000, 1.25, 8),    # narrow variant's limit
    (1920, 1080, 2000, 2.0, 5),    # untiled resize (every level >= 33 px)
    (1920, 1080, 2000, 2.5, 4),
    (1241, 376, 1000, 3.0, 3),
    (640, 480, 1000, 1.2, 15),     # levels 12-14 (60..37 px high) have no cells
])
def test_extractor_parameters(gpu, oracle, w, h, nf, sf, nl):
    """ORBextractor(nfeatures, scaleFactor, nlevels, 20, 7) for parameters other
    than the yaml defaults: scale tables, quotas, pyramid, keypoints and
    descriptors all bit-exact."""
    img = gpu.synth_image(11, 0, w, h)
    ext = gpu.ORBextractor(nf, sf, nl, 20, 7)
    k_gpu, d_gpu = ext(img)
    k_ref, d_ref, _ = oracle.extract(img, nf, sf, nl, 20, 7)
    assert len(k_gpu) > 0
    assert k_gpu.tobytes() == k_ref.tobytes(), _diff_report(k_gpu, d_gpu, k_ref, d_ref)
    assert d_gpu.tobytes() == d_ref.tobytes()
    ref_pyr = oracle.pyramid(img, sf, nl)
    for l, lv in enumerate(ext.mvImagePyramid):
        assert np.ascontiguousarray(lv).tobytes() == ref_pyr[l].tobytes(), f"level {l}"


def test_extractor_rejects_degenerate_parameters(gpu):
    """scaleFactor 1 (the reference's quota series is 0 / 0,
    src/ORBextractor.cc:453-455) is rejected at construction; a pyramid level
    of 32 px or less (where the reference's DistributeOctTree divides by zero
    or resizes its root vector to a negative size, :562-569) by the call."""
    for sf in (1.0, 0.5, float("nan"), float("inf")):
        with pytest.raises(gpu.OrbError):
            gpu.ORBextractor(1000, sf, 8, 20, 7)
    ext = gpu.ORBextractor(1000, 2.0, 8, 20, 7)  # 1241x376: level 4 is 78 x 24
    with pytest.raises(gpu.OrbError):
        ext(gpu.synth_image(1, 0, 1241, 376))
    assert ext.capacity(1241, 376) < 0


def test_extractor_100k_features(gpu, oracle):
    """nfeatures far above any ORB-SLAM2 yaml (100,000 on 1080p noise: level
    quotas 21,700 .. 6,900, 92,610 keypoints): single frame and a batch of
    two, bit-exact."""
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, (1080, 1920), dtype=np.uint8)
    k_ref, d_ref, _ = oracle.extract(img, 100000, 1.2, 8, 20, 7)
    assert len(k_ref) > 60000
    k_gpu, d_gpu = gpu.ORBextractor(100000, 1.2, 8, 20, 7)(img)
    assert k_gpu.tobytes() == k_ref.tobytes(), _diff_report(k_gpu, d_gpu, k_ref, d_ref)
    assert d_gpu.tobytes() == d_ref.tobytes()
    _batch_vs_oracle(gpu, oracle, [img, img[:, ::-1].copy()], 100000)


@pytest.mark.parametrize("w,h,stride,pitch,B", [
    (640, 480, 640, 640 * 480, 6),          # aligned rows and images
    (640, 480, 644, 644 * 480 + 2, 5),      # aligned rows, images at alternating alignment
    (641, 479, 641, 641 * 479, 3),          # odd stride and odd image pitch
    (1241, 376, 1241, 1241 * 376, 9),       # 9 images: uneven images per workgroup
    (1241, 376, 1241, 1241 * 376, 2),       # 2 images: the small-call launch shapes
    (640, 480, 648, 648 * 480 + 4, 1),      # 1 image through the batch entry point
])
def test_batch_layouts_vs_oracle(gpu, oracle, w, h, stride, pitch, B):
    """extract_batch over B images packed at (stride, pitch): the resize and blur
    workgroups walk several images each (prefetching the next), so every image
    and every alignment case is checked against the CPU oracle."""
    torch = pytest.importorskip("torch")
    ext = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    imgs = [gpu.synth_image(30 + B, f, w, h) for f in range(B)]
    buf = np.zeros(pitch * B + stride, np.uint8)
    for f, im in enumerate(imgs):
        for y in range(h):
            buf[f * pitch + y * stride: f * pitch + y * stride + w] = im[y]
    cap = ext.capacity(w, h)
    d_img = torch.from_numpy(buf).cuda()
    d_kps = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
    d_desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    d_cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ext.extract_batch(d_img.data_ptr(), B, w, h, stride, pitch, d_kps.data_ptr(),
                      d_desc.data_ptr(), cap, d_cnt.data_ptr())
    torch.cuda.synchronize()
    kps = d_kps.cpu().numpy().view(gpu.KEYPOINT_DTYPE).reshape(B, cap)
    desc = d_desc.cpu().numpy()
    cnt = d_cnt.cpu().numpy()
    for f in range(B):
        kr, dr, _ = oracle.extract(imgs[f], 1000, 1.2, 8, 20, 7)
        assert cnt[f] == len(kr), (f, cnt[f], len(kr))
        assert kps[f, : cnt[f]].tobytes() == kr.tobytes(), f
        assert desc[f, : cnt[f]].tobytes() == dr.tobytes(), f


def _batch_vs_oracle(gpu, oracle, imgs, nf=1000, sf=1.2, nl=8):
    torch = pytest.importorskip("torch")
    B = len(imgs)
    h, w = imgs[0].shape
    ext = gpu.ORBextractor(nf, sf, nl, 20, 7)
    cap = ext.capacity(w, h)
    d_img = torch.from_numpy(np.stack(imgs)).cuda()
    d_kps = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
    d_desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    d_cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ext.extract_batch(d_img.data_ptr(), B, w, h, w, w * h, d_kps.data_ptr(), d_desc.data_ptr(),
                      cap, d_cnt.data_ptr())
    torch.cuda.synchronize()
    kps = d_kps.cpu().numpy().view(gpu.KEYPOINT_DTYPE).reshape(B, cap)
    desc = d_desc.cpu().numpy()
    cnt = d_cnt.cpu().numpy()
    for f in range(B):
        kr, dr, _ = oracle.extract(imgs[f], nf, sf, nl, 20, 7)
        assert cnt[f] == len(kr), (f, cnt[f], len(kr))
        assert kps[f, : cnt[f]].tobytes() == kr.tobytes(), \
            (f, _diff_report(kps[f, : cnt[f]], desc[f, : cnt[f]], kr, dr))
        assert desc[f, : cnt[f]].tobytes() == dr.tobytes(), f


BENCH_SEED = 0x4B495454  # bench.py's default --seed
# frames of the bench stream with a keypoint 19-20 px from the top-left corner
# whose rotated pattern samples reach rows 0-3 (tools/probe/stream_parity.py:
# 43 of the stream's 8,192 frames, all on level 0)
CORNER_FRAMES = [577, 587, 597, 628, 2829, 3299, 3304, 3306]


@pytest.mark.parametrize("shift", [0, 1, 2, 3])
def test_orient_window_over_top_left_corner(gpu, oracle, shift):
    """k_orient_desc stages each keypoint's 43-row window from the 4-aligned
    byte at or below column cx - 21.  For a keypoint at x = 19 or 20 that byte
    lies before the level's first byte in row 0 (a negative offset: the first
    16-byte load fell out of the buffer's range and read as zeros, so a
    descriptor bit or two of such keypoints differed from the reference's on
    43 of the bench's 8,192 frames).  Row 0 is now loaded from byte 0 and
    shifted right.  The bench frames that showed it, through the batch entry
    point with the images `shift` bytes past a 4-byte boundary (the offset's
    sign depends on it) and through the one-frame path."""
    torch = pytest.importorskip("torch")
    w, h, B = 1241, 376, len(CORNER_FRAMES)
    imgs = [gpu.synth_image(BENCH_SEED, f, w, h) for f in CORNER_FRAMES]
    pitch = w * h + 4
    buf = np.zeros(pitch * B + 16, np.uint8)
    for f, im in enumerate(imgs):
        buf[shift + f * pitch: shift + f * pitch + w * h] = im.reshape(-1)
    ext = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    cap = ext.capacity(w, h)
    d_buf = torch.from_numpy(buf).cuda()
    d_kps = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
    d_desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    d_cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ext.extract_batch(d_buf.data_ptr() + shift, B, w, h, w, pitch, d_kps.data_ptr(),
                      d_desc.data_ptr(), cap, d_cnt.data_ptr())
    torch.cuda.synchronize()
    kps = d_kps.cpu().numpy().view(gpu.KEYPOINT_DTYPE).reshape(B, cap)
    desc = d_desc.cpu().numpy()
    cnt = d_cnt.cpu().numpy()
    for f in range(B):
        kr, dr, _ = oracle.extract(imgs[f], 1000, 1.2, 8, 20, 7)
        corner = (kr["x"] <= 20.5) & (kr["y"] <= 21.5) & (kr["octave"] == 0)
        assert corner.any(), CORNER_FRAMES[f]  # the case is really exercised
        assert cnt[f] == len(kr)
        assert kps[f, : cnt[f]].tobytes() == kr.tobytes(), CORNER_FRAMES[f]
        bad = np.nonzero((desc[f, : cnt[f]] != dr).any(1))[0]
        assert len(bad) == 0, (CORNER_FRAMES[f], kr[bad][:4])
        if shift == 0:
            k1, d1 = ext(imgs[f])
            assert k1.tobytes() == kr.tobytes() and np.array_equal(d1, dr), CORNER_FRAMES[f]


def test_batch_hard_cases_vs_oracle(gpu, oracle):
    """Batches of >= 4 frames take the one-wave-per-cell FAST kernel (level 0 on
    the side stream); single frames take the band kernel.  The hard single-frame
    cases above, as one batch: noise, low contrast (minThFAST fallback), flat."""
    rng = np.random.default_rng(3)
    noise = rng.integers(0, 256, (480, 640), dtype=np.uint8)
    rng = np.random.default_rng(4)
    base = gpu.synth_image(9, 0, 640, 480).astype(np.int32)
    low = (128 + (base - 128) // 12 + rng.integers(-3, 4, base.shape)).clip(0, 255).astype(np.uint8)
    flat = np.full((480, 640), 128, np.uint8)
    _batch_vs_oracle(gpu, oracle, [noise, low, flat, gpu.synth_image(2, 0, 640, 480)])


@pytest.mark.parametrize("w,h,nf,sf,nl", [
    (1241, 376, 1500, 1.2, 12),
    (640, 480, 800, 1.1, 8),
    (1920, 1080, 2000, 1.5, 6),
    (1241, 376, 1000, 1.9, 4),
    (1920, 1080, 2000, 2.5, 4),    # untiled resize
    (640, 480, 1000, 1.2, 1),
    (640, 480, 1000, 1.2, 2),      # the side stream's FAST covers every level >= 1,
    (1241, 376, 1000, 1.2, 3),     # the main stream's FAST launch is empty
])
def test_batch_parameters_vs_oracle(gpu, oracle, w, h, nf, sf, nl):
    _batch_vs_oracle(gpu, oracle, [gpu.synth_image(40, f, w, h) for f in range(4)], nf, sf, nl)


def test_noise_720p_dense_levels(gpu, oracle):
    """1280x720 uniform noise: level 0 holds tens of thousands of FAST
    candidates (about 10 % of its pixels), well past any 16-bit key label, so
    the octree's global-scratch path and its node / key capacities are
    exercised at a size the reference handles without limits
    (src/ORBextractor.cc:558-782).  Single frame (band FAST) and a batch of
    four (cell FAST) against the oracle."""
    rng = np.random.default_rng(720)
    imgs = [rng.integers(0, 256, (720, 1280), dtype=np.uint8) for _ in range(4)]
    k_gpu, d_gpu = gpu.ORBextractor(2000, 1.2, 8, 20, 7)(imgs[0])
    k_ref, d_ref, _ = oracle.extract(imgs[0], 2000, 1.2, 8, 20, 7)
    assert k_gpu.tobytes() == k_ref.tobytes(), _diff_report(k_gpu, d_gpu, k_ref, d_ref)
    assert d_gpu.tobytes() == d_ref.tobytes()
    cand, _ = oracle.candidates(imgs[0], 2000, 1.2, 8, 20, 7)
    assert (cand["octave"] == 0).sum() > 65535 // 4, "noise frame not dense enough to matter"
    _batch_vs_oracle(gpu, oracle, imgs, 2000)


def test_large_batch_vs_oracle(gpu, oracle):
    """More than 16 frames per call: the octree keeps its keys in LDS / global
    scratch instead of registers (the batch configuration of the bench)."""
    _batch_vs_oracle(gpu, oracle, [gpu.synth_image(50, f, 640, 480) for f in range(20)])


def test_single_batch_single_keeps_level0(gpu, oracle):
    """A replayed single-image graph must re-point level 0 at its own staged
    image: single extract, a batch on the same handle, single extract again,
    then mvImagePyramid[0] (read by Frame::ComputeStereoMatches,
    src/Frame.cc:619,633) equals the last single image, and every level equals
    the oracle's pyramid of it."""
    torch = pytest.importorskip("torch")
    w, h = 640, 480
    ext = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    a = gpu.synth_image(11, 0, w, h)
    b = gpu.synth_image(12, 0, w, h)
    ext(a)
    cap = ext.capacity(w, h)
    imgs = torch.from_numpy(np.stack([b, b])).cuda()
    k = torch.zeros((2, cap, 7), dtype=torch.int32, device="cuda")
    d = torch.zeros((2, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(2, dtype=torch.int32, device="cuda")
    ext.extract_batch(imgs.data_ptr(), 2, w, h, w, w * h, k.data_ptr(), d.data_ptr(), cap,
                      n.data_ptr())
    torch.cuda.synchronize()
    k1, d1 = ext(a)  # replays the captured graph
    del imgs  # the batch's input is gone: nothing may still point at it
    torch.cuda.empty_cache()
    pyr = ext.mvImagePyramid
    assert np.array_equal(pyr[0], a)
    ref = oracle.pyramid(a, 1.2, 8)
    for l in range(8):
        assert np.array_equal(pyr[l], ref[l]), f"level {l}"
    kr, dr, _ = oracle.extract(a, 1000, 1.2, 8, 20, 7)
    assert k1.tobytes() == kr.tobytes() and d1.tobytes() == dr.tobytes()


def test_octree_12k_features_1080p_noise(gpu, oracle):
    """The largest DistributeOctTree the configurations reach and then some:
    1920x1080 uniform noise (FAST candidates everywhere) with 12,000 features,
    on the GPU (single frame and a batch of two), bit-exact against the oracle."""
    import torch
    rng = np.random.default_rng(12)
    w, h, nf = 1920, 1080, 12000
    img = rng.integers(0, 256, (h, w), dtype=np.uint8)
    kr, dr, per = oracle.extract(img, nf)
    assert len(kr) >= nf - 8
    ext = gpu.ORBextractor(nf, 1.2, 8, 20, 7)
    k, d = ext(img)
    assert k.tobytes() == kr.tobytes() and d.tobytes() == dr.tobytes()
    cap = ext.capacity(w, h)
    imgs = torch.from_numpy(np.stack([img, img])).cuda()
    kb = torch.zeros((2, cap, 7), dtype=torch.int32, device="cuda")
    db = torch.zeros((2, cap, 32), dtype=torch.uint8, device="cuda")
    nb = torch.zeros(2, dtype=torch.int32, device="cuda")
    ext.extract_batch(imgs.data_ptr(), 2, w, h, w, w * h, kb.data_ptr(), db.data_ptr(), cap,
                      nb.data_ptr())
    torch.cuda.synchronize()
    for i in range(2):
        n = int(nb[i])
        assert n == len(kr)
        assert kb[i, :n].cpu().numpy().tobytes() == kr.tobytes()
        assert db[i, :n].cpu().numpy().tobytes() == dr.tobytes()


def test_octree_pass_bound_fails_cleanly(gpu):
    """An octree that hits its pass bound fails the image as a whole: the
    single-frame call raises ORB_EDEVICE, the batch form reports a negative
    count, and the handle keeps working afterwards (the bound lowered through
    test build lib/variants/octree_passes2.so, `make testhook`, in a child
    process: the product library has no hook)."""
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    code = f"""
import sys, numpy as np, torch
sys.path.insert(0, {str(root)!r}); sys.path.insert(0, {str(root / 'tests')!r})
from conftest import load_pkg
orb = load_pkg()
img = orb.synth_image(1, 0, 640, 480)
ext = orb.ORBextractor(1000, 1.2, 8, 20, 7)
try:
    ext(img)
    print('single: no error')
except orb.OrbError as e:
    print('single:', e.status)
cap = ext.capacity(640, 480)
imgs = torch.from_numpy(np.stack([img] * 4)).cuda()
k = torch.zeros((4, cap, 7), dtype=torch.int32, device='cuda')
d = torch.zeros((4, cap, 32), dtype=torch.uint8, device='cuda')
n = torch.zeros(4, dtype=torch.int32, device='cuda')
ext.extract_batch(imgs.data_ptr(), 4, 640, 480, 640, 640 * 480, k.data_ptr(), d.data_ptr(), cap, n.data_ptr())
torch.cuda.synchronize()
print('batch:', n.tolist())
"""
    import os
    variant = root / "orb_slam2-chinese-annotation_amd" / "lib" / "variants" / "octree_passes2.so"
    assert variant.exists(), "build the test variant first (make -C orb_slam2-chinese-annotation_amd testhook)"
    env = dict(os.environ, ORB_AMD_LIB=str(variant))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=110,
                       env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    out = dict(l.split(": ", 1) for l in r.stdout.strip().splitlines())
    assert out["single"] == str(gpu.ORB_EDEVICE)
    assert out["batch"] == str([gpu.ORB_EDEVICE] * 4)


def test_octree_12k_batch4_global_nodes(gpu, oracle):
    """12,000 features put the octree's node tables in global memory (one slice
    per (image, level)); a batch of 4 takes the cell FAST path (level 0 and
    levels 1-2 on the side stream), three calls on a stream of the caller's."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(12)
    w, h, nf = 1920, 1080, 12000
    img = rng.integers(0, 256, (h, w), dtype=np.uint8)
    ext = gpu.ORBextractor(nf, 1.2, 8, 20, 7)
    cap = ext.capacity(w, h)
    imgs = torch.from_numpy(np.stack([img] * 4)).cuda()
    k = torch.zeros((4, cap, 7), dtype=torch.int32, device="cuda")
    d = torch.zeros((4, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(4, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    for _ in range(3):
        ext.extract_batch(imgs.data_ptr(), 4, w, h, w, w * h, k.data_ptr(), d.data_ptr(), cap,
                          n.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    kr, dr, _ = oracle.extract(img, nf)
    kk, dd, nn = k.cpu().numpy().view(gpu.KEYPOINT_DTYPE).reshape(4, cap), d.cpu().numpy(), n.cpu().numpy()
    for i in range(4):
        assert nn[i] == len(kr), (i, nn[i], len(kr))
        assert kk[i, :nn[i]].tobytes() == kr.tobytes()
        assert dd[i, :nn[i]].tobytes() == dr.tobytes()


def test_host_pyramid_mirror(gpu, oracle):
    """orb_extractor_host_pyramid: the first request copies the call's levels
    once, later calls carry the copy in their graph; every level equals the
    oracle's pyramid on consecutive frames, and across frame-size changes
    (the mirror and the staging are reallocated and the graph re-captured
    while the mirror stays on)."""
    ext = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    sizes = [(1241, 376)] * 3 + [(640, 480)] * 2 + [(1920, 1080), (1241, 376), (1241, 376)]
    for f, (w, h) in enumerate(sizes):
        img = gpu.synth_image(21, f, w, h)
        k, d = ext(img)
        kr, dr, _ = oracle.extract(img, 1000)
        assert k.tobytes() == kr.tobytes() and d.tobytes() == dr.tobytes(), f
        ref = oracle.pyramid(img)
        for l in range(8):
            assert np.array_equal(ext.host_pyramid(l), ref[l]), (f, l)
    with pytest.raises(gpu.OrbError):
        ext.host_pyramid(8)
    # switched off: calls move no pyramid; the next request copies once again
    ext.host_pyramid_off()
    for f in range(2):
        img = gpu.synth_image(22, f, 1241, 376)
        k, d = ext(img)
        kr, dr, _ = oracle.extract(img, 1000)
        assert k.tobytes() == kr.tobytes() and d.tobytes() == dr.tobytes(), f
    ref = oracle.pyramid(img)
    for l in range(8):
        assert np.array_equal(ext.host_pyramid(l), ref[l]), ("off", l)
