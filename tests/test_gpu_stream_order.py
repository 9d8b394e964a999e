"""One handle driven from several caller streams with no host synchronisation.

Every extractor call reuses its handle's device scratch (pyramid arena, cell
keys, octree tables) and a frame-size change rewrites the handle's plan tables;
every matcher call reuses the grid, candidate lists and claim buffers.  The
batch entry points run asynchronously on whatever stream the caller passes, so
the library orders a call after the previous call on the same handle whenever
the stream changes (runtime.cpp CallOrder; include/orb_abi.h "Streams").  The
reference states the rule in host form: an ORBextractor is not reentrant
(include/ORBextractor.h:85; it rebuilds mvImagePyramid on every call), and
Frame runs two instances at once (src/Frame.cc:81-84).

Each test issues back-to-back calls on alternating streams, the first one
large enough to still be running when the next is issued, then compares every
frame and every problem with the oracle (bit- / index-exact).
ORB_AMD_LIB=<a build with -DORB_CALL_ORDER=0> is the negative control
(tools/archive/r06/stream_order_neg.sh): it fails these tests.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NF = 1000


def _pool(fn, items):
    with ThreadPoolExecutor(max_workers=16) as ex:
        return list(ex.map(fn, items))


def _frames(gpu, seed, n, w, h):
    return np.stack([gpu.synth_image(seed, f, w, h) for f in range(n)])


def test_extractor_across_streams_and_sizes(gpu, oracle):
    torch = pytest.importorskip("torch")
    ext = gpu.ORBextractor(NF, 1.2, 8, 20, 7)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    # (stream, width, height, frames): a size change between calls 1 -> 2 -> 3,
    # and two same-size calls on two streams (3 -> 4)
    calls = [(s1, 1241, 376, 160), (s2, 640, 480, 24), (s1, 1241, 376, 96), (s2, 1241, 376, 64)]
    bufs = []
    for i, (_, w, h, n) in enumerate(calls):
        imgs = _frames(gpu, 600 + i, n, w, h)
        cap = ext.capacity(w, h)
        bufs.append(dict(imgs=imgs, cap=cap, d_img=torch.from_numpy(imgs).cuda(),
                         d_kps=torch.full((n, cap, 7), -3, dtype=torch.int32, device="cuda"),
                         d_desc=torch.zeros((n, cap, 32), dtype=torch.uint8, device="cuda"),
                         d_cnt=torch.full((n,), -9, dtype=torch.int32, device="cuda")))
    torch.cuda.synchronize()
    for (s, w, h, n), b in zip(calls, bufs):  # no host sync between the calls
        ext.extract_batch(b["d_img"].data_ptr(), n, w, h, w, w * h, b["d_kps"].data_ptr(),
                          b["d_desc"].data_ptr(), b["cap"], b["d_cnt"].data_ptr(),
                          stream=s.cuda_stream)
    torch.cuda.synchronize()
    for (s, w, h, n), b in zip(calls, bufs):
        kps = b["d_kps"].cpu().numpy().view(gpu.KEYPOINT_DTYPE).reshape(n, b["cap"])
        desc = b["d_desc"].cpu().numpy()
        cnt = b["d_cnt"].cpu().numpy()
        ref = _pool(lambda f: oracle.extract(b["imgs"][f], NF, 1.2, 8, 20, 7)[:2], range(n))
        for f, (kr, dr) in enumerate(ref):
            assert cnt[f] == len(kr), (w, h, f, cnt[f], len(kr))
            assert kps[f, :cnt[f]].tobytes() == kr.tobytes(), (w, h, f)
            assert desc[f, :cnt[f]].tobytes() == dr.tobytes(), (w, h, f)


def test_single_frame_call_after_batch_on_caller_stream(gpu, oracle):
    # the single-frame call (the handle's own stream) right behind a batch on
    # a caller's stream, no sync in between
    torch = pytest.importorskip("torch")
    w, h, n = 1241, 376, 128
    ext = gpu.ORBextractor(NF, 1.2, 8, 20, 7)
    imgs = _frames(gpu, 700, n, w, h)
    cap = ext.capacity(w, h)
    d_img = torch.from_numpy(imgs).cuda()
    d_kps = torch.zeros((n, cap, 7), dtype=torch.int32, device="cuda")
    d_desc = torch.zeros((n, cap, 32), dtype=torch.uint8, device="cuda")
    d_cnt = torch.zeros(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    one = gpu.synth_image(701, 0, 640, 480)
    torch.cuda.synchronize()
    ext.extract_batch(d_img.data_ptr(), n, w, h, w, w * h, d_kps.data_ptr(), d_desc.data_ptr(),
                      cap, d_cnt.data_ptr(), stream=s.cuda_stream)
    k1, d1 = ext(one)
    torch.cuda.synchronize()
    kr, dr, _ = oracle.extract(one, NF, 1.2, 8, 20, 7)
    assert k1.tobytes() == kr.tobytes() and d1.tobytes() == dr.tobytes()
    kps = d_kps.cpu().numpy().view(gpu.KEYPOINT_DTYPE).reshape(n, cap)
    cnt = d_cnt.cpu().numpy()
    for f in (0, n // 2, n - 1):
        kr, dr, _ = oracle.extract(imgs[f], NF, 1.2, 8, 20, 7)
        assert kps[f, :cnt[f]].tobytes() == kr.tobytes(), f
        assert d_desc[f, :cnt[f]].cpu().numpy().tobytes() == dr.tobytes(), f


def test_matcher_alternating_streams(gpu, oracle):
    torch = pytest.importorskip("torch")
    w, h, M = 1241, 376, 5000
    ext = gpu.ORBextractor(NF, 1.2, 8, 20, 7)
    scale = np.float32(ext.GetScaleFactors())
    cap = ext.capacity(w, h)
    m = gpu.ORBmatcher(0.8)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    sizes = [192, 8, 64, 16]  # problems per call; calls alternate s1, s2, s1, s2
    imgs = _frames(gpu, 800, max(sizes), w, h)
    ext_ref = _pool(lambda f: oracle.extract(imgs[f], NF, 1.2, 8, 20, 7)[:2], range(len(imgs)))
    calls = []
    for c, B in enumerate(sizes):
        frames = [(c * 37 + i) % len(imgs) for i in range(B)]
        kps = np.zeros((B, cap), gpu.KEYPOINT_DTYPE)
        desc = np.zeros((B, cap, 32), np.uint8)
        cnt = np.zeros(B, np.int32)
        lk = np.zeros((B, cap), np.uint8)
        maps = []
        for i, f in enumerate(frames):
            k, d = ext_ref[f]
            kps[i, :len(k)] = k
            desc[i, :len(k)] = d
            cnt[i] = len(k)
            mm = gpu.synth_local_map(900 + 7 * c + i, k, d, M, w, h)
            lk[i, :len(k)] = mm[2]
            maps.append(mm)
        mps = np.stack([mm[0] for mm in maps])
        mpd = np.stack([mm[1] for mm in maps])
        calls.append(dict(
            B=B, kps=kps, desc=desc, cnt=cnt, maps=maps,
            d_k=torch.from_numpy(kps.view(np.uint8).reshape(B, -1)).cuda(),
            d_d=torch.from_numpy(desc).cuda(), d_n=torch.from_numpy(cnt).cuda(),
            d_lk=torch.from_numpy(lk).cuda(),
            d_mps=torch.from_numpy(mps.view(np.uint8).reshape(B, -1)).cuda(),
            d_mpd=torch.from_numpy(mpd).cuda(),
            d_nm=torch.full((B,), M, dtype=torch.int32, device="cuda"),
            km=torch.full((B, cap), -7, dtype=torch.int32, device="cuda"),
            nm=torch.full((B,), -7, dtype=torch.int32, device="cuda")))
    torch.cuda.synchronize()
    for c, x in enumerate(calls):  # no host sync between the calls
        s = (s1, s2)[c % 2]
        m.search_by_projection_batch(x["B"], x["d_k"].data_ptr(), x["d_d"].data_ptr(),
                                     x["d_n"].data_ptr(), x["d_lk"].data_ptr(), cap,
                                     x["d_mps"].data_ptr(), x["d_mpd"].data_ptr(),
                                     x["d_nm"].data_ptr(), M, w, h, scale, 1.0,
                                     x["km"].data_ptr(), x["nm"].data_ptr(), stream=s.cuda_stream)
    # and the host-buffer form on the handle's own stream right behind them
    x0 = calls[0]
    F = gpu.Frame(x0["kps"][0, :x0["cnt"][0]], x0["desc"][0, :x0["cnt"][0]], scale, w, h)
    n_host, km_host = m.SearchByProjection(F, x0["maps"][0][0], x0["maps"][0][1], 1.0,
                                           x0["maps"][0][2])
    torch.cuda.synchronize()
    total = 0
    for c, x in enumerate(calls):
        got_km, got_n = x["km"].cpu().numpy(), x["nm"].cpu().numpy()
        want = _pool(lambda i: oracle.match_projection_local(
            x["kps"][i, :x["cnt"][i]], x["desc"][i, :x["cnt"][i]], scale, w, h,
            x["maps"][i][0], x["maps"][i][1], 1.0, 0.8, x["maps"][i][2]), range(x["B"]))
        for i, (n_ref, km_ref) in enumerate(want):
            assert got_n[i] == n_ref, (c, i, got_n[i], n_ref)
            assert np.array_equal(got_km[i, :x["cnt"][i]], km_ref), (c, i)
            total += n_ref
        if c == 0:
            assert n_host == want[0][0] and np.array_equal(km_host, want[0][1])
    assert total > 300 * sum(sizes)
