"""GPU ComputeStereoMatches, SearchByProjection(F, LastFrame) and SearchByBoW
against the CPU oracle: float outputs bit-exact, assignments index-exact."""
import numpy as np
import pytest

import scenarios

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", [1, 2])
def test_stereo_matches(gpu, oracle, seed):
    sp = scenarios.stereo_pair(oracle, seed)
    args = (sp["kl"], sp["dl"], sp["scale"], sp["kr"], sp["dr"], sp["lpyr"], sp["rpyr"],
            sp["inv"], scenarios.BF, scenarios.FX, sp["w"], sp["h"])
    ur_ref, dp_ref = oracle.stereo_match(*args)
    F = gpu.Frame(sp["kl"], sp["dl"], sp["scale"], sp["w"], sp["h"])
    ur, dp = gpu.ORBmatcher().ComputeStereoMatches(F, sp["kr"], sp["dr"], sp["lpyr"], sp["rpyr"],
                                                   sp["inv"], scenarios.BF, scenarios.FX)
    assert (ur_ref > 0).sum() > 50
    assert ur.tobytes() == ur_ref.tobytes(), np.nonzero(ur != ur_ref)[0][:10]
    assert dp.tobytes() == dp_ref.tobytes()


def test_stereo_distance_ties(gpu, oracle):
    """Every right keypoint twice: a copy 3 px to the right with the same
    descriptor and the SMALLER index, then the original.  Each candidate's
    distance ties with its copy's, and the reference's first minimum in
    ascending iR picks the copy (src/Frame.cc:584-607), whose x moves the SAD
    search.  The device row lists hold the two in arbitrary order, so this
    pins the (distance, iR) order inside a lane as well as across lanes."""
    sp = scenarios.stereo_pair(oracle, 3)
    kr, dr = sp["kr"], sp["dr"]
    moved = kr.copy()
    moved["x"] = (moved["x"] + np.float32(3.0)).astype(np.float32)
    # blocks of 64: the copies, then their originals, so the two of a tie
    # are listed by different waves of the same round of the list builder
    n = len(kr) // 64 * 64
    parts_k, parts_d = [], []
    for b in range(0, n, 64):
        parts_k += [moved[b:b + 64], kr[b:b + 64]]
        parts_d += [dr[b:b + 64], dr[b:b + 64]]
    kr2 = np.concatenate(parts_k)
    dr2 = np.concatenate(parts_d)
    args = (sp["kl"], sp["dl"], sp["scale"], kr2, dr2, sp["lpyr"], sp["rpyr"],
            sp["inv"], scenarios.BF, scenarios.FX, sp["w"], sp["h"])
    ur_ref, dp_ref = oracle.stereo_match(*args)
    F = gpu.Frame(sp["kl"], sp["dl"], sp["scale"], sp["w"], sp["h"])
    ur, dp = gpu.ORBmatcher().ComputeStereoMatches(F, kr2, dr2, sp["lpyr"], sp["rpyr"],
                                                   sp["inv"], scenarios.BF, scenarios.FX)
    assert (ur_ref > 0).sum() > 50
    assert ur.tobytes() == ur_ref.tobytes(), np.nonzero(ur != ur_ref)[0][:10]
    assert dp.tobytes() == dp_ref.tobytes()


def test_stereo_batch_from_extractors(gpu, oracle):
    """C3 path: both images of each pair through extract_batch, stereo on device."""
    torch = pytest.importorskip("torch")
    w, h, nf, P = 1241, 376, 2000, 3
    L = gpu.ORBextractor(nf, 1.2, 8, 20, 7)
    R = gpu.ORBextractor(nf, 1.2, 8, 20, 7)
    cap = L.capacity(w, h)
    imgs_l = np.stack([oracle.synth_image(30 + i, 0, w, h, 0) for i in range(P)])
    imgs_r = np.stack([oracle.synth_image(30 + i, 0, w, h, 1) for i in range(P)])
    dev = "cuda"
    dl, dr = torch.from_numpy(imgs_l).to(dev), torch.from_numpy(imgs_r).to(dev)
    out = {}
    for name, ext, d in (("l", L, dl), ("r", R, dr)):
        k = torch.zeros((P, cap, 7), dtype=torch.int32, device=dev)
        de = torch.zeros((P, cap, 32), dtype=torch.uint8, device=dev)
        n = torch.zeros(P, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        ext.extract_batch(d.data_ptr(), P, w, h, w, w * h, k.data_ptr(), de.data_ptr(), cap,
                          n.data_ptr())
        torch.cuda.synchronize()
        out[name] = (k, de, n)
    ur = torch.zeros((P, cap), dtype=torch.float32, device=dev)
    dp = torch.zeros((P, cap), dtype=torch.float32, device=dev)
    sad = torch.zeros((P, cap), dtype=torch.int32, device=dev)
    m = gpu.ORBmatcher()
    (kl, dlsc, nl), (kr, drsc, nr) = out["l"], out["r"]
    m.stereo_match_batch(P, L, R, kl.data_ptr(), dlsc.data_ptr(), nl.data_ptr(), kr.data_ptr(),
                         drsc.data_ptr(), nr.data_ptr(), cap, scenarios.BF, scenarios.FX,
                         ur.data_ptr(), dp.data_ptr(), sad.data_ptr())
    torch.cuda.synchronize()
    p = oracle.params(nf)
    for i in range(P):
        klh, dlh, _ = oracle.extract(imgs_l[i], nf)
        krh, drh, _ = oracle.extract(imgs_r[i], nf)
        ur_ref, dp_ref = oracle.stereo_match(klh, dlh, p["scale"], krh, drh,
                                             oracle.pyramid(imgs_l[i]), oracle.pyramid(imgs_r[i]),
                                             p["inv_scale"], scenarios.BF, scenarios.FX, w, h)
        n = int(nl[i].item())
        assert n == len(klh)
        assert ur[i, :n].cpu().numpy().tobytes() == ur_ref.tobytes()
        assert dp[i, :n].cpu().numpy().tobytes() == dp_ref.tobytes()


@pytest.mark.parametrize("mono,tlc,th", [(1, 0.0, 15.0), (0, 1.0, 7.0), (0, -1.0, 7.0),
                                         (0, 0.0, 14.0)])
@pytest.mark.parametrize("check_ori", [1, 0])
def test_search_by_projection_frame(gpu, oracle, mono, tlc, th, check_ori):
    fp = scenarios.frame_pair(oracle, 2, rng_seed=int(th))
    rng = np.random.default_rng(7)
    n = len(fp["kb"])
    ur = None if mono else np.where(rng.random(n) < 0.6,
                                    fp["kb"]["x"] - rng.uniform(3, 60, n), -1).astype(np.float32)
    locked = (rng.random(n) < 0.1).astype(np.uint8)
    n_ref, km_ref = oracle.match_projection_frame(
        fp["kb"], fp["db"], fp["scale"], fp["w"], fp["h"], fp["last"], fp["last_desc"],
        scenarios.camera(), tlc, th, mono, check_ori, locked, ur)
    F = gpu.Frame(fp["kb"], fp["db"], fp["scale"], fp["w"], fp["h"], u_right=ur)
    m = gpu.ORBmatcher(0.9, bool(check_ori))
    n_gpu, km = m.SearchByProjectionFrame(F, fp["last"], fp["last_desc"], scenarios.camera(), tlc,
                                          th, bool(mono), locked)
    assert n_ref > 100
    assert n_gpu == n_ref
    assert np.array_equal(km, km_ref), np.nonzero(km != km_ref)[0][:10]


@pytest.mark.parametrize("seed,nnratio", [(4, 0.75), (5, 0.7), (6, 0.9)])
@pytest.mark.parametrize("check_ori", [1, 0])
def test_search_by_bow(gpu, oracle, seed, nnratio, check_ori):
    bp = scenarios.bow_pair(oracle, seed)
    n_ref, fm_ref = oracle.match_bow(bp["kf_desc"], bp["kf_angle"], bp["kf_mp"], bp["kf_bad"],
                                     bp["kf_fv"], bp["f_desc"], bp["f_angle"], bp["f_fv"], nnratio,
                                     check_ori)
    m = gpu.ORBmatcher(nnratio, bool(check_ori))
    n_gpu, fm = m.SearchByBoW(bp["kf_desc"], bp["kf_angle"], bp["kf_mp"], bp["kf_bad"],
                              bp["kf_fv"], bp["f_desc"], bp["f_angle"], bp["f_fv"])
    assert n_ref > 50
    assert n_gpu == n_ref
    assert np.array_equal(fm, fm_ref)


@pytest.mark.parametrize("seed", [1, 3])
def test_stereo_from_extracted_handles(gpu, oracle, seed):
    """Frame's stereo path with nothing but mvuRight / mvDepth leaving the GPU:
    both handles' last orb_extractor_extract feeds orb_stereo_match_extracted."""
    sp = scenarios.stereo_pair(oracle, seed)
    L = gpu.ORBextractor(2000, 1.2, 8, 20, 7)
    R = gpu.ORBextractor(2000, 1.2, 8, 20, 7)
    kl, dl = L(oracle.synth_image(seed, 0, sp["w"], sp["h"], 0))
    kr, dr = R(oracle.synth_image(seed, 0, sp["w"], sp["h"], 1))
    assert kl.tobytes() == sp["kl"].tobytes() and kr.tobytes() == sp["kr"].tobytes()
    ur_ref, dp_ref = oracle.stereo_match(sp["kl"], sp["dl"], sp["scale"], sp["kr"], sp["dr"],
                                         sp["lpyr"], sp["rpyr"], sp["inv"], scenarios.BF,
                                         scenarios.FX, sp["w"], sp["h"])
    ur, dp = gpu.ORBmatcher().ComputeStereoMatchesExtracted(L, R, scenarios.BF, scenarios.FX)
    assert (ur_ref > 0).sum() > 50
    assert ur.tobytes() == ur_ref.tobytes() and dp.tobytes() == dp_ref.tobytes()
    # a batch call on a handle invalidates its single-image state (the batch
    # itself must succeed: only the stereo call may raise)
    torch = pytest.importorskip("torch")
    img = torch.from_numpy(oracle.synth_image(seed, 1, sp["w"], sp["h"])).cuda()
    cap = L.capacity(sp["w"], sp["h"])
    k = torch.zeros((1, cap, 7), dtype=torch.int32, device="cuda")
    d = torch.zeros((1, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(1, dtype=torch.int32, device="cuda")
    L.extract_batch(img.data_ptr(), 1, sp["w"], sp["h"], sp["w"], sp["w"] * sp["h"],
                    k.data_ptr(), d.data_ptr(), cap, n.data_ptr())
    torch.cuda.synchronize()
    assert int(n[0]) > 0
    with pytest.raises(gpu.OrbError):
        gpu.ORBmatcher().ComputeStereoMatchesExtracted(L, R, scenarios.BF, scenarios.FX)
