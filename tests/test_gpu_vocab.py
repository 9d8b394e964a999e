"""GPU parity of the DBoW2 vocabulary transform (Frame::ComputeBoW,
src/Frame.cc:439-449 / KeyFrame::ComputeBoW src/KeyFrame.cc:60-71 ->
TemplatedVocabulary::transform, Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1128-1283)
against the CPU oracle: word ids, BowVector values (exact doubles),
FeatureVector nodes / feature lists, per-feature word and node, bit-exact.
Vocabularies are synthetic (ORBvoc.txt is not in the reference tree)."""
import numpy as np
import pytest

import scenarios

pytestmark = pytest.mark.gpu


def _voc(gpu, v, scoring=0, weighting=0):
    return gpu.ORBVocabulary(v["k"], v["L"], v["parent"], v["leaf"], v["desc"], v["weight"],
                             scoring, weighting)


def _check(got, ref):
    bw, bv, fv, fw, fn = got
    rbw, rbv, rfvn, rfvo, rfvf, rfw, rfn = ref
    assert np.array_equal(bw, rbw)
    assert np.array_equal(bv.view(np.uint64), rbv.view(np.uint64))  # bit-exact doubles
    assert np.array_equal(fv[0], rfvn) and np.array_equal(fv[1], rfvo)
    assert np.array_equal(fv[2], rfvf)
    assert np.array_equal(fw, rfw) and np.array_equal(fn, rfn)


@pytest.mark.parametrize("kw,n", [
    (dict(rng_seed=0, k=10, L=4), 1000),
    (dict(rng_seed=2, k=6, L=4, irregular=True, stop_frac=0.2), 777),
    (dict(rng_seed=3, k=10, L=3, ties=True), 2000),
    (dict(rng_seed=4, k=3, L=5, irregular=True, ties=True, order="bfs"), 64),
    (dict(rng_seed=6, k=20, L=3), 1),
    (dict(rng_seed=8, k=17, L=2, irregular=True), 8192),
])
def test_vocab_transform(gpu, oracle, kw, n):
    v = scenarios.vocabulary(**kw)
    voc = _voc(gpu, v)
    assert voc.n_nodes == len(v["parent"]) and voc.n_words == int(v["leaf"].sum())
    feats = scenarios.vocab_features(v, n, rng_seed=kw["rng_seed"] + 100)
    for levelsup in (4, 0, 1, kw["L"] + 1):
        _check(voc.transform(feats, levelsup, per_feature=True),
               oracle.vocab_transform(v, feats, levelsup, 0, 0))


@pytest.mark.parametrize("scoring,weighting", [(s, w) for s in range(6) for w in range(4)])
def test_vocab_scoring_weighting(gpu, oracle, scoring, weighting):
    v = scenarios.vocabulary(rng_seed=7, k=8, L=3, stop_frac=0.1)
    voc = _voc(gpu, v, scoring, weighting)
    feats = scenarios.vocab_features(v, 1500, rng_seed=3, flip=0.1)
    _check(voc.transform(feats, 2, per_feature=True),
           oracle.vocab_transform(v, feats, 2, scoring, weighting))


def test_vocab_orb_slam_shape(gpu, oracle):
    # ORBvoc.txt shape (k 10, L 6, TF_IDF, L1) with ORB-SLAM2's levelsup 4, on
    # descriptors from the extractor (synthetic frame) and near-leaf features
    v = scenarios.vocabulary(rng_seed=11, k=10, L=6)
    voc = _voc(gpu, v)
    img = gpu.synth_image(0, 0, 1241, 376)
    ext = gpu.ORBextractor(2000, 1.2, 8, 20, 7)
    _, d = ext(img)
    for feats in (d, scenarios.vocab_features(v, 4000, rng_seed=2)):
        _check(voc.transform(feats, 4, per_feature=True), oracle.vocab_transform(v, feats, 4))


def test_vocab_empty_inputs(gpu, oracle):
    v = scenarios.vocabulary(rng_seed=0, k=4, L=2)
    voc = _voc(gpu, v)
    bw, bv, fv = voc.transform(np.zeros((0, 32), np.uint8))
    assert len(bw) == 0 and len(fv[0]) == 0 and fv[1].tolist() == [0]
    empty = gpu.ORBVocabulary(10, 6, np.zeros(1, np.int32), np.zeros(1, np.uint8),
                              np.zeros((1, 32), np.uint8), np.zeros(1))
    assert empty.empty()
    bw, bv, fv = empty.transform(np.ones((10, 32), np.uint8))
    assert len(bw) == 0 and fv[1].tolist() == [0]
    # all words stopped
    v2 = dict(v, weight=np.zeros_like(v["weight"]))
    bw, bv, fv, fw, fn = _voc(gpu, v2).transform(scenarios.vocab_features(v, 50), per_feature=True)
    assert len(bw) == 0 and len(fv[0]) == 0 and (fw == 0xFFFFFFFF).all()
    with pytest.raises(gpu.OrbError):
        voc.transform(np.zeros((8193, 32), np.uint8))
    with pytest.raises(gpu.OrbError):  # parent >= id
        gpu.ORBVocabulary(2, 1, np.array([0, 0, 5], np.int32), np.ones(3, np.uint8),
                          np.zeros((3, 32), np.uint8), np.ones(3))


def test_vocab_load_text(gpu, oracle, tmp_path):
    v = scenarios.vocabulary(rng_seed=5, k=9, L=4, irregular=True, stop_frac=0.05)
    path = tmp_path / "voc.txt"
    scenarios.write_vocabulary_text(v, path, scoring=1, weighting=0)
    with open(path, "a") as f:
        f.write("\n")
    voc = gpu.ORBVocabulary.loadFromTextFile(path)
    assert (voc.k, voc.L, voc.scoring, voc.weighting) == (9, 4, 1, 0)
    parsed = oracle.vocab_parse_text(path)
    feats = scenarios.vocab_features(v, 1200, rng_seed=9)
    _check(voc.transform(feats, 4, per_feature=True),
           oracle.vocab_transform(parsed, feats, 4, 1, 0))
    bad = tmp_path / "bad.txt"
    bad.write_text("10 11 0 0\n")  # L > 10 rejected (:1383)
    with pytest.raises(gpu.OrbError):
        gpu.ORBVocabulary.loadFromTextFile(bad)


def test_vocab_transform_batch(gpu, oracle):
    torch = pytest.importorskip("torch")
    v = scenarios.vocabulary(rng_seed=12, k=10, L=5, irregular=True, stop_frac=0.05)
    voc = _voc(gpu, v)
    stride = 2048
    counts = np.array([2048, 1000, 0, 1, 1777, 512, 2000, 64], np.int32)
    F = len(counts)
    desc = np.zeros((F, stride, 32), np.uint8)
    for f in range(F):
        desc[f, :counts[f]] = scenarios.vocab_features(v, int(counts[f]), rng_seed=f)
    dev = torch.device("cuda:0")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_counts, d_desc = t(counts), t(desc)
    z = lambda n, dt: torch.full((n,), -7, dtype=dt, device=dev)
    fw, fwt, fn = z(F * stride, torch.int32), z(F * stride, torch.float64), z(F * stride, torch.int32)
    bw, bv, nw = z(F * stride, torch.int32), z(F * stride, torch.float64), z(F, torch.int32)
    fvn, fvo, fvf, nfv = (z(F * stride, torch.int32), z(F * (stride + 1), torch.int32),
                          z(F * stride, torch.int32), z(F, torch.int32))
    torch.cuda.synchronize()
    voc.transform_batch(F, d_counts.data_ptr(), d_desc.data_ptr(), stride, 4, fw.data_ptr(),
                        fwt.data_ptr(), fn.data_ptr(), bw.data_ptr(), bv.data_ptr(),
                        nw.data_ptr(), fvn.data_ptr(), fvo.data_ptr(), fvf.data_ptr(),
                        nfv.data_ptr())
    torch.cuda.synchronize()
    h = lambda x: x.cpu().numpy()
    fw_, bw_, bv_, nw_, fn_ = h(fw).view(np.uint32), h(bw).view(np.uint32), h(bv), h(nw), h(fn)
    fvn_, fvo_, fvf_, nfv_ = h(fvn).view(np.uint32), h(fvo), h(fvf).view(np.uint32), h(nfv)
    for f in range(F):
        n = int(counts[f])
        rbw, rbv, rfvn, rfvo, rfvf, rfw, rfn = oracle.vocab_transform(v, desc[f, :n], 4)
        a, b = int(nw_[f]), int(nfv_[f])
        o = f * stride
        assert np.array_equal(bw_[o:o + a], rbw)
        assert np.array_equal(bv_[o:o + a].view(np.uint64), rbv.view(np.uint64))
        assert np.array_equal(fvn_[o:o + b], rfvn)
        oo = f * (stride + 1)
        assert np.array_equal(fvo_[oo:oo + b + 1], rfvo)
        assert np.array_equal(fvf_[o:o + rfvo[-1]], rfvf)
        if n:
            assert np.array_equal(fw_[o:o + n], rfw) and np.array_equal(fn_[o:o + n].view(np.uint32), rfn)


def test_vocab_feeds_search_by_bow(gpu, oracle):
    # Frame::ComputeBoW -> SearchByBoW(KF, F) chain on extracted frames: the
    # FeatureVectors from the GPU transform give the same matches as the
    # oracle's transform + oracle matcher.
    v = scenarios.vocabulary(rng_seed=21, k=10, L=5)
    voc = _voc(gpu, v)
    bp = scenarios.bow_pair(oracle, 3)
    kf_fv = voc.transform(bp["kf_desc"], 4)[2]
    f_fv = voc.transform(bp["f_desc"], 4)[2]
    r1 = oracle.vocab_transform(v, bp["kf_desc"], 4)
    r2 = oracle.vocab_transform(v, bp["f_desc"], 4)
    for a, b in zip(kf_fv, r1[2:5]):
        assert np.array_equal(a, b)
    for a, b in zip(f_fv, r2[2:5]):
        assert np.array_equal(a, b)
    n, fm = gpu.ORBmatcher(0.75, True).SearchByBoW(bp["kf_desc"], bp["kf_angle"], bp["kf_mp"],
                                                   bp["kf_bad"], kf_fv, bp["f_desc"],
                                                   bp["f_angle"], f_fv)
    n_ref, fm_ref = oracle.match_bow(bp["kf_desc"], bp["kf_angle"], bp["kf_mp"], bp["kf_bad"],
                                     r1[2:5], bp["f_desc"], bp["f_angle"], r2[2:5], 0.75, True)
    assert n == n_ref and np.array_equal(fm, fm_ref) and n > 0
