"""GPU parity of the remaining ORBmatcher variants against
the CPU oracle: assignments index-exact, counts equal."""
import math

import numpy as np
import pytest

import scenarios as S

pytestmark = pytest.mark.gpu

LS = np.float32(math.log(np.float32(1.2)))


@pytest.fixture(scope="module", params=[(3, 1), (7, 2)])
def pair(request, oracle):
    seed, rs = request.param
    return S.keyframe_pair(oracle, seed, rng_seed=rs)


def _points(kf, rng, seen=0.05):
    mps = kf["mps"].copy()
    mps["bad"] |= kf["valid"] == 0
    mps["seen"] = rng.random(len(mps)) < seen
    return mps


def _frame(gpu, kf, stereo=False):
    return gpu.Frame(kf["keys"], kf["desc"], kf["scale"], kf["width"], kf["height"],
                     u_right=kf["u_right"] if stereo else None)


@pytest.mark.parametrize("th,orb_dist,ori", [(10, 100, True), (3, 64, True), (5, 50, False)])
def test_reloc_projection(gpu, oracle, pair, th, orb_dist, ori):
    kf0, kf1 = pair
    rng = np.random.default_rng(11)
    mps = _points(kf0, rng, 0.1)
    lk = (rng.random(len(kf1["keys"])) < 0.2).astype(np.uint8)
    pose = S.pose_record(oracle, kf1["Rw"], kf1["tw"])
    rn, rk = oracle.search_by_projection_reloc(kf1["keys"], kf1["desc"], kf1["scale"], 1241, 376,
                                               pose, S.camera(), mps, kf0["mp_desc"],
                                               kf0["keys"]["angle"], th, orb_dist, ori, lk, LS)
    m = gpu.ORBmatcher(0.75, ori)
    n, km = m.SearchByProjectionKF(_frame(gpu, kf1), pose, S.camera(), float(LS), mps,
                                   kf0["mp_desc"], kf0["keys"]["angle"], th, orb_dist, lk)
    assert rn > 20
    assert n == rn
    assert np.array_equal(km, rk), np.nonzero(km != rk)[0][:10]


@pytest.mark.parametrize("s,th", [(1.7, 10), (0.6, 5)])
def test_sim3_projection(gpu, oracle, pair, s, th):
    kf0, kf1 = pair
    rng = np.random.default_rng(12)
    mps = _points(kf0, rng)
    Sc = S.scw(kf1["Rw"], kf1["tw"], s)
    mm = np.where(rng.random(len(kf1["keys"])) < 0.1, rng.integers(0, 500, len(kf1["keys"])),
                  -1).astype(np.int32)
    rn, rk = oracle.search_by_projection_sim3(kf1["keys"], kf1["desc"], kf1["scale"], 1241, 376,
                                              Sc, S.camera(), mps, kf0["mp_desc"], th, mm, LS)
    n, km = gpu.ORBmatcher().SearchByProjectionSim3(_frame(gpu, kf1), Sc, S.camera(), float(LS),
                                                    mps, kf0["mp_desc"], th, mm)
    assert rn > 20
    assert n == rn
    assert np.array_equal(km, rk), np.nonzero(km != rk)[0][:10]


@pytest.mark.parametrize("th", [3.0, 1.0])
def test_fuse(gpu, oracle, pair, th):
    kf0, kf1 = pair
    rng = np.random.default_rng(13)
    mps = _points(kf0, rng)
    pose = S.pose_record(oracle, kf1["Rw"], kf1["tw"])
    rn, rb = oracle.fuse(kf1["keys"], kf1["desc"], kf1["scale"], kf1["inv_sigma2"], 1241, 376,
                         kf1["u_right"], pose, S.camera(), mps, kf0["mp_desc"], th, LS)
    n, b = gpu.ORBmatcher().Fuse(_frame(gpu, kf1, stereo=True), kf1["inv_sigma2"], pose,
                                 S.camera(), float(LS), mps, kf0["mp_desc"], th)
    assert rn > 20
    assert n == rn and np.array_equal(b, rb)


def test_fuse_sim3(gpu, oracle, pair):
    kf0, kf1 = pair
    rng = np.random.default_rng(14)
    mps = _points(kf0, rng)
    Sc = S.scw(kf1["Rw"], kf1["tw"], 2.3)
    rn, rb = oracle.fuse_sim3(kf1["keys"], kf1["desc"], kf1["scale"], 1241, 376, Sc, S.camera(),
                              mps, kf0["mp_desc"], 4.0, LS)
    n, b = gpu.ORBmatcher().FuseSim3(_frame(gpu, kf1), Sc, S.camera(), float(LS), mps,
                                     kf0["mp_desc"], 4.0)
    assert rn > 20
    assert n == rn and np.array_equal(b, rb)


@pytest.mark.parametrize("s12", [1.0, 1.05])
def test_search_by_sim3(gpu, oracle, pair, s12):
    kf0, kf1 = pair
    rng = np.random.default_rng(15)
    k0, k1 = dict(kf0), dict(kf1)
    k0["already"] = (rng.random(len(k0["keys"])) < 0.05).astype(np.uint8)
    k1["already"] = (rng.random(len(k1["keys"])) < 0.05).astype(np.uint8)
    R12 = (kf0["Rw"].astype(np.float64) @ kf1["Rw"].astype(np.float64).T).astype(np.float32)
    t12 = (kf0["tw"] - R12.astype(np.float64) @ kf1["tw"]).astype(np.float32)
    rn, rm = oracle.search_by_sim3(k0, k1, S.camera(), s12, R12, t12, 7.5, LS)
    n, m12 = gpu.ORBmatcher().SearchBySim3(
        _frame(gpu, k0), _frame(gpu, k1), float(LS), S.camera(), k0["Rw"], k0["tw"], k1["Rw"],
        k1["tw"], k0["mps"], k0["valid"], k0["already"], k0["mp_desc"], k1["mps"], k1["valid"],
        k1["already"], k1["mp_desc"], s12, R12, t12, 7.5)
    assert rn > 20
    assert n == rn and np.array_equal(m12, rm)


@pytest.mark.parametrize("ratio,ori", [(0.75, True), (0.9, False)])
def test_bow_kf(gpu, oracle, pair, ratio, ori):
    kf0, kf1 = pair
    fv0 = oracle.feature_vector(S.vocab_nodes(kf0["desc"]))
    fv1 = oracle.feature_vector(S.vocab_nodes(kf1["desc"]))
    mp0 = np.where(kf0["valid"] > 0, np.arange(len(kf0["keys"])), -1).astype(np.int32)
    mp1 = np.where(kf1["valid"] > 0, np.arange(len(kf1["keys"])) + 10000, -1).astype(np.int32)
    b0 = kf0["mps"]["bad"].astype(np.uint8)
    b1 = kf1["mps"]["bad"].astype(np.uint8)
    rn, rm = oracle.search_by_bow_kf(kf0["desc"], kf0["keys"]["angle"], mp0, b0, fv0,
                                     kf1["desc"], kf1["keys"]["angle"], mp1, b1, fv1, ratio, ori)
    n, m = gpu.ORBmatcher(ratio, ori).SearchByBoWKF(kf0["desc"], kf0["keys"]["angle"], mp0, b0,
                                                    fv0, kf1["desc"], kf1["keys"]["angle"], mp1,
                                                    b1, fv1)
    assert rn > 20
    assert n == rn and np.array_equal(m, rm)


@pytest.mark.parametrize("stereo,ori", [(False, True), (True, False), (False, False)])
def test_triangulation(gpu, oracle, stereo, ori):
    k0, k1 = S.keyframe_pair(oracle, 3, rng_seed=1, baseline=(0.5, 0.0, 0.1))
    rng = np.random.default_rng(16)
    for d in (k0, k1):
        d["has_mp"] = (rng.random(len(d["keys"])) < 0.5).astype(np.uint8)
    F12 = S.fundamental(k0, k1)
    fv0 = oracle.feature_vector(S.vocab_nodes(k0["desc"]))
    fv1 = oracle.feature_vector(S.vocab_nodes(k1["desc"]))
    rn, rm = oracle.search_for_triangulation(k0, k1, k1["sigma2"], F12, S.camera(), k0["ow"],
                                             k1["Rw"], k1["tw"], fv0, fv1, stereo, ori)
    n, m = gpu.ORBmatcher(0.6, ori).SearchForTriangulation(
        _frame(gpu, k0, True), k0["has_mp"], _frame(gpu, k1, True), k1["has_mp"], k1["sigma2"],
        F12, S.camera(), k0["ow"], k1["Rw"], k1["tw"], fv0, fv1, stereo)
    assert rn > 10
    assert n == rn and np.array_equal(m, rm)


def test_variants_empty_inputs(gpu, oracle, pair):
    kf0, kf1 = pair
    m = gpu.ORBmatcher()
    pose = S.pose_record(oracle, kf1["Rw"], kf1["tw"])
    none = kf0["mps"][:0]
    n, km = m.SearchByProjectionKF(_frame(gpu, kf1), pose, S.camera(), float(LS), none,
                                   kf0["mp_desc"][:0], kf0["keys"]["angle"][:0], 10, 100)
    assert n == 0 and (km == -1).all()
    n, b = m.Fuse(_frame(gpu, kf1), kf1["inv_sigma2"], pose, S.camera(), float(LS), none,
                  kf0["mp_desc"][:0])
    assert n == 0 and len(b) == 0
    # every keypoint already locked: nothing can match
    n, km = m.SearchByProjectionKF(_frame(gpu, kf1), pose, S.camera(), float(LS), kf0["mps"],
                                   kf0["mp_desc"], kf0["keys"]["angle"], 10, 100,
                                   np.ones(len(kf1["keys"]), np.uint8))
    assert n == 0 and (km == -1).all()
