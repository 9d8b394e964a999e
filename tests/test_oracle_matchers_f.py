"""Oracle restatements of the remaining ORBmatcher variants
against the independent Python restatements in pyref.py (test infrastructure).
The reference ships no fixtures for these functions, so parity beyond this
cross-check is unpinned."""
import math

import numpy as np
import pytest

import pyref
import scenarios as S

LS = np.float32(math.log(np.float32(1.2)))


@pytest.fixture(scope="module")
def pair(oracle):
    return S.keyframe_pair(oracle, 3, rng_seed=1)


def _points(kf, rng, seen=0.05):
    mps = kf["mps"].copy()
    mps["bad"] |= kf["valid"] == 0
    mps["seen"] = rng.random(len(mps)) < seen
    return mps


def test_reloc_matches_restatement(oracle, pair):
    kf0, kf1 = pair
    rng = np.random.default_rng(5)
    mps = _points(kf0, rng, 0.1)
    lk = (rng.random(len(kf1["keys"])) < 0.2).astype(np.uint8)
    pose = S.pose_record(oracle, kf1["Rw"], kf1["tw"])
    for th, od, ori in ((10, 100, True), (3, 50, False)):
        n, km = oracle.search_by_projection_reloc(kf1["keys"], kf1["desc"], kf1["scale"], 1241,
                                                  376, pose, S.camera(), mps, kf0["mp_desc"],
                                                  kf0["keys"]["angle"], th, od, ori, lk, LS)
        pn, pk = pyref.search_by_projection_reloc(kf1["keys"], kf1["desc"], kf1["scale"], 1241,
                                                  376, kf1["Rw"], kf1["tw"], pose["ow"][0],
                                                  S.camera(), mps, kf0["mp_desc"],
                                                  kf0["keys"]["angle"], th, od, ori, lk, LS)
        assert n == pn and n > 50
        assert np.array_equal(km, pk)


def test_sim3_projection_matches_restatement(oracle, pair):
    kf0, kf1 = pair
    rng = np.random.default_rng(6)
    mps = _points(kf0, rng)
    Sc = S.scw(kf1["Rw"], kf1["tw"], 1.7)
    mm = np.where(rng.random(len(kf1["keys"])) < 0.1, rng.integers(0, 500, len(kf1["keys"])),
                  -1).astype(np.int32)
    n, km = oracle.search_by_projection_sim3(kf1["keys"], kf1["desc"], kf1["scale"], 1241, 376,
                                             Sc, S.camera(), mps, kf0["mp_desc"], 10, mm, LS)
    pn, pk = pyref.search_by_projection_sim3(kf1["keys"], kf1["desc"], kf1["scale"], 1241, 376,
                                             Sc, S.camera(), mps, kf0["mp_desc"], 10, mm, LS)
    assert n == pn and n > 50
    assert np.array_equal(km, pk)


def test_fuse_matches_restatement(oracle, pair):
    kf0, kf1 = pair
    rng = np.random.default_rng(7)
    mps = _points(kf0, rng)
    pose = S.pose_record(oracle, kf1["Rw"], kf1["tw"])
    n, best = oracle.fuse(kf1["keys"], kf1["desc"], kf1["scale"], kf1["inv_sigma2"], 1241, 376,
                          kf1["u_right"], pose, S.camera(), mps, kf0["mp_desc"], 3.0, LS)
    pn, pb = pyref.fuse(kf1["keys"], kf1["desc"], kf1["scale"], kf1["inv_sigma2"], 1241, 376,
                        kf1["u_right"], kf1["Rw"], kf1["tw"], pose["ow"][0], S.camera(), mps,
                        kf0["mp_desc"], 3.0, LS)
    assert n == pn and n > 50
    assert np.array_equal(best, pb)


def test_search_by_sim3_matches_restatement(oracle, pair):
    kf0, kf1 = pair
    rng = np.random.default_rng(8)
    k0, k1 = dict(kf0), dict(kf1)
    k0["already"] = (rng.random(len(k0["keys"])) < 0.05).astype(np.uint8)
    k1["already"] = (rng.random(len(k1["keys"])) < 0.05).astype(np.uint8)
    R12 = (kf0["Rw"].astype(np.float64) @ kf1["Rw"].astype(np.float64).T).astype(np.float32)
    t12 = (kf0["tw"] - R12.astype(np.float64) @ kf1["tw"]).astype(np.float32)
    for s12 in (1.0, 1.05):
        n, m12 = oracle.search_by_sim3(k0, k1, S.camera(), s12, R12, t12, 7.5, LS)
        pn, pm = pyref.search_by_sim3(k0, k1, S.camera(), s12, R12, t12, 7.5, LS)
        assert n == pn and n > 50
        assert np.array_equal(m12, pm)


def test_bow_kf_matches_restatement(oracle, pair):
    kf0, kf1 = pair
    fv0 = oracle.feature_vector(S.vocab_nodes(kf0["desc"]))
    fv1 = oracle.feature_vector(S.vocab_nodes(kf1["desc"]))
    mp0 = np.where(kf0["valid"] > 0, np.arange(len(kf0["keys"])), -1).astype(np.int32)
    mp1 = np.where(kf1["valid"] > 0, np.arange(len(kf1["keys"])) + 10000, -1).astype(np.int32)
    b0 = kf0["mps"]["bad"].astype(np.uint8)
    b1 = kf1["mps"]["bad"].astype(np.uint8)
    for ratio, ori in ((0.75, True), (0.9, False)):
        n, m = oracle.search_by_bow_kf(kf0["desc"], kf0["keys"]["angle"], mp0, b0, fv0,
                                       kf1["desc"], kf1["keys"]["angle"], mp1, b1, fv1, ratio, ori)
        pn, pm = pyref.search_by_bow_kf(kf0["desc"], kf0["keys"]["angle"], mp0, b0, fv0,
                                        kf1["desc"], kf1["keys"]["angle"], mp1, b1, fv1, ratio,
                                        ori)
        assert n == pn and n > 50
        assert np.array_equal(m, pm)


def test_triangulation_matches_restatement(oracle):
    k0, k1 = S.keyframe_pair(oracle, 3, rng_seed=1, baseline=(0.5, 0.0, 0.1))
    rng = np.random.default_rng(9)
    for d in (k0, k1):
        d["has_mp"] = (rng.random(len(d["keys"])) < 0.5).astype(np.uint8)
    F12 = S.fundamental(k0, k1)
    fv0 = oracle.feature_vector(S.vocab_nodes(k0["desc"]))
    fv1 = oracle.feature_vector(S.vocab_nodes(k1["desc"]))
    for stereo, ori in ((False, True), (True, False)):
        n, m = oracle.search_for_triangulation(k0, k1, k1["sigma2"], F12, S.camera(), k0["ow"],
                                               k1["Rw"], k1["tw"], fv0, fv1, stereo, ori)
        pn, pm = pyref.search_for_triangulation(k0, k1, k1["sigma2"], F12, S.camera(), k0["ow"],
                                                k1["Rw"], k1["tw"], fv0, fv1, stereo, ori)
        assert n == pn and n > 10
        assert np.array_equal(m, pm)
