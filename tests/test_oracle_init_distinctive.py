"""Oracle restatements of the §8(f) rows (test infrastructure):
ORBmatcher::SearchForInitialization (src/ORBmatcher.cc:429-577) and
MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:250-326), C++ oracle
against the independent Python restatements in pyref.py.  The reference ships no
fixtures for either function, so beyond this cross-check parity is unpinned."""
import numpy as np
import pytest

import pyref
import scenarios


@pytest.mark.parametrize("seed,frame2", [(0, 1), (3, 2)])
def test_oracle_init_matches_restatement(oracle, seed, frame2):
    s = scenarios.init_pair(oracle, seed, frame2, w=640, h=480, nf=1000)
    n, m12, prev = oracle.search_for_initialization(s["k1"], s["d1"], s["k2"], s["d2"], s["w"],
                                                    s["h"], s["prev"], 100, 0.9, True)
    pn, pm, pp = pyref.search_for_initialization(s["k1"], s["d1"], s["k2"], s["d2"], s["w"],
                                                 s["h"], s["prev"], 100, 0.9, True)
    assert n == pn and n > 20
    assert np.array_equal(m12, pm)
    assert np.array_equal(prev, pp)
    assert n == int((m12 >= 0).sum())
    # only level-0 keypoints of both frames take part
    assert (s["k1"]["octave"][m12 >= 0] == 0).all()
    assert (s["k2"]["octave"][m12[m12 >= 0]] == 0).all()
    # one-to-one
    assert len(np.unique(m12[m12 >= 0])) == n


def test_oracle_init_no_orientation_and_small_window(oracle):
    s = scenarios.init_pair(oracle, 5, 1, w=640, h=480, nf=1000)
    for window, check in [(100, False), (15, True), (3, False)]:
        r = oracle.search_for_initialization(s["k1"], s["d1"], s["k2"], s["d2"], s["w"], s["h"],
                                             s["prev"], window, 0.9, check)
        p = pyref.search_for_initialization(s["k1"], s["d1"], s["k2"], s["d2"], s["w"], s["h"],
                                            s["prev"], window, 0.9, check)
        assert r[0] == p[0]
        assert np.array_equal(r[1], p[1]) and np.array_equal(r[2], p[2])


def test_oracle_init_steal_path(oracle):
    # duplicated frame-2 descriptors and several frame-1 copies of one point
    # exercise vMatchedDistance skipping and the steal branch (:494-499)
    rng = np.random.default_rng(1)
    n1, n2 = 40, 30
    k1 = np.zeros(n1, oracle.KEYPOINT_DTYPE)
    k2 = np.zeros(n2, oracle.KEYPOINT_DTYPE)
    k1["x"] = rng.uniform(100, 120, n1); k1["y"] = rng.uniform(100, 120, n1)
    k2["x"] = rng.uniform(100, 120, n2); k2["y"] = rng.uniform(100, 120, n2)
    k1["angle"] = rng.uniform(0, 360, n1); k2["angle"] = rng.uniform(0, 360, n2)
    base = rng.integers(0, 256, (5, 32), dtype=np.uint8)
    d2 = base[rng.integers(0, 5, n2)].copy()
    d1 = base[rng.integers(0, 5, n1)].copy()
    bits = np.unpackbits(d1, axis=1)
    bits ^= (rng.random(bits.shape) < np.linspace(0.2, 0.0, n1)[:, None]).astype(np.uint8)
    d1 = np.packbits(bits, axis=1)
    d2[::3, 0] ^= 1
    prev = np.stack([k1["x"], k1["y"]], 1)
    for check in (False, True):
        r = oracle.search_for_initialization(k1, d1, k2, d2, 640, 480, prev, 50, 0.9, check)
        p = pyref.search_for_initialization(k1, d1, k2, d2, 640, 480, prev, 50, 0.9, check)
        assert r[0] == p[0]
        assert np.array_equal(r[1], p[1]) and np.array_equal(r[2], p[2])


def test_oracle_distinctive_matches_restatement(oracle):
    rng = np.random.default_rng(7)
    offs, desc = scenarios.observation_sets(rng, 300)
    best = oracle.distinctive_descriptors(offs, desc)
    for p in range(len(offs) - 1):
        assert best[p] == pyref.distinctive_descriptor(desc[offs[p]:offs[p + 1]])
    assert (best[np.diff(offs) == 0] == -1).all()


def test_oracle_distinctive_small_cases(oracle):
    a = np.zeros((1, 32), np.uint8)
    # N = 1: BestIdx 0; N = 2: median index 0 -> both rows have median 0 -> first
    assert list(oracle.distinctive_descriptors([0, 1], a)) == [0]
    two = np.stack([np.zeros(32, np.uint8), np.full(32, 255, np.uint8)])
    assert list(oracle.distinctive_descriptors([0, 2], two)) == [0]
    # N = 3 with one outlier: the two close rows win, first of them
    three = np.stack([np.full(32, 255, np.uint8), np.zeros(32, np.uint8),
                      np.array([1] + [0] * 31, np.uint8)])
    assert list(oracle.distinctive_descriptors([0, 3], three)) == [1]
    assert list(oracle.distinctive_descriptors([0, 0, 3], three)) == [-1, 1]
