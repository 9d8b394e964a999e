"""Oracle restatement of the DBoW2 vocabulary transform (Frame::ComputeBoW,
src/Frame.cc:439-449 -> TemplatedVocabulary::transform,
Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1128-1283) against the
independent pure-Python restatement in pyref.py, plus loadFromTextFile
(:1362-1448) on the text layout.  The reference ships no vocabulary file
(ORBvoc.txt is absent from the tree) and no fixtures for transform, so parity
is unpinned beyond this cross-check and the hand-made known-answer trees."""
import numpy as np
import pytest

import pyref
import scenarios


def _cmp(o, p):
    bw, bv, fvn, fvo, fvf, fw, fn = o
    pk, pv, pn, po, pf, pw, pnode = p
    assert bw.tolist() == pk
    assert bv.tolist() == pv  # exact doubles
    assert fvn.tolist() == pn and fvo.tolist() == po and fvf.tolist() == pf
    if pw:
        assert fw.tolist() == pw and fn.tolist() == pnode


@pytest.mark.parametrize("kw", [
    dict(rng_seed=0, k=10, L=3),
    dict(rng_seed=1, k=10, L=4, order="bfs"),
    dict(rng_seed=2, k=6, L=4, irregular=True, stop_frac=0.2),
    dict(rng_seed=3, k=10, L=3, ties=True),
    dict(rng_seed=4, k=3, L=5, irregular=True, ties=True),
])
def test_oracle_vocab_matches_restatement(oracle, kw):
    voc = scenarios.vocabulary(**kw)
    feats = scenarios.vocab_features(voc, 400, rng_seed=kw["rng_seed"])
    for levelsup in (4, 1, 0, kw["L"], kw["L"] + 2):
        o = oracle.vocab_transform(voc, feats, levelsup, 0, 0)
        p = pyref.vocab_transform(voc, feats, levelsup, 0, 0)
        _cmp(o, p)


@pytest.mark.parametrize("scoring", range(6))
@pytest.mark.parametrize("weighting", range(4))
def test_oracle_vocab_scoring_weighting(oracle, scoring, weighting):
    voc = scenarios.vocabulary(rng_seed=7, k=8, L=3, stop_frac=0.1)
    feats = scenarios.vocab_features(voc, 300, rng_seed=3, flip=0.1)
    _cmp(oracle.vocab_transform(voc, feats, 2, scoring, weighting),
         pyref.vocab_transform(voc, feats, 2, scoring, weighting))


def test_oracle_vocab_known_answers(oracle):
    # root -> {1, 2}; 1 -> {3, 4}; 2 leaf.  Node 4 equals node 3 (tie: 3 wins).
    d = np.zeros((5, 32), np.uint8)
    d[1] = 0x00; d[2] = 0xFF
    d[3, 0] = 0x0F; d[4, 0] = 0x0F
    voc = dict(k=2, L=2, parent=np.array([0, 0, 0, 1, 1], np.int32),
               leaf=np.array([0, 0, 1, 1, 1], np.uint8), desc=d,
               weight=np.array([0, 0, 2.0, 1.0, 3.0]))
    # words: node 2 -> 0, node 3 -> 1, node 4 -> 2
    f = np.zeros((4, 32), np.uint8)
    f[0] = 0xFF            # -> node 2, a leaf at depth 1 = nid_level
    f[1, 0] = 0x0F         # -> node 1 -> tie 3/4 -> node 3
    f[2, 0] = 0x01         # -> node 1 -> node 3 (d 3 vs 3: tie) -> node 3
    f[3] = 0xFF; f[3, 0] = 0x00  # distance 8 to node 2 vs 248 to node 1 -> node 2
    bw, bv, fvn, fvo, fvf, fw, fn = oracle.vocab_transform(voc, f, 1, 0, 0)
    assert fw.tolist() == [0, 1, 1, 0]
    assert fn.tolist() == [2, 1, 1, 2]  # nid_level = 1
    assert bw.tolist() == [0, 1]
    # TF_IDF, L1: word 0 weight 2+2=4, word 1 weight 1+1=2 -> 4/6, 2/6
    assert bv.tolist() == [4.0 / 6.0, 2.0 / 6.0]
    assert fvn.tolist() == [1, 2] and fvo.tolist() == [0, 2, 4] and fvf.tolist() == [1, 2, 0, 3]
    # stopped word: weight 0 on node 3 drops features 1, 2 from both vectors
    voc["weight"] = np.array([0, 0, 2.0, 0.0, 3.0])
    bw, bv, fvn, fvo, fvf, fw, fn = oracle.vocab_transform(voc, f, 1, 0, 0)
    assert fw.tolist() == [0, 0xFFFFFFFF, 0xFFFFFFFF, 0]
    assert bw.tolist() == [0] and bv.tolist() == [1.0]
    assert fvn.tolist() == [2] and fvf.tolist() == [0, 3]


def test_oracle_vocab_empty(oracle):
    voc = dict(k=10, L=6, parent=np.zeros(1, np.int32), leaf=np.zeros(1, np.uint8),
               desc=np.zeros((1, 32), np.uint8), weight=np.zeros(1))
    bw, bv, fvn, fvo, fvf, _, _ = oracle.vocab_transform(voc, np.zeros((5, 32), np.uint8), 4)
    assert len(bw) == 0 and len(fvn) == 0 and fvo.tolist() == [0]
    voc = scenarios.vocabulary(rng_seed=0, k=4, L=2)
    bw, bv, fvn, fvo, fvf, _, _ = oracle.vocab_transform(voc, np.zeros((0, 32), np.uint8), 4)
    assert len(bw) == 0 and fvo.tolist() == [0]


def test_oracle_vocab_text_roundtrip(oracle, tmp_path):
    voc = scenarios.vocabulary(rng_seed=5, k=5, L=3, irregular=True, stop_frac=0.1)
    path = tmp_path / "voc.txt"
    scenarios.write_vocabulary_text(voc, path, scoring=1, weighting=2)
    with open(path, "a") as f:
        f.write("\n")  # trailing empty line, as a saved file ends
    got = oracle.vocab_parse_text(path)
    assert (got["k"], got["L"], got["scoring"], got["weighting"]) == (5, 3, 1, 2)
    for key in ("parent", "leaf", "desc", "weight"):
        assert np.array_equal(got[key][1:], np.asarray(voc[key])[1:]), key
    bad = tmp_path / "bad.txt"
    bad.write_text("30 6 0 0\n")  # k > 20 rejected (:1383)
    with pytest.raises(ValueError):
        oracle.vocab_parse_text(bad)


def test_oracle_vocab_orb_slam_shape(oracle):
    # ORBvoc.txt shape: k 10, L 6, TF_IDF, L1_NORM, transform(..., 4) -> level-2 nodes
    voc = scenarios.vocabulary(rng_seed=11, k=10, L=6)
    assert len(voc["parent"]) == 1111111
    feats = scenarios.vocab_features(voc, 1000, rng_seed=1)
    bw, bv, fvn, fvo, fvf, fw, fn = oracle.vocab_transform(voc, feats, 4, 0, 0)
    assert abs(bv.sum() - 1.0) < 1e-12 and len(bw) > 800
    # FeatureVector nodes sit at depth 2: parent of parent is the root
    par = voc["parent"]
    assert (par[par[fvn]] == 0).all() and (par[fvn] != 0).all()
    assert fvo[-1] == 1000 and sorted(fvf.tolist()) == list(range(1000))
    p = pyref.vocab_transform(voc, feats[:50], 4, 0, 0)
    o = oracle.vocab_transform(voc, feats[:50], 4, 0, 0)
    _cmp(o, p)
