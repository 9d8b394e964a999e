"""The reference-typed drop-ins, executed.

integration/ORBextractor.cc, ORBmatcher.cc and FrameStereo.cc are linked to
lib/liborb_amd.so with the test harness's own minimal cv::Mat / Frame /
KeyFrame / MapPoint (tests/integration_run/harness.cc, built by
tests/integration_run/Makefile) and run as ORB-SLAM2 calls them.  Each
scenario checks what the drop-in leaves in the caller's objects against the
CPU oracle:
  - ORBextractor::operator() (src/ORBextractor.cc:1091-1169): keypoints,
    descriptors, every mvImagePyramid level (read by src/Frame.cc:524,619,
    633,639), and an empty image leaving the outputs untouched (:1095-1096);
  - Frame::ComputeStereoMatches (src/Frame.cc:516-704) on the two extractors:
    mvuRight / mvDepth;
  - SearchByProjection(F, vpMapPoints, th): F.mvpMapPoints after the call
    (src/ORBmatcher.cc:127), including keypoints whose earlier point has no
    observations (overwritten) or has some (locked, :90-93);
  - Fuse(pKF, vpMapPoints, th): the keyframe's slots, every point's bad flag,
    observation count and slot after the call, against the reference's loop
    (src/ORBmatcher.cc:903-1077) applied in point order to a second copy of the
    same objects with the oracle's targets (Replace in both directions,
    AddObservation, points already in the keyframe, NULL and bad points,
    several points onto one keypoint);
  - SearchBySim3 (src/ORBmatcher.cc:1212-1458): vpMatches12, entries matched
    on entry kept."""
import math
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

import scenarios as S

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
HARNESS = ROOT / "tests" / "integration_run" / "dropin_harness"
LS = np.float32(math.log(np.float32(1.2)))


def _f(x):
    return repr(float(np.float32(x)))


def _run(tmp_path, scenario, files, meta):
    if not HARNESS.exists():
        pytest.fail(f"{HARNESS} not built (make -C tests/integration_run)")
    for name, arr in files.items():
        np.ascontiguousarray(arr).tofile(tmp_path / name)
    (tmp_path / "meta.txt").write_text(" ".join(_f(m) if isinstance(m, float) else str(m)
                                                for m in meta))
    r = subprocess.run([str(HARNESS), scenario, str(tmp_path)], capture_output=True, text=True,
                       timeout=100, env=dict(os.environ))
    assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.parametrize("w,h,nf,seed", [(640, 480, 1000, 1), (1241, 376, 2000, 7)])
def test_extractor_dropin(gpu, oracle, tmp_path, w, h, nf, seed):
    img = oracle.synth_image(seed, 0, w, h)
    _run(tmp_path, "extract", {"img.bin": img}, [w, h, nf])
    kr, dr, _ = oracle.extract(img, nf)
    assert (tmp_path / "kps.bin").read_bytes() == kr.tobytes()
    assert (tmp_path / "desc.bin").read_bytes() == dr.tobytes()
    ref = oracle.pyramid(img)
    sizes = [tuple(map(int, l.split())) for l in (tmp_path / "pyr_sizes.txt").read_text().split("\n") if l]
    assert len(sizes) == 8
    for l, (lw, lh) in enumerate(sizes):
        lvl = np.fromfile(tmp_path / f"pyr_{l}.bin", np.uint8).reshape(lh, lw)
        assert np.array_equal(lvl, ref[l]), f"mvImagePyramid[{l}]"
    assert (tmp_path / "empty_ok.txt").read_text() == "1"


@pytest.mark.parametrize("seed", [1, 3])
def test_stereo_dropin(gpu, oracle, tmp_path, seed):
    sp = S.stereo_pair(oracle, seed)
    _run(tmp_path, "stereo", {"imgL.bin": sp["left"], "imgR.bin": sp["right"]},
         [sp["w"], sp["h"], 2000, S.BF, S.FX])
    ur_ref, dp_ref = oracle.stereo_match(sp["kl"], sp["dl"], sp["scale"], sp["kr"], sp["dr"],
                                         sp["lpyr"], sp["rpyr"], sp["inv"], S.BF, S.FX,
                                         sp["w"], sp["h"])
    assert (ur_ref > 0).sum() > 50
    assert (tmp_path / "ur.bin").read_bytes() == ur_ref.tobytes()
    assert (tmp_path / "depth.bin").read_bytes() == dp_ref.tobytes()


@pytest.mark.parametrize("seed,n_mp,th", [(1, 2000, 1.0), (4, 5000, 3.0)])
def test_search_by_projection_dropin(gpu, oracle, tmp_path, seed, n_mp, th):
    w, h = 1241, 376
    img = oracle.synth_image(seed, 0, w, h)
    k, d, _ = oracle.extract(img, 1000)
    scale = oracle.params(1000)["scale"]
    mps, mpd, locked = oracle.synth_local_map(seed, k, d, n_mp, w, h)
    rng = np.random.default_rng(seed)
    # keypoints already holding a point: with observations (locked) or without
    pre = np.where(locked > 0, 1, np.where(rng.random(len(k)) < 0.1, 2, 0)).astype(np.uint8)
    _run(tmp_path, "local", {"keys.bin": k, "desc.bin": d, "scale.bin": scale, "tracks.bin": mps,
                             "mpdesc.bin": mpd, "pre.bin": pre}, [w, h, float(th), 0.8])
    n_ref, km = oracle.match_projection_local(k, d, scale, w, h, mps, mpd, th, 0.8,
                                              (pre == 1).astype(np.uint8))
    res = np.fromfile(tmp_path / "res.bin", np.int32)
    expect = np.where(km >= 0, km, np.where(pre > 0, -2, -1))
    assert n_ref > 100
    assert int((tmp_path / "count.txt").read_text()) == n_ref
    assert np.array_equal(res, expect), np.nonzero(res != expect)[0][:10]
    assert ((pre == 2) & (km >= 0)).any()  # a point without observations was overwritten


def _kf_files(prefix, kf):
    return {f"{prefix}keys.bin": kf["keys"], f"{prefix}desc.bin": kf["desc"],
            f"{prefix}scale.bin": kf["scale"], f"{prefix}sigma2.bin": kf["sigma2"],
            f"{prefix}invsigma2.bin": kf["inv_sigma2"], f"{prefix}uright.bin": kf["u_right"],
            f"{prefix}R.bin": np.asarray(kf["Rw"], np.float32),
            f"{prefix}t.bin": np.asarray(kf["tw"], np.float32),
            f"{prefix}ow.bin": np.asarray(kf["ow"], np.float32)}


def _kf_meta(th_or_s, th2=0.0):
    cam = S.camera()
    return [1241, 376, float(th_or_s), float(LS), float(cam[0]), float(cam[1]), float(cam[2]),
            float(cam[3]), float(cam[4]), float(cam[5]), float(th2)]


@pytest.mark.parametrize("th,rng_seed", [(3.0, 21), (1.0, 22)])
def test_fuse_dropin(gpu, oracle, tmp_path, th, rng_seed):
    kf0, kf1 = S.keyframe_pair(oracle, 3, rng_seed=1)
    rng = np.random.default_rng(rng_seed)
    n1, n0 = len(kf1["keys"]), len(kf0["keys"])
    # points already in pKF (kf1): on 40 % of its keypoints, some bad
    slots = np.nonzero(rng.random(n1) < 0.4)[0].astype(np.int32)
    ex = kf1["mps"][slots].copy()
    ex["bad"] = rng.random(len(slots)) < 0.05
    ex_obs = rng.integers(0, 6, len(slots)).astype(np.int32)
    # the points to fuse: kf0's map points (their projections land near kf1's
    # keypoints), a few entries of pKF's own points (skipped) and NULLs
    mps = kf0["mps"].copy()
    mp_obs = rng.integers(0, 6, n0).astype(np.int32)
    ref = np.full(n0, -1, np.int32)
    ref[kf0["valid"] == 0] = -2
    own_pts = np.nonzero(rng.random(n0) < 0.05)[0]
    ref[own_pts] = rng.integers(0, len(slots), len(own_pts))
    mpd = kf0["mp_desc"].copy()
    # the records the drop-in flattens (map_point_record): NULL -> bad, an
    # existing point -> its own record, seen (in pKF), observed
    rec = mps.copy()
    rec["seen"] = 0
    rec["has_obs"] = mp_obs > 0
    rec["bad"] = np.where(ref == -2, 1, rec["bad"])
    for i in np.nonzero(ref >= 0)[0]:
        e = ref[i]
        rec[i] = ex[e]
        rec[i]["seen"] = 1
        rec[i]["has_obs"] = 1
        mpd[i] = kf1["mp_desc"][slots[e]]
    pose = S.pose_record(oracle, kf1["Rw"], kf1["tw"])
    n_t, best = oracle.fuse(kf1["keys"], kf1["desc"], kf1["scale"], kf1["inv_sigma2"], 1241, 376,
                            kf1["u_right"], pose, S.camera(), rec, mpd, th, LS)
    files = _kf_files("kf_", kf1)
    files.update({"ex_mps.bin": ex, "ex_desc.bin": kf1["mp_desc"][slots], "ex_obs.bin": ex_obs,
                  "ex_slot.bin": slots, "mps.bin": mps, "mpdesc.bin": kf0["mp_desc"],
                  "mp_obs.bin": mp_obs, "mp_ref.bin": ref, "oracle_best.bin": best})
    _run(tmp_path, "fuse", files, _kf_meta(th))
    a = np.fromfile(tmp_path / "state_dropin.bin", np.int32)
    b = np.fromfile(tmp_path / "state_ref.bin", np.int32)
    n, nref = map(int, (tmp_path / "count.txt").read_text().split())
    assert n_t > 50 and n == nref
    assert np.array_equal(a, b), np.nonzero(a != b)[0][:10]
    # the scenario exercised both Replace directions and fresh slots
    tb = best[best >= 0]
    assert len(np.unique(tb)) < len(tb)          # several points onto one keypoint
    occupied = np.isin(tb, slots)
    assert occupied.any() and (~occupied).any()  # Replace and AddObservation


@pytest.mark.parametrize("s12", [1.0, 1.05])
def test_search_by_sim3_dropin(gpu, oracle, tmp_path, s12):
    kf0, kf1 = S.keyframe_pair(oracle, 3, rng_seed=1)
    rng = np.random.default_rng(31)
    k0, k1 = dict(kf0), dict(kf1)
    n0, n1 = len(k0["keys"]), len(k1["keys"])
    valid1 = np.nonzero(k1["valid"] > 0)[0]
    init = np.full(n0, -1, np.int32)
    pick = np.nonzero(rng.random(n0) < 0.06)[0]
    init[pick] = np.where(rng.random(len(pick)) < 0.7, rng.choice(valid1, len(pick)), -2)
    k0["already"] = (init != -1).astype(np.uint8)
    k1["already"] = np.zeros(n1, np.uint8)
    k1["already"][init[init >= 0]] = 1
    for k in (k0, k1):  # map_point_record: a keyframe's own points are observed
        k["mps"] = k["mps"].copy()
        k["mps"]["has_obs"] = k["valid"]
        k["mps"]["seen"] = 0
    R12 = (kf0["Rw"].astype(np.float64) @ kf1["Rw"].astype(np.float64).T).astype(np.float32)
    t12 = (kf0["tw"] - R12.astype(np.float64) @ kf1["tw"]).astype(np.float32)
    rn, rm = oracle.search_by_sim3(k0, k1, S.camera(), s12, R12, t12, 7.5, LS)
    files = _kf_files("k1_", k0)
    files.update(_kf_files("k2_", k1))
    for p, k in (("k1_", k0), ("k2_", k1)):
        files.update({f"{p}mps.bin": k["mps"], f"{p}mpdesc.bin": k["mp_desc"],
                      f"{p}valid.bin": k["valid"]})
    files.update({"init12.bin": init, "R12.bin": R12, "t12.bin": t12})
    _run(tmp_path, "sim3", files, _kf_meta(s12, 7.5))
    res = np.fromfile(tmp_path / "res.bin", np.int32)
    expect = np.where(rm >= 0, rm, np.where(init != -1, -3, -1))
    assert rn > 20
    assert int((tmp_path / "count.txt").read_text()) == rn
    assert np.array_equal(res, expect), np.nonzero(res != expect)[0][:10]
