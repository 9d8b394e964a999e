"""Synthetic matcher scenarios shared by the CPU and GPU tests (test infrastructure).

KITTI-like camera (KITTI00-02.yaml: fx 718.856, bf 386.1448), frames from the
deterministic generator, features from the CPU oracle extractor.
"""
import numpy as np

FX, FY, CX, CY = 718.856, 718.856, 607.1928, 185.2157
BF = 386.1448


def stereo_pair(oracle, seed, w=1241, h=376, nf=2000):
    left = oracle.synth_image(seed, 0, w, h, 0)
    right = oracle.synth_image(seed, 0, w, h, 1)
    kl, dl, _ = oracle.extract(left, nf)
    kr, dr, _ = oracle.extract(right, nf)
    p = oracle.params(nf)
    return dict(left=left, right=right, kl=kl, dl=dl, kr=kr, dr=dr,
                lpyr=oracle.pyramid(left), rpyr=oracle.pyramid(right),
                scale=p["scale"], inv=p["inv_scale"], w=w, h=h)


def frame_pair(oracle, seed, w=1241, h=376, nf=1000, rng_seed=0):
    """Last frame (frame 0) with map points on its keypoints, current frame 1.
    Map points are back-projected at random depth and carry the ego-motion
    shift of the synthetic sequence, so their projections land near the
    current frame's keypoints."""
    rng = np.random.default_rng(rng_seed)
    a = oracle.synth_image(seed, 0, w, h)
    b = oracle.synth_image(seed, 1, w, h)
    ka, da, _ = oracle.extract(a, nf)
    kb, db, _ = oracle.extract(b, nf)
    # ego-motion of frame 0 -> 1 in pixels (same rule as orb_synth.h ego_offset)
    shift = _ego_shift(seed)
    n = len(ka)
    z = rng.uniform(4.0, 60.0, n).astype(np.float32)
    last = np.zeros(n, oracle.LAST_MP_DTYPE)
    u = (ka["x"] + shift + rng.uniform(-1.5, 1.5, n)).astype(np.float32)
    v = (ka["y"] + rng.uniform(-1.5, 1.5, n)).astype(np.float32)
    last["xc"] = ((u - np.float32(CX)) / np.float32(FX) * z).astype(np.float32)
    last["yc"] = ((v - np.float32(CY)) / np.float32(FY) * z).astype(np.float32)
    last["invzc"] = (np.float32(1.0) / z).astype(np.float32)
    last["invzc"][rng.random(n) < 0.02] = np.float32(-0.1)  # behind the camera
    last["last_octave"] = ka["octave"]
    last["last_angle"] = ka["angle"]
    last["valid"] = rng.random(n) < 0.9
    last["has_obs"] = rng.random(n) < 0.85
    last["mp_id"] = np.arange(n, dtype=np.int32) + 1000
    p = oracle.params(nf)
    return dict(kb=kb, db=db, last=last, last_desc=da, scale=p["scale"], w=w, h=h)


def _ego_shift(seed):
    # mirror of orb_synth::ego_offset(seed, 1)
    z = (seed ^ 0xE6000000) & 0xFFFFFFFFFFFFFFFF
    z = (z + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    z ^= z >> 31
    return int(z % 7) - 3


def camera():
    return (FX, FY, CX, CY, BF, BF / FX)


def vocab_nodes(desc, bits=6):
    """Synthetic vocabulary: the node of a descriptor at the FeatureVector level
    is its first `bits` bits (stands in for DBoW2's tree descent, absent here)."""
    d = np.ascontiguousarray(desc, np.uint8)
    return (d[:, 0].astype(np.int64) & ((1 << bits) - 1)) | ((d[:, 1].astype(np.int64) & 1) << bits)


def bow_pair(oracle, seed, nf=1000, rng_seed=0):
    rng = np.random.default_rng(rng_seed)
    fp = frame_pair(oracle, seed, nf=nf, rng_seed=rng_seed)
    kf_desc = fp["last_desc"]
    n = len(kf_desc)
    kf_angle = fp["last"]["last_angle"]
    kf_mp = np.where(rng.random(n) < 0.85, np.arange(n) + 5000, -1).astype(np.int32)
    kf_bad = (rng.random(n) < 0.03).astype(np.uint8)
    kf_fv = oracle.feature_vector(vocab_nodes(kf_desc))
    f_fv = oracle.feature_vector(vocab_nodes(fp["db"]))
    return dict(kf_desc=kf_desc, kf_angle=kf_angle, kf_mp=kf_mp, kf_bad=kf_bad, kf_fv=kf_fv,
                f_desc=fp["db"], f_angle=fp["kb"]["angle"], f_fv=f_fv)
