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


def _rot(ax, ay, az):
    cx, sx, cy, sy, cz, sz = np.cos(ax), np.sin(ax), np.cos(ay), np.sin(ay), np.cos(az), np.sin(az)
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def pose(rng):
    """A camera pose Tcw with mOw computed as Frame::UpdatePoseMatrices does (float)."""
    R = _rot(*rng.uniform(-0.1, 0.1, 3)).astype(np.float32)
    t = rng.uniform(-2, 2, 3).astype(np.float32)
    ow = np.zeros(3, np.float32)
    for i in range(3):  # -Rcw^T * tcw, float dot left to right
        ow[i] = -((R[0, i] * t[0] + R[1, i] * t[1]) + R[2, i] * t[2])
    return R, t, ow


def local_map_3d(oracle, keys, desc, n_mp, width, height, rng_seed=0, scale_factor=1.2):
    """Local MapPoints in world coordinates for Frame::isInFrustum + SearchByProjection.
    70 % are back-projections of frame keypoints at random depth (descriptor = the
    keypoint's with ~8 % bit flips, distance range consistent with the keypoint's
    octave), 30 % random points (some behind the camera or out of the image).
    Normals are mostly towards the camera; ~10 % are tilted past the 0.5 cos limit.
    Returns (pose record, map points, map-point descriptors)."""
    rng = np.random.default_rng(rng_seed)
    R, t, ow = pose(rng)
    P = np.zeros(n_mp, oracle.MAP_POINT_DTYPE)
    mpd = rng.integers(0, 256, (n_mp, 32), dtype=np.uint8)
    n_kp = len(keys)
    from_kp = (rng.random(n_mp) < 0.7) & (n_kp > 0)
    kidx = rng.integers(0, max(n_kp, 1), n_mp)
    z = rng.uniform(2.0, 50.0, n_mp)
    u = np.where(from_kp, keys["x"][kidx % max(n_kp, 1)] + rng.uniform(-1, 1, n_mp),
                 rng.uniform(-100, width + 100, n_mp))
    v = np.where(from_kp, keys["y"][kidx % max(n_kp, 1)] + rng.uniform(-1, 1, n_mp),
                 rng.uniform(-100, height + 100, n_mp))
    z = np.where(~from_kp & (rng.random(n_mp) < 0.1), -z, z)
    pc = np.stack([(u - CX) / FX * z, (v - CY) / FY * z, z], 1)
    pw = (pc - t.astype(np.float64)) @ R.astype(np.float64)  # R^T (pc - t)
    P["pos"] = pw.astype(np.float32)
    d = pw - ow.astype(np.float64)
    dist = np.linalg.norm(d, axis=1)
    nrm = d / dist[:, None] + rng.normal(0, 0.15, (n_mp, 3))
    tilt = rng.random(n_mp) < 0.1
    nrm[tilt] = rng.normal(0, 1, (tilt.sum(), 3))
    P["normal"] = (nrm / np.linalg.norm(nrm, axis=1)[:, None]).astype(np.float32)
    octv = np.where(from_kp, keys["octave"][kidx % max(n_kp, 1)], rng.integers(0, 8, n_mp))
    maxd = dist * scale_factor ** octv * rng.uniform(0.9, 1.1, n_mp)
    maxd[rng.random(n_mp) < 0.05] *= 0.5  # out of the scale-invariance range
    P["max_distance"] = maxd.astype(np.float32)
    P["min_distance"] = (maxd / scale_factor ** 7).astype(np.float32)
    P["bad"] = rng.random(n_mp) < 0.03
    P["seen"] = rng.random(n_mp) < 0.05
    P["has_obs"] = rng.random(n_mp) < 0.9
    if n_kp:
        src = desc[kidx % n_kp]
        flips = rng.random((n_mp, 256)) < 0.08
        bits = np.unpackbits(src, axis=1, bitorder="little") ^ flips
        mpd = np.where(from_kp[:, None], np.packbits(bits.astype(np.uint8), axis=1,
                                                      bitorder="little"), mpd)
    rec = np.zeros(1, oracle.POSE_DTYPE)
    rec["rcw"] = R.reshape(1, 9)
    rec["tcw"] = t
    rec["ow"] = ow
    return rec, P, np.ascontiguousarray(mpd, np.uint8)


def init_pair(oracle, seed, frame2=1, w=640, h=480, nf=2000):
    """Tracking::MonocularInitialization's first SearchForInitialization call:
    the initial extractor runs with 2*nFeatures (src/Tracking.cc:126),
    vbPrevMatched starts as the initial frame's keypoint positions
    (src/Tracking.cc:661-664; call at :698-701), windowSize 100, ORBmatcher(0.9, true)."""
    a = oracle.synth_image(seed, 0, w, h)
    b = oracle.synth_image(seed, frame2, w, h)
    k1, d1, _ = oracle.extract(a, nf)
    k2, d2, _ = oracle.extract(b, nf)
    prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
    return dict(k1=k1, d1=d1, k2=k2, d2=d2, prev=prev, w=w, h=h)


def observation_sets(rng, n_mp, max_obs=40, flip=0.08):
    """CSR observation descriptors for MapPoints: noisy copies of one base
    descriptor per point (a point seen from several KeyFrames), a few empty
    lists, a few long ones; duplicated rows create median ties."""
    counts = rng.integers(1, max_obs + 1, n_mp)
    counts[rng.random(n_mp) < 0.05] = 0
    counts[rng.random(n_mp) < 0.02] = rng.integers(65, 300)
    offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    desc = np.zeros((int(offs[-1]), 32), np.uint8)
    for p in range(n_mp):
        base = rng.integers(0, 256, 32, dtype=np.uint8)
        bits = np.unpackbits(np.tile(base, (counts[p], 1)), axis=1)
        noise = rng.random(bits.shape) < rng.uniform(0.0, flip * 2)
        rows = np.packbits(bits ^ noise, axis=1)
        if counts[p] > 3 and rng.random() < 0.3:
            rows[1] = rows[0]
        desc[offs[p]:offs[p + 1]] = rows
    return offs, desc


# --------------------------------------------------------------- keyframes in 3D
def _ry(theta):
    c, s = np.cos(theta), np.sin(theta)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])


def _camera_center(R, t):
    ow = np.zeros(3, np.float32)
    for i in range(3):  # -R^T t, float dot left to right
        ow[i] = -((R[0, i] * t[0] + R[1, i] * t[1]) + R[2, i] * t[2])
    return ow


def keyframe(oracle, seed, frame, R, t, rng, w=1241, h=376, nf=1000, frac_mp=0.8,
             frac_stereo=0.5):
    """A KeyFrame of the synthetic sequence with a MapPoint behind most keypoints:
    back-projection at random depth (world frame through the pose R, t), normal
    towards the camera with noise, scale-invariance range from the keypoint
    octave, descriptor = keypoint descriptor with ~5 % bit flips; stereo
    keypoints get mvuRight = u - bf/z."""
    img = oracle.synth_image(seed, frame, w, h)
    keys, desc, _ = oracle.extract(img, nf)
    n = len(keys)
    p = oracle.params(nf)
    R = np.asarray(R, np.float32)
    t = np.asarray(t, np.float32)
    ow = _camera_center(R, t)
    z = rng.uniform(4.0, 40.0, n)
    pc = np.stack([(keys["x"] - CX) / FX * z, (keys["y"] - CY) / FY * z, z], 1)
    pw = (pc - t.astype(np.float64)) @ R.astype(np.float64)
    mps = np.zeros(n, oracle.MAP_POINT_DTYPE)
    mps["pos"] = pw.astype(np.float32)
    d = ow.astype(np.float64) - pw
    dist = np.linalg.norm(d, axis=1)
    nrm = -d / dist[:, None] + rng.normal(0, 0.2, (n, 3))
    mps["normal"] = (nrm / np.linalg.norm(nrm, axis=1)[:, None]).astype(np.float32)
    maxd = dist * 1.2 ** keys["octave"] * rng.uniform(0.9, 1.1, n)
    mps["max_distance"] = maxd.astype(np.float32)
    mps["min_distance"] = (maxd / 1.2 ** 7).astype(np.float32)
    mps["bad"] = rng.random(n) < 0.03
    valid = (rng.random(n) < frac_mp).astype(np.uint8)
    bits = np.unpackbits(desc, axis=1) ^ (rng.random((n, 256)) < 0.05)
    mp_desc = np.packbits(bits.astype(np.uint8), axis=1)
    ur = np.where(rng.random(n) < frac_stereo, keys["x"] - BF / z, -1.0).astype(np.float32)
    return dict(keys=keys, desc=desc, scale=p["scale"], inv_sigma2=p["inv_sigma2"],
                sigma2=p["sigma2"], width=w, height=h, Rw=R, tw=t, ow=ow, mps=mps, valid=valid,
                mp_desc=mp_desc, u_right=ur, already=np.zeros(n, np.uint8))


def keyframe_pair(oracle, seed, rng_seed=0, w=1241, h=376, nf=1000, baseline=None):
    """KeyFrames on frames 0 and 1 of a synthetic sequence.  Frame 1 is frame 0
    shifted by the sequence's ego shift; KF1's pose is KF0's rotated about y by
    atan(shift / fx), so KF0's points project near their KF1 keypoints.  With
    `baseline` (x, y, z) KF1's centre also moves (epipolar geometry)."""
    rng = np.random.default_rng(rng_seed)
    R0, t0, _ = pose(rng)
    th = np.arctan(_ego_shift(seed) / FX)
    Ry = _ry(th)
    R1 = (Ry @ R0.astype(np.float64)).astype(np.float32)
    t1 = (Ry @ t0.astype(np.float64))
    if baseline is not None:
        t1 = t1 - R1.astype(np.float64) @ np.asarray(baseline, np.float64)
    t1 = t1.astype(np.float32)
    kf0 = keyframe(oracle, seed, 0, R0, t0, rng, w, h, nf)
    kf1 = keyframe(oracle, seed, 1, R1, t1, rng, w, h, nf)
    return kf0, kf1


def pose_record(oracle, R, t):
    rec = np.zeros(1, oracle.POSE_DTYPE)
    rec["rcw"] = np.asarray(R, np.float32).reshape(1, 9)
    rec["tcw"] = np.asarray(t, np.float32)
    rec["ow"] = _camera_center(np.asarray(R, np.float32), np.asarray(t, np.float32))
    return rec


def scw(R, t, s):
    """Scw (3x4 row-major [sR | st]) of a similarity with rotation R, translation t."""
    S = np.zeros((3, 4), np.float32)
    S[:, :3] = (s * np.asarray(R, np.float64)).astype(np.float32)
    S[:, 3] = (s * np.asarray(t, np.float64)).astype(np.float32)
    return S


def fundamental(kf1, kf2):
    """LocalMapping::ComputeF12 in float64 (an input to SearchForTriangulation)."""
    R1, t1 = kf1["Rw"].astype(np.float64), kf1["tw"].astype(np.float64)
    R2, t2 = kf2["Rw"].astype(np.float64), kf2["tw"].astype(np.float64)
    R12 = R1 @ R2.T
    t12 = -R1 @ R2.T @ t2 + t1
    tx = np.array([[0, -t12[2], t12[1]], [t12[2], 0, -t12[0]], [-t12[1], t12[0], 0]])
    K = np.array([[FX, 0, CX], [0, FY, CY], [0, 0, 1]])
    Ki = np.linalg.inv(K)
    return (Ki.T @ tx @ R12 @ Ki).astype(np.float32)


def vocabulary(rng_seed=0, k=10, L=4, irregular=False, stop_frac=0.0, ties=False,
               order="hkmeans"):
    """Synthetic DBoW2 vocabulary tree as the node table loadFromTextFile builds
    (TemplatedVocabulary.h:1400-1444).  The ORB vocabulary (ORBvoc.txt) is not in
    the reference tree, so the tree is generated: each child descriptor is its
    parent's with bits flipped (fewer further down), leaves at depth L carry an
    idf-like weight > 0.  `order` "hkmeans" numbers nodes the way HKmeansStep
    creates them (a node's children consecutive, then each child's subtree in
    turn, :475-610) -- the order a saved vocabulary lists them in; "bfs" is
    level order.  `irregular`: nodes with fewer than k children and leaves
    above depth L (clusters with fewer than k descriptors stop early).
    `stop_frac`: words with weight 0 (stopWords, :1349-1360).  `ties`: sibling
    pairs with identical descriptors (first child must win, strict '<').
    Returns dict(k, L, parent, leaf, desc, weight) with entry 0 the root."""
    rng = np.random.default_rng(rng_seed)
    # level-order construction: per node its children's count
    levels = [np.zeros(1, np.int64)]  # node indices (bfs) per depth
    parent_bfs = [-1]
    depth = [0]
    nchild_bfs = []
    desc_bfs = [rng.integers(0, 256, 32, dtype=np.uint8)]
    n = 1
    for d in range(1, L + 1):
        prev = levels[-1]
        if irregular:
            nc = np.where(rng.random(len(prev)) < 0.15, rng.integers(2, k + 1, len(prev)), k)
            if d > 1:
                nc = np.where(rng.random(len(prev)) < 0.06, 0, nc)  # early leaf
        else:
            nc = np.full(len(prev), k)
        nchild_bfs.append(nc)
        tot = int(nc.sum())
        par = np.repeat(prev, nc)
        levels.append(np.arange(n, n + tot))
        parent_bfs.extend(par.tolist())
        depth.extend([d] * tot)
        n += tot
    parent_bfs = np.array(parent_bfs, np.int64)
    depth = np.array(depth, np.int64)
    # descriptors: flip probability per depth
    pflip = {1: 0.5, 2: 0.3, 3: 0.2, 4: 0.12, 5: 0.08, 6: 0.05}
    desc = np.zeros((n, 32), np.uint8)
    desc[0] = desc_bfs[0]
    for d in range(1, L + 1):
        idx = levels[d]
        if len(idx) == 0:
            continue
        bits = np.unpackbits(desc[parent_bfs[idx]], axis=1)
        flips = (rng.random(bits.shape) < pflip.get(d, 0.04)).astype(np.uint8)
        desc[idx] = np.packbits(bits ^ flips, axis=1)
    nchildren = np.bincount(parent_bfs[1:], minlength=n)
    leaf = (nchildren == 0).astype(np.uint8)
    leaf[0] = 0
    if ties:
        # copy the first child's descriptor onto a later sibling for ~10% of parents
        first = {}
        for i in range(1, n):
            first.setdefault(int(parent_bfs[i]), i)
        for p, c0 in first.items():
            if nchildren[p] >= 3 and rng.random() < 0.1:
                desc[c0 + 1 + rng.integers(0, nchildren[p] - 1)] = desc[c0]
    weight = np.where(leaf == 1, rng.uniform(0.5, 8.0, n), 0.0)
    if stop_frac > 0:
        weight[(leaf == 1) & (rng.random(n) < stop_frac)] = 0.0
    weight[0] = 0.0
    if order == "bfs":
        perm = np.arange(n)
    else:
        # HKmeansStep creation order: children consecutive, then recurse per child
        kids = [[] for _ in range(n)]
        for i in range(1, n):
            kids[int(parent_bfs[i])].append(i)
        perm = np.empty(n, np.int64)  # perm[new id] = bfs index
        perm[0] = 0
        nxt = 1
        stack = [0]
        while stack:
            p = stack.pop()
            ch = kids[p]
            perm[nxt:nxt + len(ch)] = ch
            nxt += len(ch)
            stack.extend(reversed(ch))  # first child's subtree first
    inv = np.empty(n, np.int64)
    inv[perm] = np.arange(n)
    parent = np.zeros(n, np.int32)
    parent[1:] = inv[parent_bfs[perm[1:]]]
    return dict(k=k, L=L, parent=parent, leaf=leaf[perm].copy(), desc=desc[perm].copy(),
                weight=weight[perm].copy())


def vocab_features(voc, n, rng_seed=0, flip=0.06, random_frac=0.1):
    """Features near vocabulary leaves: a random leaf's descriptor with bits
    flipped, plus a fraction of uniformly random descriptors."""
    rng = np.random.default_rng(rng_seed)
    leaves = np.flatnonzero(voc["leaf"])
    src = voc["desc"][rng.choice(leaves, n)]
    bits = np.unpackbits(src, axis=1)
    bits ^= (rng.random(bits.shape) < flip).astype(np.uint8)
    out = np.packbits(bits, axis=1)
    rnd = rng.random(n) < random_frac
    out[rnd] = rng.integers(0, 256, (int(rnd.sum()), 32), dtype=np.uint8)
    return out


def write_vocabulary_text(voc, path, scoring=0, weighting=0):
    """ORBvoc.txt layout read by loadFromTextFile (:1362-1448): header
    "k L scoring weighting", then per node "parent isLeaf d0 .. d31 weight"."""
    with open(path, "w") as f:
        f.write(f"{voc['k']} {voc['L']}  {scoring} {weighting}\n")
        for i in range(1, len(voc["parent"])):
            d = " ".join(str(int(x)) for x in voc["desc"][i])
            f.write(f"{int(voc['parent'][i])} {int(voc['leaf'][i])} {d} {float(voc['weight'][i])!r}\n")


# Camera models for Frame::UndistortKeyPoints / ComputeImageBounds: mK as 3x3
# float rows and mDistCoef as Tracking builds it (src/Tracking.cc:66-78: 4
# coefficients, a 5th only when k3 != 0).  TUM1/TUM2 from Examples/Monocular.
def cameras():
    def K(fx, fy, cx, cy):
        return np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]], np.float32)
    return {
        "tum1": (K(517.306408, 516.469215, 318.643040, 255.313989),
                 np.array([0.262383, -0.953104, -0.005358, 0.002628, 1.163314], np.float32)),
        "tum2": (K(520.908620, 521.007327, 325.141442, 249.701764),
                 np.array([0.231222, -0.784899, -0.003257, -0.000105, 0.917205], np.float32)),
        "kitti": (K(718.856, 718.856, 607.1928, 185.2157), np.zeros(4, np.float32)),
        "k4": (K(458.654, 457.296, 367.215, 248.375),
               np.array([-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05], np.float32)),
        "rational8": (K(500.0, 505.0, 320.5, 240.25),
                      np.array([0.1, -0.05, 0.001, -0.002, 0.01, 0.02, -0.01, 0.005], np.float32)),
        "prism12": (K(600.0, 600.0, 310.0, 250.0),
                    np.array([-0.2, 0.05, 0.0005, 0.0003, 0.0, 0.0, 0.0, 0.0, 0.001, -0.0005,
                              0.0008, 0.0002], np.float32)),
    }


def undistort_points_grid(w=640, h=480, rng_seed=0, n_random=500):
    """Image corners, a grid and random sub-pixel points (some outside)."""
    rng = np.random.default_rng(rng_seed)
    gx, gy = np.meshgrid(np.linspace(0, w, 17), np.linspace(0, h, 13))
    pts = [np.array([[0, 0], [w, 0], [0, h], [w, h]], np.float32),
           np.stack([gx.ravel(), gy.ravel()], 1).astype(np.float32),
           rng.uniform([-20, -20], [w + 20, h + 20], (n_random, 2)).astype(np.float32)]
    return np.concatenate(pts)
