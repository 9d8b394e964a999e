"""ctypes wrapper of the CPU oracle (oracle/liborb_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker / CPU baseline -- never by the
product package.  Parity status: unpinned against a reference binary (see the
header of orb_oracle.cpp and DESIGN.md §2).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
# ORB_ORACLE_VARIANT=glibc (read at import) selects the build with the
# reference's own glibc cosf/sinf/logf calls instead of the pins (tools/parity_libm.py)
LIB_PATH = HERE / ("liborb_oracle_glibc.so" if os.environ.get("ORB_ORACLE_VARIANT") == "glibc"
                   else "liborb_oracle.so")

KEYPOINT_DTYPE = np.dtype(
    [("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
     ("octave", "<i4"), ("class_id", "<i4")]
)
MP_TRACK_DTYPE = np.dtype(
    [("proj_x", "<f4"), ("proj_y", "<f4"), ("proj_xr", "<f4"), ("view_cos", "<f4"),
     ("level", "<i4"), ("in_view", "u1"), ("bad", "u1"), ("has_obs", "u1"), ("_pad", "u1")]
)

_lib = None


class _Frame(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int32), ("keys", ctypes.c_void_p), ("descriptors", ctypes.c_void_p),
        ("u_right", ctypes.c_void_p), ("min_x", ctypes.c_float), ("max_x", ctypes.c_float),
        ("min_y", ctypes.c_float), ("max_y", ctypes.c_float), ("n_levels", ctypes.c_int32),
        ("scale_factors", ctypes.c_void_p),
    ]


def build():
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        build()
    L = ctypes.CDLL(str(LIB_PATH))
    vp, i32, f32, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
    sig = {
        "oracle_params": (i32, [i32, f32, i32, vp, vp, vp, vp, vp, vp]),
        "oracle_level_sizes": (i32, [i32, i32, f32, i32, vp]),
        "oracle_pyramid": (i32, [vp, i32, i32, sz, f32, i32, vp]),
        "oracle_resize": (i32, [vp, i32, i32, vp, i32, i32]),
        "oracle_blur7": (i32, [vp, i32, i32, vp]),
        "oracle_fast": (i32, [vp, i32, i32, i32, vp, i32]),
        "oracle_fast_atan2": (f32, [f32, f32]),
        "oracle_sincos": (None, [f32, vp, vp]),
        "oracle_descriptor_distance": (i32, [vp, vp]),
        "oracle_candidates": (i32, [vp, i32, i32, sz, i32, f32, i32, i32, i32, vp, i32, vp]),
        "oracle_distribute": (i32, [vp, i32, i32, i32, i32, i32, i32, vp, i32]),
        "oracle_extract": (i32, [vp, i32, i32, sz, i32, f32, i32, i32, i32, vp, vp, i32, vp]),
        "oracle_match_projection_local": (i32, [vp, vp, i32, vp, vp, f32, f32, vp]),
        "oracle_grid": (i32, [vp, i32, f32, f32, f32, f32, vp, vp]),
        "oracle_synth_image": (None, [ctypes.c_uint64, i32, i32, i32, i32, vp, sz]),
        "oracle_synth_local_map": (None, [ctypes.c_uint64, vp, vp, i32, i32, i32, i32, vp, vp, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def _p(a):
    return a.ctypes.data


def params(nfeatures=1000, scale_factor=1.2, nlevels=8):
    sc, isc, s2, is2 = (np.zeros(nlevels, np.float32) for _ in range(4))
    q = np.zeros(nlevels, np.int32)
    um = np.zeros(16, np.int32)
    lib().oracle_params(nfeatures, scale_factor, nlevels, _p(sc), _p(isc), _p(s2), _p(is2), _p(q), _p(um))
    return dict(scale=sc, inv_scale=isc, sigma2=s2, inv_sigma2=is2, quota=q, umax=um)


def level_sizes(w, h, scale_factor=1.2, nlevels=8):
    wh = np.zeros(2 * nlevels, np.int32)
    lib().oracle_level_sizes(w, h, scale_factor, nlevels, _p(wh))
    return [(int(wh[2 * l]), int(wh[2 * l + 1])) for l in range(nlevels)]


def pyramid(img, scale_factor=1.2, nlevels=8):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    sizes = level_sizes(w, h, scale_factor, nlevels)
    out = np.zeros(sum(a * b for a, b in sizes), np.uint8)
    lib().oracle_pyramid(_p(img), w, h, w, scale_factor, nlevels, _p(out))
    levels, off = [], 0
    for (lw, lh) in sizes:
        levels.append(out[off: off + lw * lh].reshape(lh, lw))
        off += lw * lh
    return levels


def resize(src, dw, dh):
    src = np.ascontiguousarray(src, np.uint8)
    dst = np.zeros((dh, dw), np.uint8)
    lib().oracle_resize(_p(src), src.shape[1], src.shape[0], _p(dst), dw, dh)
    return dst


def blur7(src):
    src = np.ascontiguousarray(src, np.uint8)
    dst = np.zeros_like(src)
    lib().oracle_blur7(_p(src), src.shape[1], src.shape[0], _p(dst))
    return dst


def fast(img, threshold):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    cap = w * h
    out = np.zeros(cap, KEYPOINT_DTYPE)
    n = lib().oracle_fast(_p(img), w, h, threshold, _p(out), cap)
    return out[:n].copy()


def fast_atan2(y, x):
    return lib().oracle_fast_atan2(y, x)


def sincos(angle):
    s, c = ctypes.c_float(), ctypes.c_float()
    lib().oracle_sincos(angle, ctypes.byref(s), ctypes.byref(c))
    return s.value, c.value


def descriptor_distance(a, b):
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    return lib().oracle_descriptor_distance(_p(a), _p(b))


def candidates(img, nfeatures=1000, scale_factor=1.2, nlevels=8, ini=20, mn=7):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    per = np.zeros(nlevels, np.int32)
    n = lib().oracle_candidates(_p(img), w, h, w, nfeatures, scale_factor, nlevels, ini, mn, None, 0, _p(per))
    out = np.zeros(max(n, 1), KEYPOINT_DTYPE)
    lib().oracle_candidates(_p(img), w, h, w, nfeatures, scale_factor, nlevels, ini, mn, _p(out), n, _p(per))
    return out[:n], per


def distribute(keys, min_x, max_x, min_y, max_y, n):
    keys = np.ascontiguousarray(keys, KEYPOINT_DTYPE)
    cap = max(len(keys), 1)
    out = np.zeros(cap, KEYPOINT_DTYPE)
    k = lib().oracle_distribute(_p(keys), len(keys), min_x, max_x, min_y, max_y, n, _p(out), cap)
    return out[:k].copy()


def extract(img, nfeatures=1000, scale_factor=1.2, nlevels=8, ini=20, mn=7):
    """ORBextractor::operator() on the CPU: (keypoints, descriptors, per_level)."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    cap = nfeatures + 64 * nlevels
    while True:
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        per = np.zeros(nlevels, np.int32)
        n = lib().oracle_extract(_p(img), w, h, w, nfeatures, scale_factor, nlevels, ini, mn,
                                 _p(kps), _p(desc), cap, _p(per))
        if n >= 0:
            return kps[:n].copy(), desc[:n].copy(), per
        cap = -n - 1


def frame_struct(keys, desc, scale, width, height, u_right=None):
    keys = np.ascontiguousarray(keys, KEYPOINT_DTYPE)
    desc = np.ascontiguousarray(desc, np.uint8)
    scale = np.ascontiguousarray(scale, np.float32)
    f = _Frame()
    f.n = len(keys)
    f.keys = _p(keys)
    f.descriptors = _p(desc)
    f.u_right = _p(u_right) if u_right is not None else None
    f.min_x, f.max_x, f.min_y, f.max_y = 0.0, float(width), 0.0, float(height)
    f.n_levels = len(scale)
    f.scale_factors = _p(scale)
    return f, (keys, desc, scale, u_right)


def match_projection_local(keys, desc, scale, width, height, mps, mp_desc, th, nnratio,
                           kp_locked=None, u_right=None):
    f, keep = frame_struct(keys, desc, scale, width, height, u_right)
    mps = np.ascontiguousarray(mps, MP_TRACK_DTYPE)
    mp_desc = np.ascontiguousarray(mp_desc, np.uint8)
    km = np.full(len(keys), -1, np.int32)
    lk = None if kp_locked is None else np.ascontiguousarray(kp_locked, np.uint8)
    n = lib().oracle_match_projection_local(ctypes.byref(f), _p(lk) if lk is not None else None,
                                            len(mps), _p(mps), _p(mp_desc), th, nnratio, _p(km))
    return n, km


def grid(keys, width, height):
    keys = np.ascontiguousarray(keys, KEYPOINT_DTYPE)
    cs = np.zeros(64 * 48 + 1, np.int32)
    idx = np.zeros(max(len(keys), 1), np.int32)
    n = lib().oracle_grid(_p(keys), len(keys), 0.0, float(width), 0.0, float(height), _p(cs), _p(idx))
    return cs, idx[:n]


def synth_image(seed, frame, width, height, view=0):
    img = np.empty((height, width), np.uint8)
    lib().oracle_synth_image(seed, frame, view, width, height, _p(img), width)
    return img


def synth_local_map(seed, keys, desc, n_mp, width, height):
    keys = np.ascontiguousarray(keys, KEYPOINT_DTYPE)
    desc = np.ascontiguousarray(desc, np.uint8)
    mps = np.zeros(n_mp, MP_TRACK_DTYPE)
    mpd = np.zeros((n_mp, 32), np.uint8)
    lk = np.zeros(len(keys), np.uint8)
    lib().oracle_synth_local_map(seed, _p(keys), _p(desc), len(keys), n_mp, width, height,
                                 _p(mps), _p(mpd), _p(lk))
    return mps, mpd, lk


# ------------------------------------------------------------ stereo / frame / BoW
class _StereoInput(ctypes.Structure):
    _fields_ = [
        ("left", ctypes.c_void_p), ("n_right", ctypes.c_int32), ("right_keys", ctypes.c_void_p),
        ("right_desc", ctypes.c_void_p), ("n_levels", ctypes.c_int32),
        ("left_levels", ctypes.c_void_p), ("right_levels", ctypes.c_void_p),
        ("level_width", ctypes.c_void_p), ("level_height", ctypes.c_void_p),
        ("level_stride", ctypes.c_void_p), ("inv_scale_factors", ctypes.c_void_p),
        ("bf", ctypes.c_float), ("fx", ctypes.c_float),
    ]


class _Camera(ctypes.Structure):
    _fields_ = [("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float),
                ("cy", ctypes.c_float), ("bf", ctypes.c_float), ("mb", ctypes.c_float)]


LAST_MP_DTYPE = np.dtype([("xc", "<f4"), ("yc", "<f4"), ("invzc", "<f4"), ("last_octave", "<i4"),
                          ("last_angle", "<f4"), ("valid", "u1"), ("has_obs", "u1"),
                          ("_pad", "u1", 2), ("mp_id", "<i4")])
assert LAST_MP_DTYPE.itemsize == 28


def stereo_struct(lkeys, ldesc, scale, rkeys, rdesc, lpyr, rpyr, inv_scale, bf, fx, width, height):
    """Build an orb_stereo_input_t (shared by the oracle and the product wrappers)."""
    f, keep = frame_struct(lkeys, ldesc, scale, width, height)
    rkeys = np.ascontiguousarray(rkeys, KEYPOINT_DTYPE)
    rdesc = np.ascontiguousarray(rdesc, np.uint8)
    L = len(lpyr)
    lp = [np.ascontiguousarray(a) for a in lpyr]
    rp = [np.ascontiguousarray(a) for a in rpyr]
    lptr = (ctypes.c_void_p * L)(*[a.ctypes.data for a in lp])
    rptr = (ctypes.c_void_p * L)(*[a.ctypes.data for a in rp])
    w = np.array([a.shape[1] for a in lp], np.int32)
    h = np.array([a.shape[0] for a in lp], np.int32)
    st = np.array([a.strides[0] for a in lp], np.int64)
    inv = np.ascontiguousarray(inv_scale, np.float32)
    s = _StereoInput()
    s.left = ctypes.addressof(f)
    s.n_right = len(rkeys)
    s.right_keys, s.right_desc = _p(rkeys), _p(rdesc)
    s.n_levels = L
    s.left_levels = ctypes.addressof(lptr)
    s.right_levels = ctypes.addressof(rptr)
    s.level_width, s.level_height, s.level_stride = _p(w), _p(h), _p(st)
    s.inv_scale_factors = _p(inv)
    s.bf, s.fx = bf, fx
    return s, (f, keep, rkeys, rdesc, lp, rp, lptr, rptr, w, h, st, inv)


def stereo_match(*args):
    s, keep = stereo_struct(*args)
    n = keep[0].n
    ur = np.full(n, -1, np.float32)
    dp = np.full(n, -1, np.float32)
    lib().oracle_stereo_match.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib().oracle_stereo_match(ctypes.byref(s), _p(ur), _p(dp))
    return ur, dp


def match_projection_frame(keys, desc, scale, width, height, last, last_desc, cam, tlc_z, th,
                           mono, check_ori, kp_locked=None, u_right=None):
    f, keep = frame_struct(keys, desc, scale, width, height, u_right)
    last = np.ascontiguousarray(last, LAST_MP_DTYPE)
    last_desc = np.ascontiguousarray(last_desc, np.uint8)
    c = _Camera(*cam)
    km = np.full(len(keys), -1, np.int32)
    lk = None if kp_locked is None else np.ascontiguousarray(kp_locked, np.uint8)
    fn = lib().oracle_match_projection_frame
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float, ctypes.c_float, ctypes.c_int,
                   ctypes.c_int, ctypes.c_void_p]
    fn.restype = ctypes.c_int
    n = fn(ctypes.byref(f), _p(lk) if lk is not None else None, len(last), _p(last),
           _p(last_desc), ctypes.byref(c), tlc_z, th, int(mono), int(check_ori), _p(km))
    return n, km


def feature_vector(node_of):
    """DBoW2 FeatureVector as CSR: (sorted node ids, offsets, feature indices ascending)."""
    node_of = np.asarray(node_of, np.int64)
    order = np.argsort(node_of, kind="stable")
    ids, counts = np.unique(node_of, return_counts=True)
    offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    return ids.astype(np.uint32), offs, order.astype(np.uint32)


def match_bow(kf_desc, kf_angle, kf_mp, kf_bad, kf_fv, f_desc, f_angle, f_fv, nnratio, check_ori):
    kf_desc = np.ascontiguousarray(kf_desc, np.uint8)
    f_desc = np.ascontiguousarray(f_desc, np.uint8)
    kf_angle = np.ascontiguousarray(kf_angle, np.float32)
    f_angle = np.ascontiguousarray(f_angle, np.float32)
    kf_mp = np.ascontiguousarray(kf_mp, np.int32)
    kf_bad = None if kf_bad is None else np.ascontiguousarray(kf_bad, np.uint8)
    fm = np.full(len(f_desc), -1, np.int32)
    vp, i32, f32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    fn = lib().oracle_match_bow
    fn.argtypes = [i32, vp, vp, vp, vp, i32, vp, vp, vp, i32, vp, vp, i32, vp, vp, vp, f32, i32, vp]
    fn.restype = i32
    n = fn(len(kf_desc), _p(kf_desc), _p(kf_angle), _p(kf_mp),
           _p(kf_bad) if kf_bad is not None else None, len(kf_fv[0]), _p(kf_fv[0]), _p(kf_fv[1]),
           _p(kf_fv[2]), len(f_desc), _p(f_desc), _p(f_angle), len(f_fv[0]), _p(f_fv[0]),
           _p(f_fv[1]), _p(f_fv[2]), nnratio, int(check_ori), _p(fm))
    return n, fm


MAP_POINT_DTYPE = np.dtype([("pos", "<f4", (3,)), ("normal", "<f4", (3,)), ("min_distance", "<f4"),
                            ("max_distance", "<f4"), ("bad", "u1"), ("seen", "u1"),
                            ("has_obs", "u1"), ("_pad", "u1")])
POSE_DTYPE = np.dtype([("rcw", "<f4", (9,)), ("tcw", "<f4", (3,)), ("ow", "<f4", (3,))])


def pinned_log(x):
    fn = lib().oracle_log
    fn.restype, fn.argtypes = ctypes.c_double, [ctypes.c_double]
    return fn(float(x))


def frustum(mps, pose, cam, width, height, cos_limit=0.5, log_scale=None, n_levels=8,
            min_x=0.0, min_y=0.0):
    """Tracking::SearchLocalPoints' isInFrustum loop on the CPU: (n_in_view, tracks)."""
    mps = np.ascontiguousarray(mps, MAP_POINT_DTYPE)
    pose = np.ascontiguousarray(pose, POSE_DTYPE).reshape(1)
    if log_scale is None:
        log_scale = np.float32(pinned_log(np.float32(1.2)))
    tracks = np.zeros(len(mps), MP_TRACK_DTYPE)
    c = _Camera(*cam)
    fn = lib().oracle_frustum
    vp, f32 = ctypes.c_void_p, ctypes.c_float
    fn.argtypes = [ctypes.c_int, vp, vp, vp, f32, f32, f32, f32, f32, f32, ctypes.c_int, vp]
    fn.restype = ctypes.c_int
    n = fn(len(mps), _p(mps), _p(pose), ctypes.byref(c), min_x, float(width), min_y, float(height),
           cos_limit, float(log_scale), n_levels, _p(tracks))
    return n, tracks


def search_for_initialization(keys1, desc1, keys2, desc2, width, height, prev_matched,
                              window_size=100, nnratio=0.9, check_ori=True, scale=None):
    """ORBmatcher(nnratio, check_ori).SearchForInitialization(F1, F2, vbPrevMatched,
    vnMatches12, windowSize) on the CPU (src/ORBmatcher.cc:429-577).

    Returns (nmatches, matches12, prev_matched_updated)."""
    scale = np.ones(8, np.float32) if scale is None else scale
    f1, k1 = frame_struct(keys1, desc1, scale, width, height)
    f2, k2 = frame_struct(keys2, desc2, scale, width, height)
    prev = np.array(prev_matched, np.float32).reshape(len(keys1), 2).copy()
    m12 = np.full(len(keys1), -1, np.int32)
    fn = lib().oracle_search_for_initialization
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                   ctypes.c_float, ctypes.c_int, ctypes.c_void_p]
    fn.restype = ctypes.c_int
    n = fn(ctypes.byref(f1), ctypes.byref(f2), _p(prev), int(window_size), float(nnratio),
           int(check_ori), _p(m12))
    return n, m12, prev


def distinctive_descriptors(offs, desc):
    """MapPoint::ComputeDistinctiveDescriptors over CSR observation lists
    (src/MapPoint.cc:250-326): BestIdx per point, -1 for an empty list."""
    offs = np.ascontiguousarray(offs, np.int32)
    desc = np.ascontiguousarray(desc, np.uint8)
    n = len(offs) - 1
    best = np.full(max(n, 0), -1, np.int32)
    fn = lib().oracle_distinctive_descriptors
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    fn.restype = None
    if n > 0:
        fn(n, _p(offs), _p(desc), _p(best))
    return best


def _fr(keys, desc, scale, width, height, u_right=None):
    """orb_frame_t for a (Key)Frame; keeps the numpy buffers alive with it."""
    keys = np.ascontiguousarray(keys, KEYPOINT_DTYPE)
    ur = None if u_right is None else np.ascontiguousarray(u_right, np.float32)
    f, keep = frame_struct(keys, desc, scale, width, height, ur)
    return f, keep


def _f32(a, n=None):
    a = np.ascontiguousarray(a, np.float32)
    return a if n is None else a.reshape(n)


def search_by_projection_reloc(keys, desc, scale, width, height, pose, cam, mps, mp_desc,
                               kf_angle, th, orb_dist, check_ori=True, kp_locked=None,
                               log_scale=None):
    """SearchByProjection(F, pKF, sAlreadyFound, th, ORBdist) (src/ORBmatcher.cc:1622-1759):
    (nmatches, kp_match) with kp_match[j] = point index, -1 untouched, -2 reset."""
    f, keep = _fr(keys, desc, scale, width, height)
    pose = np.ascontiguousarray(pose, POSE_DTYPE).reshape(1)
    mps = np.ascontiguousarray(mps, MAP_POINT_DTYPE)
    mpd = np.ascontiguousarray(mp_desc, np.uint8)
    ka = _f32(kf_angle)
    lk = None if kp_locked is None else np.ascontiguousarray(kp_locked, np.uint8)
    km = np.full(len(keys), -1, np.int32)
    ls = np.float32(pinned_log(np.float32(1.2))) if log_scale is None else log_scale
    c = _Camera(*cam)
    vp, i32, f32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    fn = lib().oracle_search_by_projection_reloc
    fn.argtypes = [vp, vp, vp, vp, f32, i32, vp, vp, vp, f32, i32, i32, vp]
    fn.restype = i32
    n = fn(ctypes.byref(f), _p(lk) if lk is not None else None, _p(pose), ctypes.byref(c), ls,
           len(mps), _p(mps), _p(mpd), _p(ka), th, int(orb_dist), int(check_ori), _p(km))
    return n, km


def search_by_projection_sim3(keys, desc, scale, width, height, scw, cam, mps, mp_desc, th,
                              kp_matched, log_scale=None):
    """SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (src/ORBmatcher.cc:311-425):
    (nmatches, kp_matched updated)."""
    f, keep = _fr(keys, desc, scale, width, height)
    S = _f32(scw, 12)
    mps = np.ascontiguousarray(mps, MAP_POINT_DTYPE)
    mpd = np.ascontiguousarray(mp_desc, np.uint8)
    km = np.array(kp_matched, np.int32).copy()
    ls = np.float32(pinned_log(np.float32(1.2))) if log_scale is None else log_scale
    c = _Camera(*cam)
    vp, i32, f32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    fn = lib().oracle_search_by_projection_sim3
    fn.argtypes = [vp, vp, vp, f32, i32, vp, vp, f32, vp]
    fn.restype = i32
    n = fn(ctypes.byref(f), _p(S), ctypes.byref(c), ls, len(mps), _p(mps), _p(mpd), th, _p(km))
    return n, km


def fuse(keys, desc, scale, inv_sigma2, width, height, u_right, pose, cam, mps, mp_desc, th,
         log_scale=None):
    """Fuse(pKF, vpMapPoints, th) target selection (src/ORBmatcher.cc:903-1077):
    (n_with_target, best keypoint per point or -1)."""
    f, keep = _fr(keys, desc, scale, width, height, u_right)
    inv = _f32(inv_sigma2)
    pose = np.ascontiguousarray(pose, POSE_DTYPE).reshape(1)
    mps = np.ascontiguousarray(mps, MAP_POINT_DTYPE)
    mpd = np.ascontiguousarray(mp_desc, np.uint8)
    best = np.full(len(mps), -1, np.int32)
    ls = np.float32(pinned_log(np.float32(1.2))) if log_scale is None else log_scale
    c = _Camera(*cam)
    vp, i32, f32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    fn = lib().oracle_fuse
    fn.argtypes = [vp, vp, vp, vp, f32, i32, vp, vp, f32, vp]
    fn.restype = i32
    n = fn(ctypes.byref(f), _p(inv), _p(pose), ctypes.byref(c), ls, len(mps), _p(mps), _p(mpd),
           th, _p(best))
    return n, best


def fuse_sim3(keys, desc, scale, width, height, scw, cam, mps, mp_desc, th, log_scale=None):
    """Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) target selection
    (src/ORBmatcher.cc:1079-1210): (n_with_target, best keypoint per point or -1)."""
    f, keep = _fr(keys, desc, scale, width, height)
    S = _f32(scw, 12)
    mps = np.ascontiguousarray(mps, MAP_POINT_DTYPE)
    mpd = np.ascontiguousarray(mp_desc, np.uint8)
    best = np.full(len(mps), -1, np.int32)
    ls = np.float32(pinned_log(np.float32(1.2))) if log_scale is None else log_scale
    c = _Camera(*cam)
    vp, i32, f32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    fn = lib().oracle_fuse_sim3
    fn.argtypes = [vp, vp, vp, f32, i32, vp, vp, f32, vp]
    fn.restype = i32
    n = fn(ctypes.byref(f), _p(S), ctypes.byref(c), ls, len(mps), _p(mps), _p(mpd), th,
           _p(best))
    return n, best


def search_by_sim3(kf1, kf2, cam, s12, R12, t12, th, log_scale=None):
    """SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th)
    (src/ORBmatcher.cc:1212-1458).  kfX = dict(keys, desc, scale, width, height,
    Rw (3x3), tw (3), mps (MAP_POINT_DTYPE per keypoint), valid, already, mp_desc).
    Returns (nFound, match12)."""
    ls = np.float32(pinned_log(np.float32(1.2))) if log_scale is None else log_scale
    f1, k1 = _fr(kf1["keys"], kf1["desc"], kf1["scale"], kf1["width"], kf1["height"])
    f2, k2 = _fr(kf2["keys"], kf2["desc"], kf2["scale"], kf2["width"], kf2["height"])
    arrs = []
    for kf in (kf1, kf2):
        arrs.append([_f32(kf["Rw"], 9), _f32(kf["tw"], 3),
                     np.ascontiguousarray(kf["mps"], MAP_POINT_DTYPE),
                     np.ascontiguousarray(kf["valid"], np.uint8),
                     np.ascontiguousarray(kf["already"], np.uint8),
                     np.ascontiguousarray(kf["mp_desc"], np.uint8)])
    R12, t12 = _f32(R12, 9), _f32(t12, 3)
    m12 = np.full(len(kf1["keys"]), -1, np.int32)
    c = _Camera(*cam)
    vp, i32, f32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    fn = lib().oracle_search_by_sim3
    fn.argtypes = [vp, vp, f32, f32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, f32, vp,
                   vp, f32, vp]
    fn.restype = i32
    a1, a2 = arrs
    n = fn(ctypes.byref(f1), ctypes.byref(f2), ls, ls, ctypes.byref(c), _p(a1[0]), _p(a1[1]),
           _p(a2[0]), _p(a2[1]), _p(a1[2]), _p(a1[3]), _p(a1[4]), _p(a1[5]), _p(a2[2]),
           _p(a2[3]), _p(a2[4]), _p(a2[5]), s12, _p(R12), _p(t12), th, _p(m12))
    return n, m12


def search_by_bow_kf(d1, a1, mp1, bad1, fv1, d2, a2, mp2, bad2, fv2, nnratio, check_ori):
    """SearchByBoW(pKF1, pKF2, vpMatches12) (src/ORBmatcher.cc:581-716):
    (nmatches, match12 = MapPoint id of KF2 or -1)."""
    d1, d2 = np.ascontiguousarray(d1, np.uint8), np.ascontiguousarray(d2, np.uint8)
    a1, a2 = _f32(a1), _f32(a2)
    mp1, mp2 = np.ascontiguousarray(mp1, np.int32), np.ascontiguousarray(mp2, np.int32)
    b1 = None if bad1 is None else np.ascontiguousarray(bad1, np.uint8)
    b2 = None if bad2 is None else np.ascontiguousarray(bad2, np.uint8)
    m12 = np.full(len(d1), -1, np.int32)
    vp, i32, f32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    fn = lib().oracle_search_by_bow_kf
    fn.argtypes = [vp, vp, vp, vp, i32, i32, vp, vp, vp, vp, vp, vp, vp, i32, i32, vp, vp, vp,
                   f32, i32, vp]
    fn.restype = i32
    n = fn(_p(d1), _p(a1), _p(mp1), _p(b1) if b1 is not None else None, len(d1), len(fv1[0]),
           _p(fv1[0]), _p(fv1[1]), _p(fv1[2]), _p(d2), _p(a2), _p(mp2),
           _p(b2) if b2 is not None else None, len(d2), len(fv2[0]), _p(fv2[0]), _p(fv2[1]),
           _p(fv2[2]), nnratio, int(check_ori), _p(m12))
    return n, m12


def search_for_triangulation(kf1, kf2, level_sigma2, F12, cam, Cw, R2w, t2w, fv1, fv2,
                             only_stereo=False, check_ori=True):
    """SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo)
    (src/ORBmatcher.cc:718-901): (nmatches, match12 = KF2 index or -1).
    kfX = dict(keys, desc, scale, width, height, u_right, has_mp)."""
    f1, k1 = _fr(kf1["keys"], kf1["desc"], kf1["scale"], kf1["width"], kf1["height"],
                 kf1["u_right"])
    f2, k2 = _fr(kf2["keys"], kf2["desc"], kf2["scale"], kf2["width"], kf2["height"],
                 kf2["u_right"])
    h1 = np.ascontiguousarray(kf1["has_mp"], np.uint8)
    h2 = np.ascontiguousarray(kf2["has_mp"], np.uint8)
    ls2, F, C, R, t = _f32(level_sigma2), _f32(F12, 9), _f32(Cw, 3), _f32(R2w, 9), _f32(t2w, 3)
    m12 = np.full(len(kf1["keys"]), -1, np.int32)
    c = _Camera(*cam)
    vp, i32 = ctypes.c_void_p, ctypes.c_int
    fn = lib().oracle_search_for_triangulation
    fn.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, vp, vp, vp, i32, vp, vp, vp, i32,
                   i32, vp]
    fn.restype = i32
    n = fn(ctypes.byref(f1), _p(h1), ctypes.byref(f2), _p(h2), _p(ls2), _p(F), ctypes.byref(c),
           _p(C), _p(R), _p(t), len(fv1[0]), _p(fv1[0]), _p(fv1[1]), _p(fv1[2]), len(fv2[0]),
           _p(fv2[0]), _p(fv2[1]), _p(fv2[2]), int(only_stereo), int(check_ori), _p(m12))
    return n, m12


def vocab_transform(voc, desc, levelsup=4, scoring=0, weighting=0):
    """TemplatedVocabulary::transform(features, BowVector, FeatureVector, levelsup)
    (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1128-1283) on the node table
    `voc` (dict parent/leaf/desc/weight, k, L).  Returns (bow_words, bow_values,
    fv_nodes, fv_offs, fv_feats, feat_word, feat_node)."""
    desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    n = len(desc)
    parent = np.ascontiguousarray(voc["parent"], np.int32)
    leaf = np.ascontiguousarray(voc["leaf"], np.uint8)
    nd = np.ascontiguousarray(voc["desc"], np.uint8)
    nw = np.ascontiguousarray(voc["weight"], np.float64)
    cap = max(n, 1)
    bw = np.zeros(cap, np.uint32)
    bv = np.zeros(cap, np.float64)
    fvn = np.zeros(cap, np.uint32)
    fvo = np.zeros(cap + 1, np.int32)
    fvf = np.zeros(cap, np.uint32)
    fw = np.zeros(cap, np.uint32)
    fnode = np.zeros(cap, np.uint32)
    n_words = ctypes.c_int(0)
    n_fv = ctypes.c_int(0)
    fn = lib().oracle_vocab_transform
    vp, i32 = ctypes.c_void_p, ctypes.c_int
    fn.argtypes = [i32, i32, i32, i32, i32, vp, vp, vp, vp, i32, vp, i32, vp, vp, vp, vp, vp, vp,
                   vp, vp, vp]
    fn.restype = i32
    r = fn(int(voc["k"]), int(voc["L"]), scoring, weighting, len(parent), _p(parent), _p(leaf),
           _p(nd), _p(nw), n, _p(desc), levelsup, _p(bw), _p(bv), ctypes.byref(n_words), _p(fvn),
           _p(fvo), _p(fvf), ctypes.byref(n_fv), _p(fw), _p(fnode))
    if r != 0:
        raise ValueError("malformed vocabulary node table")
    a, b = n_words.value, n_fv.value
    return (bw[:a], bv[:a], fvn[:b], fvo[:b + 1], fvf[:fvo[b]], fw[:n], fnode[:n])


def vocab_parse_text(path):
    """loadFromTextFile (TemplatedVocabulary.h:1362-1448): the header and node
    table, as a dict like tests/scenarios.vocabulary returns (plus scoring,
    weighting)."""
    fn = lib().oracle_vocab_parse_text
    vp = ctypes.c_void_p
    fn.argtypes = [ctypes.c_char_p, vp, ctypes.c_int, vp, vp, vp, vp]
    fn.restype = ctypes.c_int
    hdr = np.zeros(4, np.int32)
    n = fn(str(path).encode(), _p(hdr), 0, None, None, None, None)
    if n < 0:
        raise ValueError(f"cannot parse vocabulary {path}")
    parent = np.zeros(n, np.int32)
    leaf = np.zeros(n, np.uint8)
    desc = np.zeros((n, 32), np.uint8)
    weight = np.zeros(n, np.float64)
    fn(str(path).encode(), _p(hdr), n, _p(parent), _p(leaf), _p(desc), _p(weight))
    return dict(k=int(hdr[0]), L=int(hdr[1]), scoring=int(hdr[2]), weighting=int(hdr[3]),
                parent=parent, leaf=leaf, desc=desc, weight=weight)


def vocab_time(voc, desc, n_frames, n_per_frame, levelsup=4, scoring=0, weighting=0):
    """Seconds the oracle spends in transform() over n_frames frames (tree built
    once, outside the timed region).  CPU baseline only."""
    desc = np.ascontiguousarray(desc, np.uint8)
    parent = np.ascontiguousarray(voc["parent"], np.int32)
    leaf = np.ascontiguousarray(voc["leaf"], np.uint8)
    nd = np.ascontiguousarray(voc["desc"], np.uint8)
    nw = np.ascontiguousarray(voc["weight"], np.float64)
    fn = lib().oracle_vocab_time
    vp, i32 = ctypes.c_void_p, ctypes.c_int
    fn.argtypes = [i32, i32, i32, i32, i32, vp, vp, vp, vp, i32, i32, vp, i32]
    fn.restype = ctypes.c_double
    return fn(int(voc["k"]), int(voc["L"]), scoring, weighting, len(parent), _p(parent),
              _p(leaf), _p(nd), _p(nw), n_frames, n_per_frame, _p(desc), levelsup)


def _cam_args(K, dist):
    K = np.ascontiguousarray(K, np.float32).reshape(9)
    dist = np.ascontiguousarray(dist, np.float32).reshape(-1)
    return K, dist


def undistort_points(xy, K, dist):
    """cv::undistortPoints(src, dst, K, D, noArray(), K) on (n, 2) float points
    (OpenCV cvUndistortPoints arithmetic; see camera_oracle.cpp)."""
    xy = np.ascontiguousarray(xy, np.float32).reshape(-1, 2)
    K, dist = _cam_args(K, dist)
    out = np.zeros_like(xy)
    fn = lib().oracle_undistort_points
    vp = ctypes.c_void_p
    fn.argtypes = [ctypes.c_int, vp, vp, vp, ctypes.c_int, vp]
    fn.restype = ctypes.c_int
    if fn(len(xy), _p(xy), _p(K), _p(dist), len(dist), _p(out)) != 0:
        raise ValueError("unsupported distortion model")
    return out


def undistort_keypoints(keys, K, dist):
    """Frame::UndistortKeyPoints (src/Frame.cc:452-482) -> mvKeysUn."""
    keys = np.ascontiguousarray(keys, KEYPOINT_DTYPE)
    K, dist = _cam_args(K, dist)
    out = np.zeros_like(keys)
    fn = lib().oracle_undistort_keypoints
    vp = ctypes.c_void_p
    fn.argtypes = [ctypes.c_int, vp, vp, vp, ctypes.c_int, vp]
    fn.restype = ctypes.c_int
    if fn(len(keys), _p(keys) if len(keys) else None, _p(K), _p(dist), len(dist),
          _p(out) if len(keys) else None) != 0:
        raise ValueError("unsupported distortion model")
    return out


def compute_image_bounds(cols, rows, K, dist):
    """Frame::ComputeImageBounds (src/Frame.cc:484-514) -> (minX, maxX, minY, maxY)."""
    K, dist = _cam_args(K, dist)
    b = np.zeros(4, np.float32)
    fn = lib().oracle_compute_image_bounds
    vp = ctypes.c_void_p
    fn.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_int, vp]
    fn.restype = ctypes.c_int
    if fn(cols, rows, _p(K), _p(dist), len(dist), _p(b)) != 0:
        raise ValueError("unsupported distortion model")
    return b
