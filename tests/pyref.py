"""Independent pure-Python / numpy restatements used to cross-check the C++ oracle
on small inputs (test infrastructure only).

They follow the reference text directly, written a second time and differently
(numpy where the rule is arithmetic, plain lists where it is control flow), so a
transcription slip in oracle/orb_oracle.cpp shows up as a disagreement.
"""
from __future__ import annotations

import math

import numpy as np

CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3),
          (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def f32(x):
    return np.float32(x)


# ------------------------------------------------------------------ FAST (A.1)
def fast(img: np.ndarray, t: int):
    """cv::FAST(img, kps, t, nonmax=True) from its mathematical definition:
    corner iff 9 contiguous circle pixels are all < v-t or all > v+t; score =
    max(t, best dark arc, best bright arc) - 1; NMS vs 8-neighbours with
    non-corners (and everything outside rows/cols 3..n-4) at 0."""
    t = min(max(t, 0), 255)
    h, w = img.shape
    I = img.astype(np.int32)
    score = np.zeros((h, w), np.int32)
    corner = np.zeros((h, w), bool)
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            v = I[y, x]
            ring = [I[y + dy, x + dx] for dx, dy in CIRCLE]
            dark = [v - r for r in ring]  # > t for dark pixels
            best_d = max(min(dark[(k + j) % 16] for j in range(9)) for k in range(16))
            best_b = max(min(-dark[(k + j) % 16] for j in range(9)) for k in range(16))
            if best_d > t or best_b > t:
                corner[y, x] = True
                score[y, x] = max(t, best_d, best_b) - 1
    out = []
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            if not corner[y, x]:
                continue
            s = score[y, x]
            if all(s > score[y + dy, x + dx] for dy in (-1, 0, 1) for dx in (-1, 0, 1)
                   if dy or dx):
                out.append((x, y, s))
    return out


# --------------------------------------------------------- resize INTER_LINEAR (A.2)
def resize_linear(src: np.ndarray, dw: int, dh: int) -> np.ndarray:
    sh, sw = src.shape
    scale_x = 1.0 / (dw / sw)
    scale_y = 1.0 / (dh / sh)

    def coeffs(n_dst, n_src, scale, clamp):
        idx = np.zeros(n_dst, np.int64)
        w0 = np.zeros(n_dst, np.int64)
        w1 = np.zeros(n_dst, np.int64)
        edge = np.zeros(n_dst, bool)
        for d in range(n_dst):
            f = f32((d + 0.5) * scale - 0.5)
            s = int(math.floor(f))
            f = f32(f - f32(s))
            if clamp:
                if s < 0:
                    f, s = f32(0), 0
                if s + 1 >= n_src:
                    edge[d] = True
                    if s >= n_src - 1:
                        f, s = f32(0), n_src - 1
            idx[d] = s
            w0[d] = int(np.rint(f32(f32(1) - f) * f32(2048)))
            w1[d] = int(np.rint(f * f32(2048)))
        return idx, w0, w1, edge

    xi, a0, a1, xedge = coeffs(dw, sw, scale_x, True)
    yi, b0, b1, _ = coeffs(dh, sh, scale_y, False)
    first_edge = int(np.argmax(xedge)) if xedge.any() else dw
    S = src.astype(np.int64)
    x1 = np.minimum(xi + 1, sw - 1)
    H = S[:, xi] * a0 + S[:, x1] * a1
    H[:, first_edge:] = S[:, xi[first_edge:]] * 2048
    r0 = np.clip(yi, 0, sh - 1)
    r1 = np.clip(yi + 1, 0, sh - 1)
    D = (H[r0] * b0[:, None] + H[r1] * b1[:, None] + (1 << 21)) >> 22
    return np.clip(D, 0, 255).astype(np.uint8)


# ------------------------------------------------------ GaussianBlur 7x7 (A.3)
def gaussian_kernel_int():
    """getGaussianKernel(7, 2, CV_32F) then cvRound(k * 256)."""
    x = np.arange(7) - 3.0
    k = np.array([f32(math.exp(-0.5 / (2.0 * 2.0) * v * v)) for v in x], np.float32)
    s = 0.0
    for v in k:
        s += float(v)
    k = np.array([f32(float(v) * (1.0 / s)) for v in k], np.float32)
    return [int(np.rint(f32(v) * f32(256))) for v in k]


def blur7(src: np.ndarray) -> np.ndarray:
    k = np.array(gaussian_kernel_int(), np.int64)
    p = np.pad(src.astype(np.int64), 3, mode="reflect")  # numpy 'reflect' == BORDER_REFLECT_101
    h, w = src.shape
    rows = sum(k[i] * p[:, i:i + w] for i in range(7))
    cols = sum(k[j] * rows[j:j + h, :] for j in range(7))
    return np.clip((cols + (1 << 15)) >> 16, 0, 255).astype(np.uint8)


# ----------------------------------------------------------- fastAtan2 (A.4)
def fast_atan2(y, x):
    y, x = f32(y), f32(x)
    r2d = f32(180.0 / math.pi)
    p1, p3 = f32(0.9997878412794807) * r2d, f32(-0.3258083974640975) * r2d
    p5, p7 = f32(0.1555786518463281) * r2d, f32(-0.04432655554792128) * r2d
    ax, ay = abs(x), abs(y)
    eps = f32(2.220446049250313e-16)
    if ax >= ay:
        c = f32(ay / f32(ax + eps))
        c2 = f32(c * c)
        a = f32(f32(f32(f32(f32(f32(f32(p7 * c2) + p5) * c2) + p3) * c2) + p1) * c)
    else:
        c = f32(ax / f32(ay + eps))
        c2 = f32(c * c)
        a = f32(f32(90) - f32(f32(f32(f32(f32(f32(f32(p7 * c2) + p5) * c2) + p3) * c2) + p1) * c))
    if x < 0:
        a = f32(f32(180) - a)
    if y < 0:
        a = f32(f32(360) - a)
    return a


# ------------------------------------------------- DistributeOctTree (a5)
class _Node:
    __slots__ = ("keys", "ul", "ur", "bl", "br", "nomore", "seq")

    def __init__(self, ul, ur, bl, br, seq):
        self.keys, self.ul, self.ur, self.bl, self.br = [], ul, ur, bl, br
        self.nomore, self.seq = False, seq


def distribute(keys, minX, maxX, minY, maxY, N):
    """keys: list of (x, y, response) relative to the border origin.
    Python list as the std::list (index 0 = front); node creation sequence as
    the pointer tie-break."""
    nIni = int(math.floor(float(f32(f32(maxX - minX) / f32(maxY - minY))) + 0.5))  # roundf
    hX = f32(f32(maxX - minX) / f32(nIni))
    seq = [0]

    def new(ul, ur, bl, br):
        n = _Node(ul, ur, bl, br, seq[0])
        seq[0] += 1
        return n

    lst = []
    ini = []
    for i in range(nIni):
        ulx, urx = int(f32(hX * f32(i))), int(f32(hX * f32(i + 1)))
        n = new((ulx, 0), (urx, 0), (ulx, maxY - minY), (urx, maxY - minY))
        lst.append(n)
        ini.append(n)
    for k in keys:
        ini[int(f32(f32(k[0]) / hX))].keys.append(k)
    lst = [n for n in lst if n.keys]
    for n in lst:
        n.nomore = len(n.keys) == 1

    def divide(p):
        hx = int(math.ceil(float(f32(p.ur[0] - p.ul[0]) / f32(2))))
        hy = int(math.ceil(float(f32(p.br[1] - p.ul[1]) / f32(2))))
        c1 = new(p.ul, (p.ul[0] + hx, p.ul[1]), (p.ul[0], p.ul[1] + hy), (p.ul[0] + hx, p.ul[1] + hy))
        c2 = new(c1.ur, p.ur, c1.br, (p.ur[0], p.ul[1] + hy))
        c3 = new(c1.bl, c1.br, p.bl, (c1.br[0], p.bl[1]))
        c4 = new(c3.ur, c2.br, c3.br, p.br)
        for k in p.keys:
            if k[0] < c1.ur[0]:
                (c1 if k[1] < c1.br[1] else c3).keys.append(k)
            elif k[1] < c1.br[1]:
                c2.keys.append(k)
            else:
                c4.keys.append(k)
        out = []
        for c in (c1, c2, c3, c4):
            c.nomore = len(c.keys) == 1
            if c.keys:
                out.append(c)
        return out

    # creation numbers only matter among pushed nodes: renumber at push time
    counter = [nIni]

    def push_children(children, sized):
        nonlocal lst
        for c in children:
            c.seq = counter[0]
            counter[0] += 1
            lst.insert(0, c)
            if len(c.keys) > 1:
                sized.append(c)

    finish = False
    sized = []
    while not finish:
        prev = len(lst)
        sized = []
        n_expand = 0
        i = 0
        while i < len(lst):
            nd = lst[i]
            if nd.nomore:
                i += 1
                continue
            before = len(sized)
            kids = divide(nd)
            lst.pop(i)
            push_children(kids, sized)
            n_expand += len(sized) - before
            i += len(kids)  # skip the children now in front of the cursor
        if len(lst) >= N or len(lst) == prev:
            finish = True
        elif len(lst) + n_expand * 3 > N:
            while not finish:
                prev = len(lst)
                cand = sorted(sized, key=lambda n: (len(n.keys), n.seq))
                sized = []
                for nd in reversed(cand):
                    kids = divide(nd)
                    lst.remove(nd)
                    push_children(kids, sized)
                    if len(lst) >= N:
                        break
                if len(lst) >= N or len(lst) == prev:
                    finish = True
    result = []
    for nd in lst:
        best = nd.keys[0]
        for k in nd.keys[1:]:
            if k[2] > best[2]:
                best = k
        result.append(best)
    return result


# ------------------------------------------------- grid + GetFeaturesInArea
def grid_cells(keys, width, height):
    invW = f32(f32(64) / f32(width))
    invH = f32(f32(48) / f32(height))
    cells = {}
    for i, k in enumerate(keys):
        vx, vy = f32(f32(k["x"]) * invW), f32(f32(k["y"]) * invH)
        px = int(math.floor(float(vx) + 0.5)) if vx >= 0 else -int(math.floor(-float(vx) + 0.5))
        py = int(math.floor(float(vy) + 0.5)) if vy >= 0 else -int(math.floor(-float(vy) + 0.5))
        if 0 <= px < 64 and 0 <= py < 48:
            cells.setdefault((px, py), []).append(i)
    return cells, invW, invH


def features_in_area(keys, cells, invW, invH, x, y, r, minL, maxL):
    x, y, r = f32(x), f32(y), f32(r)
    x0 = max(0, int(math.floor(float(f32(f32(x - r) * invW)))))
    if x0 >= 64:
        return []
    x1 = min(63, int(math.ceil(float(f32(f32(x + r) * invW)))))
    if x1 < 0:
        return []
    y0 = max(0, int(math.floor(float(f32(f32(y - r) * invH)))))
    if y0 >= 48:
        return []
    y1 = min(47, int(math.ceil(float(f32(f32(y + r) * invH)))))
    if y1 < 0:
        return []
    check = minL > 0 or maxL >= 0
    out = []
    for ix in range(x0, x1 + 1):
        for iy in range(y0, y1 + 1):
            for i in cells.get((ix, iy), []):
                k = keys[i]
                if check and (k["octave"] < minL or (maxL >= 0 and k["octave"] > maxL)):
                    continue
                if abs(f32(k["x"] - x)) < r and abs(f32(k["y"] - y)) < r:
                    out.append(i)
    return out


def hamming(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def search_by_projection_local(keys, desc, scale, width, height, mps, mp_desc, th, nnratio,
                               locked=None):
    cells, invW, invH = grid_cells(keys, width, height)
    lock = np.zeros(len(keys), bool) if locked is None else locked.astype(bool).copy()
    km = np.full(len(keys), -1, np.int32)
    n = 0
    for m, mp in enumerate(mps):
        if not mp["in_view"] or mp["bad"]:
            continue
        lvl = int(mp["level"])
        r = f32(2.5) if float(mp["view_cos"]) > 0.998 else f32(4.0)  # float vs double literal
        if f32(th) != f32(1.0):
            r = f32(r * f32(th))
        rs = f32(r * f32(scale[lvl]))
        idxs = features_in_area(keys, cells, invW, invH, mp["proj_x"], mp["proj_y"], rs, lvl - 1, lvl)
        best, bl, best2, bl2, bi = 256, -1, 256, -1, -1
        for i in idxs:
            if lock[i]:
                continue
            d = hamming(mp_desc[m], desc[i])
            if d < best:
                best2, bl2 = best, bl
                best, bl, bi = d, int(keys[i]["octave"]), i
            elif d < best2:
                best2, bl2 = d, int(keys[i]["octave"])
        if best <= 100:
            if bl == bl2 and f32(best) > f32(f32(nnratio) * f32(best2)):
                continue
            km[bi] = m
            if mp["has_obs"]:
                lock[bi] = True
            n += 1
    return n, km


def frustum(mps, rcw, tcw, ow, cam, width, height, cos_limit, log_scale, n_levels):
    """Vectorised numpy restatement of Frame::isInFrustum + MapPoint::PredictScale
    (src/Frame.cc:303-366, src/MapPoint.cc:435-450) with the oracle's pinned
    arithmetic: float32 Pc / projection, float64 norm and dot.  log via numpy
    float64 (the oracle pins fdlibm's scheme; both agree after rounding to float)."""
    f32 = np.float32
    fx, fy, cx, cy, bf, _ = (f32(c) for c in cam)
    R = np.asarray(rcw, f32).reshape(3, 3)
    t = np.asarray(tcw, f32)
    P = mps["pos"].astype(f32)
    pc = [((R[i, 0] * P[:, 0] + R[i, 1] * P[:, 1]) + R[i, 2] * P[:, 2]) + t[i] for i in range(3)]
    X, Y, Z = pc
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        invz = f32(1.0) / Z
        u = fx * X * invz + cx
        v = fy * Y * invz + cy
        O = P - np.asarray(ow, f32)
        dist = np.sqrt(((O[:, 0].astype(np.float64) ** 2) + O[:, 1].astype(np.float64) ** 2)
                       + O[:, 2].astype(np.float64) ** 2).astype(f32)
        N = mps["normal"].astype(np.float64)
        dot = ((O[:, 0] * N[:, 0]) + O[:, 1] * N[:, 1]) + O[:, 2] * N[:, 2]
        view_cos = (dot / dist.astype(np.float64)).astype(f32)
        maxd = f32(1.2) * mps["max_distance"]
        mind = f32(0.8) * mps["min_distance"]
        ok = (mps["seen"] == 0) & (mps["bad"] == 0) & ~(Z < 0)
        ok &= ~((u < 0) | (u > f32(width)) | (v < 0) | (v > f32(height)))
        ok &= ~((dist < mind) | (dist > maxd))
        ok &= ~(view_cos < f32(cos_limit))
        ratio = mps["max_distance"] / dist
        lr = np.log(ratio.astype(np.float64)).astype(f32)
        q = np.ceil(lr / f32(log_scale))
        level = np.where(q < 0, 0, np.where(q >= n_levels, n_levels - 1,
                                            np.nan_to_num(q).astype(np.int64)))
    return ok, u, v, u - bf * invz, view_cos, level


def _rot_bin(a1, a2):
    # ORBmatcher's histogram bin with factor 1/HISTO_LENGTH (src/ORBmatcher.cc:516-524)
    rot = f32(f32(a1) - f32(a2))
    if rot < 0.0:
        rot = f32(rot + f32(360.0))
    v = f32(rot * f32(f32(1.0) / f32(30)))
    b = int(math.floor(float(v) + 0.5))
    return 0 if b == 30 else b


def _three_maxima(counts):
    m1 = m2 = m3 = 0
    i1 = i2 = i3 = -1
    for i, s in enumerate(counts):
        if s > m1:
            m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, i
        elif s > m2:
            m3, m2, i3, i2 = m2, s, i2, i
        elif s > m3:
            m3, i3 = s, i
    if m2 < f32(0.1) * f32(m1):
        i2 = i3 = -1
    elif m3 < f32(0.1) * f32(m1):
        i3 = -1
    return i1, i2, i3


def search_for_initialization(keys1, desc1, keys2, desc2, width, height, prev, window,
                              nnratio, check_ori):
    """Independent restatement of ORBmatcher::SearchForInitialization
    (src/ORBmatcher.cc:429-577) in plain Python."""
    cells, invW, invH = grid_cells(keys2, width, height)
    prev = np.array(prev, np.float32).reshape(len(keys1), 2).copy()
    m12 = np.full(len(keys1), -1, np.int32)
    mdist = [1 << 31] * len(keys2)
    m21 = [-1] * len(keys2)
    hist = [[] for _ in range(30)]
    n = 0
    for i1 in range(len(keys1)):
        if keys1[i1]["octave"] > 0:
            continue
        idx = features_in_area(keys2, cells, invW, invH, prev[i1, 0], prev[i1, 1], window, 0, 0)
        if not idx:
            continue
        b1, b2, bi = 1 << 31, 1 << 31, -1
        for i2 in idx:
            d = hamming(desc1[i1], desc2[i2])
            if mdist[i2] <= d:
                continue
            if d < b1:
                b2, b1, bi = b1, d, i2
            elif d < b2:
                b2 = d
        if b1 <= 50 and f32(b1) < f32(f32(b2) * f32(nnratio)):
            if m21[bi] >= 0:
                m12[m21[bi]] = -1
                n -= 1
            m12[i1], m21[bi], mdist[bi] = bi, i1, b1
            n += 1
            if check_ori:
                hist[_rot_bin(keys1[i1]["angle"], keys2[bi]["angle"])].append(i1)
    if check_ori:
        keep = _three_maxima([len(h) for h in hist])
        for b in range(30):
            if b in keep:
                continue
            for i1 in hist[b]:
                if m12[i1] >= 0:
                    m12[i1] = -1
                    n -= 1
    for i1 in range(len(keys1)):
        if m12[i1] >= 0:
            prev[i1] = (keys2[m12[i1]]["x"], keys2[m12[i1]]["y"])
    return n, m12, prev


def distinctive_descriptor(desc):
    """MapPoint::ComputeDistinctiveDescriptors' BestIdx (src/MapPoint.cc:285-318)."""
    n = len(desc)
    if n == 0:
        return -1
    bits = np.unpackbits(desc, axis=1).astype(np.int32)
    D = (bits[:, None, :] != bits[None, :, :]).sum(-1)
    best, bi = 1 << 31, 0
    for i in range(n):
        med = int(np.sort(D[i])[int(0.5 * (n - 1))])
        if med < best:
            best, bi = med, i
    return bi


# ------------------------------------------- §8(f) ORBmatcher variants (scalar)
def _xf(R, t, P):
    R = np.asarray(R, np.float32).reshape(3, 3)
    return [f32(f32(f32(R[r, 0] * f32(P[0])) + f32(R[r, 1] * f32(P[1]))) + f32(R[r, 2] * f32(P[2])))
            + f32(t[r]) for r in range(3)]


def _norm(a):
    return f32(math.sqrt(sum(float(x) * float(x) for x in a)))


def _dotd(a, b):
    return sum(float(x) * float(y) for x, y in zip(a, b))


def _level(maxd, dist, log_scale, n_levels):
    ratio = f32(f32(maxd) / f32(dist))
    q = np.ceil(f32(f32(math.log(float(ratio))) / f32(log_scale)))
    return 0 if q < 0 else (n_levels - 1 if q >= n_levels else int(q))


def _sim3_pose(S):
    S = np.asarray(S, np.float32).reshape(3, 4)
    scw = f32(math.sqrt(sum(float(S[0, k]) ** 2 for k in range(3))))
    inv = 1.0 / float(scw)
    R = np.array([[f32(float(S[r, c]) * inv) for c in range(3)] for r in range(3)], np.float32)
    t = np.array([f32(float(S[r, 3]) * inv) for r in range(3)], np.float32)
    ow = np.array([-(f32(f32(R[0, i] * t[0]) + f32(R[1, i] * t[1])) + f32(R[2, i] * t[2]))
                   for i in range(3)], np.float32)
    return R, t, ow


def _in_kf(x, y, w, h):
    return 0 <= x < w and 0 <= y < h


def _best(keys, desc, cells, invW, invH, dq, u, v, r, lo, hi, skip=None, gate=None,
          check_levels=False, init=256):
    """GetFeaturesInArea + first-minimum scan; the level filter is either the
    function's (check_levels) or the loop's (kpLevel < lo || > hi)."""
    idx = features_in_area(keys, cells, invW, invH, u, v, r, lo if check_levels else -1,
                           hi if check_levels else -1)
    bd, bi = init, -1
    for j in idx:
        if skip is not None and skip(j):
            continue
        o = int(keys[j]["octave"])
        if not check_levels and (o < lo or o > hi):
            continue
        if gate is not None and not gate(j):
            continue
        d = hamming(dq, desc[j])
        if d < bd:
            bd, bi = d, j
    return bd, bi


def search_by_projection_sim3(keys, desc, scale, width, height, S, cam, mps, mp_desc, th,
                              kp_matched, log_scale, n_levels=8):
    fx, fy, cx, cy = (f32(c) for c in cam[:4])
    cells, invW, invH = grid_cells(keys, width, height)
    R, t, ow = _sim3_pose(S)
    km = np.array(kp_matched, np.int32).copy()
    n = 0
    for i, mp in enumerate(mps):
        if mp["bad"] or mp["seen"]:
            continue
        Pc = _xf(R, t, mp["pos"])
        if Pc[2] < 0:
            continue
        invz = f32(f32(1) / Pc[2])
        u = f32(f32(fx * f32(Pc[0] * invz)) + cx)
        v = f32(f32(fy * f32(Pc[1] * invz)) + cy)
        if not _in_kf(u, v, width, height):
            continue
        PO = [f32(f32(mp["pos"][k]) - ow[k]) for k in range(3)]
        dist = _norm(PO)
        if dist < f32(f32(0.8) * mp["min_distance"]) or dist > f32(f32(1.2) * mp["max_distance"]):
            continue
        if _dotd(PO, mp["normal"]) < 0.5 * float(dist):
            continue
        lvl = _level(mp["max_distance"], dist, log_scale, n_levels)
        bd, bi = _best(keys, desc, cells, invW, invH, mp_desc[i], u, v,
                       f32(f32(th) * f32(scale[lvl])), lvl - 1, lvl, skip=lambda j: km[j] >= 0)
        if bd <= 50:
            km[bi] = i
            n += 1
    return n, km


def fuse(keys, desc, scale, inv_sigma2, width, height, u_right, R, t, ow, cam, mps, mp_desc, th,
         log_scale, n_levels=8):
    fx, fy, cx, cy, bf = (f32(c) for c in cam[:5])
    cells, invW, invH = grid_cells(keys, width, height)
    best = np.full(len(mps), -1, np.int32)
    n = 0
    for i, mp in enumerate(mps):
        if mp["bad"] or mp["seen"]:
            continue
        Pc = _xf(R, t, mp["pos"])
        if Pc[2] < 0:
            continue
        invz = f32(f32(1) / Pc[2])
        u = f32(f32(fx * f32(Pc[0] * invz)) + cx)
        v = f32(f32(fy * f32(Pc[1] * invz)) + cy)
        if not _in_kf(u, v, width, height):
            continue
        ur = f32(u - f32(bf * invz))
        PO = [f32(f32(mp["pos"][k]) - f32(ow[k])) for k in range(3)]
        dist = _norm(PO)
        if dist < f32(f32(0.8) * mp["min_distance"]) or dist > f32(f32(1.2) * mp["max_distance"]):
            continue
        if _dotd(PO, mp["normal"]) < 0.5 * float(dist):
            continue
        lvl = _level(mp["max_distance"], dist, log_scale, n_levels)

        def gate(j):
            k = keys[j]
            ex, ey = f32(u - f32(k["x"])), f32(v - f32(k["y"]))
            e2 = f32(f32(ex * ex) + f32(ey * ey))
            if u_right[j] >= 0:
                er = f32(ur - f32(u_right[j]))
                return float(f32(f32(e2 + f32(er * er)) * f32(inv_sigma2[k["octave"]]))) <= 7.8
            return float(f32(e2 * f32(inv_sigma2[k["octave"]]))) <= 5.99

        bd, bi = _best(keys, desc, cells, invW, invH, mp_desc[i], u, v,
                       f32(f32(th) * f32(scale[lvl])), lvl - 1, lvl, gate=gate)
        if bd <= 50:
            best[i] = bi
            n += 1
    return n, best


def search_by_sim3(kf1, kf2, cam, s12, R12, t12, th, log_scale, n_levels=8):
    fx, fy, cx, cy = (f32(c) for c in cam[:4])
    R12 = np.asarray(R12, np.float32).reshape(3, 3)
    sR12 = np.array([[f32(float(s12) * float(R12[r, c])) for c in range(3)] for r in range(3)])
    sR21 = np.array([[f32((1.0 / float(s12)) * float(R12[c, r])) for c in range(3)]
                     for r in range(3)])
    t21 = np.array([-(f32(f32(sR21[r, 0] * f32(t12[0])) + f32(sR21[r, 1] * f32(t12[1])))
                      + f32(sR21[r, 2] * f32(t12[2]))) for r in range(3)], np.float32)

    def direction(A, B, sR, tt):
        cells, invW, invH = grid_cells(B["keys"], B["width"], B["height"])
        out = np.full(len(A["keys"]), -1, np.int32)
        for i, mp in enumerate(A["mps"]):
            if not A["valid"][i] or A["already"][i] or mp["bad"]:
                continue
            Pb = _xf(sR, tt, _xf(A["Rw"], A["tw"], mp["pos"]))
            if Pb[2] < 0:
                continue
            invz = f32(1.0 / float(Pb[2]))
            u = f32(f32(fx * f32(Pb[0] * invz)) + cx)
            v = f32(f32(fy * f32(Pb[1] * invz)) + cy)
            if not _in_kf(u, v, B["width"], B["height"]):
                continue
            dist = _norm(Pb)
            if dist < f32(f32(0.8) * mp["min_distance"]) or dist > f32(f32(1.2) * mp["max_distance"]):
                continue
            lvl = _level(mp["max_distance"], dist, log_scale, n_levels)
            bd, bi = _best(B["keys"], B["desc"], cells, invW, invH, A["mp_desc"][i], u, v,
                           f32(f32(th) * f32(B["scale"][lvl])), lvl - 1, lvl, init=1 << 31)
            if bd <= 100:
                out[i] = bi
        return out

    m1 = direction(kf1, kf2, sR21, t21)
    m2 = direction(kf2, kf1, sR12, np.asarray(t12, np.float32))
    m12 = np.array([j if j >= 0 and m2[j] == i else -1 for i, j in enumerate(m1)], np.int32)
    return int((m12 >= 0).sum()), m12


def search_by_bow_kf(d1, a1, mp1, bad1, fv1, d2, a2, mp2, bad2, fv2, nnratio, check_ori):
    m12 = np.full(len(d1), -1, np.int32)
    matched2 = np.zeros(len(d2), bool)
    hist = [[] for _ in range(30)]
    nodes2 = {int(fv2[0][k]): fv2[2][fv2[1][k]:fv2[1][k + 1]] for k in range(len(fv2[0]))}
    for k in range(len(fv1[0])):
        f2 = nodes2.get(int(fv1[0][k]))
        if f2 is None:
            continue
        for i1 in fv1[2][fv1[1][k]:fv1[1][k + 1]]:
            if mp1[i1] < 0 or bad1[i1]:
                continue
            b1, b2, bi = 256, 256, -1
            for i2 in f2:
                if matched2[i2] or mp2[i2] < 0 or bad2[i2]:
                    continue
                d = hamming(d1[i1], d2[i2])
                if d < b1:
                    b2, b1, bi = b1, d, i2
                elif d < b2:
                    b2 = d
            if b1 < 50 and f32(b1) < f32(f32(nnratio) * f32(b2)):
                m12[i1] = mp2[bi]
                matched2[bi] = True
                if check_ori:
                    hist[_rot_bin(a1[i1], a2[bi])].append(i1)
    if check_ori:
        keep = _three_maxima([len(h) for h in hist])
        for b in range(30):
            if b not in keep:
                for i1 in hist[b]:
                    m12[i1] = -1
    return int((m12 >= 0).sum()), m12


def search_by_projection_reloc(keys, desc, scale, width, height, R, t, ow, cam, mps, mp_desc,
                               kf_angle, th, orb_dist, check_ori, kp_locked, log_scale,
                               n_levels=8):
    fx, fy, cx, cy = (f32(c) for c in cam[:4])
    cells, invW, invH = grid_cells(keys, width, height)
    lock = np.asarray(kp_locked, bool).copy()
    km = np.full(len(keys), -1, np.int32)
    hist = [[] for _ in range(30)]
    for i, mp in enumerate(mps):
        if mp["bad"] or mp["seen"]:
            continue
        Pc = _xf(R, t, mp["pos"])
        invz = f32(1.0 / float(Pc[2]))
        u = f32(f32(f32(fx * Pc[0]) * invz) + cx)
        v = f32(f32(f32(fy * Pc[1]) * invz) + cy)
        if u < 0 or u > width or v < 0 or v > height:
            continue
        PO = [f32(f32(mp["pos"][k]) - f32(ow[k])) for k in range(3)]
        dist = _norm(PO)
        if dist < f32(f32(0.8) * mp["min_distance"]) or dist > f32(f32(1.2) * mp["max_distance"]):
            continue
        lvl = _level(mp["max_distance"], dist, log_scale, n_levels)
        bd, bi = _best(keys, desc, cells, invW, invH, mp_desc[i], u, v,
                       f32(f32(th) * f32(scale[lvl])), lvl - 1, lvl + 1, skip=lambda j: lock[j],
                       check_levels=True)
        if bd <= orb_dist:
            lock[bi] = True
            km[bi] = i
            if check_ori:
                hist[_rot_bin(kf_angle[i], keys[bi]["angle"])].append(bi)
    if check_ori:
        keep = _three_maxima([len(h) for h in hist])
        for b in range(30):
            if b not in keep:
                for j in hist[b]:
                    km[j] = -2
    return int((km >= 0).sum()), km


def search_for_triangulation(kf1, kf2, level_sigma2, F12, cam, Cw, R2w, t2w, fv1, fv2,
                             only_stereo, check_ori):
    fx, fy, cx, cy = (f32(c) for c in cam[:4])
    F = np.asarray(F12, np.float32).reshape(3, 3)
    C2 = _xf(R2w, t2w, Cw)
    invz = f32(f32(1) / C2[2])
    ex = f32(f32(f32(fx * C2[0]) * invz) + cx)
    ey = f32(f32(f32(fy * C2[1]) * invz) + cy)
    k1s, k2s = kf1["keys"], kf2["keys"]
    m12 = np.full(len(k1s), -1, np.int32)
    hist = [[] for _ in range(30)]
    nodes2 = {int(fv2[0][k]): fv2[2][fv2[1][k]:fv2[1][k + 1]] for k in range(len(fv2[0]))}
    for k in range(len(fv1[0])):
        f2 = nodes2.get(int(fv1[0][k]))
        if f2 is None:
            continue
        for i1 in fv1[2][fv1[1][k]:fv1[1][k + 1]]:
            if kf1["has_mp"][i1]:
                continue
            st1 = kf1["u_right"][i1] >= 0
            if only_stereo and not st1:
                continue
            kp1 = k1s[i1]
            a = f32(f32(f32(kp1["x"] * F[0, 0]) + f32(kp1["y"] * F[1, 0])) + F[2, 0])
            b = f32(f32(f32(kp1["x"] * F[0, 1]) + f32(kp1["y"] * F[1, 1])) + F[2, 1])
            c = f32(f32(f32(kp1["x"] * F[0, 2]) + f32(kp1["y"] * F[1, 2])) + F[2, 2])
            bd, bi = 50, -1
            for i2 in f2:
                if kf2["has_mp"][i2]:
                    continue
                st2 = kf2["u_right"][i2] >= 0
                if only_stereo and not st2:
                    continue
                d = hamming(kf1["desc"][i1], kf2["desc"][i2])
                if d > 50 or d > bd:
                    continue
                kp2 = k2s[i2]
                if not st1 and not st2:
                    dx, dy = f32(ex - kp2["x"]), f32(ey - kp2["y"])
                    if f32(f32(dx * dx) + f32(dy * dy)) < f32(100 * kf2["scale"][kp2["octave"]]):
                        continue
                num = f32(f32(f32(a * kp2["x"]) + f32(b * kp2["y"])) + c)
                den = f32(f32(a * a) + f32(b * b))
                if den == 0:
                    continue
                if float(f32(f32(num * num) / den)) < 3.84 * float(level_sigma2[kp2["octave"]]):
                    bd, bi = d, i2
            if bi >= 0:
                m12[i1] = bi
                if check_ori:
                    hist[_rot_bin(kp1["angle"], k2s[bi]["angle"])].append(i1)
    if check_ori:
        keep = _three_maxima([len(h) for h in hist])
        for bb in range(30):
            if bb not in keep:
                for i1 in hist[bb]:
                    m12[i1] = -1
    return int((m12 >= 0).sum()), m12


_POP8 = np.array([bin(i).count("1") for i in range(256)], np.int64)


def vocab_transform(voc, desc, levelsup, scoring, weighting):
    """DBoW2 TemplatedVocabulary::transform (TemplatedVocabulary.h:1128-1283),
    written from the text a second time: children lists rebuilt from the
    parent table in file order, descent by a first-index argmin (strict '<'),
    BowVector / FeatureVector as dicts sorted at the end."""
    parent = np.asarray(voc["parent"])
    n_nodes = len(parent)
    children = [[] for _ in range(n_nodes)]
    for i in range(1, n_nodes):
        children[int(parent[i])].append(i)
    words = {}
    for i in range(1, n_nodes):
        if voc["leaf"][i]:
            words[i] = len(words)
    nd = np.asarray(voc["desc"], np.uint8)
    L = int(voc["L"])
    nid_level = L - levelsup
    bow, fv = {}, {}
    fword, fnode = [], []
    tf = weighting in (0, 1)
    if not words:
        return [], [], [], [0], [], [], []
    for i, f in enumerate(np.asarray(desc, np.uint8).reshape(-1, 32)):
        node, level, nid = 0, 0, 0
        nid_set = nid_level <= 0
        while True:
            level += 1
            ch = children[node]
            d = _POP8[np.bitwise_xor(nd[ch], f)].sum(axis=1)
            node = ch[int(np.argmin(d))]  # first minimum
            if level == nid_level:
                nid, nid_set = node, True
            if not children[node]:
                break
        if not nid_set:
            nid = node
        w = float(voc["weight"][node])
        wid = words.get(node, 0)
        fword.append(wid if w > 0 else 0xFFFFFFFF)
        fnode.append(nid)
        if w > 0:
            if tf:
                bow[wid] = bow[wid] + w if wid in bow else w
            elif wid not in bow:
                bow[wid] = w
            fv.setdefault(nid, []).append(i)
    keys = sorted(bow)
    vals = [bow[k] for k in keys]
    must = scoring != 5
    if tf and vals and not must:
        vals = [v / float(len(vals)) for v in vals]
    if must:
        norm = 0.0
        if scoring == 1:
            for v in vals:
                norm += v * v
            norm = math.sqrt(norm)
        else:
            for v in vals:
                norm += abs(v)
        if norm > 0.0:
            vals = [v / norm for v in vals]
    nodes = sorted(fv)
    offs = [0]
    feats = []
    for k in nodes:
        feats.extend(fv[k])
        offs.append(len(feats))
    return keys, vals, nodes, offs, feats, fword, fnode


def undistort_points(xy, K, dist):
    """cvUndistortPoints (OpenCV, as Frame::UndistortKeyPoints calls it with
    P = mK, src/Frame.cc:468), restated a second time with Python floats
    (IEEE doubles, no fused multiply-add): widen, 5 fixed-point iterations,
    map through RR = K, narrow to float32."""
    K = [float(np.float32(v)) for v in np.asarray(K, np.float32).reshape(9)]
    k = [float(np.float32(v)) for v in np.asarray(dist, np.float32).reshape(-1)]
    k = k + [0.0] * (12 - len(k))
    fx, fy, cx, cy = K[0], K[4], K[2], K[5]
    ifx, ify = 1.0 / fx, 1.0 / fy
    out = np.zeros((len(xy), 2), np.float32)
    for i, (u, v) in enumerate(np.asarray(xy, np.float32).reshape(-1, 2)):
        x = (float(u) - cx) * ifx
        y = (float(v) - cy) * ify
        x0, y0 = x, y
        for _ in range(5):
            r2 = x * x + y * y
            icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / \
                (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2)
            dx = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2
            dy = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2
            x = (x0 - dx) * icdist
            y = (y0 - dy) * icdist
        xx = K[0] * x + K[1] * y + K[2]
        yy = K[3] * x + K[4] * y + K[5]
        ww = 1.0 / (K[6] * x + K[7] * y + K[8])
        out[i] = (np.float32(xx * ww), np.float32(yy * ww))
    return out
