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
