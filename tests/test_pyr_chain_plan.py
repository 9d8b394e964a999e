"""k_pyr_chain's band plan (`orb_pyr_chain_plan`, host code of the product
library, callable without a GPU): the one-launch resize chain of single-frame
calls reads, at level l - 1, only rows its band has computed there.  Checked
for the ORB-SLAM2 configurations and the parameter edge cases of
test_gpu_extractor: every row of every level is owned by exactly one band, a
band's computed rows contain its owned rows, and they cover every source row
(OpenCV INTER_LINEAR taps yofs and yofs + 1, clamped; src/ORBextractor.cc:1172-1207)
of the rows it computes one level up.  The kernel's pixels themselves are
checked bit-exact against the oracle on the GPU (test_gpu_extractor)."""
import ctypes

import numpy as np
import pytest

MAXL = 16
I = ctypes.c_int


class Level(ctypes.Structure):  # csrc/orb_plan.h OrbLevelDesc
    _fields_ = [("w", I), ("h", I), ("pitch", I), ("blurPitch", I), ("arenaOff", ctypes.c_longlong),
                ("blurOff", ctypes.c_longlong), ("cellBeg", I), ("cellEnd", I), ("quota", I),
                ("nodeCap", I), ("outOff", I), ("nIni", I), ("hX", ctypes.c_float), ("Wr", I),
                ("Hr", I), ("scale", ctypes.c_float), ("sizeF", ctypes.c_float), ("rtabX", I),
                ("rtabY", I), ("xmax", I), ("tileBeg", I), ("cellMaxRows", I), ("cellMaxCols", I)]


class Plan(ctypes.Structure):  # csrc/orb_plan.h OrbPlanDesc
    _fields_ = [(n, I) for n in ("nlevels", "ncells", "keyCap", "slotsPerImage", "iniTh", "minTh",
                                 "maxCellRows", "maxCellCols", "srcW", "srcH", "nBlurTiles",
                                 "nBands", "maxBandBytes")] + [("lv", Level * MAXL)]


class Band(ctypes.Structure):  # csrc/orb_plan.h OrbChainBand
    _fields_ = [("lo", ctypes.c_int16 * MAXL), ("hi", ctypes.c_int16 * MAXL),
                ("own", ctypes.c_int16 * MAXL), ("ownEnd", ctypes.c_int16 * MAXL)]


def yofs(h, sh):
    """runtime.cpp's row table: sy = floor((float)((dy + 0.5) * scale_y - 0.5))."""
    scale_y = 1.0 / (h / sh)
    fy = np.float32((np.arange(h, dtype=np.float64) + 0.5) * scale_y - 0.5)
    return np.floor(fy).astype(np.int32)


@pytest.mark.parametrize("w,h,sf,nl", [(1241, 376, 1.2, 8), (640, 480, 1.2, 8), (1920, 1080, 1.2, 8),
                                       (1920, 1080, 1.5, 6), (1241, 376, 1.2, 12), (1241, 376, 1.9, 4),
                                       (641, 479, 1.1, 8), (403, 301, 1.2, 8)])
def test_chain_bands_cover_their_reads(orb, oracle, w, h, sf, nl):
    lib = orb.lib()
    sizes = oracle.level_sizes(w, h, sf, nl)
    plan = Plan()
    plan.nlevels = nl
    rtab = []
    for l, (lw, lh) in enumerate(sizes):
        plan.lv[l].w, plan.lv[l].h = lw, lh
        if l:
            plan.lv[l].rtabY = len(rtab)
            rtab.extend(yofs(lh, sizes[l - 1][1]).tolist())
    rt = np.array(rtab or [0], np.int32)
    bands = (Band * 128)()
    buf = (ctypes.c_int * 2)()
    lds = 150 * 1024
    fn = lib.orb_pyr_chain_plan
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int,
                   ctypes.c_void_p]
    nb = fn(ctypes.byref(plan), rt.ctypes.data, lds, ctypes.byref(bands), 128, ctypes.byref(buf))
    assert nb >= 16, "no band count fits the LDS budget"
    assert buf[0] + buf[1] <= lds
    for l, (lw, lh) in enumerate(sizes):
        owned = np.zeros(lh, np.int32)
        for b in range(nb):
            B = bands[b]
            lo, hi, o0, o1 = B.lo[l], B.hi[l], B.own[l], B.ownEnd[l]
            owned[o0:o1] += 1
            assert 0 <= lo <= hi <= lh
            if o1 > o0:
                assert lo <= o0 and o1 <= hi, (l, b)
            assert (hi - lo) * ((lw + 3) & ~3) <= buf[l & 1], (l, b)
            if l and hi > lo:
                sh = sizes[l - 1][1]
                yo = rt[plan.lv[l].rtabY + lo: plan.lv[l].rtabY + hi]
                need = np.concatenate([np.clip(yo, 0, sh - 1), np.clip(yo + 1, 0, sh - 1)])
                assert need.min() >= B.lo[l - 1] and need.max() < B.hi[l - 1], (l, b)
        assert (owned == 1).all(), f"level {l}: rows owned {owned.min()}..{owned.max()} times"
