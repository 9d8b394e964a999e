#!/usr/bin/env python3
"""What the A.6 / A.7 primitive pins change at the outputs.

The oracle (and the GPU, bit-exact to it) evaluates the descriptor's
cos/sin (src/ORBextractor.cc:125) and PredictScale's log (src/MapPoint.cc:443)
with pinned double-precision routines rounded once to float.  The reference
calls glibc cosf / sinf / logf.  This script runs both oracle builds
(liborb_oracle.so = pinned, liborb_oracle_glibc.so = glibc calls; oracle/Makefile)
over the committed golden inputs plus >= 1,000 synthetic frames and counts
what differs: keypoint records, descriptor rows / bytes / bits, local-map
match assignments (SearchByProjection), and isInFrustum scale levels.

CPU only, test infrastructure (loads the oracle).  Output: one JSON object,
committed as profiles/r02_parity_libm.json.
Usage: python tools/parity_libm.py [--frames 1000] [--threads 8]
"""
import argparse
import importlib.util
import json
import math
import os
import sys
import time
import multiprocessing as mp
from concurrent.futures import ProcessPoolExecutor
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tests"))


def load_oracle(variant):
    """A separate module instance of oracle/oracle.py bound to one build."""
    old = os.environ.get("ORB_ORACLE_VARIANT")
    os.environ["ORB_ORACLE_VARIANT"] = variant
    try:
        spec = importlib.util.spec_from_file_location(f"oracle_{variant}", ROOT / "oracle" / "oracle.py")
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        if old is None:
            os.environ.pop("ORB_ORACLE_VARIANT", None)
        else:
            os.environ["ORB_ORACLE_VARIANT"] = old
    mod.lib()
    return mod


PIN = GL = None


# 1) sin/cos: per-angle comparison of the two primitive builds on every
# angle fastAtan2 can produce from the frames' keypoints, and the end effect
# on the descriptors
def run(case):
    pin, gl = PIN, GL
    import scenarios
    seed, frame, w, h, nf = case
    img = pin.synth_image(seed, frame, w, h)
    kp, dp, _ = pin.extract(img, nf)
    kg, dg, _ = gl.extract(img, nf)
    res = {"kp_equal": kp.tobytes() == kg.tobytes(), "n": len(kp)}
    rows = np.any(dp != dg, axis=1)
    res["desc_rows_diff"] = int(rows.sum())
    res["desc_bytes_diff"] = int((dp != dg).sum())
    res["desc_bits_diff"] = int(np.unpackbits(dp ^ dg).sum())
    ang = kp["angle"].astype(np.float32) * np.float32(math.pi / 180.0)
    sc_diff = 0
    for a in ang:
        s1, c1 = pin.sincos(np.float32(a))
        s2, c2 = gl.sincos(np.float32(a))
        sc_diff += (s1 != s2) or (c1 != c2)
    res["sincos_diff"] = int(sc_diff)
    # 2) SearchByProjection against a local map derived from the pinned keys
    mps, mpd, lk = pin.synth_local_map(seed * 131 + frame, kp, dp, 3000, w, h)
    scale = np.float32(pin.params(nf)["scale"])
    n1, m1 = pin.match_projection_local(kp, dp, scale, w, h, mps, mpd, 1.0, 0.8, lk)
    n2, m2 = gl.match_projection_local(kg, dg, scale, w, h, mps, mpd, 1.0, 0.8, lk)
    res["matches"] = int(n1)
    res["match_count_diff"] = int(n1 != n2)
    res["match_assign_diff"] = int((m1 != m2).sum())
    # 3) isInFrustum + PredictScale on a 3-D local map
    pose, P, _ = scenarios.local_map_3d(pin, kp, dp, 3000, w, h, rng_seed=seed * 7 + frame)
    ls = np.float32(math.log(np.float32(1.2)))
    a_n, ta = pin.frustum(P, pose, scenarios.camera(), w, h, 0.5, ls, 8)
    b_n, tb = gl.frustum(P, pose, scenarios.camera(), w, h, 0.5, ls, 8)
    ok = ta["in_view"].astype(bool)
    res["mp_in_view"] = int(ok.sum())
    res["mp_level_diff"] = int((ta["level"][ok] != tb["level"][ok]).sum())
    return res



def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 4)
    ap.add_argument("--out", default=str(ROOT / "profiles" / "r02_parity_libm.json"))
    args = ap.parse_args()
    global PIN, GL
    PIN, GL = load_oracle("pinned"), load_oracle("glibc")
    pin = PIN

    # inputs: the golden fixtures' images (tests/golden/golden.json) + synthetic frames
    golden = json.loads((ROOT / "tests" / "golden" / "golden.json").read_text())
    cases = [(c["seed"], 0, c["w"], c["h"], c["nf"]) for c in golden["extract"]]
    for f in range(args.frames):
        w, h = (1241, 376) if f % 5 < 3 else (640, 480)
        cases.append((1000 + f // 50, f % 50, w, h, 1000 if f % 7 else 2000))

    t0 = time.time()
    # processes, not threads: the oracle wrappers set ctypes signatures per call
    with ProcessPoolExecutor(args.threads, mp_context=mp.get_context("fork")) as ex:
        rs = list(ex.map(run, cases, chunksize=4))
    # 4) the primitives alone against glibc's float entry points (ctypes into
    # libm): logf over float ratios, sinf/cosf over descriptor angles
    import ctypes
    libm = ctypes.CDLL("libm.so.6")
    for fn in ("logf", "sinf", "cosf"):
        getattr(libm, fn).restype = ctypes.c_float
        getattr(libm, fn).argtypes = [ctypes.c_float]
    rng = np.random.default_rng(0)
    ratios = np.concatenate([rng.uniform(0.05, 20.0, 200000).astype(np.float32),
                             np.float32(1.2) ** np.arange(-40, 41, dtype=np.float32)])
    log_diff = sum(np.float32(pin.pinned_log(float(r))) != np.float32(libm.logf(float(r)))
                   for r in ratios)
    angles = (rng.uniform(0.0, 360.0, 200000).astype(np.float32) *
              np.float32(math.pi / 180.0)).astype(np.float32)
    sc_sweep = 0
    for a in angles:
        s1, c1 = pin.sincos(float(a))
        sc_sweep += (np.float32(s1) != np.float32(libm.sinf(float(a)))) or \
            (np.float32(c1) != np.float32(libm.cosf(float(a))))
    tot = lambda k: int(sum(r[k] for r in rs))
    out = {
        "what": "pinned (A.6 double sincos, A.7 double log, rounded to float; = GPU) vs "
                "glibc cosf/sinf/logf (the reference's calls), same oracle otherwise",
        "frames": len(rs), "golden_cases": len(golden["extract"]),
        "keypoints": tot("n"),
        "frames_with_keypoint_diff": int(sum(not r["kp_equal"] for r in rs)),
        "keypoint_angles_with_sincos_diff": tot("sincos_diff"),
        "descriptor_rows_diff": tot("desc_rows_diff"),
        "descriptor_bytes_diff": tot("desc_bytes_diff"),
        "descriptor_bits_diff": tot("desc_bits_diff"),
        "descriptor_rows_diff_frac": tot("desc_rows_diff") / max(tot("n"), 1),
        "frames_with_descriptor_diff": int(sum(r["desc_rows_diff"] > 0 for r in rs)),
        "local_map_matches": tot("matches"),
        "frames_with_match_count_diff": tot("match_count_diff"),
        "match_assignments_diff": tot("match_assign_diff"),
        "map_points_in_view": tot("mp_in_view"),
        "map_point_levels_diff": tot("mp_level_diff"),
        "logf_sweep_ratios": int(len(ratios)),
        "logf_sweep_diff_pinned_vs_glibc": int(log_diff),
        "sincosf_sweep_angles": int(len(angles)),
        "sincosf_sweep_diff_pinned_vs_glibc": int(sc_sweep),
        "seconds": time.time() - t0,
        "libc": os.confstr("CS_GNU_LIBC_VERSION") if hasattr(os, "confstr") else None,
    }
    txt = json.dumps(out, indent=1)
    print(txt)
    Path(args.out).write_text(txt + "\n")


if __name__ == "__main__":
    main()
