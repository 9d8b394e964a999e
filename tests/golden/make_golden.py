"""Generate tests/golden/ fixtures from the CPU oracle (dev tool, run here).

The reference ships no golden vectors or tests and cannot be
built offline (§8(c)), so these fixtures are produced by oracle/orb_oracle.cpp
and freeze its behaviour: they pin regressions of the oracle and let the GPU
tests check against stored answers, not a live CPU run.  They are NOT
reference-binary outputs (parity vs a reference binary stays unpinned).

    python tests/golden/make_golden.py
"""
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
sys.path.insert(0, str(HERE.parents[1] / "oracle"))
import oracle  # noqa: E402
import scenarios  # noqa: E402

EXTRACT = [(640, 480, 1000, 1), (640, 480, 1000, 2), (640, 480, 1000, 3), (1241, 376, 1000, 0),
           (1241, 376, 2000, 7), (1920, 1080, 4000, 5)]
FULL = {(640, 480, 1000, 1), (1241, 376, 1000, 0)}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    out = {"extract": [], "match": {}}
    for (w, h, nf, seed) in EXTRACT:
        img = oracle.synth_image(seed, 0, w, h)
        k, d, per = oracle.extract(img, nf)
        pyr = oracle.pyramid(img)
        out["extract"].append(dict(w=w, h=h, nf=nf, seed=seed, image=sha(img),
                                   pyramid=[sha(l) for l in pyr], per_level=per.tolist(),
                                   n=int(len(k)), keypoints=sha(k), descriptors=sha(d)))
        if (w, h, nf, seed) in FULL:
            np.savez_compressed(HERE / f"extract_{w}x{h}_n{nf}_s{seed}.npz",
                                keypoints=k.view(np.uint8).reshape(len(k), 28), descriptors=d)
    # local map matching (C4 shape)
    img = oracle.synth_image(0, 0, 1241, 376)
    k, d, _ = oracle.extract(img, 1000)
    mps, mpd, lk = oracle.synth_local_map(0, k, d, 5000, 1241, 376)
    sc = oracle.params(1000)["scale"]
    n, km = oracle.match_projection_local(k, d, sc, 1241, 376, mps, mpd, 1.0, 0.8, lk)
    out["match"]["local_1241x376_s0_m5000"] = dict(nmatches=int(n), kp_match=sha(km))
    sp = scenarios.stereo_pair(oracle, 1)
    ur, dp = oracle.stereo_match(sp["kl"], sp["dl"], sp["scale"], sp["kr"], sp["dr"], sp["lpyr"],
                                 sp["rpyr"], sp["inv"], scenarios.BF, scenarios.FX, sp["w"], sp["h"])
    out["match"]["stereo_1241x376_s1_n2000"] = dict(u_right=sha(ur), depth=sha(dp),
                                                    valid=int((ur > 0).sum()))
    fp = scenarios.frame_pair(oracle, 2, rng_seed=15)
    n, km = oracle.match_projection_frame(fp["kb"], fp["db"], fp["scale"], fp["w"], fp["h"],
                                          fp["last"], fp["last_desc"], scenarios.camera(), 0.0,
                                          15.0, 1, 1)
    out["match"]["frame_mono_s2_th15"] = dict(nmatches=int(n), kp_match=sha(km))
    bp = scenarios.bow_pair(oracle, 4)
    n, fm = oracle.match_bow(bp["kf_desc"], bp["kf_angle"], bp["kf_mp"], bp["kf_bad"], bp["kf_fv"],
                             bp["f_desc"], bp["f_angle"], bp["f_fv"], 0.75, 1)
    out["match"]["bow_s4_r075"] = dict(nmatches=int(n), f_match=sha(fm))
    (HERE / "golden.json").write_text(json.dumps(out, indent=1) + "\n")
    print("wrote", HERE / "golden.json")


if __name__ == "__main__":
    main()
