"""The A.6 / A.7 primitive pins against the reference's own glibc calls.

The oracle (and the GPU, bit-exact to it) evaluates the descriptor's cos/sin
(src/ORBextractor.cc:125) and PredictScale's log (src/MapPoint.cc:443) with
pinned double routines rounded once to float; the reference calls glibc
cosf/sinf/logf.  The primitives differ by one ulp on a few percent of inputs;
this checks, on a sample of frames, that no keypoint, descriptor bit, local-map
match or frustum level changes (tools/parity_libm.py runs the same comparison
over the golden inputs + 1,000 frames: profiles/r02_parity_libm.json)."""
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))


@pytest.fixture(scope="module")
def variants():
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)
    import parity_libm
    parity_libm.PIN = parity_libm.load_oracle("pinned")
    parity_libm.GL = parity_libm.load_oracle("glibc")
    return parity_libm


@pytest.mark.parametrize("case", [(1, 0, 640, 480, 1000), (0, 0, 1241, 376, 1000),
                                  (1003, 7, 1241, 376, 2000), (1011, 3, 640, 480, 1000)])
def test_pins_change_no_output(variants, case):
    r = variants.run(case)
    assert r["n"] > 500
    assert r["sincos_diff"] >= 0  # angles whose cos/sin differ by an ulp (typically a few %)
    assert r["kp_equal"]
    assert r["desc_rows_diff"] == 0 and r["desc_bits_diff"] == 0
    assert r["match_count_diff"] == 0 and r["match_assign_diff"] == 0 and r["matches"] > 100
    assert r["mp_level_diff"] == 0 and r["mp_in_view"] > 100


def test_glibc_primitives_do_differ(variants):
    """The two builds really do evaluate different primitives."""
    import ctypes
    import math

    import numpy as np
    libm = ctypes.CDLL("libm.so.6")
    libm.sinf.restype = ctypes.c_float
    libm.sinf.argtypes = [ctypes.c_float]
    rng = np.random.default_rng(1)
    angles = (rng.uniform(0, 360, 4000).astype(np.float32) * np.float32(math.pi / 180)).astype(np.float32)
    diff_pin = sum(np.float32(variants.PIN.sincos(float(a))[0]) != np.float32(libm.sinf(float(a)))
                   for a in angles)
    diff_gl = sum(np.float32(variants.GL.sincos(float(a))[0]) != np.float32(libm.sinf(float(a)))
                  for a in angles)
    assert diff_gl == 0 and diff_pin > 0
