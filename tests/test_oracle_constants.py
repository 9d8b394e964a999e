"""Constants the reference embeds -- its only built-in known answers:
the rBRIEF sampling table, umax, per-level quotas, scale tables, Appendix B
level sizes, matcher thresholds.  Checked against the reference source text when
/root/reference is present (this container), and against the survey's derived
values always."""
import re

import numpy as np
import pytest

from conftest import PKG_DIR, REFERENCE

SRC = REFERENCE / "src" / "ORBextractor.cc"
needs_ref = pytest.mark.skipif(not SRC.exists(), reason="reference tree not mounted")


def _pattern_header():
    text = (PKG_DIR / "csrc" / "orb_pattern_data.h").read_text()
    body = text.split("{", 1)[1].split("}", 1)[0]
    return [int(v) for v in re.findall(r"-?\d+", body)]


@needs_ref
def test_pattern_table_is_the_reference_table():
    text = SRC.read_text(encoding="utf-8", errors="replace")
    body = text.split("bit_pattern_31_[256*4] =", 1)[1].split("};", 1)[0]
    body = re.sub(r"/\*.*?\*/", " ", body, flags=re.S)
    ref = [int(v) for v in re.findall(r"-?\d+", body)]
    assert len(ref) == 1024 and _pattern_header() == ref


def test_pattern_table_shape():
    p = np.array(_pattern_header()).reshape(512, 2)
    assert p.min() >= -13 and p.max() <= 12 and len(p) == 512
    assert np.sqrt((p.astype(float) ** 2).sum(1)).max() < 18.5  # samples stay within +-18 px


def test_umax(oracle):
    assert oracle.params()["umax"].tolist() == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
    # 749-pixel circular patch used by IC_Angle
    um = oracle.params()["umax"]
    assert 31 + 2 * sum(2 * int(um[v]) + 1 for v in range(1, 16)) == 749


@pytest.mark.parametrize("nf,quota", [
    (1000, [217, 181, 151, 126, 105, 87, 73, 60]),
    (2000, [434, 362, 302, 251, 209, 175, 145, 122]),
    (4000, [869, 724, 603, 503, 419, 349, 291, 242]),
])
def test_quotas(oracle, nf, quota):
    assert oracle.params(nf)["quota"].tolist() == quota


def test_scale_tables(oracle):
    p = oracle.params()
    sf = np.float64(np.float32(1.2))  # `double scaleFactor` member, include/ORBextractor.h:98
    s = [np.float32(1.0)]
    for _ in range(7):
        s.append(np.float32(np.float64(s[-1]) * sf))
    assert p["scale"].tolist() == [float(v) for v in s]
    assert p["inv_scale"].tolist() == [float(np.float32(1) / v) for v in s]
    assert p["sigma2"].tolist() == [float(v * v) for v in s]
    assert [int(31 * v) for v in p["scale"]] == [31, 37, 44, 53, 64, 77, 92, 111]


@pytest.mark.parametrize("w,h,sizes", [
    (640, 480, [(640, 480), (533, 400), (444, 333), (370, 278), (309, 231), (257, 193), (214, 161), (179, 134)]),
    (1241, 376, [(1241, 376), (1034, 313), (862, 261), (718, 218), (598, 181), (499, 151), (416, 126), (346, 105)]),
    (1920, 1080, [(1920, 1080), (1600, 900), (1333, 750), (1111, 625), (926, 521), (772, 434), (643, 362), (536, 301)]),
])
def test_level_sizes(oracle, w, h, sizes):
    assert oracle.level_sizes(w, h) == sizes


@needs_ref
def test_matcher_thresholds_in_reference():
    m = (REFERENCE / "src" / "ORBmatcher.cc").read_text(encoding="utf-8", errors="replace")
    assert "TH_HIGH = 100" in m and "TH_LOW = 50" in m and "HISTO_LENGTH = 30" in m
    f = (REFERENCE / "include" / "Frame.h").read_text(encoding="utf-8", errors="replace")
    assert re.search(r"FRAME_GRID_ROWS\s+48", f) and re.search(r"FRAME_GRID_COLS\s+64", f)
    e = SRC.read_text(encoding="utf-8", errors="replace")
    assert "EDGE_THRESHOLD = 19" in e and "HALF_PATCH_SIZE = 15" in e and "PATCH_SIZE = 31" in e
