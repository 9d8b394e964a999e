"""The C-ABI library: builds, loads without a GPU, exports exactly what
include/orb_abi.h declares, and refuses to compute without a gfx950 device."""
import ctypes
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG_DIR, ROOT

HEADER = ROOT / "include" / "orb_abi.h"


def declared_functions():
    text = re.sub(r"/\*.*?\*/", " ", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"\b(orb_[a-z0-9_]+)\s*\(", text)))


def exported(lib_path):
    out = subprocess.run(["nm", "-D", "--defined-only", str(lib_path)], check=True,
                         capture_output=True, text=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if " T " in ln}


def test_header_declares_the_drop_in_surface():
    fns = declared_functions()
    for must in ["orb_extractor_create", "orb_extractor_extract", "orb_extractor_extract_batch",
                 "orb_extractor_pyramid_level", "orb_descriptor_distance", "orb_hamming_batch",
                 "orb_match_projection_local", "orb_match_projection_local_batch",
                 "orb_stereo_match", "orb_match_projection_frame", "orb_match_bow"]:
        assert must in fns


def test_library_exports_every_declared_symbol(orb):
    orb.lib()
    missing = set(declared_functions()) - exported(orb.LIB_PATH)
    assert not missing, f"declared in orb_abi.h but not exported: {sorted(missing)}"


def test_library_has_gfx950_code_object(orb):
    blob = orb.LIB_PATH.read_bytes()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # offload bundle entry for gfx950
    for k in (b"k_fast_band", b"k_octree", b"k_orient_desc", b"k_proj_resolve", b"k_stereo_match"):
        assert k in blob


def test_abi_version_and_status_strings(orb):
    L = orb.lib()
    assert L.orb_abi_version() == 1
    assert L.orb_status_string(0) == b"ok"
    assert L.orb_status_string(-5) == b"no gfx950 device"


def test_host_descriptor_distance(orb):
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (200, 32), dtype=np.uint8)
    b = rng.integers(0, 256, (200, 32), dtype=np.uint8)
    for i in range(200):
        assert orb.ORBmatcher.DescriptorDistance(a[i], b[i]) == int(np.unpackbits(a[i] ^ b[i]).sum())


def test_no_cpu_fallback_without_gpu(orb):
    """Without a gfx950 device the product refuses to compute (fails loudly)."""
    if orb.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(orb.OrbError) as e:
        orb.ORBextractor(1000, 1.2, 8, 20, 7)
    assert e.value.status == orb.ORB_ENODEV
    with pytest.raises(orb.OrbError):
        orb.ORBmatcher(0.8)


def test_product_does_not_link_the_oracle(orb):
    out = subprocess.run(["ldd", str(orb.LIB_PATH)], capture_output=True, text=True).stdout
    assert "oracle" not in out
    syms = exported(orb.LIB_PATH)
    assert not any(s.startswith("oracle_") for s in syms)


def test_stereo_rejects_short_level_stride(orb):
    """orb_stereo_match validates every level's stride before staging (a stride
    shorter than the width would read rows past their end)."""
    import ctypes
    import numpy as np
    L = orb.lib()
    lvl = np.zeros((8, 8), np.uint8)
    ptrs = (ctypes.c_void_p * 1)(lvl.ctypes.data)
    w = np.array([64], np.int32)
    h = np.array([8], np.int32)
    st = np.array([8], np.int64)  # < width
    inv = np.ones(1, np.float32)
    keys = np.zeros(1, orb.KEYPOINT_DTYPE)
    desc = np.zeros((1, 32), np.uint8)
    f = orb.Frame(keys, desc, np.ones(1, np.float32), 64, 8)._c()
    s = orb._StereoInput()
    s.left = ctypes.addressof(f)
    s.n_right = 0
    s.n_levels = 1
    s.left_levels = s.right_levels = ctypes.addressof(ptrs)
    s.level_width, s.level_height, s.level_stride = (orb._ptr(w), orb._ptr(h), orb._ptr(st))
    s.inv_scale_factors = orb._ptr(inv)
    s.bf, s.fx = 40.0, 500.0
    ur = np.zeros(1, np.float32)
    dp = np.zeros(1, np.float32)
    # validation happens before any device work (no GPU needed)
    assert L.orb_stereo_match(ctypes.c_void_p(1), ctypes.byref(s), orb._ptr(ur), orb._ptr(dp)) == orb.ORB_EINVAL


def test_resolve_kernel_routing(orb):
    """The resolve kernel orb_matcher_resolve_kernel reports (its host routing,
    matcher_kernels.hip orb_k_proj_resolve_kernel) for the shapes the bench
    and the tests use; host logic only, no GPU."""
    L = orb.lib()
    f = L.orb_k_proj_resolve_kernel
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int] * 4
    AUTO, PREFIX, FP, JAC = 0, 1, 2, 3
    W1, W4, W8, FPK, JACK = 1, 4, 8, 16, 32
    cap = 1100  # keypoint slots of a 1241x376, 1000-feature frame (order of)
    assert f(1024, cap, 5000, AUTO) == W1      # the headline's batches
    assert f(256, cap, 5000, AUTO) == W1
    assert f(32, cap, 5000, AUTO) == W4        # 9-127 problems
    assert f(9, cap, 5000, AUTO) == W4
    assert f(8, cap, 5000, AUTO) == FPK        # calls of <= 8 problems: fixed point
    assert f(1, cap, 5000, AUTO) == FPK
    assert f(16, 4400, 50000, AUTO) == FPK     # C5: large maps
    assert f(16, 4400, 50000, PREFIX) == W8
    assert f(1024, cap, 5000, PREFIX) == W1
    assert f(4, cap, 5000, PREFIX) == W4
    assert f(1024, cap, 5000, FP) == FPK
    assert f(16, 4400, 50000, JAC) == JACK
    # claims that do not fit in LDS (12 B per keypoint slot): prefix windows
    assert f(1, 15000, 50000, AUTO) == W8
    assert f(1, 15000, 50000, JAC) == W8
    assert f(1, 15000, 5000, FP) == W4
    jb = L.orb_k_proj_jacobi_bytes
    jb.restype = ctypes.c_size_t
    jb.argtypes = [ctypes.c_int] * 4
    assert jb(cap, 5000, 1024, AUTO) == 0
    assert jb(4400, 50000, 16, JAC) > 0
