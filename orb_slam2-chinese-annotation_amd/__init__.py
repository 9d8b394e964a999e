"""MI355X-native ORB front-end: Python host mirror of the reference interface.

Mirrors, over the C ABI in ``include/orb_abi.h`` (library ``lib/liborb_amd.so``):

* ``ORBextractor``  -- ORB_SLAM2::ORBextractor (reference include/ORBextractor.h:45-114):
  same constructor arguments, ``__call__(image, mask)`` = ``operator()``
  (src/ORBextractor.cc:1091-1169), the ``Get*`` scale accessors and
  ``mvImagePyramid``.
* ``ORBmatcher``    -- ORB_SLAM2::ORBmatcher (include/ORBmatcher.h:37-102):
  ``DescriptorDistance`` and ``SearchByProjection(Frame, local map, th)``
  (src/ORBmatcher.cc:47-133).

Every result is computed by the gfx950 HIP kernels; there is no CPU path.  If
the library is missing or no gfx950 device is visible the calls raise.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
# ORB_AMD_LIB selects another build of the same library (A/B kernel experiments)
LIB_PATH = Path(os.environ.get("ORB_AMD_LIB", PKG_DIR / "lib" / "liborb_amd.so"))

ORB_OK, ORB_EEMPTY, ORB_EINVAL, ORB_ENOMEM, ORB_EDEVICE, ORB_ECAPACITY, ORB_ENODEV = 0, 1, -1, -2, -3, -4, -5

KEYPOINT_DTYPE = np.dtype(
    [("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
     ("octave", "<i4"), ("class_id", "<i4")]
)
MP_TRACK_DTYPE = np.dtype(
    [("proj_x", "<f4"), ("proj_y", "<f4"), ("proj_xr", "<f4"), ("view_cos", "<f4"),
     ("level", "<i4"), ("in_view", "u1"), ("bad", "u1"), ("has_obs", "u1"), ("_pad", "u1")]
)
LAST_MP_DTYPE = np.dtype([("xc", "<f4"), ("yc", "<f4"), ("invzc", "<f4"), ("last_octave", "<i4"),
                          ("last_angle", "<f4"), ("valid", "u1"), ("has_obs", "u1"),
                          ("_pad", "u1", 2), ("mp_id", "<i4")])
assert KEYPOINT_DTYPE.itemsize == 28 and MP_TRACK_DTYPE.itemsize == 24
assert LAST_MP_DTYPE.itemsize == 28


MAP_POINT_DTYPE = np.dtype([("pos", "<f4", (3,)), ("normal", "<f4", (3,)), ("min_distance", "<f4"),
                            ("max_distance", "<f4"), ("bad", "u1"), ("seen", "u1"),
                            ("has_obs", "u1"), ("_pad", "u1")])
POSE_DTYPE = np.dtype([("rcw", "<f4", (9,)), ("tcw", "<f4", (3,)), ("ow", "<f4", (3,))])


class OrbError(RuntimeError):
    def __init__(self, status: int, what: str):
        self.status = status
        super().__init__(f"{what}: {_status_str(status)} ({status})")


_lib = None


def _status_str(s: int) -> str:
    if _lib is None:
        return str(s)
    return _lib.orb_status_string(s).decode()


class _Frame(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int32), ("keys", ctypes.c_void_p), ("descriptors", ctypes.c_void_p),
        ("u_right", ctypes.c_void_p), ("min_x", ctypes.c_float), ("max_x", ctypes.c_float),
        ("min_y", ctypes.c_float), ("max_y", ctypes.c_float), ("n_levels", ctypes.c_int32),
        ("scale_factors", ctypes.c_void_p),
    ]


def lib() -> ctypes.CDLL:
    """Load liborb_amd.so (fails loudly if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise OrbError(ORB_ENODEV, f"{LIB_PATH} not built (run __graft_entry__.build())")
    # One HIP runtime per process: torch-ROCm ships its own libamdhip64 (soname
    # libamdhip64.so.7).  Loading torch first lets liborb_amd.so's DT_NEEDED on
    # libamdhip64.so.7 bind to that same copy, so device pointers and streams
    # can be shared with torch (plumbing for device memory / torch.distributed).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(str(LIB_PATH))
    vp, i32, f32, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
    sig = {
        "orb_abi_version": (i32, []),
        "orb_status_string": (ctypes.c_char_p, [i32]),
        "orb_device_count": (i32, [vp]),
        "orb_extractor_create": (i32, [i32, f32, i32, i32, i32, i32, vp]),
        "orb_extractor_destroy": (None, [vp]),
        "orb_extractor_get_levels": (i32, [vp]),
        "orb_extractor_get_scale_factor": (f32, [vp]),
        "orb_extractor_get_scale_factors": (None, [vp, vp]),
        "orb_extractor_get_inverse_scale_factors": (None, [vp, vp]),
        "orb_extractor_get_scale_sigma_squares": (None, [vp, vp]),
        "orb_extractor_get_inverse_scale_sigma_squares": (None, [vp, vp]),
        "orb_extractor_get_features_per_level": (None, [vp, vp]),
        "orb_extractor_capacity": (i32, [vp, i32, i32]),
        "orb_extractor_extract": (i32, [vp, vp, i32, i32, sz, vp, vp, i32, vp]),
        "orb_extractor_pyramid_level": (i32, [vp, i32, vp, sz, vp, vp]),
        "orb_extractor_blurred_level": (i32, [vp, i32, vp, sz, vp, vp]),
        "orb_extractor_host_pyramid": (i32, [vp, i32, vp, vp, vp, vp]),
        "orb_extractor_host_pyramid_off": (i32, [vp]),
        "orb_extractor_extract_batch": (i32, [vp, vp, i32, i32, i32, sz, sz, vp, vp, i32, vp, vp]),
        "orb_extractor_batch_level": (i32, [vp, i32, i32, vp, vp, vp, vp]),
        "orb_match_projection_local_stage": (i32, [vp, i32, i32, vp]),
        "orb_match_projection_local_begin": (i32, [vp, vp, i32, i32]),
        "orb_match_projection_local_staged": (i32, [vp, vp, i32, i32, i32, f32, f32, vp, vp]),
        "orb_extractor_stream": (vp, [vp]),
        "orb_extractor_profile": (i32, [vp, i32]),
        "orb_extractor_profile_read": (i32, [vp, i32, vp, vp, vp]),
        "orb_descriptor_distance": (i32, [vp, vp]),
        "orb_matcher_create": (i32, [i32, vp]),
        "orb_matcher_destroy": (None, [vp]),
        "orb_matcher_stream": (vp, [vp]),
        "orb_matcher_profile": (i32, [vp, i32]),
        "orb_matcher_set_resolve": (i32, [vp, i32, i32]),
        "orb_matcher_resolve_kernel": (i32, [vp, i32, i32, i32, vp]),
        "orb_matcher_profile_read": (i32, [vp, i32, vp, vp, vp]),
        "orb_hamming_batch": (i32, [vp, vp, vp, i32, vp, vp]),
        "orb_match_projection_local": (i32, [vp, vp, vp, i32, vp, vp, f32, f32, vp, vp]),
        "orb_match_projection_local_batch": (
            i32, [vp, i32, vp, vp, vp, vp, i32, vp, vp, vp, i32, f32, f32, f32, f32, i32, vp,
                  f32, f32, vp, vp, vp]),
        "orb_stereo_match": (i32, [vp, vp, vp, vp]),
        "orb_stereo_match_extracted": (i32, [vp, vp, vp, f32, f32, vp, vp, i32, vp]),
        "orb_stereo_match_batch": (i32, [vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, i32, f32, f32,
                                         vp, vp, vp, vp]),
        "orb_match_projection_frame": (i32, [vp, vp, vp, i32, vp, vp, vp, f32, f32, i32, i32, vp,
                                             vp]),
        "orb_match_bow": (i32, [vp, i32, vp, vp, vp, vp, i32, vp, vp, vp, i32, vp, vp, i32, vp,
                                vp, vp, f32, i32, vp, vp]),
        "orb_frustum": (i32, [vp, i32, vp, vp, vp, f32, f32, f32, f32, f32, f32, i32, vp, vp]),
        "orb_frustum_batch": (i32, [vp, i32, vp, vp, i32, vp, vp, f32, f32, f32, f32, f32, f32,
                                    i32, vp, vp, vp]),
        "orb_search_for_initialization": (i32, [vp, vp, vp, vp, i32, f32, i32, vp, vp]),
        "orb_search_for_initialization_batch": (
            i32, [vp, i32, vp, vp, vp, vp, vp, vp, i32, f32, f32, f32, f32, i32, f32, i32, vp, vp,
                  vp, vp]),
        "orb_distinctive_descriptors": (i32, [vp, i32, vp, vp, vp, vp]),
        "orb_distinctive_descriptors_batch": (i32, [vp, i32, vp, vp, vp, vp, vp]),
        "orb_search_by_projection_reloc": (i32, [vp, vp, vp, vp, vp, f32, i32, vp, vp, vp, f32,
                                                 i32, i32, vp, vp]),
        "orb_search_by_projection_sim3": (i32, [vp, vp, vp, vp, f32, i32, vp, vp, f32, vp, vp]),
        "orb_fuse": (i32, [vp, vp, vp, vp, vp, f32, i32, vp, vp, f32, vp, vp]),
        "orb_fuse_sim3": (i32, [vp, vp, vp, vp, f32, i32, vp, vp, f32, vp, vp]),
        "orb_search_by_sim3": (i32, [vp, vp, vp, f32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                     vp, vp, f32, vp, vp, f32, vp, vp]),
        "orb_match_bow_kf": (i32, [vp, i32, vp, vp, vp, vp, i32, vp, vp, vp, i32, vp, vp, vp, vp,
                                   i32, vp, vp, vp, f32, i32, vp, vp]),
        "orb_search_for_triangulation": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32,
                                               vp, vp, vp, i32, vp, vp, vp, i32, i32, vp, vp]),
        "orb_vocabulary_create": (i32, [i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp]),
        "orb_vocabulary_load_text": (i32, [i32, ctypes.c_char_p, vp]),
        "orb_vocabulary_destroy": (None, [vp]),
        "orb_vocabulary_info": (i32, [vp, vp]),
        "orb_vocabulary_stream": (vp, [vp]),
        "orb_vocabulary_transform": (i32, [vp, i32, vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        "orb_vocabulary_transform_batch": (i32, [vp, i32, vp, vp, i32, i32, vp, vp, vp, vp, vp,
                                                 vp, vp, vp, vp, vp, vp]),
        "orb_undistort_points": (i32, [vp, i32, vp, vp, vp, i32, vp]),
        "orb_undistort_keypoints": (i32, [vp, i32, vp, vp, vp, i32, vp]),
        "orb_compute_image_bounds": (i32, [vp, i32, i32, vp, vp, i32, vp]),
        "orb_undistort_keypoints_batch": (i32, [vp, i32, vp, vp, i32, vp, vp, i32, vp, vp]),
        "orb_synth_image": (None, [ctypes.c_uint64, i32, i32, i32, i32, vp, sz]),
        "orb_synth_local_map": (None, [ctypes.c_uint64, vp, vp, i32, i32, i32, i32, vp, vp, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


_HIP_RT = None


def _hip_runtime() -> ctypes.CDLL:
    """The HIP runtime this process already uses: liborb_amd.so's dependency,
    looked up by its SONAME, so the loaded copy (torch's, when torch came
    first) is returned rather than a second runtime."""
    global _HIP_RT
    if _HIP_RT is None:
        lib()
        _HIP_RT = ctypes.CDLL("libamdhip64.so.7")
    return _HIP_RT


def _check(status: int, what: str) -> int:
    if status not in (ORB_OK,):
        raise OrbError(status, what)
    return status


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def device_count() -> int:
    n = ctypes.c_int(0)
    lib().orb_device_count(ctypes.byref(n))
    return n.value


# --------------------------------------------------------------- synthetic input
def synth_image(seed: int, frame: int, width: int, height: int, view: int = 0) -> np.ndarray:
    """Deterministic synthetic grayscale frame (orb_synth_image)."""
    img = np.empty((height, width), np.uint8)
    lib().orb_synth_image(seed, frame, view, width, height, _ptr(img), width)
    return img


def synth_local_map(seed: int, keys: np.ndarray, desc: np.ndarray, n_mp: int, width: int,
                    height: int):
    """SURVEY §8(d) C5 synthetic local map: (mps, mp_desc, kp_locked)."""
    keys = np.ascontiguousarray(keys, KEYPOINT_DTYPE)
    desc = np.ascontiguousarray(desc, np.uint8)
    mps = np.zeros(n_mp, MP_TRACK_DTYPE)
    mp_desc = np.zeros((n_mp, 32), np.uint8)
    locked = np.zeros(len(keys), np.uint8)
    lib().orb_synth_local_map(seed, _ptr(keys), _ptr(desc), len(keys), n_mp, width, height,
                              _ptr(mps), _ptr(mp_desc), _ptr(locked))
    return mps, mp_desc, locked


# ------------------------------------------------------------------- extractor
class ORBextractor:
    """ORB_SLAM2::ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)."""

    def __init__(self, nfeatures: int, scaleFactor: float, nlevels: int, iniThFAST: int,
                 minThFAST: int, device: int = 0):
        L = lib()
        h = ctypes.c_void_p()
        _check(L.orb_extractor_create(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST,
                                      device, ctypes.byref(h)), "orb_extractor_create")
        self._h = h
        self.nlevels = nlevels
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            lib().orb_extractor_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def _floats(self, fn) -> list:
        out = np.zeros(self.nlevels, np.float32)
        fn(self._h, _ptr(out))
        return out.tolist()

    def GetLevels(self) -> int:
        return lib().orb_extractor_get_levels(self._h)

    def GetScaleFactor(self) -> float:
        return lib().orb_extractor_get_scale_factor(self._h)

    def GetScaleFactors(self) -> list:
        return self._floats(lib().orb_extractor_get_scale_factors)

    def GetInverseScaleFactors(self) -> list:
        return self._floats(lib().orb_extractor_get_inverse_scale_factors)

    def GetScaleSigmaSquares(self) -> list:
        return self._floats(lib().orb_extractor_get_scale_sigma_squares)

    def GetInverseScaleSigmaSquares(self) -> list:
        return self._floats(lib().orb_extractor_get_inverse_scale_sigma_squares)

    def features_per_level(self) -> list:
        out = np.zeros(self.nlevels, np.int32)
        lib().orb_extractor_get_features_per_level(self._h, _ptr(out))
        return out.tolist()

    def capacity(self, width: int, height: int) -> int:
        return lib().orb_extractor_capacity(self._h, width, height)

    def __call__(self, image: np.ndarray, mask=None):
        """operator(): returns (keypoints[KEYPOINT_DTYPE], descriptors uint8 N x 32).

        An empty image returns (None, None) -- the reference returns with its
        outputs untouched (src/ORBextractor.cc:1095-1096).  A non-uint8 or
        non-2D image is rejected like the reference's assert (:1100)."""
        if image is None or image.size == 0:
            return None, None
        if image.dtype != np.uint8 or image.ndim != 2:
            raise OrbError(ORB_EINVAL, "image must be 8UC1 (CV_8UC1)")
        image = np.ascontiguousarray(image)
        H, W = image.shape
        cap = self.capacity(W, H)
        if cap < 0:
            raise OrbError(ORB_EINVAL, f"unsupported image size {W}x{H}")
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = ctypes.c_int(0)
        _check(lib().orb_extractor_extract(self._h, _ptr(image), W, H, image.strides[0], _ptr(kps),
                                           _ptr(desc), cap, ctypes.byref(n)),
               "orb_extractor_extract")
        return kps[: n.value].copy(), desc[: n.value].copy()

    def host_pyramid(self, level: int) -> np.ndarray:
        """Level `level` of the last __call__ through the library's pinned host
        mirror (orb_extractor_host_pyramid), copied into a new array."""
        p, w, h, st = ctypes.c_void_p(), ctypes.c_int(0), ctypes.c_int(0), ctypes.c_size_t(0)
        _check(lib().orb_extractor_host_pyramid(self._h, level, ctypes.byref(p), ctypes.byref(w),
                                                ctypes.byref(h), ctypes.byref(st)), "host_pyramid")
        buf = (ctypes.c_uint8 * (st.value * (h.value - 1) + w.value)).from_address(p.value)
        a = np.frombuffer(buf, np.uint8)
        return np.lib.stride_tricks.as_strided(a, (h.value, w.value), (st.value, 1)).copy()

    def host_pyramid_off(self):
        """Stop the per-call host mirror of levels 1.. (orb_extractor_host_pyramid_off)."""
        _check(lib().orb_extractor_host_pyramid_off(self._h), "host_pyramid_off")

    @property
    def mvImagePyramid(self) -> list:
        """Host copies of the last image's pyramid levels."""
        L = lib()
        out = []
        for l in range(self.nlevels):
            w, h = ctypes.c_int(0), ctypes.c_int(0)
            _check(L.orb_extractor_pyramid_level(self._h, l, None, 0, ctypes.byref(w),
                                                 ctypes.byref(h)), "pyramid_level")
            a = np.zeros((h.value, w.value), np.uint8)
            _check(L.orb_extractor_pyramid_level(self._h, l, _ptr(a), w.value, None, None),
                   "pyramid_level")
            out.append(a)
        return out

    def blurred_levels(self) -> list:
        """Host copies of the last image's 7x7-blurred levels (what rBRIEF samples)."""
        L = lib()
        out = []
        for l in range(self.nlevels):
            w, h = ctypes.c_int(0), ctypes.c_int(0)
            _check(L.orb_extractor_blurred_level(self._h, l, None, 0, ctypes.byref(w),
                                                 ctypes.byref(h)), "blurred_level")
            a = np.zeros((h.value, w.value), np.uint8)
            _check(L.orb_extractor_blurred_level(self._h, l, _ptr(a), w.value, None, None),
                   "blurred_level")
            out.append(a)
        return out

    def extract_batch(self, d_images: int, n_images: int, width: int, height: int, stride: int,
                      image_pitch: int, d_keypoints: int, d_descriptors: int, capacity: int,
                      d_counts: int, stream: int = 0):
        """Device-resident batch form (raw device pointers, e.g. torch .data_ptr())."""
        _check(lib().orb_extractor_extract_batch(self._h, d_images, n_images, width, height,
                                                 stride, image_pitch, d_keypoints, d_descriptors,
                                                 capacity, d_counts, stream or None),
               "orb_extractor_extract_batch")

    def stream(self) -> int:
        return lib().orb_extractor_stream(self._h) or 0

    def batch_level(self, image: int, level: int) -> np.ndarray:
        """Host copy of pyramid level `level` of batch image `image` after
        extract_batch (orb_extractor_batch_level's device view, copied with the
        process's HIP runtime; call after the batch's stream is synchronised)."""
        p, w, h, st = ctypes.c_void_p(), ctypes.c_int(), ctypes.c_int(), ctypes.c_size_t()
        _check(lib().orb_extractor_batch_level(self._h, image, level, ctypes.byref(p), ctypes.byref(w),
                                               ctypes.byref(h), ctypes.byref(st)),
               "orb_extractor_batch_level")
        out = np.zeros((h.value, w.value), np.uint8)
        hip = _hip_runtime()
        rc = hip.hipMemcpy2D(ctypes.c_void_p(out.ctypes.data), ctypes.c_size_t(w.value), p, st,
                             ctypes.c_size_t(w.value), ctypes.c_size_t(h.value), ctypes.c_int(2))
        if rc != 0:
            raise OrbError(ORB_EDEVICE, f"hipMemcpy2D -> {rc}")
        return out

    def profile(self, enable: bool = True):
        _check(lib().orb_extractor_profile(self._h, int(enable)), "profile")

    def profile_read(self, stage: int):
        ms = ctypes.c_double(0)
        n = ctypes.c_int(0)
        name = ctypes.c_char_p()
        _check(lib().orb_extractor_profile_read(self._h, stage, ctypes.byref(ms), ctypes.byref(n),
                                                ctypes.byref(name)), "profile_read")
        return name.value.decode(), ms.value, n.value


# --------------------------------------------------------------------- matcher
class Frame:
    """The Frame members ORBmatcher reads (src/Frame.cc, include/Frame.h)."""

    def __init__(self, keys, descriptors, scale_factors, width, height, u_right=None,
                 min_x=0.0, min_y=0.0):
        self.mvKeysUn = np.ascontiguousarray(keys, KEYPOINT_DTYPE)
        self.mDescriptors = np.ascontiguousarray(descriptors, np.uint8).reshape(-1, 32)
        self.mvScaleFactors = np.ascontiguousarray(scale_factors, np.float32)
        self.mvuRight = None if u_right is None else np.ascontiguousarray(u_right, np.float32)
        self.mnMinX, self.mnMaxX = float(min_x), float(width)
        self.mnMinY, self.mnMaxY = float(min_y), float(height)
        self.N = len(self.mvKeysUn)

    def _c(self) -> _Frame:
        f = _Frame()
        f.n = self.N
        f.keys = _ptr(self.mvKeysUn) if self.N else None
        f.descriptors = _ptr(self.mDescriptors) if self.N else None
        f.u_right = _ptr(self.mvuRight) if self.mvuRight is not None else None
        f.min_x, f.max_x, f.min_y, f.max_y = self.mnMinX, self.mnMaxX, self.mnMinY, self.mnMaxY
        f.n_levels = len(self.mvScaleFactors)
        f.scale_factors = _ptr(self.mvScaleFactors)
        return f


class _LocalStage(ctypes.Structure):  # orb_local_stage_t
    _fields_ = [("keys", ctypes.c_void_p), ("descriptors", ctypes.c_void_p),
                ("u_right", ctypes.c_void_p), ("kp_locked", ctypes.c_void_p),
                ("mps", ctypes.c_void_p), ("mp_desc", ctypes.c_void_p)]


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


class ORBmatcher:
    """ORB_SLAM2::ORBmatcher(nnratio=0.6, checkOri=true)."""

    TH_HIGH, TH_LOW, HISTO_LENGTH = 100, 50, 30

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True, device: int = 0):
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)
        h = ctypes.c_void_p()
        _check(lib().orb_matcher_create(device, ctypes.byref(h)), "orb_matcher_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().orb_matcher_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    @staticmethod
    def DescriptorDistance(a: np.ndarray, b: np.ndarray) -> int:
        a = np.ascontiguousarray(a, np.uint8)
        b = np.ascontiguousarray(b, np.uint8)
        return lib().orb_descriptor_distance(_ptr(a), _ptr(b))

    def profile(self, enable: bool = True):
        _check(lib().orb_matcher_profile(self._h, int(enable)), "profile")

    def profile_read(self, stage: int):
        ms = ctypes.c_double(0)
        n = ctypes.c_int(0)
        name = ctypes.c_char_p()
        _check(lib().orb_matcher_profile_read(self._h, stage, ctypes.byref(ms), ctypes.byref(n),
                                              ctypes.byref(name)), "profile_read")
        return name.value.decode(), ms.value, n.value

    def stream(self) -> int:
        return lib().orb_matcher_stream(self._h) or 0

    # resolve schedules of SearchByProjection(F, localMap) (orb_abi.h)
    RESOLVE_AUTO, RESOLVE_PREFIX, RESOLVE_FIXED_POINT, RESOLVE_JACOBI = 0, 1, 2, 3
    RESOLVE_KERNELS = {1: "k_proj_resolve<1>", 4: "k_proj_resolve<4>", 8: "k_proj_resolve<8>",
                       16: "k_proj_resolve_fp<1024>", 32: "k_proj_jacobi+k_proj_resolve_fp"}

    def set_resolve(self, schedule: int, jacobi_rounds: int = 6):
        """Resolve schedule of the local-map matcher (every schedule is exact)."""
        _check(lib().orb_matcher_set_resolve(self._h, schedule, jacobi_rounds), "set_resolve")

    def resolve_kernel(self, n_problems: int, kp_stride: int, mp_stride: int) -> str:
        """Name of the resolve kernel a call of this shape launches."""
        k = ctypes.c_int(0)
        _check(lib().orb_matcher_resolve_kernel(self._h, n_problems, kp_stride, mp_stride,
                                                ctypes.byref(k)), "resolve_kernel")
        return self.RESOLVE_KERNELS[k.value]

    def search_by_projection_batch(self, n_problems, d_keys, d_desc, d_nkeys, d_locked, kp_stride,
                                   d_mps, d_mp_desc, d_nmps, mp_stride, width, height,
                                   scale_factors, th, d_kp_match, d_nmatches, stream: int = 0,
                                   min_x=0.0, min_y=0.0):
        """Device-batched SearchByProjection(F, localMap, th) over P problems."""
        sc = np.ascontiguousarray(scale_factors, np.float32)
        _check(lib().orb_match_projection_local_batch(
            self._h, n_problems, d_keys, d_desc, d_nkeys, d_locked or None, kp_stride, d_mps,
            d_mp_desc, d_nmps, mp_stride, min_x, float(width), min_y, float(height), len(sc),
            _ptr(sc), th, self.mfNNratio, d_kp_match, d_nmatches, stream or None),
            "orb_match_projection_local_batch")

    def hamming_batch(self, d_a: int, d_b: int, n: int, d_out: int, stream: int = 0):
        _check(lib().orb_hamming_batch(self._h, d_a, d_b, n, d_out, stream or None), "hamming")

    def SearchByProjection(self, F: Frame, mps: np.ndarray, mp_desc: np.ndarray, th: float,
                           kp_locked: np.ndarray | None = None):
        """SearchByProjection(F, vpMapPoints, th): returns (nmatches, kp_match).

        kp_match[i] = index of the map point assigned to keypoint i by this
        call (F.mvpMapPoints[i] = vpMapPoints[kp_match[i]]) or -1."""
        mps = np.ascontiguousarray(mps, MP_TRACK_DTYPE)
        mp_desc = np.ascontiguousarray(mp_desc, np.uint8).reshape(-1, 32)
        locked = None if kp_locked is None else np.ascontiguousarray(kp_locked, np.uint8)
        kp_match = np.full(F.N, -1, np.int32)
        nm = ctypes.c_int32(0)
        f = F._c()
        _check(lib().orb_match_projection_local(
            self._h, ctypes.byref(f), _ptr(locked) if locked is not None else None, len(mps),
            _ptr(mps) if len(mps) else None, _ptr(mp_desc) if len(mps) else None, th,
            self.mfNNratio, _ptr(kp_match), ctypes.byref(nm)), "SearchByProjection")
        return nm.value, kp_match

    def SearchByProjectionStaged(self, F: Frame, mps: np.ndarray, mp_desc: np.ndarray, th: float,
                                 kp_locked: np.ndarray | None = None, begin: bool = True):
        """SearchByProjection through the zero-copy pair
        orb_match_projection_local_stage / _staged: the inputs are written
        straight into the handle's pinned block (as the C++ drop-in does);
        with `begin`, _begin sends the frame's part before the map is written."""
        mps = np.ascontiguousarray(mps, MP_TRACK_DTYPE)
        mp_desc = np.ascontiguousarray(mp_desc, np.uint8).reshape(-1, 32)
        n, M = F.N, len(mps)
        if n == 0:
            return 0, np.zeros(0, np.int32)
        st = _LocalStage()
        _check(lib().orb_match_projection_local_stage(self._h, n, M, ctypes.byref(st)), "stage")

        def view(ptr, dtype, count):
            nbytes = count * np.dtype(dtype).itemsize
            buf = (ctypes.c_uint8 * max(nbytes, 1)).from_address(ptr)
            return np.frombuffer(buf, np.uint8, nbytes).view(dtype)
        view(st.keys, KEYPOINT_DTYPE, n)[:] = F.mvKeysUn
        view(st.descriptors, np.uint8, n * 32)[:] = F.mDescriptors.reshape(-1)
        stereo = F.mvuRight is not None
        if stereo:
            view(st.u_right, np.float32, n)[:] = F.mvuRight
        if kp_locked is not None:
            view(st.kp_locked, np.uint8, n)[:] = kp_locked
        f = F._c()
        if begin:
            _check(lib().orb_match_projection_local_begin(self._h, ctypes.byref(f), int(stereo),
                                                          int(kp_locked is not None)), "begin")
        if M:
            view(st.mps, MP_TRACK_DTYPE, M)[:] = mps
            view(st.mp_desc, np.uint8, M * 32)[:] = mp_desc.reshape(-1)
        kp_match = np.full(n, -1, np.int32)
        nm = ctypes.c_int32(0)
        _check(lib().orb_match_projection_local_staged(
            self._h, ctypes.byref(f), M, int(stereo), int(kp_locked is not None), th, self.mfNNratio,
            _ptr(kp_match), ctypes.byref(nm)), "SearchByProjectionStaged")
        return nm.value, kp_match


    # ---------------------------------------------------- Frame::ComputeStereoMatches
    def ComputeStereoMatchesExtracted(self, left_ext, right_ext, bf: float, fx: float):
        """Frame::ComputeStereoMatches for the pair last extracted by the two
        handles' __call__ (orb_stereo_match_extracted): nothing but mvuRight /
        mvDepth crosses PCIe.  Returns (mvuRight, mvDepth)."""
        n = ctypes.c_int(0)
        L = lib()
        _check(L.orb_stereo_match_extracted(self._h, left_ext.handle, right_ext.handle, bf, fx,
                                            None, None, 0, ctypes.byref(n)),
               "orb_stereo_match_extracted")
        ur = np.full(n.value, -1, np.float32)
        dp = np.full(n.value, -1, np.float32)
        if n.value:
            _check(L.orb_stereo_match_extracted(self._h, left_ext.handle, right_ext.handle, bf,
                                                fx, _ptr(ur), _ptr(dp), n.value, ctypes.byref(n)),
                   "orb_stereo_match_extracted")
        return ur, dp

    def ComputeStereoMatches(self, left: Frame, right_keys, right_desc, left_pyramid,
                             right_pyramid, inv_scale_factors, bf: float, fx: float):
        """Frame::ComputeStereoMatches (src/Frame.cc:516-704): (mvuRight, mvDepth)."""
        rk = np.ascontiguousarray(right_keys, KEYPOINT_DTYPE)
        rd = np.ascontiguousarray(right_desc, np.uint8).reshape(-1, 32)
        L = len(left_pyramid)
        lp = [np.ascontiguousarray(a, np.uint8) for a in left_pyramid]
        rp = [np.ascontiguousarray(a, np.uint8) for a in right_pyramid]
        for a, b in zip(lp, rp):
            if a.shape != b.shape:
                raise OrbError(ORB_EINVAL, "left/right pyramid level shapes differ")
        lptr = (ctypes.c_void_p * L)(*[a.ctypes.data for a in lp])
        rptr = (ctypes.c_void_p * L)(*[a.ctypes.data for a in rp])
        w = np.array([a.shape[1] for a in lp], np.int32)
        h = np.array([a.shape[0] for a in lp], np.int32)
        st = np.array([a.strides[0] for a in lp], np.int64)
        inv = np.ascontiguousarray(inv_scale_factors, np.float32)
        f = left._c()
        s = _StereoInput()
        s.left = ctypes.addressof(f)
        s.n_right = len(rk)
        s.right_keys = _ptr(rk) if len(rk) else None
        s.right_desc = _ptr(rd) if len(rk) else None
        s.n_levels = L
        s.left_levels, s.right_levels = ctypes.addressof(lptr), ctypes.addressof(rptr)
        s.level_width, s.level_height, s.level_stride = _ptr(w), _ptr(h), _ptr(st)
        s.inv_scale_factors = _ptr(inv)
        s.bf, s.fx = bf, fx
        ur = np.full(left.N, -1, np.float32)
        dp = np.full(left.N, -1, np.float32)
        _check(lib().orb_stereo_match(self._h, ctypes.byref(s), _ptr(ur), _ptr(dp)),
               "ComputeStereoMatches")
        return ur, dp

    def stereo_match_batch(self, n_pairs, left_ext, right_ext, d_lk, d_ld, d_ln, d_rk, d_rd,
                           d_rn, kp_stride, bf, fx, d_ur, d_depth, d_sad, stream: int = 0):
        _check(lib().orb_stereo_match_batch(self._h, n_pairs, left_ext.handle, right_ext.handle,
                                            d_lk, d_ld, d_ln, d_rk, d_rd, d_rn, kp_stride, bf, fx,
                                            d_ur, d_depth, d_sad, stream or None),
               "orb_stereo_match_batch")

    # -------------------------------------------- SearchByProjection(F, LastFrame)
    def SearchByProjectionFrame(self, current: Frame, last, last_desc, cam, tlc_z: float,
                                th: float, bMono: bool, kp_locked=None):
        """SearchByProjection(CurrentFrame, LastFrame, th, bMono): (nmatches, kp_match).
        kp_match: MapPoint id assigned, -1 untouched, -2 reset by the rotation filter."""
        last = np.ascontiguousarray(last, LAST_MP_DTYPE)
        last_desc = np.ascontiguousarray(last_desc, np.uint8).reshape(-1, 32)
        locked = None if kp_locked is None else np.ascontiguousarray(kp_locked, np.uint8)
        c = _Camera(*cam)
        km = np.full(current.N, -1, np.int32)
        nm = ctypes.c_int32(0)
        f = current._c()
        _check(lib().orb_match_projection_frame(
            self._h, ctypes.byref(f), _ptr(locked) if locked is not None else None, len(last),
            _ptr(last) if len(last) else None, _ptr(last_desc) if len(last) else None,
            ctypes.byref(c), tlc_z, th, int(bMono), int(self.mbCheckOrientation), _ptr(km),
            ctypes.byref(nm)), "SearchByProjection(F, LastFrame)")
        return nm.value, km

    # ------------------------------------------------------------ isInFrustum
    def isInFrustum(self, mps, pose, cam, min_x: float, max_x: float, min_y: float, max_y: float,
                    viewingCosLimit: float, logScaleFactor: float, nLevels: int):
        """Tracking::SearchLocalPoints' loop of Frame::isInFrustum over the local map
        (src/Tracking.cc:1360-1377): (nToMatch, tracks as MP_TRACK_DTYPE)."""
        mps = np.ascontiguousarray(mps, MAP_POINT_DTYPE)
        pose = np.ascontiguousarray(pose, POSE_DTYPE).reshape(1)
        tracks = np.zeros(len(mps), MP_TRACK_DTYPE)
        n = ctypes.c_int32(0)
        c = _Camera(*cam)
        _check(lib().orb_frustum(self._h, len(mps), _ptr(mps) if len(mps) else None, _ptr(pose),
                                 ctypes.byref(c), min_x, max_x, min_y, max_y, viewingCosLimit,
                                 logScaleFactor, nLevels, _ptr(tracks) if len(mps) else None,
                                 ctypes.byref(n)), "isInFrustum")
        return n.value, tracks

    def frustum_batch(self, n_problems, d_mps, d_nmps, mp_stride, d_poses, cam, min_x, max_x,
                      min_y, max_y, viewingCosLimit, logScaleFactor, nLevels, d_tracks,
                      d_n_in_view, stream: int = 0):
        c = _Camera(*cam)
        _check(lib().orb_frustum_batch(self._h, n_problems, d_mps, d_nmps, mp_stride, d_poses,
                                       ctypes.byref(c), min_x, max_x, min_y, max_y,
                                       viewingCosLimit, logScaleFactor, nLevels, d_tracks,
                                       d_n_in_view, stream or None), "frustum_batch")

    # ------------------------------------------------------------- SearchByBoW
    def SearchByBoW(self, kf_desc, kf_angle, kf_mp, kf_bad, kf_fv, f_desc, f_angle, f_fv):
        """SearchByBoW(pKF, F, vpMapPointMatches): (nmatches, f_match).
        *_fv = DBoW2 FeatureVector as (node ids ascending, offsets, feature indices)."""
        kd = np.ascontiguousarray(kf_desc, np.uint8)
        ka = np.ascontiguousarray(kf_angle, np.float32)
        km = np.ascontiguousarray(kf_mp, np.int32)
        kb = None if kf_bad is None else np.ascontiguousarray(kf_bad, np.uint8)
        fd = np.ascontiguousarray(f_desc, np.uint8)
        fa = np.ascontiguousarray(f_angle, np.float32)
        kfv = [np.ascontiguousarray(kf_fv[0], np.uint32), np.ascontiguousarray(kf_fv[1], np.int32),
               np.ascontiguousarray(kf_fv[2], np.uint32)]
        ffv = [np.ascontiguousarray(f_fv[0], np.uint32), np.ascontiguousarray(f_fv[1], np.int32),
               np.ascontiguousarray(f_fv[2], np.uint32)]
        fm = np.full(len(fd), -1, np.int32)
        nm = ctypes.c_int32(0)
        _check(lib().orb_match_bow(
            self._h, len(kd), _ptr(kd), _ptr(ka), _ptr(km), _ptr(kb) if kb is not None else None,
            len(kfv[0]), _ptr(kfv[0]), _ptr(kfv[1]), _ptr(kfv[2]), len(fd), _ptr(fd), _ptr(fa),
            len(ffv[0]), _ptr(ffv[0]), _ptr(ffv[1]), _ptr(ffv[2]), self.mfNNratio,
            int(self.mbCheckOrientation), _ptr(fm), ctypes.byref(nm)), "SearchByBoW")
        return nm.value, fm

    # ------------------------------------------- projection-window variants (§8(f))
    @staticmethod
    def _mps(mps):
        return np.ascontiguousarray(mps, MAP_POINT_DTYPE)

    def SearchByProjectionKF(self, F: Frame, pose, cam, logScaleFactor: float, mps, mp_desc,
                             kf_angle, th: float, ORBdist: int, kp_locked=None):
        """SearchByProjection(F, pKF, sAlreadyFound, th, ORBdist) (src/ORBmatcher.cc:1622-1759):
        (nmatches, kp_match) -- point index per frame keypoint, -1 none, -2 reset."""
        mps = self._mps(mps)
        md = np.ascontiguousarray(mp_desc, np.uint8).reshape(-1, 32)
        ka = np.ascontiguousarray(kf_angle, np.float32)
        pose = np.ascontiguousarray(pose, POSE_DTYPE).reshape(1)
        lk = None if kp_locked is None else np.ascontiguousarray(kp_locked, np.uint8)
        km = np.full(F.N, -1, np.int32)
        nm = ctypes.c_int32(0)
        f, c = F._c(), _Camera(*cam)
        _check(lib().orb_search_by_projection_reloc(
            self._h, ctypes.byref(f), _ptr(lk) if lk is not None else None, _ptr(pose),
            ctypes.byref(c), logScaleFactor, len(mps), _ptr(mps) if len(mps) else None,
            _ptr(md) if len(mps) else None, _ptr(ka) if len(mps) else None, th, int(ORBdist),
            int(self.mbCheckOrientation), _ptr(km) if F.N else None, ctypes.byref(nm)),
            "SearchByProjection(F, KF)")
        return nm.value, km

    def SearchByProjectionSim3(self, KF: Frame, Scw, cam, logScaleFactor: float, mps, mp_desc,
                               th: float, kp_matched):
        """SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (src/ORBmatcher.cc:311-425):
        (nmatches, kp_matched updated)."""
        mps = self._mps(mps)
        md = np.ascontiguousarray(mp_desc, np.uint8).reshape(-1, 32)
        S = np.ascontiguousarray(Scw, np.float32).reshape(12)
        km = np.array(kp_matched, np.int32).copy()
        nm = ctypes.c_int32(0)
        f, c = KF._c(), _Camera(*cam)
        _check(lib().orb_search_by_projection_sim3(
            self._h, ctypes.byref(f), _ptr(S), ctypes.byref(c), logScaleFactor, len(mps),
            _ptr(mps) if len(mps) else None, _ptr(md) if len(mps) else None, th,
            _ptr(km) if KF.N else None, ctypes.byref(nm)), "SearchByProjection(KF, Scw)")
        return nm.value, km

    def Fuse(self, KF: Frame, invLevelSigma2, pose, cam, logScaleFactor: float, mps, mp_desc,
             th: float = 3.0):
        """Fuse(pKF, vpMapPoints, th) targets (src/ORBmatcher.cc:903-1077): (n, fuse_idx)."""
        mps = self._mps(mps)
        md = np.ascontiguousarray(mp_desc, np.uint8).reshape(-1, 32)
        inv = np.ascontiguousarray(invLevelSigma2, np.float32)
        pose = np.ascontiguousarray(pose, POSE_DTYPE).reshape(1)
        out = np.full(len(mps), -1, np.int32)
        nm = ctypes.c_int32(0)
        f, c = KF._c(), _Camera(*cam)
        _check(lib().orb_fuse(self._h, ctypes.byref(f), _ptr(inv), _ptr(pose), ctypes.byref(c),
                              logScaleFactor, len(mps), _ptr(mps) if len(mps) else None,
                              _ptr(md) if len(mps) else None, th,
                              _ptr(out) if len(mps) else None, ctypes.byref(nm)), "Fuse")
        return nm.value, out

    def FuseSim3(self, KF: Frame, Scw, cam, logScaleFactor: float, mps, mp_desc, th: float):
        """Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) targets (src/ORBmatcher.cc:1079-1210)."""
        mps = self._mps(mps)
        md = np.ascontiguousarray(mp_desc, np.uint8).reshape(-1, 32)
        S = np.ascontiguousarray(Scw, np.float32).reshape(12)
        out = np.full(len(mps), -1, np.int32)
        nm = ctypes.c_int32(0)
        f, c = KF._c(), _Camera(*cam)
        _check(lib().orb_fuse_sim3(self._h, ctypes.byref(f), _ptr(S), ctypes.byref(c),
                                   logScaleFactor, len(mps), _ptr(mps) if len(mps) else None,
                                   _ptr(md) if len(mps) else None, th,
                                   _ptr(out) if len(mps) else None, ctypes.byref(nm)),
               "Fuse(Scw)")
        return nm.value, out

    def SearchBySim3(self, KF1: Frame, KF2: Frame, logScaleFactor: float, cam, R1w, t1w, R2w,
                     t2w, mps1, valid1, already1, mp_desc1, mps2, valid2, already2, mp_desc2,
                     s12: float, R12, t12, th: float):
        """SearchBySim3 (src/ORBmatcher.cc:1212-1458): (nFound, match12 = idx2 or -1)."""
        f32a = lambda a, n: np.ascontiguousarray(a, np.float32).reshape(n)
        u8 = lambda a: np.ascontiguousarray(a, np.uint8)
        keep = [f32a(R1w, 9), f32a(t1w, 3), f32a(R2w, 9), f32a(t2w, 3), self._mps(mps1),
                u8(valid1), u8(already1), u8(mp_desc1), self._mps(mps2), u8(valid2),
                u8(already2), u8(mp_desc2), f32a(R12, 9), f32a(t12, 3)]
        m12 = np.full(KF1.N, -1, np.int32)
        nm = ctypes.c_int32(0)
        f1, f2, c = KF1._c(), KF2._c(), _Camera(*cam)
        p = [_ptr(a) if a.size else None for a in keep]
        _check(lib().orb_search_by_sim3(self._h, ctypes.byref(f1), ctypes.byref(f2),
                                        logScaleFactor, ctypes.byref(c), *p[:12], s12, p[12],
                                        p[13], th, _ptr(m12) if KF1.N else None,
                                        ctypes.byref(nm)), "SearchBySim3")
        return nm.value, m12

    def SearchByBoWKF(self, desc1, angle1, mp1, bad1, fv1, desc2, angle2, mp2, bad2, fv2):
        """SearchByBoW(pKF1, pKF2, vpMatches12) (src/ORBmatcher.cc:581-716):
        (nmatches, match12 = MapPoint id of KF2 or -1)."""
        d1 = np.ascontiguousarray(desc1, np.uint8)
        d2 = np.ascontiguousarray(desc2, np.uint8)
        a1, a2 = (np.ascontiguousarray(a, np.float32) for a in (angle1, angle2))
        m1, m2 = (np.ascontiguousarray(a, np.int32) for a in (mp1, mp2))
        b1 = None if bad1 is None else np.ascontiguousarray(bad1, np.uint8)
        b2 = None if bad2 is None else np.ascontiguousarray(bad2, np.uint8)
        v1 = [np.ascontiguousarray(fv1[0], np.uint32), np.ascontiguousarray(fv1[1], np.int32),
              np.ascontiguousarray(fv1[2], np.uint32)]
        v2 = [np.ascontiguousarray(fv2[0], np.uint32), np.ascontiguousarray(fv2[1], np.int32),
              np.ascontiguousarray(fv2[2], np.uint32)]
        out = np.full(len(d1), -1, np.int32)
        nm = ctypes.c_int32(0)
        _check(lib().orb_match_bow_kf(
            self._h, len(d1), _ptr(d1), _ptr(a1), _ptr(m1), _ptr(b1) if b1 is not None else None,
            len(v1[0]), _ptr(v1[0]), _ptr(v1[1]), _ptr(v1[2]), len(d2), _ptr(d2), _ptr(a2),
            _ptr(m2), _ptr(b2) if b2 is not None else None, len(v2[0]), _ptr(v2[0]), _ptr(v2[1]),
            _ptr(v2[2]), self.mfNNratio, int(self.mbCheckOrientation), _ptr(out),
            ctypes.byref(nm)), "SearchByBoW(KF, KF)")
        return nm.value, out

    def SearchForTriangulation(self, KF1: Frame, has_mp1, KF2: Frame, has_mp2, levelSigma2, F12,
                               cam, Cw, R2w, t2w, fv1, fv2, bOnlyStereo: bool = False):
        """SearchForTriangulation (src/ORBmatcher.cc:718-901): (nmatches, match12)."""
        h1, h2 = (np.ascontiguousarray(a, np.uint8) for a in (has_mp1, has_mp2))
        keep = [np.ascontiguousarray(a, np.float32).reshape(-1)
                for a in (levelSigma2, F12, Cw, R2w, t2w)]
        v1 = [np.ascontiguousarray(fv1[0], np.uint32), np.ascontiguousarray(fv1[1], np.int32),
              np.ascontiguousarray(fv1[2], np.uint32)]
        v2 = [np.ascontiguousarray(fv2[0], np.uint32), np.ascontiguousarray(fv2[1], np.int32),
              np.ascontiguousarray(fv2[2], np.uint32)]
        out = np.full(KF1.N, -1, np.int32)
        nm = ctypes.c_int32(0)
        f1, f2, c = KF1._c(), KF2._c(), _Camera(*cam)
        _check(lib().orb_search_for_triangulation(
            self._h, ctypes.byref(f1), _ptr(h1), ctypes.byref(f2), _ptr(h2), _ptr(keep[0]),
            _ptr(keep[1]), ctypes.byref(c), _ptr(keep[2]), _ptr(keep[3]), _ptr(keep[4]),
            len(v1[0]), _ptr(v1[0]), _ptr(v1[1]), _ptr(v1[2]), len(v2[0]), _ptr(v2[0]),
            _ptr(v2[1]), _ptr(v2[2]), int(bOnlyStereo), int(self.mbCheckOrientation), _ptr(out),
            ctypes.byref(nm)), "SearchForTriangulation")
        return nm.value, out

    # ------------------------------------------------- SearchForInitialization
    def SearchForInitialization(self, F1: Frame, F2: Frame, vbPrevMatched, windowSize: int = 10):
        """SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize)
        (src/ORBmatcher.cc:429-577): returns (nmatches, vnMatches12, vbPrevMatched
        updated).  vbPrevMatched: (N1, 2) float32 points."""
        prev = np.array(vbPrevMatched, np.float32).reshape(F1.N, 2).copy()
        m12 = np.full(F1.N, -1, np.int32)
        nm = ctypes.c_int32(0)
        f1, f2 = F1._c(), F2._c()
        _check(lib().orb_search_for_initialization(
            self._h, ctypes.byref(f1), ctypes.byref(f2), _ptr(prev) if F1.N else None,
            int(windowSize), self.mfNNratio, int(self.mbCheckOrientation),
            _ptr(m12) if F1.N else None, ctypes.byref(nm)), "SearchForInitialization")
        return nm.value, m12, prev

    def search_for_initialization_batch(self, n_problems, d_keys1, d_desc1, d_n1, d_keys2,
                                        d_desc2, d_n2, kp_stride, min_x, max_x, min_y, max_y,
                                        windowSize, d_prev, d_matches12, d_nmatches,
                                        stream: int = 0):
        _check(lib().orb_search_for_initialization_batch(
            self._h, n_problems, d_keys1, d_desc1, d_n1, d_keys2, d_desc2, d_n2, kp_stride,
            min_x, max_x, min_y, max_y, int(windowSize), self.mfNNratio,
            int(self.mbCheckOrientation), d_prev, d_matches12, d_nmatches, stream or None),
            "search_for_initialization_batch")

    # ----------------------------------------------------- undistortion (Frame)
    @staticmethod
    def _cam(K, dist):
        K = np.ascontiguousarray(K, np.float32).reshape(9)
        dist = np.ascontiguousarray(dist, np.float32).reshape(-1)
        return K, dist

    def undistort_points(self, xy, K, dist):
        """cv::undistortPoints(src, dst, K, D, noArray(), K) on (n, 2) float points."""
        xy = np.ascontiguousarray(xy, np.float32).reshape(-1, 2)
        K, dist = self._cam(K, dist)
        out = np.zeros_like(xy)
        _check(lib().orb_undistort_points(self._h, len(xy), _ptr(xy) if len(xy) else None,
                                          _ptr(K), _ptr(dist), len(dist),
                                          _ptr(out) if len(xy) else None), "undistortPoints")
        return out

    def UndistortKeyPoints(self, mvKeys, K, dist):
        """Frame::UndistortKeyPoints (src/Frame.cc:452-482): returns mvKeysUn."""
        keys = np.ascontiguousarray(mvKeys, KEYPOINT_DTYPE)
        K, dist = self._cam(K, dist)
        out = np.zeros_like(keys)
        _check(lib().orb_undistort_keypoints(self._h, len(keys), _ptr(keys) if len(keys) else None,
                                             _ptr(K), _ptr(dist), len(dist),
                                             _ptr(out) if len(keys) else None),
               "UndistortKeyPoints")
        return out

    def ComputeImageBounds(self, cols, rows, K, dist):
        """Frame::ComputeImageBounds (src/Frame.cc:484-514): (mnMinX, mnMaxX, mnMinY, mnMaxY)."""
        K, dist = self._cam(K, dist)
        b = np.zeros(4, np.float32)
        _check(lib().orb_compute_image_bounds(self._h, cols, rows, _ptr(K), _ptr(dist), len(dist),
                                              _ptr(b)), "ComputeImageBounds")
        return tuple(float(v) for v in b)

    def undistort_keypoints_batch(self, n_frames, d_n, d_keys, stride, K, dist, d_keys_un,
                                  stream: int = 0):
        K, dist = self._cam(K, dist)
        _check(lib().orb_undistort_keypoints_batch(self._h, n_frames, d_n, d_keys, stride, _ptr(K),
                                                   _ptr(dist), len(dist), d_keys_un,
                                                   stream or None), "undistort_keypoints_batch")

    # ------------------------------------------ MapPoint::ComputeDistinctiveDescriptors
    def ComputeDistinctiveDescriptors(self, obs_offs, obs_desc, descriptors=None):
        """MapPoint::ComputeDistinctiveDescriptors for many points (src/MapPoint.cc:250-326).
        obs_offs (n_mp + 1) CSR offsets into obs_desc rows (observations in map
        order, bad KeyFrames dropped).  Returns (best_idx, descriptors): best_idx
        -1 for empty lists, whose descriptor rows keep their input value."""
        offs = np.ascontiguousarray(obs_offs, np.int32)
        od = np.ascontiguousarray(obs_desc, np.uint8).reshape(-1, 32)
        n = len(offs) - 1
        best = np.full(max(n, 0), -1, np.int32)
        out = (np.zeros((max(n, 0), 32), np.uint8) if descriptors is None
               else np.array(descriptors, np.uint8).reshape(n, 32))
        if n <= 0:
            return best, out
        _check(lib().orb_distinctive_descriptors(
            self._h, n, _ptr(offs), _ptr(od) if len(od) else None, _ptr(best), _ptr(out)),
            "ComputeDistinctiveDescriptors")
        return best, out

    def distinctive_descriptors_batch(self, n_mp, d_offs, d_desc, d_best, d_out=None,
                                      stream: int = 0):
        _check(lib().orb_distinctive_descriptors_batch(self._h, n_mp, d_offs, d_desc, d_best,
                                                       d_out, stream or None),
               "distinctive_descriptors_batch")


# ------------------------------------------------------------------ vocabulary
class ORBVocabulary:
    """DBoW2 TemplatedVocabulary<FORB::TDescriptor, FORB> (include/ORBVocabulary.h),
    device-resident.  Built from a loadFromTextFile node table
    (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1362-1448) or a text file.
    Scoring / weighting codes as BowVector.h:36-53 (L1_NORM 0 ... DOT_PRODUCT 5;
    TF_IDF 0, TF 1, IDF 2, BINARY 3)."""

    def __init__(self, k: int, L: int, parent, leaf, descriptors, weights, scoring: int = 0,
                 weighting: int = 0, device: int = 0, _handle=None):
        if _handle is not None:
            self._h = _handle
        else:
            parent = np.ascontiguousarray(parent, np.int32)
            leaf = np.ascontiguousarray(leaf, np.uint8)
            desc = np.ascontiguousarray(descriptors, np.uint8).reshape(-1, 32)
            w = np.ascontiguousarray(weights, np.float64)
            n = len(parent)
            if not (len(leaf) == n and len(desc) == n and len(w) == n):
                raise ValueError("vocabulary node table arrays differ in length")
            h = ctypes.c_void_p()
            _check(lib().orb_vocabulary_create(device, k, L, scoring, weighting, n, _ptr(parent),
                                               _ptr(leaf), _ptr(desc), _ptr(w), ctypes.byref(h)),
                   "orb_vocabulary_create")
            self._h = h
        info = np.zeros(6, np.int32)
        _check(lib().orb_vocabulary_info(self._h, _ptr(info)), "orb_vocabulary_info")
        self.k, self.L, self.scoring, self.weighting, self.n_nodes, self.n_words = map(int, info)

    @classmethod
    def loadFromTextFile(cls, path, device: int = 0) -> "ORBVocabulary":
        h = ctypes.c_void_p()
        _check(lib().orb_vocabulary_load_text(device, str(path).encode(), ctypes.byref(h)),
               "orb_vocabulary_load_text")
        return cls(0, 0, None, None, None, None, _handle=h)

    def close(self):
        if getattr(self, "_h", None):
            lib().orb_vocabulary_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def size(self) -> int:
        return self.n_words

    def empty(self) -> bool:
        return self.n_words == 0

    @property
    def stream(self) -> int:
        return lib().orb_vocabulary_stream(self._h) or 0

    def transform(self, descriptors, levelsup: int = 4, per_feature: bool = False):
        """transform(features, BowVector&, FeatureVector&, levelsup) as called by
        Frame::ComputeBoW (src/Frame.cc:439-449).  Returns (bow_words, bow_values,
        feat_vec) with feat_vec = (node ids, CSR offsets, feature indices) in the
        layout ORBmatcher.SearchByBoW takes; with per_feature also (word per
        feature, 0xFFFFFFFF if stopped; FeatureVector node per feature)."""
        d = np.ascontiguousarray(descriptors, np.uint8).reshape(-1, 32)
        n = len(d)
        cap = max(n, 1)
        bw = np.zeros(cap, np.uint32)
        bv = np.zeros(cap, np.float64)
        fvn = np.zeros(cap, np.uint32)
        fvo = np.zeros(cap + 1, np.int32)
        fvf = np.zeros(cap, np.uint32)
        fw = np.zeros(cap, np.uint32) if per_feature else None
        fn = np.zeros(cap, np.uint32) if per_feature else None
        nw = ctypes.c_int(0)
        nf = ctypes.c_int(0)
        _check(lib().orb_vocabulary_transform(
            self._h, n, _ptr(d) if n else None, levelsup, _ptr(bw), _ptr(bv), ctypes.byref(nw),
            _ptr(fvn), _ptr(fvo), _ptr(fvf), ctypes.byref(nf),
            _ptr(fw) if per_feature else None, _ptr(fn) if per_feature else None), "transform")
        a, b = nw.value, nf.value
        fv = (fvn[:b], fvo[:b + 1], fvf[:fvo[b]])
        if per_feature:
            return bw[:a], bv[:a], fv, fw[:n], fn[:n]
        return bw[:a], bv[:a], fv

    def transform_batch(self, n_frames, d_counts, d_desc, stride, levelsup, d_feat_word,
                        d_feat_weight, d_feat_node, d_bow_words, d_bow_values, d_n_words,
                        d_fv_nodes, d_fv_offs, d_fv_feats, d_n_fv_nodes, stream: int = 0):
        """Device-resident batch form (raw device pointers, e.g. torch .data_ptr())."""
        _check(lib().orb_vocabulary_transform_batch(
            self._h, n_frames, d_counts, d_desc, stride, levelsup, d_feat_word, d_feat_weight,
            d_feat_node, d_bow_words, d_bow_values, d_n_words, d_fv_nodes, d_fv_offs, d_fv_feats,
            d_n_fv_nodes, stream or None), "transform_batch")
