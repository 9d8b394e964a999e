"""Oracle restatement of cv::undistortPoints as Frame::UndistortKeyPoints and
Frame::ComputeImageBounds call it (src/Frame.cc:452-514) against the
independent Python restatement (pyref.py).  OpenCV is a third-party
dependency that is absent here and the reference has no fixtures for it, so
parity with OpenCV itself is unpinned; the restatement follows
cvUndistortPoints' double arithmetic (camera_oracle.cpp header)."""
import numpy as np
import pytest

import pyref
import scenarios


@pytest.mark.parametrize("cam", ["tum1", "tum2", "kitti", "k4", "rational8", "prism12"])
def test_undistort_points_matches_restatement(oracle, cam):
    K, D = scenarios.cameras()[cam]
    pts = scenarios.undistort_points_grid(rng_seed=len(cam))
    got = oracle.undistort_points(pts, K, D)
    ref = pyref.undistort_points(pts, K, D)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_undistort_keypoints_fields(oracle):
    K, D = scenarios.cameras()["tum1"]
    img = oracle.synth_image(1, 0, 640, 480)
    keys, _, _ = oracle.extract(img, 1000)
    un = oracle.undistort_keypoints(keys, K, D)
    for f in ("size", "angle", "response", "octave", "class_id"):
        assert np.array_equal(un[f], keys[f])
    xy = np.stack([keys["x"], keys["y"]], 1)
    ref = pyref.undistort_points(xy, K, D)
    assert np.array_equal(un["x"], ref[:, 0]) and np.array_equal(un["y"], ref[:, 1])
    # barrel distortion at TUM1: points move, the centre barely
    assert np.abs(un["x"] - keys["x"]).max() > 1.0
    # zero k1: mvKeysUn = mvKeys (:454-458), even with other coefficients set
    D0 = D.copy()
    D0[0] = 0
    assert oracle.undistort_keypoints(keys, K, D0).tobytes() == keys.tobytes()


def test_compute_image_bounds(oracle):
    K, D = scenarios.cameras()["tum1"]
    b = oracle.compute_image_bounds(640, 480, K, D)
    c = pyref.undistort_points(np.array([[0, 0], [640, 0], [0, 480], [640, 480]], np.float32), K, D)
    assert b.tolist() == [min(c[0, 0], c[2, 0]), max(c[1, 0], c[3, 0]), min(c[0, 1], c[1, 1]),
                          max(c[2, 1], c[3, 1])]
    Kk, Dk = scenarios.cameras()["kitti"]
    assert oracle.compute_image_bounds(1241, 376, Kk, Dk).tolist() == [0, 1241, 0, 376]
    with pytest.raises(ValueError):
        oracle.undistort_points(np.zeros((1, 2), np.float32), K, np.zeros(6, np.float32))
