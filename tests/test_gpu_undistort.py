"""GPU parity of keypoint undistortion (Frame::UndistortKeyPoints,
Frame::ComputeImageBounds, src/Frame.cc:452-514; cv::undistortPoints with
P = mK) against the CPU oracle: float32 outputs bit-exact (double arithmetic
in the same order, no contraction, IEEE division on both sides)."""
import numpy as np
import pytest

import scenarios

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cam", ["tum1", "tum2", "kitti", "k4", "rational8", "prism12"])
def test_undistort_points(gpu, oracle, cam):
    K, D = scenarios.cameras()[cam]
    pts = scenarios.undistort_points_grid(rng_seed=len(cam), n_random=20000)
    got = gpu.ORBmatcher().undistort_points(pts, K, D)
    ref = oracle.undistort_points(pts, K, D)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("cam", ["tum1", "kitti"])
def test_undistort_keypoints_and_bounds(gpu, oracle, cam):
    K, D = scenarios.cameras()[cam]
    img = gpu.synth_image(2, 0, 640, 480)
    keys, _ = gpu.ORBextractor(1000, 1.2, 8, 20, 7)(img)
    m = gpu.ORBmatcher()
    un = m.UndistortKeyPoints(keys, K, D)
    assert un.tobytes() == oracle.undistort_keypoints(keys, K, D).tobytes()
    b = m.ComputeImageBounds(640, 480, K, D)
    assert list(b) == oracle.compute_image_bounds(640, 480, K, D).tolist()
    assert len(m.UndistortKeyPoints(keys[:0], K, D)) == 0
    with pytest.raises(gpu.OrbError):
        m.UndistortKeyPoints(keys, K, np.zeros(3, np.float32))


def test_undistort_keypoints_batch(gpu, oracle):
    torch = pytest.importorskip("torch")
    K, D = scenarios.cameras()["tum1"]
    ext = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    frames = [ext(gpu.synth_image(3, f, 640, 480))[0] for f in range(6)]
    stride = 1100
    counts = np.array([len(f) for f in frames] + [0, 17], np.int32)
    F = len(counts)
    keys = np.zeros((F, stride), gpu.KEYPOINT_DTYPE)
    for f in range(6):
        keys[f, :counts[f]] = frames[f]
    keys[7, :17] = frames[0][:17]
    dev = torch.device("cuda:0")
    d_keys = torch.from_numpy(keys.view(np.uint8).reshape(-1)).to(dev)
    d_n = torch.from_numpy(counts).to(dev)
    d_out = torch.full((keys.nbytes,), 0xAB, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    m = gpu.ORBmatcher()
    m.undistort_keypoints_batch(F, d_n.data_ptr(), d_keys.data_ptr(), stride, K, D,
                                d_out.data_ptr())
    torch.cuda.synchronize()
    out = d_out.cpu().numpy().view(gpu.KEYPOINT_DTYPE).reshape(F, stride)
    for f in range(F):
        n = int(counts[f])
        ref = oracle.undistort_keypoints(keys[f, :n], K, D)
        assert out[f, :n].tobytes() == ref.tobytes()
        assert (out[f, n:].view(np.uint8) == 0xAB).all()  # untouched past the count
