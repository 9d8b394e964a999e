"""GPU Frame::isInFrustum over the local map and the chained
SearchLocalPoints path (frustum -> SearchByProjection) against the CPU oracle."""
import math

import numpy as np
import pytest

import scenarios

pytestmark = pytest.mark.gpu
LS = np.float32(math.log(np.float32(1.2)))
TRACK_FIELDS = ("proj_x", "proj_y", "proj_xr", "view_cos", "level", "in_view", "bad", "has_obs")


def _case(oracle, seed, n_mp=8000):
    img = oracle.synth_image(seed, 0, 1241, 376)
    k, d, _ = oracle.extract(img, 1000)
    pose, P, mpd = scenarios.local_map_3d(oracle, k, d, n_mp, 1241, 376, rng_seed=seed)
    return k, d, pose, P, mpd


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_frustum_bit_exact(gpu, oracle, seed):
    k, d, pose, P, _ = _case(oracle, seed)
    n_ref, tr_ref = oracle.frustum(P, pose, scenarios.camera(), 1241, 376, 0.5, LS, 8)
    n, tr = gpu.ORBmatcher().isInFrustum(P, pose, scenarios.camera(), 0.0, 1241.0, 0.0, 376.0,
                                         0.5, LS, 8)
    assert n == n_ref > 1000
    assert tr.tobytes() == tr_ref.tobytes()


def test_frustum_edge_cases(gpu, oracle):
    P = np.zeros(5, gpu.MAP_POINT_DTYPE)
    rec = np.zeros(1, gpu.POSE_DTYPE)
    rec["rcw"] = np.eye(3, dtype=np.float32).reshape(1, 9)
    P["pos"] = [[0, 0, 10], [0, 0, -10], [0, 0, 0], [1e4, 0, 1], [0.5, 0.2, 3]]
    P["normal"] = [[0, 0, 1]] * 5
    P["max_distance"] = 100.0
    P["seen"] = [0, 0, 0, 0, 1]
    cam = (500.0, 500.0, 320.0, 240.0, 40.0, 0.08)
    n_ref, tr_ref = oracle.frustum(P, rec, cam, 640, 480, 0.5, LS, 8)
    n, tr = gpu.ORBmatcher().isInFrustum(P, rec, cam, 0.0, 640.0, 0.0, 480.0, 0.5, LS, 8)
    assert n == n_ref == 2
    assert tr.tobytes() == tr_ref.tobytes()  # incl. the NaN projection of the z=0 point
    assert gpu.ORBmatcher().isInFrustum(P[:0], rec, cam, 0, 640, 0, 480, 0.5, LS, 8)[0] == 0


@pytest.mark.parametrize("seed", [4, 5])
def test_search_local_points_chain(gpu, oracle, seed):
    """SearchLocalPoints = isInFrustum(0.5) over the local map, then
    SearchByProjection(F, localMap, th=1) with ORBmatcher(0.8)."""
    k, d, pose, P, mpd = _case(oracle, seed, 10000)
    rng = np.random.default_rng(seed)
    locked = (rng.random(len(k)) < 0.2).astype(np.uint8)
    scale = oracle.params(1000)["scale"]
    _, tr_ref = oracle.frustum(P, pose, scenarios.camera(), 1241, 376, 0.5, LS, 8)
    n_ref, km_ref = oracle.match_projection_local(k, d, scale, 1241, 376, tr_ref, mpd, 1.0, 0.8,
                                                  locked)
    m = gpu.ORBmatcher(0.8)
    _, tr = m.isInFrustum(P, pose, scenarios.camera(), 0.0, 1241.0, 0.0, 376.0, 0.5, LS, 8)
    F = gpu.Frame(k, d, scale, 1241, 376)
    n, km = m.SearchByProjection(F, tr, mpd, 1.0, locked)
    assert n == n_ref > 300
    assert np.array_equal(km, km_ref)


def test_frustum_batch_per_problem_pose(gpu, oracle):
    torch = pytest.importorskip("torch")
    cases = [_case(oracle, s, 3000 + 500 * s) for s in range(3)]
    stride = max(len(c[3]) for c in cases)
    Pall = np.zeros((3, stride), gpu.MAP_POINT_DTYPE)
    poses = np.zeros(3, gpu.POSE_DTYPE)
    for i, c in enumerate(cases):
        Pall[i, :len(c[3])] = c[3]
        poses[i] = c[2][0]
    dev = "cuda"
    d_mps = torch.from_numpy(Pall.view(np.uint8).reshape(3, -1)).to(dev)
    d_n = torch.tensor([len(c[3]) for c in cases], dtype=torch.int32, device=dev)
    d_pose = torch.from_numpy(poses.view(np.uint8)).to(dev)
    d_tr = torch.zeros((3, stride * gpu.MP_TRACK_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    d_cnt = torch.zeros(3, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    m = gpu.ORBmatcher()
    m.frustum_batch(3, d_mps.data_ptr(), d_n.data_ptr(), stride, d_pose.data_ptr(),
                    scenarios.camera(), 0.0, 1241.0, 0.0, 376.0, 0.5, LS, 8, d_tr.data_ptr(),
                    d_cnt.data_ptr())
    torch.cuda.synchronize()
    tr_all = d_tr.cpu().numpy().view(gpu.MP_TRACK_DTYPE).reshape(3, stride)
    for i, c in enumerate(cases):
        n_ref, tr_ref = oracle.frustum(c[3], c[2], scenarios.camera(), 1241, 376, 0.5, LS, 8)
        assert int(d_cnt[i].item()) == n_ref
        assert tr_all[i, :len(c[3])].tobytes() == tr_ref.tobytes()
