"""Synthetic inputs are identical from the product library and the oracle build
(integer-only generator), deterministic, and shaped like the survey's configs."""
import numpy as np


def test_images_identical_across_builds(orb, oracle):
    for (w, h, seed, frame, view) in [(640, 480, 1, 0, 0), (1241, 376, 7, 3, 1), (1920, 1080, 5, 0, 0)]:
        a = orb.synth_image(seed, frame, w, h, view)
        b = oracle.synth_image(seed, frame, w, h, view)
        assert a.shape == (h, w) and np.array_equal(a, b)


def test_sequence_moves_and_stereo_shifts(orb):
    f0 = orb.synth_image(3, 0, 640, 480)
    f5 = orb.synth_image(3, 5, 640, 480)
    r0 = orb.synth_image(3, 0, 640, 480, view=1)
    assert not np.array_equal(f0, f5) and not np.array_equal(f0, r0)
    assert 20 < f0.std() < 120


def test_local_map_identical(orb, oracle):
    rng = np.random.default_rng(0)
    keys = np.zeros(500, orb.KEYPOINT_DTYPE)
    keys["x"] = rng.uniform(0, 640, 500)
    keys["y"] = rng.uniform(0, 480, 500)
    keys["octave"] = rng.integers(0, 8, 500)
    desc = rng.integers(0, 256, (500, 32), dtype=np.uint8)
    a = orb.synth_local_map(9, keys, desc, 3000, 640, 480)
    b = oracle.synth_local_map(9, keys, desc, 3000, 640, 480)
    for x, y in zip(a, b):
        assert x.tobytes() == y.tobytes()
    mps = a[0]
    assert 0.9 < mps["in_view"].mean() < 1.0 and set(np.unique(mps["view_cos"])) <= {np.float32(0.999), np.float32(0.9)}
