"""The CPU oracle on many host threads at once (bench.py's all-cores CPU
baseline): every call's result equals the same call made alone.  The
matchers' grid scratch is per thread (a shared function-local grid was
rebuilt under another thread's SearchByProjection and crashed the bench)."""
import threading

import numpy as np


def test_oracle_extract_and_match_threads(oracle):
    w, h = 640, 480
    imgs = [oracle.synth_image(70 + f, 0, w, h) for f in range(6)]
    scale = oracle.params(1000)["scale"]
    ref = []
    for i, im in enumerate(imgs):
        k, d, _ = oracle.extract(im, 1000)
        mps, mpd, locked = oracle.synth_local_map(i, k, d, 2000, w, h)
        ref.append((k, d, mps, mpd, locked,
                    oracle.match_projection_local(k, d, scale, w, h, mps, mpd, 1.0, 0.8, locked)))
    bad = []

    def work(t):
        for it in range(4):
            i = (t + it) % len(imgs)
            k, d, mps, mpd, locked, (n_ref, km_ref) = ref[i]
            k2, d2, _ = oracle.extract(imgs[i], 1000)
            n, km = oracle.match_projection_local(k, d, scale, w, h, mps, mpd, 1.0, 0.8, locked)
            if k2.tobytes() != k.tobytes() or d2.tobytes() != d.tobytes() or n != n_ref or \
                    not np.array_equal(km, km_ref):
                bad.append((t, i))

    ths = [threading.Thread(target=work, args=(t,)) for t in range(8)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not bad, bad
