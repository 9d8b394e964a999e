import sys, numpy as np
sys.path[:0] = ["tests", "oracle", "."]
import torch  # noqa
from conftest import PKG_DIR
import importlib.util
spec = importlib.util.spec_from_file_location("orb_amd", PKG_DIR / "__init__.py", submodule_search_locations=[str(PKG_DIR)])
gpu = importlib.util.module_from_spec(spec); sys.modules["orb_amd"] = gpu; spec.loader.exec_module(gpu)
import oracle
for (w, h) in [(640, 480), (1241, 376)]:
    img = gpu.synth_image(1, 0, w, h)
    ext = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    ext(img)
    for l, (a, b) in enumerate(zip(ext.mvImagePyramid, oracle.pyramid(img))):
        bad = np.argwhere(a != b)
        if len(bad):
            print(w, h, "level", l, a.shape, len(bad), bad[:8].tolist(), a[tuple(bad[0])], b[tuple(bad[0])])
            rows = sorted(set(bad[:, 0].tolist())); cols = sorted(set(bad[:, 1].tolist()))
            print("  rows", rows[:20], "... cols", cols[:20], cols[-5:])
