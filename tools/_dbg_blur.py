import sys, numpy as np
sys.path[:0] = ["tests", "oracle", "."]
import torch  # noqa
from conftest import PKG_DIR
import importlib.util
spec = importlib.util.spec_from_file_location("orb_amd", PKG_DIR / "__init__.py", submodule_search_locations=[str(PKG_DIR)])
gpu = importlib.util.module_from_spec(spec); sys.modules["orb_amd"] = gpu; spec.loader.exec_module(gpu)
import oracle
img = gpu.synth_image(12, 0, 640, 480)
ext = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
ext(img)
a = ext.blurred_levels()[0]
b = oracle.blur7(img)
bad = np.argwhere(a != b)
print(len(bad))
rows = sorted(set(bad[:, 0].tolist()))
print("rows", rows[:40])
for r in rows[:6]:
    cs = bad[bad[:, 0] == r][:, 1]
    print(r, cs.tolist()[:40])
    print(" got", a[r, cs[:12]].tolist(), "exp", b[r, cs[:12]].tolist())
