import sys, numpy as np
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tests")]
import bench, oracle, scenarios
orb = bench.load_package()
bad = 0
for i in range(16):
    s = scenarios.init_pair(oracle, 100 + i, 1 + i % 3, w=640, h=480, nf=2000)
    rn, rm, rp = oracle.search_for_initialization(s["k1"], s["d1"], s["k2"], s["d2"], 640, 480, s["prev"], 100, 0.9, True)
    rn0, rm0, _ = oracle.search_for_initialization(s["k1"], s["d1"], s["k2"], s["d2"], 640, 480, s["prev"], 100, 0.9, False)
    m = orb.ORBmatcher(0.9, True)
    F1 = orb.Frame(s["k1"], s["d1"], np.ones(8, np.float32), 640, 480)
    F2 = orb.Frame(s["k2"], s["d2"], np.ones(8, np.float32), 640, 480)
    n, m12, prev = m.SearchForInitialization(F1, F2, s["prev"], 100)
    m0 = orb.ORBmatcher(0.9, False)
    n0, m120, _ = m0.SearchForInitialization(F1, F2, s["prev"], 100)
    d = np.nonzero(m12 != rm)[0]
    d0 = np.nonzero(m120 != rm0)[0]
    print(i, "n", n, rn, "noori", n0, rn0, "diff", d[:8], "diff_noori", d0[:8], [(int(m120[j]), int(rm0[j])) for j in d0[:8]], flush=True)
