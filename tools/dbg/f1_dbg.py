import sys, numpy as np
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tests"), str(ROOT / "tools")]
import torch, bench, oracle, scenarios, bench_configs as bc
orb = bench.load_package()
W, H, P, U = 640, 480, 64, 16
pairs = [scenarios.init_pair(oracle, 100 + i, 1 + i % 3, w=W, h=H, nf=2000) for i in range(U)]
stride = max(max(len(s["k1"]), len(s["k2"])) for s in pairs)
K1 = np.zeros((P, stride), orb.KEYPOINT_DTYPE); K2 = np.zeros((P, stride), orb.KEYPOINT_DTYPE)
D1 = np.zeros((P, stride, 32), np.uint8); D2 = np.zeros((P, stride, 32), np.uint8)
PR = np.zeros((P, stride, 2), np.float32); n1 = np.zeros(P, np.int32); n2 = np.zeros(P, np.int32)
for i in range(P):
    s = pairs[i % U]
    n1[i], n2[i] = len(s["k1"]), len(s["k2"])
    K1[i, :n1[i]], D1[i, :n1[i]], PR[i, :n1[i]] = s["k1"], s["d1"], s["prev"]
    K2[i, :n2[i]], D2[i, :n2[i]] = s["k2"], s["d2"]
t = {k: torch.from_numpy(np.ascontiguousarray(v).view(np.uint8)).cuda() for k, v in dict(K1=K1, K2=K2, D1=D1, D2=D2, n1=n1, n2=n2).items()}
pr0 = torch.from_numpy(PR).cuda(); pr = pr0.clone()
m12 = torch.zeros((P, stride), dtype=torch.int32, device="cuda"); nm = torch.zeros(P, dtype=torch.int32, device="cuda")
mt = orb.ORBmatcher(0.9, True)
s_ = torch.cuda.current_stream().cuda_stream
def step():
    pr.copy_(pr0)
    mt.search_for_initialization_batch(P, t["K1"].data_ptr(), t["D1"].data_ptr(), t["n1"].data_ptr(), t["K2"].data_ptr(), t["D2"].data_ptr(), t["n2"].data_ptr(), stride, 0.0, float(W), 0.0, float(H), 100, pr.data_ptr(), m12.data_ptr(), nm.data_ptr(), s_)
refs = [oracle.search_for_initialization(s["k1"], s["d1"], s["k2"], s["d2"], W, H, s["prev"], 100, 0.9, True) for s in pairs]
for it in range(4):
    step(); torch.cuda.synchronize()
    mm = m12.cpu().numpy(); nn = nm.cpu().numpy()
    out = []
    for i in range(P):
        rn, rm, rp = refs[i % U]
        d = np.nonzero(mm[i, :n1[i]] != rm)[0]
        if nn[i] != rn or len(d): out.append((i, int(nn[i]), rn, len(d), d[:3].tolist(), [(int(mm[i, j]), int(rm[j])) for j in d[:3]]))
    print("iter", it, "bad problems", len(out), out[:6], flush=True)
