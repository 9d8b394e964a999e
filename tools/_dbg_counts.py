import sys, ctypes, numpy as np
sys.path[:0] = ["tests", "oracle", "."]
import torch
import bench
orb = bench.load_package()
L = orb.lib()
W, H, B = 1241, 376, 64
imgs = np.stack([orb.synth_image(0x4B495454, f, W, H) for f in range(B)])
ext = orb.ORBextractor(1000, 1.2, 8, 20, 7)
cap = ext.capacity(W, H)
d = torch.from_numpy(imgs).cuda()
k = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda"); de = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda"); n = torch.zeros(B, dtype=torch.int32, device="cuda")
ext.extract_batch(d.data_ptr(), B, W, H, W, W * H, k.data_ptr(), de.data_ptr(), cap, n.data_ptr())
torch.cuda.synchronize()
c = (ctypes.c_ulonglong * 8)()
L.orb_dbg_counters(c)
px = 1444097 * B
print("pixels", px, "queuedA", c[0], c[0] / px, "cornersA", c[1], c[1] / px, "queuedB", c[2], "cornersB", c[3], "kps", int(n.sum()))
