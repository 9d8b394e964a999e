"""Every frame of the bench's synthetic stream through the batch extractor,
checked against the CPU oracle (keypoints and descriptors), with the details
of any mismatch: which keypoints, their level / position / angle, how many
descriptor bits differ, and what the one-frame path gives for that frame.

  stream_parity.py [--frames 8192] [--start 0] [--batch 1024] [--threads 16]
"""
import argparse
import json
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=8192)
    ap.add_argument("--start", type=int, default=0)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--seed", type=int, default=0x4B495454)
    ap.add_argument("--width", type=int, default=1241)
    ap.add_argument("--height", type=int, default=376)
    ap.add_argument("--features", type=int, default=1000)
    a = ap.parse_args()
    import torch
    from conftest import load_pkg
    import oracle
    orb = load_pkg()
    W, H, B, NF = a.width, a.height, a.batch, a.features
    ids = list(range(a.start, a.start + a.frames))
    lib = orb.lib()
    imgs = np.empty((len(ids), H, W), np.uint8)
    with ThreadPoolExecutor(a.threads) as ex:
        list(ex.map(lambda i: lib.orb_synth_image(a.seed, ids[i], 0, W, H, imgs[i].ctypes.data, W),
                    range(len(ids))))
    ext = orb.ORBextractor(NF, 1.2, 8, 20, 7)
    cap = ext.capacity(W, H)
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    k_all = np.zeros((len(ids), cap), orb.KEYPOINT_DTYPE)
    d_all = np.zeros((len(ids), cap, 32), np.uint8)
    n_all = np.zeros(len(ids), np.int32)
    for b0 in range(0, len(ids), B):
        nb = min(B, len(ids) - b0)
        d_img = torch.from_numpy(imgs[b0:b0 + nb]).to(dev)
        dk = torch.zeros((nb, cap, 7), dtype=torch.int32, device=dev)
        dd = torch.zeros((nb, cap, 32), dtype=torch.uint8, device=dev)
        dn = torch.zeros(nb, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        ext.extract_batch(d_img.data_ptr(), nb, W, H, W, W * H, dk.data_ptr(), dd.data_ptr(), cap,
                          dn.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        k_all[b0:b0 + nb] = dk.cpu().numpy().view(orb.KEYPOINT_DTYPE).reshape(nb, cap)
        d_all[b0:b0 + nb] = dd.cpu().numpy()
        n_all[b0:b0 + nb] = dn.cpu().numpy()
    print(f"extracted {len(ids)} frames on the GPU", flush=True)

    def check(i):
        kr, dr, _ = oracle.extract(imgs[i], NF, 1.2, 8, 20, 7)
        n = int(n_all[i])
        if n != len(kr):
            return i, {"count": [n, len(kr)]}
        kg, dg = k_all[i, :n], d_all[i, :n]
        kd = [j for j in range(n) if kg[j].tobytes() != kr[j].tobytes()]
        dd = [j for j in range(n) if not np.array_equal(dg[j], dr[j])]
        if not kd and not dd:
            return i, None
        det = []
        for j in (dd or kd)[:6]:
            det.append({"kp": j, "x": float(kr[j]["x"]), "y": float(kr[j]["y"]),
                        "octave": int(kr[j]["octave"]), "angle_ref": float(kr[j]["angle"]),
                        "angle_gpu": float(kg[j]["angle"]),
                        "bits": int(np.unpackbits(dg[j] ^ dr[j]).sum())})
        return i, {"keys_differ": len(kd), "desc_differ": len(dd), "detail": det}

    with ThreadPoolExecutor(a.threads) as ex:
        res = list(ex.map(check, range(len(ids))))
    bad = [(i, r) for i, r in res if r is not None]
    print(f"{len(bad)} of {len(ids)} frames differ from the oracle", flush=True)
    for i, r in bad[:12]:
        single = None
        k1, d1 = ext(imgs[i])
        kr, dr, _ = oracle.extract(imgs[i], NF, 1.2, 8, 20, 7)
        single = bool(len(k1) == len(kr) and np.array_equal(d1, dr) and
                      k1.tobytes() == kr.tobytes())
        print(json.dumps({"frame": ids[i], **r, "one_frame_path_exact": single}), flush=True)


if __name__ == "__main__":
    main()
