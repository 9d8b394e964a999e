"""Every frame of the bench's synthetic stream through the batch extractor,
checked against the CPU oracle (keypoints and descriptors), with the details
of any mismatch: which keypoints, their level / position / angle, how many
descriptor bits differ, and what the one-frame path gives for that frame.

  stream_parity.py [--frames 8192] [--start 0] [--batch 1024] [--threads 16]
                   [--width W --height H --features N] [--match M]

--match M: also SearchByProjection(F, localMap) of every frame against its own
M-point synthetic local map (bench.py's maps), device-batched, against the
oracle's assignments.
--one-frame: every frame through the one-frame entry point (ORBextractor
operator(): k_fast_band, the register octree, k_orient_desc<1>) instead.
--stereo: every frame is a stereo pair (view 0 left, view 1 right): both
extractions and ComputeStereoMatches (device-batched, orb_stereo_match_batch)
against the oracle's mvuRight / mvDepth, bit for bit.
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
    ap.add_argument("--match", type=int, default=0)
    ap.add_argument("--stereo", action="store_true")
    ap.add_argument("--one-frame", action="store_true")
    a = ap.parse_args()
    if a.stereo:
        return stereo(a)
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
        if a.one_frame:
            for i in range(b0, b0 + nb):
                k1, d1 = ext(imgs[i])
                n_all[i] = len(k1)
                k_all[i, :len(k1)] = k1
                d_all[i, :len(k1)] = d1
            continue
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
    print(f"extracted {len(ids)} frames on the GPU ({'one-frame calls' if a.one_frame else 'batches'})",
          flush=True)

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
    if a.match:
        M = a.match
        scale = np.float32(ext.GetScaleFactors())
        maps = [None] * len(ids)

        def mk(i):
            n = int(n_all[i])
            maps[i] = orb.synth_local_map(a.seed + ids[i], k_all[i, :n], d_all[i, :n], M, W, H)
        with ThreadPoolExecutor(a.threads) as ex:
            list(ex.map(mk, range(len(ids))))
        mt = orb.ORBmatcher(0.8)
        km_all = np.zeros((len(ids), cap), np.int32)
        nm_all = np.zeros(len(ids), np.int32)
        for b0 in range(0, len(ids), B):
            nb = min(B, len(ids) - b0)
            mps = np.stack([maps[i][0] for i in range(b0, b0 + nb)])
            mpd = np.stack([maps[i][1] for i in range(b0, b0 + nb)])
            lk = np.zeros((nb, cap), np.uint8)
            for j in range(nb):
                lk[j, :n_all[b0 + j]] = maps[b0 + j][2]
            t = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.uint8)).to(dev)
            dk, dd, dl = t(k_all[b0:b0 + nb]), t(d_all[b0:b0 + nb]), t(lk)
            dm, dmd = t(mps), t(mpd)
            dn = torch.from_numpy(n_all[b0:b0 + nb].copy()).to(dev)
            dnm = torch.full((nb,), M, dtype=torch.int32, device=dev)
            dkm = torch.zeros((nb, cap), dtype=torch.int32, device=dev)
            dnmt = torch.zeros(nb, dtype=torch.int32, device=dev)
            torch.cuda.synchronize()
            mt.search_by_projection_batch(nb, dk.data_ptr(), dd.data_ptr(), dn.data_ptr(),
                                          dl.data_ptr(), cap, dm.data_ptr(), dmd.data_ptr(),
                                          dnm.data_ptr(), M, W, H, scale, 1.0, dkm.data_ptr(),
                                          dnmt.data_ptr(), s.cuda_stream)
            torch.cuda.synchronize()
            km_all[b0:b0 + nb] = dkm.cpu().numpy()
            nm_all[b0:b0 + nb] = dnmt.cpu().numpy()

        def mcheck(i):
            n = int(n_all[i])
            mps, mpd, lk = maps[i]
            n_ref, km_ref = oracle.match_projection_local(k_all[i, :n], d_all[i, :n], scale, W, H,
                                                          mps, mpd, 1.0, 0.8, lk)
            ok = n_ref == nm_all[i] and np.array_equal(km_all[i, :n], km_ref)
            return i, None if ok else {"nmatch": [int(nm_all[i]), int(n_ref)],
                                       "kp_diff": int((km_all[i, :n] != km_ref).sum())}
        with ThreadPoolExecutor(a.threads) as ex:
            mres = list(ex.map(mcheck, range(len(ids))))
        mbad = [(i, r) for i, r in mres if r is not None]
        print(f"SearchByProjection vs {M} map points: {len(mbad)} of {len(ids)} frames differ "
              f"(mean matches {nm_all.mean():.1f})", flush=True)
        for i, r in mbad[:10]:
            print(json.dumps({"frame": ids[i], **r}), flush=True)
    for i, r in bad[:12]:
        single = None
        k1, d1 = ext(imgs[i])
        kr, dr, _ = oracle.extract(imgs[i], NF, 1.2, 8, 20, 7)
        single = bool(len(k1) == len(kr) and np.array_equal(d1, dr) and
                      k1.tobytes() == kr.tobytes())
        print(json.dumps({"frame": ids[i], **r, "one_frame_path_exact": single}), flush=True)


def stereo(a):
    import torch
    from conftest import load_pkg
    import oracle
    orb = load_pkg()
    W, H, B, NF = a.width, a.height, a.batch, a.features
    bf, fx = 386.1448, 718.856
    ids = list(range(a.start, a.start + a.frames))
    lib = orb.lib()
    views = []
    for v in (0, 1):
        im = np.empty((len(ids), H, W), np.uint8)
        with ThreadPoolExecutor(a.threads) as ex:
            list(ex.map(lambda i: lib.orb_synth_image(a.seed, ids[i], v, W, H, im[i].ctypes.data, W),
                        range(len(ids))))
        views.append(im)
    L = orb.ORBextractor(NF, 1.2, 8, 20, 7)
    R = orb.ORBextractor(NF, 1.2, 8, 20, 7)
    mt = orb.ORBmatcher()
    cap = L.capacity(W, H)
    dev = torch.device("cuda", 0)
    ur_all = np.zeros((len(ids), cap), np.float32)
    dp_all = np.zeros((len(ids), cap), np.float32)
    n_all = np.zeros(len(ids), np.int32)
    for b0 in range(0, len(ids), B):
        nb = min(B, len(ids) - b0)
        outs = []
        for ext, im in ((L, views[0]), (R, views[1])):
            d_img = torch.from_numpy(im[b0:b0 + nb]).to(dev)
            k = torch.zeros((nb, cap, 7), dtype=torch.int32, device=dev)
            de = torch.zeros((nb, cap, 32), dtype=torch.uint8, device=dev)
            n = torch.zeros(nb, dtype=torch.int32, device=dev)
            torch.cuda.synchronize()
            ext.extract_batch(d_img.data_ptr(), nb, W, H, W, W * H, k.data_ptr(), de.data_ptr(), cap,
                              n.data_ptr())
            torch.cuda.synchronize()
            outs.append((d_img, k, de, n))
        ur = torch.zeros((nb, cap), dtype=torch.float32, device=dev)
        dp = torch.zeros((nb, cap), dtype=torch.float32, device=dev)
        sad = torch.zeros((nb, cap), dtype=torch.int32, device=dev)
        (_, kl, dl, nl), (_, kr, dr, nr) = outs
        mt.stereo_match_batch(nb, L, R, kl.data_ptr(), dl.data_ptr(), nl.data_ptr(), kr.data_ptr(),
                              dr.data_ptr(), nr.data_ptr(), cap, bf, fx, ur.data_ptr(), dp.data_ptr(),
                              sad.data_ptr())
        torch.cuda.synchronize()
        ur_all[b0:b0 + nb] = ur.cpu().numpy()
        dp_all[b0:b0 + nb] = dp.cpu().numpy()
        n_all[b0:b0 + nb] = nl.cpu().numpy()
    print(f"extracted and stereo-matched {len(ids)} pairs on the GPU", flush=True)
    p = oracle.params(NF)

    def check(i):
        kl, dl, _ = oracle.extract(views[0][i], NF, 1.2, 8, 20, 7)
        kr, dr, _ = oracle.extract(views[1][i], NF, 1.2, 8, 20, 7)
        ur_ref, dp_ref = oracle.stereo_match(kl, dl, p["scale"], kr, dr, oracle.pyramid(views[0][i]),
                                             oracle.pyramid(views[1][i]), p["inv_scale"], bf, fx, W, H)
        n = int(n_all[i])
        if n != len(kl):
            return i, {"count": [n, len(kl)]}
        bad = np.nonzero((ur_all[i, :n].view(np.uint32) != ur_ref.view(np.uint32)) |
                         (dp_all[i, :n].view(np.uint32) != dp_ref.view(np.uint32)))[0]
        if len(bad) == 0:
            return i, None
        return i, {"differ": int(len(bad)), "first": [int(j) for j in bad[:4]],
                   "gpu": [float(ur_all[i, j]) for j in bad[:4]], "ref": [float(ur_ref[j]) for j in bad[:4]]}

    with ThreadPoolExecutor(a.threads) as ex:
        res = list(ex.map(check, range(len(ids))))
    bad = [(i, r) for i, r in res if r is not None]
    matched = float((ur_all > 0).sum()) / len(ids)
    print(f"ComputeStereoMatches: {len(bad)} of {len(ids)} pairs differ from the oracle "
          f"(mean {matched:.1f} left keypoints with a match)", flush=True)
    for i, r in bad[:10]:
        print(json.dumps({"pair": ids[i], **r}), flush=True)


if __name__ == "__main__":
    main()
