"""Does another process's idle GPU state slow the drop-in's one-frame calls?

Runs `harness time DIR` (prepared by dropin_timeline.py prepare) three ways:
alone; as a child of this process after it has created the bench's set of
streams and library handles and run one batch on each (then left idle, as
bench.py's process is while its drop-in leg runs); alone again.
Prints each run's time.json.  Usage: dropin_idle_queues.py DIR
"""
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
HARNESS = ROOT / "tests/integration_run/dropin_harness_gpustereo"


def run(d, tag):
    r = subprocess.run([str(HARNESS), "time", d], capture_output=True, text=True, timeout=300)
    if r.returncode:
        raise SystemExit(f"{tag}: harness failed: {r.stderr[-800:]}")
    print(tag, json.dumps(json.loads((Path(d) / "time.json").read_text())), flush=True)


def main():
    d = sys.argv[1]
    run(d, "alone")
    sys.path.insert(0, str(ROOT / "tests"))
    import torch
    from conftest import load_pkg
    orb = load_pkg()
    W, H, B = 1241, 376, 64
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(dev) for _ in range(8)]
    exts = [orb.ORBextractor(1000, 1.2, 8, 20, 7) for _ in range(2)]
    mts = [orb.ORBmatcher(0.8) for _ in range(4)]
    img = torch.zeros((B, H, W), dtype=torch.uint8, device=dev)
    cap = exts[0].capacity(W, H)
    k = torch.zeros((B, cap, 7), dtype=torch.int32, device=dev)
    de = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
    n = torch.zeros(B, dtype=torch.int32, device=dev)
    for i, e in enumerate(exts):
        e.extract_batch(img.data_ptr(), B, W, H, W, W * H, k.data_ptr(), de.data_ptr(), cap,
                        n.data_ptr(), streams[i].cuda_stream)
    for s in streams:
        torch.zeros(1, device=dev).add_(1)  # touch each stream's queue
        with torch.cuda.stream(s):
            torch.ones(16, device=dev).sum()
    torch.cuda.synchronize()
    run(d, "beside_idle_process_state")
    del mts, exts
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
    # (the third run is a separate invocation: see the gpurun command in DESIGN §5)
