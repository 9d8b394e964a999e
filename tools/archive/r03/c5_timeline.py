#!/usr/bin/env python3
"""Probe: timeline of C5's pipelined steps (extract on stream E, match on
stream M) -- per-step start/end of both by timing events -- for a call that
lands in the slow mode and one in the fast mode (tools/probe/c5_streams.py)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[3]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

orb = bench.load_package()
dev = torch.device("cuda:0")
orig = bench.pipelined


def traced(torch, dev, extract, match, n_sets, steps, warmup):
    es, ms = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    ext_done = [torch.cuda.Event() for _ in range(n_sets)]
    match_done = [torch.cuda.Event() for _ in range(n_sets)]
    n = warmup + steps
    T = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(n)]
    for g in range(n):
        j = g % n_sets
        if g >= n_sets:
            es.wait_event(match_done[j])
        T[g][0].record(es)
        extract(j, es.cuda_stream)
        T[g][1].record(es)
        ext_done[j].record(es)
        ms.wait_event(ext_done[j])
        T[g][2].record(ms)
        match(j, ms.cuda_stream)
        T[g][3].record(ms)
        match_done[j].record(ms)
    torch.cuda.synchronize()
    t0 = T[warmup][0]
    rel = np.array([[t0.elapsed_time(T[g][k]) for k in range(4)] for g in range(warmup, n)])
    e_dur = rel[:, 1] - rel[:, 0]
    m_dur = rel[:, 3] - rel[:, 2]
    step = np.diff(rel[:, 0])
    e_gap = rel[1:, 0] - rel[:-1, 1]  # extraction idle between steps
    m_lag = rel[:, 2] - rel[:, 1]      # match start after its extraction ended
    print(f"  step {step.mean():.3f} ms; extract {e_dur.mean():.3f}; match {m_dur.mean():.3f}; "
          f"extract idle between steps {e_gap.mean():.3f}; match starts {m_lag.mean():.3f} after "
          f"its extraction", flush=True)
    for g in range(3):
        print("   ", np.round(rel[g], 3), flush=True)
    return (rel[-1, 3] - rel[0, 0]) / 1e3 / steps


bench.pipelined = traced
for tag in ("fresh process", "again", "third"):
    r, _ = bench.proj_workload(orb, torch, dev, 16, 1920, 1080, 4000, 50000, 16, bench.C5_SEED,
                               steps=200, warmup=10)
    print(f"{tag}: {r['value']:.0f} problems/s", flush=True)
