#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) into per-kernel HBM
bytes per launch, the `traffic` figure bench.py reports.

Usage: tools/pmc_summary.py <fetch_dir> <write_dir> <batch> <out.json>

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  Values are reported raw (no
x2 correction): the gfx950 halving applies to 16-B/lane streaming loads, and our
kernels load bytes and dwords; on k_pyr_resize (dword loads, known byte count)
raw FETCH_SIZE matches the algorithmic read bytes within a few per cent
(DESIGN.md §5).
"""
import collections
import csv
import json
import sys
from pathlib import Path


def kname(full):
    """'void k_pyr_resize<true>(...)' -> 'k_pyr_resize'"""
    n = full.split("(")[0]
    n = n[5:] if n.startswith("void ") else n
    return n.split("<")[0]


def per_kernel(d, counter):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(Path(d) / "run_counter_collection.csv")):
        if r["Counter_Name"] == counter:
            vals[kname(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)
    return vals


def main():
    fetch_dir, write_dir, batch, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    f, w = per_kernel(fetch_dir, "FETCH_SIZE"), per_kernel(write_dir, "WRITE_SIZE")
    res = {"batch": batch, "unit": "bytes per launch (mean over dispatches)", "kernels": {}}
    for k in sorted(set(f) | set(w)):
        if not k.startswith("k_"):
            continue
        fb = sum(f.get(k, [0])) / max(len(f.get(k, [])), 1)
        wb = sum(w.get(k, [0])) / max(len(w.get(k, [])), 1)
        res["kernels"][k] = {"fetch_bytes": fb, "write_bytes": wb, "traffic_bytes": fb + wb,
                             "dispatches": len(f.get(k, []))}
    Path(out).write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res["kernels"], indent=1))


if __name__ == "__main__":
    main()
