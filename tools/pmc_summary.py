#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) into per-kernel HBM
bytes per launch, the `traffic` figure bench.py reports.

Usage: tools/pmc_summary.py <fetch_dir> <write_dir> <batch> <out.json>

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  FETCH_SIZE is doubled: on
gfx950 it reports half the bytes of every load shape the kernels use --
dword, 16-B and 64-B-per-lane reads of a known 1 GiB all read back as 0.5 GiB
(tools/probe/fetch_calib.hip, profiles/r02_fetch_calib.txt).  WRITE_SIZE is
used raw (exact for the same probe's dword and 16-B stores).
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
            scale = 2.0 if counter == "FETCH_SIZE" else 1.0  # calibrated, see above
            vals[kname(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0 * scale)
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
