#!/usr/bin/env python3
"""Per-kernel mean of every PMC counter in one or more rocprofv3 output dirs.
Usage: tools/pmc_table.py [--json OUT --batch B] <dir> [<dir> ...]
With --json, also writes {"batch": B, "kernels": {kernel: {counter: mean}}}
(per-launch means, read by bench.py for the VALU issue bound)."""
import argparse
import collections
import csv
import json
from pathlib import Path


def kname(full):
    """'void k_pyr_resize<true>(...)' -> 'k_pyr_resize'"""
    n = full.split("(")[0]
    n = n[5:] if n.startswith("void ") else n
    return n.split("<")[0]


ap = argparse.ArgumentParser()
ap.add_argument("--json")
ap.add_argument("--batch", type=int, default=512)
ap.add_argument("dirs", nargs="+")
args = ap.parse_args()

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for d in args.dirs:
    for f in Path(d).glob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            if k.startswith("k_"):
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
names = sorted({c for k in vals for c in vals[k]})
print("kernel".ljust(18), " ".join(n[:14].rjust(14) for n in names))
for k in sorted(vals):
    print(k.ljust(18), " ".join(
        (f"{sum(vals[k][n]) / len(vals[k][n]):14.4g}" if vals[k][n] else " " * 14) for n in names))
if args.json:
    out = {"batch": args.batch, "unit": "counter value per launch (mean over dispatches)",
           "kernels": {k: {n: sum(v) / len(v) for n, v in sorted(vals[k].items()) if v}
                       for k in sorted(vals)}}
    Path(args.json).write_text(json.dumps(out, indent=1) + "\n")
