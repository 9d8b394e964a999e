#!/usr/bin/env python3
"""Per-kernel mean of every PMC counter in one or more rocprofv3 output dirs.
Usage: tools/pmc_table.py <dir> [<dir> ...]"""
import collections
import csv
import sys
from pathlib import Path


def kname(full):
    """'void k_pyr_resize<true>(...)' -> 'k_pyr_resize'"""
    n = full.split("(")[0]
    n = n[5:] if n.startswith("void ") else n
    return n.split("<")[0]

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
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
