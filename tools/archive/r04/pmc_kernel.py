#!/usr/bin/env python3
"""Mean per-dispatch PMC counters of one kernel in each rocprofv3 --pmc run
directory given.  Usage: pmc_kernel.py <kernel> <dir> [<dir> ...]"""
import collections
import csv
import sys
from pathlib import Path


def kname(full):
    n = full.split("(")[0]
    n = n[5:] if n.startswith("void ") else n
    return n.split("<")[0]


kern = sys.argv[1]
for d in sys.argv[2:]:
    f = Path(d) / "run_counter_collection.csv"
    if not f.exists():
        print(f"{Path(d).name}: no counters")
        continue
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if kname(r["Kernel_Name"]) == kern:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(Path(d).name + ": " + ", ".join(f"{c} {sum(v) / len(v):.4g}" for c, v in sorted(vals.items())),
          flush=True)
