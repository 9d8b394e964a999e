#!/usr/bin/env python3
"""Per-kernel launch durations from a rocprofv3 kernel trace, split by grid
shape (the bench's isolated table runs each stage as one launch; its
pipelined region splits FAST into three).  Usage: trace_summary.py <trace.csv>"""
import collections
import csv
import json
import sys


def kname(full):
    n = full.split("(")[0]
    n = n[5:] if n.startswith("void ") else n
    return n


rows = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if r.get("Kind") != "KERNEL_DISPATCH":
        continue
    k = kname(r["Kernel_Name"])
    if not k.startswith("k_"):
        continue
    g = (int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), int(r["Grid_Size_Y"]),
         int(r["Workgroup_Size_X"]))
    rows[(k, g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
out = []
for (k, g), v in sorted(rows.items()):
    v.sort()
    out.append({"kernel": k, "workgroups_x": g[0], "grid_y": g[1], "workgroup_size": g[2],
                "launches": len(v), "mean_ms": sum(v) / len(v), "median_ms": v[len(v) // 2],
                "min_ms": v[0], "max_ms": v[-1]})
for o in out:
    print(json.dumps(o))
