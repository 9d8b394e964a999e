"""One call's kernel timeline from a rocprofv3 kernel trace: the last `--calls`
groups of launches (a group = the kernels between two gaps of > --gap-us), each
kernel's start offset, duration and the gap before it, in microseconds.
Usage: timeline.py <run_kernel_trace.csv> [--last 3] [--gap-us 50]"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--last", type=int, default=3)
ap.add_argument("--gap-us", type=float, default=50.0)
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
groups, cur, prev_end = [], [], None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if prev_end is not None and s - prev_end > a.gap_us * 1e3 and cur:
        groups.append(cur)
        cur = []
    cur.append((s, e, r["Kernel_Name"].split("(")[0][:40], r.get("Grid_Size", "")))
    prev_end = e if prev_end is None else max(prev_end, e)
if cur:
    groups.append(cur)
for g in groups[-a.last:]:
    t0 = g[0][0]
    pe = t0
    print(f"-- call: {(max(e for _, e, _, _ in g) - t0) / 1e3:.1f} us, {len(g)} kernels")
    for s, e, name, grid in g:
        print(f"  +{(s - t0) / 1e3:7.1f}  {((e - s) / 1e3):6.1f} us  gap {(s - pe) / 1e3:5.1f}  {name} grid={grid}")
        pe = max(pe, e)
