"""Which kernels run beside which in bench.py's timed region, from a rocprofv3
kernel trace (--kernel-trace --output-format csv): per queue, the busy time of
each kernel family, and for the pairs of families on different queues the time
they overlap, over the timed region (the longest run of the match stream's
k_proj_resolve launches less than --gap-ms apart).
Usage: lane_phase.py <kernel_trace.csv> [--gap-ms 6]"""
import argparse
import csv
import collections

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--gap-ms", type=float, default=6.0)
a = ap.parse_args()
rows = list(csv.DictReader(open(a.trace)))
qkey = "Queue_Id" if "Queue_Id" in rows[0] else ("Stream_Id" if "Stream_Id" in rows[0] else None)


def fam(name):
    n = name.split("(")[0].replace("void ", "")
    return n.split("<")[0]


ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), fam(r["Kernel_Name"]),
              r.get(qkey, "?") if qkey else "?") for r in rows), key=lambda k: k[0])
res = [k for k in ks if k[2] == "k_proj_resolve"]
best, cur = (0, 0), 0
for i in range(1, len(res)):
    if res[i][0] - res[i - 1][0] > a.gap_ms * 1e6:
        cur = i
    if i - cur > best[1] - best[0]:
        best = (cur, i)
t0, t1 = res[best[0]][0], res[best[1]][1]
win = [k for k in ks if k[0] >= t0 and k[1] <= t1]
span = (t1 - t0) / 1e6
print(f"timed region: {best[1] - best[0] + 1} resolves, {span:.2f} ms, {len(win)} kernels; "
      f"{span / max(1, best[1] - best[0] + 1):.3f} ms per resolve")
busy = collections.defaultdict(float)
for s, e, f, q in win:
    busy[(q, f)] += (e - s) / 1e6
for (q, f), v in sorted(busy.items()):
    print(f"  queue {q:>4} {f:22s} busy {v:8.2f} ms ({100 * v / span:5.1f} %)")
# pairwise overlap of families on different queues (sweep over intervals)
ov = collections.defaultdict(float)
byq = collections.defaultdict(list)
for k in win:
    byq[k[3]].append(k)
qs = sorted(byq)
for i, qa in enumerate(qs):
    for qb in qs[i + 1:]:
        A, B = byq[qa], byq[qb]
        j = 0
        for s, e, f, _ in A:
            while j < len(B) and B[j][1] <= s:
                j += 1
            m = j
            while m < len(B) and B[m][0] < e:
                o = min(e, B[m][1]) - max(s, B[m][0])
                if o > 0:
                    ov[(qa, f, qb, B[m][2])] += o / 1e6
                m += 1
print("overlap (ms) of family pairs on different queues, >= 2 % of the region:")
for (qa, fa, qb, fb), v in sorted(ov.items(), key=lambda x: -x[1]):
    if v >= 0.02 * span:
        print(f"  {qa:>4}:{fa:22s} x {qb:>4}:{fb:22s} {v:8.2f}")
