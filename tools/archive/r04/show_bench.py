#!/usr/bin/env python3
"""Print the headline keys of a bench.py JSON line (last line of the file)."""
import json
import sys

r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", round(r["value"]), "ms/step", round(r["ms_per_step"], 3), "n_gpus", r["n_gpus"])
ro = r["roofline"]
print("roofline", ro["kernel"], "frac", round(ro["frac"], 4), "achieved", round(ro["achieved"], 1),
      "ms", round(ro["ms_per_launch"], 4), "pipelined", ro.get("ms_per_launch_pipelined"))
for k, v in r.get("kernels", {}).items():
    print(" ", k, {a: round(b, 4) for a, b in v.items()})
for key in ("C5_problems_per_s", "C3_stereo_pairs_per_s"):
    if key in r:
        c = r[key]
        print(key, round(c["value"]), {a: round(b) for a, b in c.items()
                                       if a.startswith("match_only_problems")})
if "cpu_baseline" in r:
    c = r["cpu_baseline"]
    print("cpu 1-thread", round(c["value"], 2), "all-cores", c.get("all_cores"))
print("dropin", json.dumps(r.get("dropin")))
if r.get("host_input"):
    print("host_input", round(r["host_input"]["frames_per_s"]))
