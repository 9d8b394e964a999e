"""Print value + selected kernels' (isolated, pipelined) ms from bench_ab.sh logs.
Usage: ab_kernels.py DIR"""
import glob
import json
import sys

for f in sorted(glob.glob(sys.argv[1] + "/bench_*.log")):
    for line in open(f):
        if line.startswith('{"metric'):
            d = json.loads(line)
            k = d["kernels"]
            print(f.split("/")[-1], round(d["value"]),
                  {n: (round(v["ms_per_launch_isolated"], 3), round(v["ms_per_call_pipelined"], 3))
                   for n, v in k.items() if n in ("k_proj_candidates", "k_proj_resolve", "k_orient_desc",
                                                  "k_fast_cells", "k_octree")})
