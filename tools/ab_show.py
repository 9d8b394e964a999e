#!/usr/bin/env python3
"""Summarise gpurun_out/ab_<tag>.jsonl (tools/ab_variants.sh)."""
import json
import sys

for line in open(sys.argv[1]):
    r = json.loads(line)
    b = r["bench"]
    k = {n: round(v, 3) for n, v in b["kernels_ms_per_launch"].items()}
    print(f'{r["variant"]:>10} {b["value"]:10.0f} fr/s  call {b.get("extraction_call_ms_per_launch", 0):.3f} ms  {k}')
