#!/bin/bash
# round-4 step 1: full GPU suite, C5 stage probe, default bench line
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$O/s1_tests.log" 2>&1 || { tail -30 "$O/s1_tests.log"; exit 1; }
tail -2 "$O/s1_tests.log"
timeout -k 10 200 python -u tools/r04/c5_stages.py 16 128 > "$O/s1_c5.log" 2>&1
ORB_PROJ_WG_LARGE=512 timeout -k 10 200 python -u tools/r04/c5_stages.py 16 >> "$O/s1_c5.log" 2>&1
ORB_RESOLVE_JACOBI=0 timeout -k 10 200 python -u tools/r04/c5_stages.py 16 >> "$O/s1_c5.log" 2>&1
for R in 3; do ORB_JACOBI_ROUNDS=$R timeout -k 10 200 python -u tools/r04/c5_stages.py 16 >> "$O/s1_c5.log" 2>&1; done
cat "$O/s1_c5.log"
timeout -k 10 400 python bench.py > "$O/s1_bench.json" 2> "$O/s1_bench.err"
python - <<'PY'
import json
r=json.loads(open("gpurun_out/s1_bench.json").read().strip().splitlines()[-1])
print("value", r["value"], "roof", r["roofline"]["kernel"], r["roofline"]["frac"])
for k,v in r["kernels"].items(): print(k, {a: round(b,4) for a,b in v.items()})
print("C5", r["C5_problems_per_s"]["value"], r["C5_problems_per_s"]["match_only_problems_per_s"])
print("C3", r["C3_stereo_pairs_per_s"]["value"])
print("cpu", r["cpu_baseline"]["value"], r["cpu_baseline"]["all_cores"])
print("dropin", r.get("dropin"))
print("host", r["host_input"]["frames_per_s"])
PY
