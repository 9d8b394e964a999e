#!/bin/bash
# round-4 step 3: the default bench line, then the profile set (trace + PMC)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
timeout -k 10 400 python -X faulthandler bench.py > "$O/s3_bench.json" 2> "$O/s3_bench.err" || { tail -30 "$O/s3_bench.err"; exit 1; }
python3 tools/r04/show_bench.py "$O/s3_bench.json"
bash tools/r04/gpu_profile.sh r04 > "$O/s3_prof.log" 2>&1 || { tail -20 "$O/s3_prof.log"; exit 1; }
cat "$O/profr04/trace_summary.jsonl" | head -40
