#!/bin/bash
# round-4 final pass: the whole GPU suite, then the default bench line
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
bash tools/r04/gpu_tests.sh final
timeout -k 10 600 python -u bench.py > "$O/final_bench.json" 2> "$O/final_bench.err" || { tail -20 "$O/final_bench.err"; exit 1; }
python3 tools/r04/show_bench.py "$O/final_bench.json" || tail -c 3000 "$O/final_bench.json"
