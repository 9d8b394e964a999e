#!/bin/bash
# Round 3: the secondary configurations through the shared, pipelined
# workloads: tools/bench_configs.py (with oracle checks) and bench.py's keys.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
timeout -k 10 300 python "$R/tools/bench_configs.py" --configs ${1:-C3,C5,C4M} --steps 20 > "$O/r03_configs.jsonl" 2> "$O/r03_configs.err" || exit 1
timeout -k 10 300 python "$R/bench.py" --no-cpu --frames 2048 --steps 20 > "$O/r03_bench_sec.json" 2> "$O/r03_bench_sec.err" || exit 1
cat "$O/r03_configs.jsonl"
python3 -c "
import json
b = json.load(open('$O/r03_bench_sec.json'))
print(round(b['value']), b['C3_stereo_pairs_per_s']['value'], b['C5_problems_per_s']['value'], b['host_input']['frames_per_s'])
"
