#!/bin/bash
# Round 3: full GPU suite, then HIP hardware-queue count A/B (the bench uses
# ~6 streams against the default 4 queues per process) and the C3/C5
# reconciliation (tools/bench_configs.py standalone vs bench.py's secondaries).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > "$O/tests_r03.log" 2>&1 || { tail -30 "$O/tests_r03.log"; exit 1; }
tail -n 1 "$O/tests_r03.log"
bash "$R/tools/sweep_envsets.sh" r03_hwq "GPU_MAX_HW_QUEUES=4" "GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=16" "GPU_MAX_HW_QUEUES=4" || exit 1
timeout -k 10 300 python "$R/tools/bench_configs.py" --configs C3,C5 --steps 20 > "$O/r03_configs_c3c5.jsonl" 2> "$O/r03_configs_c3c5.err" || exit 1
timeout -k 10 300 python "$R/bench.py" --no-cpu --frames 2048 --steps 20 --host-frames 0 > "$O/r03_bench_sec.json" 2> "$O/r03_bench_sec.err" || exit 1
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python "$R/bench.py" --no-cpu --frames 2048 --steps 20 --host-frames 0 > "$O/r03_bench_sec16.json" 2> "$O/r03_bench_sec16.err" || exit 1
cat "$O/r03_configs_c3c5.jsonl"
python3 -c "
import json
for f in ('r03_bench_sec.json','r03_bench_sec16.json'):
    b=json.load(open('$O/'+f)); print(f, round(b['value']), b['C3_stereo_pairs_per_s']['value'], b['C5_problems_per_s']['value'])
"
