#!/bin/bash
# Round 3: isolate the C5 gap between bench.py and tools/bench_configs.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
timeout -k 10 200 python "$R/tools/probe/c5_probe.py" 2>/dev/null || exit 1
timeout -k 10 300 python "$R/bench.py" --no-cpu --frames 512 --steps 2 --host-frames 0 > "$O/r03_c5_small.json" 2>/dev/null || exit 1
python3 -c "import json; b=json.load(open('$O/r03_c5_small.json')); print('bench.py tiny main then C5', round(b['C5_problems_per_s']['value']), round(b['C3_stereo_pairs_per_s']['value']))"
timeout -k 10 300 python "$R/bench.py" --no-cpu --frames 8192 --steps 60 --host-frames 0 > "$O/r03_c5_big.json" 2>/dev/null || exit 1
python3 -c "import json; b=json.load(open('$O/r03_c5_big.json')); print('bench.py default main then C5', round(b['value']), round(b['C5_problems_per_s']['value']), round(b['C3_stereo_pairs_per_s']['value']))"
