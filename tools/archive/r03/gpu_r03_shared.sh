#!/bin/bash
# Round 3: one side stream per device shared by all extractor handles
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
OUT=$O/shared.txt; : > "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extractor.py tests/test_gpu_concurrency.py > "$O/shared_parity.log" 2>&1 || exit 1
tail -1 "$O/shared_parity.log" >> "$OUT"
AMD_LOG_LEVEL=3 timeout -k 10 300 python "$R/bench.py" --no-cpu > "$O/sh_b.json" 2> "$O/sh.log" || exit 1
python3 -c "import json;b=json.load(open('$O/sh_b.json'));print('log3 bench', round(b['value']), 'C3', round(b['C3_stereo_pairs_per_s']['value']), 'C5', round(b['C5_problems_per_s']['value']), 'host', round(b['host_input']['frames_per_s']))" >> "$OUT"
grep "Number of allocated hardware queues" "$O/sh.log" | tail -1 >> "$OUT" || true
rm -f "$O/sh.log"
for set in "X=0" "X=0" "ORB_SIDE_SHARED=0" "GPU_MAX_HW_QUEUES=2"; do
  env $set timeout -k 10 300 python "$R/bench.py" --no-cpu > "$O/sh_b.json" 2>/dev/null || exit 1
  python3 -c "import json;b=json.load(open('$O/sh_b.json'));print('$set bench', round(b['value']), 'C3', round(b['C3_stereo_pairs_per_s']['value']), 'C5', round(b['C5_problems_per_s']['value']), 'host', round(b['host_input']['frames_per_s']))" >> "$OUT"
done
cat "$OUT"
