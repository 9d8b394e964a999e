#!/bin/bash
# Round 3: --batch 512 vs 1024, full default line, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
OUT=$O/batch2.txt; : > "$OUT"
for b in 1024 512 1024 512; do
  timeout -k 10 300 python "$R/bench.py" --no-cpu --batch $b --steps 20 --warmup 5 > "$O/batch_b.json" 2>/dev/null || exit 1
  python3 -c "import json;b=json.load(open('$O/batch_b.json'));print('batch $b', round(b['value']), round(b['ms_per_step'],3), 'C3', round(b['C3_stereo_pairs_per_s']['value']), 'C5', round(b['C5_problems_per_s']['value']), 'host', round(b['host_input']['frames_per_s']))" >> "$OUT"
done
cat "$OUT"
