#!/bin/bash
# Round 3: bench streams by priority pool (extract normal, match least, side
# stream greatest): C5 repeat probe, queue log, two full bench lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
OUT=$O/streams3.txt; : > "$OUT"
timeout -k 10 200 python "$R/tools/probe/c5_swap.py" --repeat 2>/dev/null >> "$OUT" || exit 1
timeout -k 10 200 python "$R/tools/probe/c5_swap.py" 2>/dev/null >> "$OUT" || exit 1
for i in 1 2; do
  timeout -k 10 300 python "$R/bench.py" --no-cpu > "$O/streams3_b.json" 2>/dev/null || exit 1
  python3 -c "import json;b=json.load(open('$O/streams3_b.json'));print('bench', round(b['value']), 'C3', round(b['C3_stereo_pairs_per_s']['value']), 'C5', round(b['C5_problems_per_s']['value']), 'host', round(b['host_input']['frames_per_s']))" >> "$OUT"
done
ORB_BENCH_STREAMS=torch timeout -k 10 300 python "$R/bench.py" --no-cpu > "$O/streams3_b.json" 2>/dev/null || exit 1
python3 -c "import json;b=json.load(open('$O/streams3_b.json'));print('torch streams: bench', round(b['value']), 'C3', round(b['C3_stereo_pairs_per_s']['value']), 'C5', round(b['C5_problems_per_s']['value']), 'host', round(b['host_input']['frames_per_s']))" >> "$OUT"
cat "$OUT"
