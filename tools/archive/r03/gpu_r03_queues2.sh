#!/bin/bash
# Round 3: how many HSA queues does the bench process create, and does C5's
# mode follow the queue count?  (AMD_LOG_LEVEL=3 acquireQueue lines)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
OUT=$O/queues2.txt; : > "$OUT"
AMD_LOG_LEVEL=3 timeout -k 10 300 python "$R/bench.py" --no-cpu --frames 2048 --steps 20 > "$O/q2_b.json" 2> "$O/q2.log" || exit 1
python3 -c "import json;b=json.load(open('$O/q2_b.json'));print('log3 bench', round(b['value']), 'C3', round(b['C3_stereo_pairs_per_s']['value']), 'C5', round(b['C5_problems_per_s']['value']))" >> "$OUT"
grep -c "acquireQueue" "$O/q2.log" >> "$OUT" || true
grep "Number of allocated hardware queues" "$O/q2.log" | tail -2 >> "$OUT" || true
grep -i "cooperative\|oversubscri\|HQD\|map" "$O/q2.log" | head -5 >> "$OUT" || true
rm -f "$O/q2.log"
for q in 2 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python "$R/bench.py" --no-cpu --frames 2048 --steps 20 > "$O/q2_b.json" 2>/dev/null || exit 1
  python3 -c "import json;b=json.load(open('$O/q2_b.json'));print('queues $q bench', round(b['value']), 'C3', round(b['C3_stereo_pairs_per_s']['value']), 'C5', round(b['C5_problems_per_s']['value']))" >> "$OUT"
done
cat "$OUT"
