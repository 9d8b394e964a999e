#!/bin/bash
# Round 3: is C5's slow mode tied to the extractor's side stream?  C5 repeat
# probe and full bench lines with level 0's FAST inline (no side stream).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
OUT=$O/inline.txt; : > "$OUT"
for set in "ORB_FAST_L0_INLINE=1" "X=0"; do
  echo "== $set" >> "$OUT"
  env $set timeout -k 10 200 python "$R/tools/probe/c5_swap.py" --repeat 2>/dev/null >> "$OUT" || exit 1
  for i in 1 2; do
    env $set timeout -k 10 300 python "$R/bench.py" --no-cpu > "$O/inline_b.json" 2>/dev/null || exit 1
    python3 -c "import json;b=json.load(open('$O/inline_b.json'));print('bench', round(b['value']), 'C3', round(b['C3_stereo_pairs_per_s']['value']), 'C5', round(b['C5_problems_per_s']['value']), 'host', round(b['host_input']['frames_per_s']))" >> "$OUT"
  done
done
cat "$OUT"
