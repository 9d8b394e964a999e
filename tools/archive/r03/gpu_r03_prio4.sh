#!/bin/bash
# Round 3: full bench line vs (side stream, bench match stream) priorities
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
OUT=$O/prio4.txt; : > "$OUT"
for rep in 1 2; do
for set in "ORB_STREAM2_PRIO=greatest ORB_BENCH_PRIO_MATCH=least" "ORB_STREAM2_PRIO=least ORB_BENCH_PRIO_MATCH=greatest" "ORB_STREAM2_PRIO=least ORB_BENCH_PRIO_MATCH=least" "ORB_STREAM2_PRIO=least ORB_BENCH_PRIO_MATCH=normal"; do
  env $set timeout -k 10 200 python "$R/bench.py" --no-cpu > "$O/prio4_b.json" 2>/dev/null || exit 1
  python3 -c "import json;b=json.load(open('$O/prio4_b.json'));print('$set', 'bench', round(b['value']), 'C3', round(b['C3_stereo_pairs_per_s']['value']), 'C5', round(b['C5_problems_per_s']['value']), 'host', round(b['host_input']['frames_per_s']))" >> "$OUT"
done
done
cat "$OUT"
