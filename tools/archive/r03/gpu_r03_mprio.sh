#!/bin/bash
# Round 3: bench match-stream priority with the shared side stream
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
OUT=$O/mprio.txt; : > "$OUT"
for set in "ORB_BENCH_PRIO_MATCH=greatest" "ORB_BENCH_PRIO_MATCH=least" "ORB_BENCH_PRIO_MATCH=normal" "ORB_BENCH_PRIO_MATCH=greatest" "ORB_BENCH_PRIO_MATCH=least"; do
  env $set timeout -k 10 300 python "$R/bench.py" --no-cpu --steps 20 > "$O/mp_b.json" 2>/dev/null || exit 1
  python3 -c "import json;b=json.load(open('$O/mp_b.json'));print('$set bench', round(b['value']), 'C3', round(b['C3_stereo_pairs_per_s']['value']), 'C5', round(b['C5_problems_per_s']['value']), 'host', round(b['host_input']['frames_per_s']), {k:round(x,3) for k,x in b['kernels_ms_per_launch'].items()})" >> "$OUT"
done
cat "$OUT"
