#!/bin/bash
# Round 3: frames per extraction launch (bench --batch) A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
OUT=$O/batch.txt; : > "$OUT"
for b in 512 1024 2048 256 512; do
  timeout -k 10 300 python "$R/bench.py" --no-cpu --no-secondary --host-frames 0 --batch $b > "$O/batch_b.json" 2>/dev/null || exit 1
  python3 -c "import json;b=json.load(open('$O/batch_b.json'));print('batch $b', round(b['value']), round(b['ms_per_step'],3), {k:round(v,3) for k,v in b['kernels_ms_per_launch'].items()})" >> "$OUT"
done
for b in 512 1024 2048; do
  timeout -k 10 120 python "$R/tools/probe/stage_times.py" --batch $b 2>/dev/null | grep B= >> "$OUT" || exit 1
done
cat "$OUT"
