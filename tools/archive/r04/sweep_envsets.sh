#!/bin/bash
# A/B several environment settings: extraction-only stage times and a short
# bench per setting.  Usage (GPU box): tools/sweep_envsets.sh <tag> "A=1 B=2" "A=0" ...
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
OUT=$O/sweep_$TAG.txt; : > "$OUT"
i=0
for set in "$@"; do
  i=$((i + 1))
  echo -n "[$set] stage: " >> "$OUT"
  env $set timeout -k 10 120 python "$R/tools/probe/stage_times.py" 2>> "$O/sweep_$TAG.err" | grep B= >> "$OUT" || exit 1
  env $set timeout -k 10 200 python "$R/bench.py" --no-cpu --no-secondary --frames 2048 --steps 30 --host-frames 0 > "$O/sweep_${TAG}_$i.json" 2>> "$O/sweep_$TAG.err" || exit 1
  python3 -c "import json;b=json.load(open('$O/sweep_${TAG}_$i.json'));print('[$set] bench:', round(b['value']), round(b['extraction_call_ms_per_launch'],3), {k:round(x,3) for k,x in b['kernels_ms_per_launch'].items()})" >> "$OUT"
done
cat "$OUT"
