#!/bin/bash
# Sweep one environment knob: extraction-only stage times and a short bench per value.
# Usage (GPU box): tools/sweep_env.sh <tag> <VAR> <v1> [v2 ...]
set -o pipefail
TAG=$1; VAR=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
OUT=$O/sweep_$TAG.txt; : > "$OUT"
for v in "$@"; do
  export "$VAR=$v"
  echo -n "$VAR=$v stage: " >> "$OUT"
  timeout -k 10 120 python "$R/tools/probe/stage_times.py" 2>> "$O/sweep_$TAG.err" | grep B= >> "$OUT" || exit 1
  timeout -k 10 200 python "$R/bench.py" --no-cpu --no-secondary --frames 2048 --steps 30 > "$O/sweep_${TAG}_$v.json" 2>> "$O/sweep_$TAG.err" || exit 1
  python3 -c "import json;b=json.load(open('$O/sweep_${TAG}_$v.json'));print('$VAR=$v bench:', round(b['value']), round(b['extraction_call_ms_per_launch'],3), {k:round(x,3) for k,x in b['kernels_ms_per_launch'].items()})" >> "$OUT"
done
echo done
