#!/bin/bash
# GPU box: extractor parity of the default build, then an env-knob sweep
# (tools/sweep_env.sh).  Usage: tools/gpu_parity_sweep.sh <tag> <VAR> <v1> [v2 ...]
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_extractor.py tests/test_golden.py > "$O/${TAG}_t.log" 2>&1 || { tail -30 "$O/${TAG}_t.log"; exit 1; }
tail -1 "$O/${TAG}_t.log"
"$R/tools/sweep_env.sh" "$@" || exit 1
cat "$O/sweep_$TAG.txt"
