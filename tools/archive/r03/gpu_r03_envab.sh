#!/bin/bash
# GPU box: an environment knob A/B on the default build: extractor + golden
# parity with the knob set, extraction stage times and a short bench without
# and with it.  Usage: tools/gpu_r03_envab.sh <tag> VAR=value [VAR=value ...]
set -eo pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
cd "$R"
env "$@" timeout -k 10 300 python -u -m pytest tests/test_gpu_extractor.py tests/test_golden.py -x -q \
  --timeout 120 --timeout-method thread > "$O/t_$TAG.log" 2>&1
tail -1 "$O/t_$TAG.log"
ARGS="--no-cpu --no-secondary --frames 2048 --steps 30 --host-frames 0"
for rep in 1 2; do
  timeout -k 10 120 python tools/probe/stage_times.py --batch 512 2>/dev/null | tail -1 | sed "s/^/base: /"
  env "$@" timeout -k 10 120 python tools/probe/stage_times.py --batch 512 2>/dev/null | tail -1 | sed "s/^/knob: /"
  timeout -k 10 200 python bench.py $ARGS 2>/dev/null | python -c "import json,sys;print('bench base', round(json.loads(sys.stdin.read().strip().splitlines()[-1])['value']))"
  env "$@" timeout -k 10 200 python bench.py $ARGS 2>/dev/null | python -c "import json,sys;print('bench knob', round(json.loads(sys.stdin.read().strip().splitlines()[-1])['value']))"
done
