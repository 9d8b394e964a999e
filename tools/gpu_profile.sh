#!/bin/bash
# Round profile recipe (run on the GPU box through gpurun from the repo root):
#   GPU parity tests, the default bench line, a rocprofv3 kernel-trace/stats
#   pass and two PMC passes (FETCH_SIZE and WRITE_SIZE cannot share a pass).
# Usage: tools/gpu_profile.sh <tag>
set -eo pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$O/tests_$TAG.log" 2>&1
timeout -k 10 400 python bench.py > "$O/bench_$TAG.json" 2> "$O/bench_$TAG.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_$TAG" -o run --output-format csv \
  -- python3 "$R/bench.py" --no-cpu --steps 10 --warmup 2 > "$O/prof_$TAG.json" 2> "$O/prof_$TAG.err"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$O/pmcf_$TAG" -o run --output-format csv \
  -- python3 "$R/bench.py" --no-cpu --steps 2 --warmup 1 > "$O/pmcf_$TAG.json" 2> "$O/pmcf_$TAG.err"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$O/pmcw_$TAG" -o run --output-format csv \
  -- python3 "$R/bench.py" --no-cpu --steps 2 --warmup 1 > "$O/pmcw_$TAG.json" 2> "$O/pmcw_$TAG.err"
echo done
