#!/bin/bash
# GPU test pass for round 4 (run through gpurun from the repo root):
#   tools/r04/gpu_tests.sh <tag> [pytest selectors...]
set -eo pipefail
TAG=${1:-t}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd "$R"
SEL=${@:-tests}
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu $SEL \
  > "gpurun_out/tests_$TAG.log" 2>&1
tail -3 "gpurun_out/tests_$TAG.log"
