#!/bin/bash
# Round 3, k_fast_cells byte tile: extractor parity on the new build, then a
# short A/B bench against the pre-change build (lib/variants/base.so) and the
# extraction stage times of both.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
TAG=${1:-r03_fast}
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 200 $PYT tests/test_gpu_extractor.py tests/test_golden.py > "$O/${TAG}_t.log" 2>&1 || { echo "parity failed"; tail -30 "$O/${TAG}_t.log"; exit 1; }
"$R/tools/ab_variants.sh" "$TAG" base || exit 1
timeout -k 10 120 python "$R/tools/probe/stage_times.py" > "$O/${TAG}_stages_new.txt" 2>&1 || exit 1
ORB_AMD_LIB=$R/orb_slam2-chinese-annotation_amd/lib/variants/base.so timeout -k 10 120 python "$R/tools/probe/stage_times.py" > "$O/${TAG}_stages_base.txt" 2>&1 || exit 1
timeout -k 10 200 $PYT tests/test_gpu_distributed.py > "$O/${TAG}_dist.log" 2>&1 || { echo "dist tests failed"; tail -30 "$O/${TAG}_dist.log"; exit 1; }
echo ok
