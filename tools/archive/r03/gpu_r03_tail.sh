#!/bin/bash
# Round 3: split tail (side stream also runs octree + orient of levels 0..2)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
ORB_SIDE_TAIL=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_extractor.py tests/test_golden.py tests/test_gpu_matcher.py > "$O/tail_parity.log" 2>&1 || exit 1
bash "$R/tools/sweep_envsets.sh" tail "X=0" "ORB_SIDE_TAIL=1" "ORB_SIDE_TAIL=1 ORB_FAST_SIDE_LEVELS=1" "ORB_SIDE_TAIL=1 ORB_FAST_SIDE_LEVELS=3" "X=0"
