#!/bin/bash
# Round 3: resize chain on a third stream (ORB_CHAIN_STREAM=1) with the side
# FAST stream at various priorities, side-levels schedule
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
timeout -k 10 200 env ORB_CHAIN_STREAM=1 ORB_STREAM2_PRIO=least python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extractor.py > "$O/chain_parity.log" 2>&1 || exit 1
bash "$R/tools/sweep_envsets.sh" chain "X=0" "ORB_CHAIN_STREAM=1 ORB_STREAM2_PRIO=least" "ORB_CHAIN_STREAM=1 ORB_STREAM2_PRIO=normal ORB_CHAIN_PRIO=greatest" "ORB_STREAM2_PRIO=least" "X=0"
