#!/bin/bash
# round-4 step 5: FAST / orient variant times (alone), then the schedule A/B
# and the PMC passes (step 4)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
ATTR_NOPMC=1 bash tools/r04/attr.sh v5 k_fast_cells q640 q640l3 q640cpw8 q640cpw2 pkrot pk5 pkdb4 pkdb db > "$O/s5_var.log" 2>&1 || { tail -20 "$O/s5_var.log"; exit 1; }
cat "$O/s5_var.log"
bash tools/r04/gpu_step4.sh
