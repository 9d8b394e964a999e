#!/bin/bash
# round-4 step 4: schedule A/B, then the PMC passes of the profile set
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
bash tools/r04/gpu_sched_ab.sh > "$O/s4_sched.log" 2>&1 || { tail -20 "$O/s4_sched.log"; exit 1; }
cat "$O/s4_sched.log"
bash tools/r04/gpu_profile.sh r04 > "$O/s4_prof.log" 2>&1 || { tail -20 "$O/s4_prof.log"; exit 1; }
echo profile done
