#!/bin/bash
# round-4 step 2: k_fast_cells / k_orient_desc attribution builds, schedule A/B
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
bash tools/r04/attr.sh fast k_fast_cells tight0 q640 q640c128 fstub1 fstub2 fstub3 fstub4 fstub5 > "$O/s1_fattr.log" 2>&1 || { tail -20 "$O/s1_fattr.log"; exit 1; }
tail -20 "$O/s1_fattr.log"
bash tools/r04/attr.sh orient k_orient_desc pkrot dstub1 dstub2 dstub3 dstub4 dstub5 > "$O/s1_oattr.log" 2>&1 || { tail -20 "$O/s1_oattr.log"; exit 1; }
tail -14 "$O/s1_oattr.log"
bash tools/r04/gpu_sched_ab.sh > "$O/s1_sched.log" 2>&1 || { tail -20 "$O/s1_sched.log"; exit 1; }
cat "$O/s1_sched.log"
