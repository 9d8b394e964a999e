#!/bin/bash
# round-4 step 2: k_fast_cells / k_orient_desc attribution builds
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
bash tools/r04/attr.sh fast k_fast_cells tight0 q640 q640c128 fstub1 fstub2 fstub3 fstub4 fstub5 > "$O/s2_fattr.log" 2>&1 || { tail -20 "$O/s2_fattr.log"; exit 1; }
tail -22 "$O/s2_fattr.log"
bash tools/r04/attr.sh orient k_orient_desc pkrot dstub1 dstub2 dstub3 dstub4 dstub5 > "$O/s2_oattr.log" 2>&1 || { tail -20 "$O/s2_oattr.log"; exit 1; }
tail -16 "$O/s2_oattr.log"
