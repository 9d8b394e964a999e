#!/bin/bash
# k_fast_cells attribution: the default library and the FC_STUB=1..5 builds
# (tools/build_variant.sh fstubK "-DFC_STUB=K"), each timed alone
# (fast_attr.py) and counted in one rocprofv3 SQ pass.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/fattr; mkdir -p "$O"; cd "$R"
V="default tight0 fstub1 fstub2 fstub3 fstub4 fstub5"
for v in $V; do
  lib=$R/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so
  [ "$v" != default ] && lib=$R/orb_slam2-chinese-annotation_amd/lib/variants/$v.so
  ORB_AMD_LIB=$lib timeout -k 10 120 python -u tools/r04/fast_attr.py >> "$O/times.txt" 2>> "$O/err.txt"
done
cat "$O/times.txt"
cd /tmp && export TMPDIR=/tmp
for v in $V; do
  lib=$R/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so
  [ "$v" != default ] && lib=$R/orb_slam2-chinese-annotation_amd/lib/variants/$v.so
  ORB_AMD_LIB=$lib ATTR_CALLS=2 timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT \
    -d "$O/pmc_$v" -o run --output-format csv -- python3 "$R/tools/r04/fast_attr.py" > "$O/pmc_$v.log" 2>&1
done
cd "$R"
python3 tools/r04/pmc_kernel.py k_fast_cells $(for v in $V; do echo "$O/pmc_$v"; done) | tee "$O/pmc.txt"
