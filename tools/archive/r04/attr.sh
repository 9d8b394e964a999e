#!/bin/bash
# Kernel attribution: the default library and the variant builds named (each
# tools/build_variant.sh NAME FLAGS), each timed alone (fast_attr.py: every
# stage one after another on one stream) and counted in one rocprofv3 SQ pass.
# Usage: tools/r04/attr.sh <tag> <kernel> <variant> ...
set -eo pipefail
TAG=$1; K=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/attr_$TAG; mkdir -p "$O"; cd "$R"
V="default $*"
for v in $V; do
  lib=$R/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so
  [ "$v" != default ] && lib=$R/orb_slam2-chinese-annotation_amd/lib/variants/$v.so
  ORB_AMD_LIB=$lib timeout -k 10 120 python -u tools/r04/fast_attr.py >> "$O/times.txt" 2>> "$O/err.txt"
done
cat "$O/times.txt"
[ -n "$ATTR_NOPMC" ] && exit 0
cd /tmp && export TMPDIR=/tmp
for v in $V; do
  lib=$R/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so
  [ "$v" != default ] && lib=$R/orb_slam2-chinese-annotation_amd/lib/variants/$v.so
  ORB_AMD_LIB=$lib ATTR_CALLS=2 timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT \
    -d "$O/pmc_$v" -o run --output-format csv -- python3 "$R/tools/r04/fast_attr.py" > "$O/pmc_$v.log" 2>&1
done
cd "$R"
python3 tools/r04/pmc_kernel.py "$K" $(for v in $V; do echo "$O/pmc_$v"; done) | tee "$O/pmc.txt"
