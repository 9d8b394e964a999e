#!/bin/bash
# Occupancy / instruction-mix PMC passes over the bench (tools/pmc_table.py reads them).
# Usage: tools/gpu_pmc.sh <tag> [bench args...]
set -eo pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
# FAST as one dispatch per call: tools/build_variant.sh l0inline -DFAST_L0_INLINE=1
L0LIB=$R/orb_slam2-chinese-annotation_amd/lib/variants/l0inline.so
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu --steps 2 --warmup 1 --host-frames 0 $*"
ORB_AMD_LIB=$L0LIB timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH GRBM_GUI_ACTIVE \
  -d "$O/pmcA_$TAG" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$O/pmcA_$TAG.log" 2>&1
ORB_AMD_LIB=$L0LIB timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU \
  -d "$O/pmcB_$TAG" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$O/pmcB_$TAG.log" 2>&1
echo done  # then: tools/pmc_table.py --json profiles/rNN_pmc.json gpurun_out/pmcA_<tag> gpurun_out/pmcB_<tag>
