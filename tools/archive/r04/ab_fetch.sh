#!/bin/bash
# FETCH_SIZE pass over the small bench for the base library and each variant:
# gpurun_out/abf_<tag>_<variant>/ (tools/pmc_summary.py reads them).
# Usage (GPU box): tools/ab_fetch.sh <tag> [variant ...]
set -eo pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu --no-secondary --frames 512 --steps 2 --warmup 1"
ORB_FAST_L0_INLINE=1 timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d "$O/abf_${TAG}_base" -o run \
  --output-format csv -- python3 "$R/bench.py" $ARGS > "$O/abf_${TAG}_base.log" 2>&1
for v in "$@"; do
  ORB_AMD_LIB=$R/orb_slam2-chinese-annotation_amd/lib/variants/$v.so ORB_FAST_L0_INLINE=1 \
    timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d "$O/abf_${TAG}_$v" -o run \
    --output-format csv -- python3 "$R/bench.py" $ARGS > "$O/abf_${TAG}_$v.log" 2>&1
done
echo done
