#!/bin/bash
# Extraction-only stage times (tools/probe/stage_times.py) for the base library
# and each variant, with level 0's FAST beside the resize chain and inline.
# Usage (GPU box): tools/ab_stage.sh <tag> [variant ...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
OUT=$O/abst_$TAG.txt; : > "$OUT"
for v in base "$@"; do
  if [ "$v" = base ]; then unset ORB_AMD_LIB; else export ORB_AMD_LIB=$R/orb_slam2-chinese-annotation_amd/lib/variants/$v.so; fi
  for inl in 0 1; do
    echo -n "$v inline=$inl: " >> "$OUT"
    ORB_FAST_L0_INLINE=$inl timeout -k 10 120 python "$R/tools/probe/stage_times.py" \
      2>> "$O/abst_$TAG.err" | grep B= >> "$OUT" || exit 1
  done
done
echo done
