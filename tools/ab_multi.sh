#!/bin/bash
# GPU box: extractor parity for each variant, then one A/B bench series.
# Usage: tools/ab_multi.sh <tag> <variant> [variant ...]
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
for V in "$@"; do
  ORB_AMD_LIB=$R/orb_slam2-chinese-annotation_amd/lib/variants/$V.so timeout -k 10 200 \
    python -u -m pytest tests/test_gpu_extractor.py tests/test_golden.py -x -q --timeout 120 \
    --timeout-method thread > "$R/gpurun_out/t_${TAG}_$V.log" 2>&1 || { echo "parity failed: $V"; exit 1; }
done
"$R/tools/ab_variants.sh" "$TAG" "$@"
