#!/bin/bash
# GPU box: parity of one library variant (extractor tests) then a short A/B
# bench against the default build.  Usage: tools/run_ab.sh <tag> <variant>
TAG=$1; V=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
ORB_AMD_LIB=$R/orb_slam2-chinese-annotation_amd/lib/variants/$V.so timeout -k 10 200 \
  python -u -m pytest tests/test_gpu_extractor.py tests/test_golden.py -x -q --timeout 120 \
  --timeout-method thread > "$R/gpurun_out/t_$TAG.log" 2>&1 || exit 1
"$R/tools/ab_variants.sh" "$TAG" "$V"
