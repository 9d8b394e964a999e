#!/bin/bash
# GPU box: extractor + golden parity of the default build, extraction stage
# times of the default build and of each variant, then the bench A/B.
# Usage: tools/gpu_r03_ab.sh <tag> <variant> ...
set -eo pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_extractor.py tests/test_golden.py -x -q \
  --timeout 120 --timeout-method thread > "$O/t_$TAG.log" 2>&1
tail -1 "$O/t_$TAG.log"
for v in "$@"; do  # each variant's extractor + golden parity too
  ORB_AMD_LIB=$R/orb_slam2-chinese-annotation_amd/lib/variants/$v.so timeout -k 10 300 \
    python -u -m pytest tests/test_gpu_extractor.py tests/test_golden.py -x -q \
    --timeout 120 --timeout-method thread > "$O/t_${TAG}_$v.log" 2>&1
  echo "$v: $(tail -1 "$O/t_${TAG}_$v.log")"
done
timeout -k 10 120 python tools/probe/stage_times.py --batch 512 > "$O/st_${TAG}_base.txt" 2>&1
for v in "$@"; do
  ORB_AMD_LIB=$R/orb_slam2-chinese-annotation_amd/lib/variants/$v.so timeout -k 10 120 \
    python tools/probe/stage_times.py --batch 512 > "$O/st_${TAG}_$v.txt" 2>&1
done
tools/ab_variants.sh "$TAG" "$@"
for f in "$O"/st_${TAG}_*.txt; do echo "== $f"; tail -12 "$f"; done
python tools/ab_show.py "$O/ab_$TAG.jsonl" 2>/dev/null || cat "$O/ab_$TAG.jsonl" | cut -c1-200
