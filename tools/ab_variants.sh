#!/bin/bash
# A/B the library variants under lib/variants/ (tools/build_variant.sh) with a
# short bench each; one JSON line per variant in gpurun_out/ab_<tag>.jsonl.
# Usage (GPU box): tools/ab_variants.sh <tag> [variant ...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
OUT=$O/ab_$TAG.jsonl; : > "$OUT"
ARGS="--no-cpu --no-secondary --frames 2048 --steps 30"
timeout -k 10 200 python "$R/bench.py" $ARGS > "$O/ab_base.json" 2>> "$O/ab_$TAG.err" || exit 1
echo "{\"variant\": \"base\", \"bench\": $(cat "$O/ab_base.json")}" >> "$OUT"
for v in "$@"; do
  ORB_AMD_LIB=$R/orb_slam2-chinese-annotation_amd/lib/variants/$v.so \
    timeout -k 10 200 python "$R/bench.py" $ARGS > "$O/ab_$v.json" 2>> "$O/ab_$TAG.err" || exit 1
  echo "{\"variant\": \"$v\", \"bench\": $(cat "$O/ab_$v.json")}" >> "$OUT"
done
echo done
