#!/bin/bash
# Round 6 bench A/B (GPU box): bench_ab.sh OUT REPS "label:lib:ENV=V,ENV=V" ...
# lib "product" = lib/liborb_amd.so, else lib/variants/<lib>.so; the headline
# without the CPU / secondary / drop-in legs, specs interleaved REPS times.
O=$1; REPS=$2; shift 2
mkdir -p "$O"
for r in $(seq 1 $REPS); do
  for spec in "$@"; do
    IFS=: read -r label lib envs <<< "$spec"
    (
      if [ "$lib" != product ]; then export ORB_AMD_LIB=orb_slam2-chinese-annotation_amd/lib/variants/$lib.so; fi
      IFS=, ; for e in $envs; do [ -n "$e" ] && export "$e"; done
      timeout -k 10 240 python -u bench.py --no-secondary --no-cpu --no-dropin > "$O/bench_${label}_$r.log" 2>&1
    ) || { echo "FAIL $label"; tail -20 "$O/bench_${label}_$r.log"; exit 1; }
    echo "bench $label $r: $(grep -o '"value": [0-9.]*' "$O/bench_${label}_$r.log" | head -1)"
  done
done
