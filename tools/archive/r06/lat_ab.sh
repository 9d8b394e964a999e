#!/bin/bash
# one-frame latency A/B (tools/probe/latency_probe.py) over library variants:
# lat_ab.sh OUT REPS name:lib ...  (lib "product" = lib/liborb_amd.so)
O=$1; REPS=$2; shift 2
for r in $(seq 1 $REPS); do
  for spec in "$@"; do
    IFS=: read -r name lib <<< "$spec"
    if [ "$lib" = product ]; then unset ORB_AMD_LIB; else export ORB_AMD_LIB=orb_slam2-chinese-annotation_amd/lib/variants/$lib.so; fi
    timeout -k 10 120 python -u tools/probe/latency_probe.py --calls 300 --tag "$name" >> "$O" 2>/dev/null || { echo "FAIL $name" >> "$O"; exit 1; }
  done
done
