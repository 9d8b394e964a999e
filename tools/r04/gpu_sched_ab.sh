#!/bin/bash
# Schedule A/B in the two-lane bench: the side stream (default) against one
# stream per lane (ORB_FAST_L0_INLINE=1: FAST of every level in one launch
# after the resize chain), interleaved, with the C5 / C3 keys.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/sched; mkdir -p "$O"; cd "$R"
ARGS="--no-cpu --no-dropin --host-frames 0 --steps 40"
for i in 1; do
  for v in side inline; do
    E=""; [ $v = inline ] && E="ORB_FAST_L0_INLINE=1"
    env $E timeout -k 10 300 python bench.py $ARGS > "$O/$v$i.json" 2> "$O/$v$i.err"
    python3 -c "
import json,sys; r=json.loads(open('$O/$v$i.json').read().strip().splitlines()[-1])
print('$v$i', round(r['value']), 'C5', round(r['C5_problems_per_s']['value']), round(r['C5_problems_per_s']['match_only_problems_per_s']), 'C3', round(r['C3_stereo_pairs_per_s']['value']))"
  done
done
