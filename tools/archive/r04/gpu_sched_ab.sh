#!/bin/bash
# Schedule A/B in the two-lane bench, interleaved, with the C5 / C3 keys:
#   side    the default (level 0..2 FAST on the side stream)
#   inline  one stream per lane (ORB_FAST_L0_INLINE=1: FAST of every level in
#           one launch after the resize chain)
#   jac     C4's SearchByProjection through the Jacobi resolve too
#           (ORB_RESOLVE_FP_MIN=1000; default: local maps of 20,000+ points)
#   inlane  each lane runs its launch's matcher after its extraction on its own
#           stream (no match stream)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/sched; mkdir -p "$O"; cd "$R"
ARGS="--no-cpu --no-dropin --host-frames 0 --steps 40"
for v in side inline jac inlane side2; do
  E="ORB_NOTHING=1"
  [ $v = inline ] && E="ORB_FAST_L0_INLINE=1"
  [ $v = jac ] && E="ORB_RESOLVE_FP_MIN=1000"
  [ $v = inlane ] && E="ORB_BENCH_LANE_MATCH=inlane"
  env $E timeout -k 10 300 python bench.py $ARGS > "$O/$v.json" 2> "$O/$v.err"
  python3 -c "
import json; r=json.loads(open('$O/$v.json').read().strip().splitlines()[-1])
k=r['kernels']
print('$v', round(r['value']), 'C5', round(r['C5_problems_per_s']['value']), round(r['C5_problems_per_s']['match_only_problems_per_s']), 'C3', round(r['C3_stereo_pairs_per_s']['value']), {n: round(v['ms_per_call_pipelined'], 3) for n, v in k.items() if 'ms_per_call_pipelined' in v})"
done
