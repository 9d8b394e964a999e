#!/bin/bash
# round-4 step 19: the headline's resolve as the fixed-point kernel (256 and
# 1024 threads per problem) instead of the one-wave prefix kernel, interleaved
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
for env in "" "ORB_RESOLVE_FP_MIN=0 ORB_RESOLVE_FP=256" "ORB_RESOLVE_FP_MIN=0" "" "ORB_RESOLVE_FP_MIN=0 ORB_RESOLVE_FP=256"; do
  env $env timeout -k 10 300 python bench.py --no-cpu --no-dropin --no-secondary --host-frames 0 --steps 40 > "$O/s19_b.json" 2> "$O/s19_b.err" || { tail -20 "$O/s19_b.err"; exit 1; }
  python3 -c "import json; r=json.loads(open('$O/s19_b.json').read().strip().splitlines()[-1]); k=r['kernels']['k_proj_resolve']; print('[$env]', round(r['value']), round(k['ms_per_call_isolated'],4), round(k['ms_per_call_pipelined'],4))"
done
