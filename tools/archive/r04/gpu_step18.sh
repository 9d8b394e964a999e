#!/bin/bash
# round-4 step 18: map points per candidate-scan workgroup for the headline's
# 5,000-point maps (PROJ_WG 512 default vs 1024 / 256 variants), interleaved
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
VD=$R/orb_slam2-chinese-annotation_amd/lib/variants
for lib in "" "$VD/pw1024.so" "$VD/pw256.so" "" "$VD/pw1024.so" "$VD/pw256.so"; do
  if [ -n "$lib" ]; then export ORB_AMD_LIB=$lib; else unset ORB_AMD_LIB; fi
  timeout -k 10 300 python bench.py --no-cpu --no-dropin --no-secondary --host-frames 0 --steps 40 > "$O/s18_b.json" 2> "$O/s18_b.err" || { tail -20 "$O/s18_b.err"; exit 1; }
  python3 -c "import json; r=json.loads(open('$O/s18_b.json').read().strip().splitlines()[-1]); k=r['kernels']['k_proj_candidates']; print('${lib##*/}', round(r['value']), round(k['ms_per_call_isolated'],4), round(k['ms_per_call_pipelined'],4))"
done
