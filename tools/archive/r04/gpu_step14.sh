#!/bin/bash
# round-4 step 14: candidate scan with each point's record and descriptor
# loaded before the grid staging; matcher parity; C5 stages; headline bench
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_matcher.py tests/test_gpu_dropin.py tests/test_gpu_mapping.py > "$O/s14_tests.log" 2>&1 || { tail -30 "$O/s14_tests.log"; exit 1; }
tail -1 "$O/s14_tests.log"
for env in "" "ORB_PROJ_PPT=2" "ORB_RESOLVE_JACOBI=1 ORB_JACOBI_ROUNDS=6"; do
  env $env timeout -k 10 150 python -u tools/r04/c5_stages.py 16 >> "$O/s14_c5.log" 2>&1 || { tail -20 "$O/s14_c5.log"; exit 1; }
done
grep C5 "$O/s14_c5.log"
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu --no-dropin --no-secondary --host-frames 0 --steps 40 > "$O/s14_b.json" 2> "$O/s14_b.err" || { tail -20 "$O/s14_b.err"; exit 1; }
  python3 -c "import json; r=json.loads(open('$O/s14_b.json').read().strip().splitlines()[-1]); k=r['kernels']; print(round(r['value']), {n: (round(v['ms_per_call_isolated'],4), round(v['ms_per_call_pipelined'],4)) for n, v in k.items() if 'proj' in n})"
done
