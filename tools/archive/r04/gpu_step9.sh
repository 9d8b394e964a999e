#!/bin/bash
# round-4 step 9: C5 resolve without loop-head memory waits (LDS kpMatch,
# two windows of inputs in flight, slow re-scan out of line), candidate scan
# from global (ORB_PROJ_DIRECT); matcher / drop-in parity; stage A/B; drop-in
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_matcher.py tests/test_gpu_dropin.py tests/test_cpp_host.py > "$O/s9_tests.log" 2>&1 || { tail -30 "$O/s9_tests.log"; exit 1; }
tail -1 "$O/s9_tests.log"
for env in "" "ORB_PROJ_DIRECT=1" "ORB_RESOLVE_FP=512" "ORB_PROJ_DIRECT=1 ORB_RESOLVE_FP=512"; do
  env $env timeout -k 10 150 python -u tools/r04/c5_stages.py 16 >> "$O/s9_c5.log" 2>&1 || { tail -20 "$O/s9_c5.log"; exit 1; }
done
grep C5 "$O/s9_c5.log"
timeout -k 10 200 python -u tools/r04/dropin_probe.py > "$O/s9_dropin.json" 2> "$O/s9_dropin.err" || { tail -20 "$O/s9_dropin.err"; exit 1; }
cat "$O/s9_dropin.json"
