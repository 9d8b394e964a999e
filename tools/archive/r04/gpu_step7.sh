#!/bin/bash
# round-4 step 7: matcher / drop-in tests and the drop-in timing
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dropin.py tests/test_gpu_matcher.py tests/test_cpp_host.py tests/test_gpu_concurrency.py > "$O/s7_tests.log" 2>&1 || { tail -30 "$O/s7_tests.log"; exit 1; }
tail -1 "$O/s7_tests.log"
timeout -k 10 200 python -u tools/r04/dropin_probe.py > "$O/s7_dropin.json" 2> "$O/s7_dropin.err" || { tail -20 "$O/s7_dropin.err"; exit 1; }
cat "$O/s7_dropin.json"
