#!/bin/bash
# round-4 step 8: drop-in timing after CopyDescriptor; kernel variants alone;
# bench launch-size A/B
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dropin.py tests/test_cpp_host.py > "$O/s8_tests.log" 2>&1 || { tail -30 "$O/s8_tests.log"; exit 1; }
tail -1 "$O/s8_tests.log"
timeout -k 10 200 python -u tools/r04/dropin_probe.py > "$O/s8_dropin.json" 2> "$O/s8_dropin.err" || { tail -20 "$O/s8_dropin.err"; exit 1; }
cat "$O/s8_dropin.json"
ATTR_NOPMC=1 bash tools/r04/attr.sh v8 k_fast_cells mw5 c192 cpw8 > "$O/s8_var.log" 2>&1 || { tail -20 "$O/s8_var.log"; exit 1; }
cat "$O/s8_var.log"
for b in 1024 2048 512 1024; do
  timeout -k 10 300 python bench.py --no-cpu --no-dropin --no-secondary --host-frames 0 --steps 40 --batch $b > "$O/s8_b$b.json" 2> "$O/s8_b$b.err"
  python3 -c "import json; r=json.loads(open('$O/s8_b$b.json').read().strip().splitlines()[-1]); print('batch $b', round(r['value']))"
done
