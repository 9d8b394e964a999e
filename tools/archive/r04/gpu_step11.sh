#!/bin/bash
# round-4 step 11: batched claim reads (fixed-point and Jacobi resolve),
# batched candidate staging, k_pyr_chain v2; parity, C5 stages, single-frame
# extraction (chain on / off), drop-in
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extractor.py tests/test_gpu_matcher.py tests/test_cpp_host.py tests/test_gpu_dropin.py > "$O/s11_tests.log" 2>&1 || { tail -30 "$O/s11_tests.log"; exit 1; }
tail -1 "$O/s11_tests.log"
for env in "" "ORB_PROJ_PPT=2" "ORB_RESOLVE_JACOBI=1 ORB_JACOBI_ROUNDS=6" "ORB_RESOLVE_JACOBI=1 ORB_JACOBI_ROUNDS=7" "ORB_PROJ_PPT=2 ORB_RESOLVE_JACOBI=1 ORB_JACOBI_ROUNDS=7"; do
  env $env timeout -k 10 150 python -u tools/r04/c5_stages.py 16 >> "$O/s11_c5.log" 2>&1 || { tail -20 "$O/s11_c5.log"; exit 1; }
done
grep C5 "$O/s11_c5.log"
for env in "ORB_PYR_CHAIN=1" "ORB_PYR_CHAIN=0" "ORB_PYR_CHAIN=1"; do
  env $env timeout -k 10 100 python -u tools/r04/single_wall.py >> "$O/s11_single.log" 2>&1 || { tail -20 "$O/s11_single.log"; exit 1; }
  env $env ATTR_BATCH=1 ATTR_CALLS=300 timeout -k 10 100 python -u tools/r04/fast_attr.py >> "$O/s11_single.log" 2>&1 || { tail -20 "$O/s11_single.log"; exit 1; }
done
grep -v amdgpu.ids "$O/s11_single.log"
timeout -k 10 200 python -u tools/r04/dropin_probe.py > "$O/s11_dropin.json" 2> "$O/s11_dropin.err" || { tail -20 "$O/s11_dropin.err"; exit 1; }
cat "$O/s11_dropin.json"
ORB_RESOLVE_FP_MIN=0 timeout -k 10 200 python -u tools/r04/dropin_probe.py > "$O/s11_dropin_fp.json" 2> "$O/s11_dropin_fp.err" || { tail -20 "$O/s11_dropin_fp.err"; exit 1; }
cat "$O/s11_dropin_fp.json"
