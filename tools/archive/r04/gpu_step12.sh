#!/bin/bash
# round-4 step 12: fixed-point resolve with three claim buffers (one barrier
# per round) vs two (FP_NBUF=2 variant); matcher parity; C5 stages; drop-in
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_matcher.py tests/test_cpp_host.py tests/test_gpu_dropin.py > "$O/s12_tests.log" 2>&1 || { tail -30 "$O/s12_tests.log"; exit 1; }
tail -1 "$O/s12_tests.log"
V=$R/orb_slam2-chinese-annotation_amd/lib/variants/nbuf2.so
for lib in "" "$V" "" "$V"; do
  if [ -n "$lib" ]; then export ORB_AMD_LIB=$lib; else unset ORB_AMD_LIB; fi
  timeout -k 10 150 python -u tools/r04/c5_stages.py 16 2>&1 | grep C5 | sed "s|^|${lib##*/} |" >> "$O/s12_c5.log"
done
unset ORB_AMD_LIB
cat "$O/s12_c5.log"
timeout -k 10 200 python -u tools/r04/dropin_probe.py > "$O/s12_dropin.json" 2> "$O/s12_dropin.err" || { tail -20 "$O/s12_dropin.err"; exit 1; }
cat "$O/s12_dropin.json"
