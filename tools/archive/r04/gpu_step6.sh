#!/bin/bash
# round-4 step 6: GPU suite, the default bench line, the profile set
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$O/s6_tests.log" 2>&1 || { tail -30 "$O/s6_tests.log"; exit 1; }
tail -2 "$O/s6_tests.log"
ORB_AMD_LIB=$R/orb_slam2-chinese-annotation_amd/lib/variants/pkrot.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_golden.py tests/test_gpu_extractor.py -k "not 12k" > "$O/s6_pkrot.log" 2>&1 || { tail -30 "$O/s6_pkrot.log"; exit 1; }
tail -1 "$O/s6_pkrot.log"
ATTR_NOPMC=1 bash tools/r04/attr.sh v6 k_orient_desc pkrot > "$O/s6_var.log" 2>&1 && cat "$O/s6_var.log"
timeout -k 10 400 python -X faulthandler bench.py > "$O/s6_bench.json" 2> "$O/s6_bench.err" || { tail -30 "$O/s6_bench.err"; exit 1; }
python3 tools/r04/show_bench.py "$O/s6_bench.json"
bash tools/r04/gpu_profile.sh r04b > "$O/s6_prof.log" 2>&1 || { tail -20 "$O/s6_prof.log"; exit 1; }
echo profile done
