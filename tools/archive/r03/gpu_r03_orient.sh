#!/bin/bash
# Round 3, k_orient_desc readlane fix: full GPU suite on the default build
# (one-pair calls now on k_orient_desc<1>), the extractor parity tests on the
# __launch_bounds__(256, 5) build, a short A/B bench of both variants and the
# single-frame host-API rate (<1> vs the run-time-count <0>).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
V=$R/orb_slam2-chinese-annotation_amd/lib/variants
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $PYT tests -m gpu > "$O/r03_t_default.log" 2>&1 || { echo "default suite failed"; exit 1; }
ORB_AMD_LIB=$V/desc5.so timeout -k 10 200 $PYT tests/test_gpu_extractor.py tests/test_golden.py \
  > "$O/r03_t_desc5.log" 2>&1 || { echo "desc5 parity failed"; exit 1; }
"$R/tools/ab_variants.sh" r03_desc desc5 desc0rt || exit 1
timeout -k 10 120 "$R/tools/probe/host_api_rate" 2000 > "$O/r03_host_api_ct1.txt" 2>&1 || exit 1
mkdir -p /tmp/rt0 && cp "$V/desc0rt.so" /tmp/rt0/liborb_amd.so
LD_LIBRARY_PATH=/tmp/rt0 timeout -k 10 120 "$R/tools/probe/host_api_rate" 2000 > "$O/r03_host_api_rt0.txt" 2>&1 || exit 1
echo ok
