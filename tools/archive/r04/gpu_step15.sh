#!/bin/bash
# round-4 step 15: k_orient_desc at 5 waves per SIMD (DESC_MIN_WAVES=5: 96
# VGPRs, no scratch) vs the default 4; alone and in the bench, interleaved
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
V=$R/orb_slam2-chinese-annotation_amd/lib/variants/mw5.so
ORB_AMD_LIB=$V timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extractor.py -k "bit_exact or batch" > "$O/s15_tests.log" 2>&1 || { tail -30 "$O/s15_tests.log"; exit 1; }
tail -1 "$O/s15_tests.log"
ATTR_NOPMC=1 bash tools/r04/attr.sh v15 k_orient_desc mw5 > "$O/s15_var.log" 2>&1 || { tail -20 "$O/s15_var.log"; exit 1; }
cat "$O/s15_var.log"
for lib in "" "$V" "" "$V"; do
  if [ -n "$lib" ]; then export ORB_AMD_LIB=$lib; else unset ORB_AMD_LIB; fi
  timeout -k 10 300 python bench.py --no-cpu --no-dropin --no-secondary --host-frames 0 --steps 40 > "$O/s15_b.json" 2> "$O/s15_b.err" || { tail -20 "$O/s15_b.err"; exit 1; }
  python3 -c "import json; r=json.loads(open('$O/s15_b.json').read().strip().splitlines()[-1]); k=r['kernels']['k_orient_desc']; print('${lib##*/}', round(r['value']), round(k['ms_per_call_isolated'],4), round(k['ms_per_call_pipelined'],4))"
done
