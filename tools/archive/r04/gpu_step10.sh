#!/bin/bash
# round-4 step 10: the one-launch resize chain for single frames (extractor
# parity, drop-in timing); fixed-point resolve clocks (FP_DEBUG build); drop-in with the
# fixed-point resolve for 5,000-point maps; headline bench with the candidate
# scan reading the staged grid from global (no LDS beside the extraction)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extractor.py tests/test_gpu_matcher.py tests/test_cpp_host.py > "$O/s10_tests.log" 2>&1 || { tail -30 "$O/s10_tests.log"; exit 1; }
tail -1 "$O/s10_tests.log"
for env in "" "ORB_PROJ_PPT=2" "ORB_RESOLVE_FP_PPT=2" "ORB_RESOLVE_FP_PPT=4" "ORB_RESOLVE_JACOBI=1 ORB_JACOBI_ROUNDS=7" "ORB_RESOLVE_JACOBI=1 ORB_JACOBI_ROUNDS=10"; do
  env $env timeout -k 10 150 python -u tools/r04/c5_stages.py 16 >> "$O/s10_c5.log" 2>&1 || { tail -20 "$O/s10_c5.log"; exit 1; }
done
grep C5 "$O/s10_c5.log"
ORB_AMD_LIB=$R/orb_slam2-chinese-annotation_amd/lib/variants/fpdbg.so timeout -k 10 150 python -u tools/r04/fp_debug.py > "$O/s10_fpdbg.log" 2>&1 || { tail -20 "$O/s10_fpdbg.log"; exit 1; }
grep -v amdgpu.ids "$O/s10_fpdbg.log"
ORB_RESOLVE_FP_MIN=0 timeout -k 10 200 python -u tools/r04/dropin_probe.py > "$O/s10_dropin_fp.json" 2> "$O/s10_dropin_fp.err" || { tail -20 "$O/s10_dropin_fp.err"; exit 1; }
cat "$O/s10_dropin_fp.json"
for env in "" "ORB_PROJ_DIRECT=1" "" "ORB_PROJ_DIRECT=1"; do
  env $env timeout -k 10 300 python bench.py --no-cpu --no-dropin --no-secondary --host-frames 0 --steps 40 > "$O/s10_b.json" 2> "$O/s10_b.err" || { tail -20 "$O/s10_b.err"; exit 1; }
  python3 -c "import json; r=json.loads(open('$O/s10_b.json').read().strip().splitlines()[-1]); k=r['kernels']; print('[$env]', round(r['value']), {n: (v.get('ms_per_call_isolated'), v.get('ms_per_call_pipelined')) for n, v in k.items() if 'proj' in n})"
done
ATTR_NOPMC=1 bash tools/r04/attr.sh v10 k_fast_cells wpe0 wpe8 cpw8 > "$O/s10_var.log" 2>&1 || { tail -20 "$O/s10_var.log"; exit 1; }
cat "$O/s10_var.log"
cd /tmp && export TMPDIR=/tmp
ORB_RESOLVE_JACOBI=1 ORB_JACOBI_ROUNDS=8 timeout -k 10 150 rocprofv3 --kernel-trace --stats -d "$O/s10_jac" -o run --output-format csv -- python3 "$R/tools/r04/c5_stages.py" 16 > "$O/s10_jac.log" 2>&1 || { tail -20 "$O/s10_jac.log"; exit 1; }
cd "$R"
grep C5 "$O/s10_jac.log"
f=$(find "$O/s10_jac" -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 "$f" | head -25
