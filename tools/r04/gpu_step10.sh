#!/bin/bash
# round-4 step 10: fixed-point resolve clocks (FP_DEBUG build); drop-in with the
# fixed-point resolve for 5,000-point maps; headline bench with the candidate
# scan reading the staged grid from global (no LDS beside the extraction)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
ORB_AMD_LIB=$R/orb_slam2-chinese-annotation_amd/lib/variants/fpdbg.so timeout -k 10 150 python -u tools/r04/fp_debug.py > "$O/s10_fpdbg.log" 2>&1 || { tail -20 "$O/s10_fpdbg.log"; exit 1; }
grep -v amdgpu.ids "$O/s10_fpdbg.log"
ORB_RESOLVE_FP_MIN=0 timeout -k 10 200 python -u tools/r04/dropin_probe.py > "$O/s10_dropin_fp.json" 2> "$O/s10_dropin_fp.err" || { tail -20 "$O/s10_dropin_fp.err"; exit 1; }
cat "$O/s10_dropin_fp.json"
for env in "" "ORB_PROJ_DIRECT=1" "" "ORB_PROJ_DIRECT=1"; do
  env $env timeout -k 10 300 python bench.py --no-cpu --no-dropin --no-secondary --host-frames 0 --steps 40 > "$O/s10_b.json" 2> "$O/s10_b.err" || { tail -20 "$O/s10_b.err"; exit 1; }
  python3 -c "import json; r=json.loads(open('$O/s10_b.json').read().strip().splitlines()[-1]); k=r['kernels']; print('[$env]', round(r['value']), {n: (v.get('ms_per_call_isolated'), v.get('ms_per_call_pipelined')) for n, v in k.items() if 'proj' in n})"
done
ATTR_NOPMC=1 bash tools/r04/attr.sh v10 k_fast_cells mw5 c192 cpw8 > "$O/s10_var.log" 2>&1 || { tail -20 "$O/s10_var.log"; exit 1; }
cat "$O/s10_var.log"
