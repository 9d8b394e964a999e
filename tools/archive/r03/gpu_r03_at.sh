#!/bin/bash
# Round 3: branchless fastAtan2 (default) vs before (variant pre_at); resolve
# waves per problem for C4 (ORB_RESOLVE_NW 1 / 2 / 4)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extractor.py tests/test_golden.py tests/test_gpu_matcher.py > "$O/at_parity.log" 2>&1 || exit 1
OUT=$O/at.txt; tail -1 "$O/at_parity.log" > "$OUT"
ORB_RESOLVE_NW=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matcher.py > "$O/at_parity1.log" 2>&1 || exit 1
tail -1 "$O/at_parity1.log" >> "$OUT"
for v in new pre_at new pre_at; do
  if [ $v = new ]; then L=""; else L="ORB_AMD_LIB=$R/orb_slam2-chinese-annotation_amd/lib/variants/$v.so"; fi
  env $L timeout -k 10 120 python "$R/tools/probe/stage_times.py" 2>/dev/null | grep B= | sed "s/^/$v /" >> "$OUT" || exit 1
  env $L timeout -k 10 300 python "$R/bench.py" --no-cpu --no-secondary --host-frames 0 --steps 20 > "$O/at_b.json" 2>/dev/null || exit 1
  python3 -c "import json;b=json.load(open('$O/at_b.json'));print('$v bench', round(b['value']), {k:round(x,3) for k,x in b['kernels_ms_per_launch'].items()})" >> "$OUT"
done
for nw in 1 2 4 1; do
  ORB_RESOLVE_NW=$nw timeout -k 10 300 python "$R/bench.py" --no-cpu --no-secondary --host-frames 0 --steps 20 > "$O/at_b.json" 2>/dev/null || exit 1
  python3 -c "import json;b=json.load(open('$O/at_b.json'));print('nw$nw bench', round(b['value']), {k:round(x,3) for k,x in b['kernels_ms_per_launch'].items()})" >> "$OUT"
done
cat "$OUT"
