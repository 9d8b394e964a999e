#!/bin/bash
# Round 3: k_orient_desc row sums packed by v_perm (default) vs before (variant
# or1); then the side-levels split re-swept with the faster FAST
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extractor.py tests/test_golden.py > "$O/or2_parity.log" 2>&1 || exit 1
OUT=$O/or2.txt; tail -1 "$O/or2_parity.log" > "$OUT"
for v in new or1 new or1; do
  if [ $v = new ]; then L=""; else L="ORB_AMD_LIB=$R/orb_slam2-chinese-annotation_amd/lib/variants/$v.so"; fi
  env $L timeout -k 10 120 python "$R/tools/probe/stage_times.py" 2>/dev/null | grep B= | sed "s/^/$v /" >> "$OUT" || exit 1
  env $L timeout -k 10 300 python "$R/bench.py" --no-cpu --no-secondary --host-frames 0 --steps 20 > "$O/or_b.json" 2>/dev/null || exit 1
  python3 -c "import json;b=json.load(open('$O/or_b.json'));print('$v bench', round(b['value']), {k:round(x,3) for k,x in b['kernels_ms_per_launch'].items()})" >> "$OUT"
done
for n in 1 3 4 2; do
  ORB_FAST_SIDE_LEVELS=$n timeout -k 10 120 python "$R/tools/probe/stage_times.py" 2>/dev/null | grep B= | sed "s/^/side$n /" >> "$OUT" || exit 1
  ORB_FAST_SIDE_LEVELS=$n timeout -k 10 300 python "$R/bench.py" --no-cpu --no-secondary --host-frames 0 --steps 20 > "$O/or_b.json" 2>/dev/null || exit 1
  python3 -c "import json;b=json.load(open('$O/or_b.json'));print('side$n bench', round(b['value']))" >> "$OUT"
done
cat "$OUT"
