#!/bin/bash
# Round 3: k_fast_cells with a row-major candidate queue and keys written by NMS
# in place (default build) vs the bitmap + compaction path (variant fcold)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extractor.py tests/test_golden.py tests/test_gpu_dropin.py > "$O/rm_parity.log" 2>&1 || exit 1
OUT=$O/rowmajor.txt; tail -1 "$O/rm_parity.log" > "$OUT"
for v in new fcold new fcold; do
  if [ $v = new ]; then L=""; else L="ORB_AMD_LIB=$R/orb_slam2-chinese-annotation_amd/lib/variants/$v.so"; fi
  env $L timeout -k 10 120 python "$R/tools/probe/stage_times.py" 2>/dev/null | grep B= | sed "s/^/$v /" >> "$OUT" || exit 1
  env $L timeout -k 10 300 python "$R/bench.py" --no-cpu --no-secondary --host-frames 0 --steps 20 > "$O/rm_b.json" 2>/dev/null || exit 1
  python3 -c "import json;b=json.load(open('$O/rm_b.json'));print('$v bench', round(b['value']), {k:round(x,3) for k,x in b['kernels_ms_per_launch'].items()})" >> "$OUT"
done
cat "$OUT"
