#!/bin/bash
# Round 3: orient loop restructure -- parity, A/B against the previous build
# (pre_orient) and the level-lookup-only build (oneblock0), stage times; then
# the secondary configurations (tools/gpu_r03_configs.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
V=$R/orb_slam2-chinese-annotation_amd/lib/variants
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extractor.py tests/test_golden.py tests/test_gpu_dropin.py > "$O/r03_or2_t.log" 2>&1 || { tail -30 "$O/r03_or2_t.log"; exit 1; }
tail -n 1 "$O/r03_or2_t.log"
"$R/tools/ab_variants.sh" r03_or2 pre_orient oneblock0 || exit 1
for v in new pre_orient; do
  if [ $v = new ]; then L=""; else L="ORB_AMD_LIB=$V/$v.so"; fi
  env $L timeout -k 10 120 python "$R/tools/probe/stage_times.py" 2>/dev/null | grep B= > "$O/r03_or2_stages_$v.txt" || exit 1
done
cat "$O/r03_or2_stages_new.txt" "$O/r03_or2_stages_pre_orient.txt"
python3 -c "
import json
for l in open('$O/ab_r03_or2.jsonl'):
    d = json.loads(l); b = d['bench']
    print(d['variant'], round(b['value']), round(b['extraction_call_ms_per_launch'], 4), round(b['kernels_ms_per_launch']['k_orient_desc'], 4))
"
bash "$R/tools/gpu_r03_configs.sh" || exit 1
