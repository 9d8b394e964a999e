# resize offsets / weights computed in-kernel (base, PYR_TAB_INLINE=1) vs loaded from the plan's tables (tabload): parity, one-frame latency, batch stages
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pyrtab; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_headline.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity failed"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for v in base tabload base tabload; do
  if [ $v = base ]; then L=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else L=$V/$v.so; fi
  ORB_AMD_LIB=$L timeout -k 10 180 python3 tools/probe/latency_probe.py --calls 300 --tag $v >> $O/lat.jsonl 2> $O/err_lat.txt || exit 1
  ORB_AMD_LIB=$L timeout -k 10 180 python3 tools/probe/stage_times.py --batch 1024 --calls 20 > $O/st_$v.txt 2>&1 || exit 1
  echo "$v $(tail -1 $O/st_$v.txt)" >> $O/stages.txt
done
python3 -c "
import json
for l in open('$O/lat.jsonl'):
    d=json.loads(l); print(d['tag'], round(d['extract_ms'],4), round(d['match_ms'],4), round(d['both_ms'],4), {k:round(v,4) for k,v in d['stage_ms'].items() if k.startswith('k_pyr') or k=='extract_total'})
"
cat $O/stages.txt
