# GPU box (round 5): matcher tests (grid build change), latency, lane / stream A/B of the headline
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_matcher.py tests/test_gpu_headline.py tests/test_gpu_matchers_more.py tests/test_gpu_matchers_f.py tests/test_gpu_mapping.py tests/test_gpu_dropin.py > gpurun_out/r05_t7.log 2>&1; rc=$?; echo "matcher tests rc=$rc"; tail -2 gpurun_out/r05_t7.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python tools/probe/latency_probe.py --tag grid4 > gpurun_out/r05_latency4.jsonl || exit 1
cat gpurun_out/r05_latency4.jsonl
O=gpurun_out/r05_lanes.jsonl; : > $O
B="timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-dropin --no-cpu --no-secondary --host-frames 0"
for cfg in "2 prio" "3 prio" "2 cumask" "3 cumask" "2 prio"; do
  set -- $cfg
  ORB_BENCH_STREAMS=$2 $B --lanes $1 > gpurun_out/r05_lane.json 2>> gpurun_out/r05_lanes.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r05_lane.json').read().strip().splitlines()[-1]);print(json.dumps({'lanes':$1,'streams':'$2','value':d['value'],'parity':d['parity_sample']['bit_exact']}))" >> $O
done
cat $O
