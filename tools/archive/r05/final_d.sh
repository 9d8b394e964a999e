# Round 5 last check of HEAD: every GPU test, smoke, the default bench line
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final_d; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { echo "GPU tests failed"; tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['C3_stereo_pairs_per_s']['value'], d['C5_problems_per_s']['value'], d['C4_latency']['frames_per_call_1']['serial_ms_per_call'], d['parity_sample']['bit_exact'], d['roofline']['frac'], d['cpu_baseline']['value'])"
