# Round 5 closing validation: every GPU test, smoke, then the round profile set (bench line, kernel trace, HBM / SQ PMC passes)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final_c; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { echo "GPU tests failed"; tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_profile.sh r05c > $O/profile.log 2>&1 || { echo "profile failed"; tail -20 $O/profile.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_r05c.json').read().strip().splitlines()[-1]); print(d['value'], d['C3_stereo_pairs_per_s']['value'], d['C5_problems_per_s']['value'], d['C4_latency']['frames_per_call_1']['serial_ms_per_call'], d['parity_sample']['bit_exact'], d['roofline']['frac'])"
