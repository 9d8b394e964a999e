# C5 resolve: whole-problem Jacobi in one workgroup (k_proj_resolve_wj, RESOLVE_WJ=1) vs the fixed-point windows: parity, then C5 rates
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/wj; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
lib() { if [ $1 = base ]; then echo $GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else echo $V/$1.so; fi; }
ORB_AMD_LIB=$V/wj8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_matcher.py -m gpu -x -q --timeout 120 --timeout-method thread -k "large_maps or headline or schedules and not auto" > $O/parity.log 2>&1 || { echo "parity failed"; tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
ORB_AMD_LIB=$V/wj.so timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity2.log 2>&1 || { echo "parity2 failed"; tail -40 $O/parity2.log; exit 1; }
tail -1 $O/parity2.log
for v in base wj2 wj wj8 wj wj8; do
  ORB_AMD_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --no-cpu --host-frames 0 > $O/bench_$v.json 2> $O/bench_$v.err || { echo "bench $v failed"; tail -5 $O/bench_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); c=d['C5_problems_per_s']; print('$v', round(d['value']), 'C5', round(c['value']), 'alone', round(c['match_only_problems_per_s']), 'two', round(c['two_match_streams']['problems_per_s']), round(c['two_match_streams']['match_only_problems_per_s']))" | tee -a $O/bench.txt
done
