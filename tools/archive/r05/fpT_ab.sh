# k_proj_resolve_fp with 512 / 256 threads (2 / 4 points per thread, same 1024-point windows): parity, C5 rates
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fpT; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
lib() { if [ $1 = base ]; then echo $GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else echo $V/$1.so; fi; }
for v in fp512 fp256; do
ORB_AMD_LIB=$V/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_matcher.py tests/test_gpu_headline.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity_$v.log 2>&1 || { echo "parity $v failed"; tail -30 $O/parity_$v.log; exit 1; }
tail -1 $O/parity_$v.log
done
for v in base fp512 fp256 base fp512 fp256; do
  ORB_AMD_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --no-cpu --host-frames 0 > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); c=d['C5_problems_per_s']; print('$v', round(d['value']), 'C5', round(c['value']), round(c['match_only_problems_per_s']), 'two', round(c['two_match_streams']['problems_per_s']), round(c['two_match_streams']['match_only_problems_per_s']))" | tee -a $O/bench.txt
done
