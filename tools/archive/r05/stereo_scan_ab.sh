# stereo candidate scan: 2 row-list entries per lane per step (base, STEREO_SCAN_UNROLL 2), 1 (su1), 3 (su3), with the record (su2h1) or
# image-pointer loads hoisted (su2h2), and the previous kernel (stold): parity, C3
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/stscan; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
lib() { if [ $1 = base ]; then echo $GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else echo $V/$1.so; fi; }
ORB_AMD_LIB=$V/stold.so timeout -k 10 120 python -u -m pytest tests/test_gpu_matchers_more.py -k ties -m gpu -x -q --timeout 120 --timeout-method thread > $O/ties_old.log 2>&1; rc=$?; echo "old kernel on the ties test: rc $rc $(tail -1 $O/ties_old.log)"
if [ $rc -gt 1 ]; then exit 1; fi  # a fault / timeout, not a test failure
timeout -k 10 300 python -u -m pytest tests/test_gpu_matchers_more.py tests/test_gpu_dropin.py tests/test_gpu_concurrency.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity failed"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for v in base stold su1 su3 su2h2 su2h1 base stold; do
  ORB_AMD_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --no-cpu --host-frames 0 > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); c=d['C3_stereo_pairs_per_s']; print('$v', round(d['value']), round(c['value']), round(c['extraction_only_ms_per_step'],3), round(c['stereo_match_only_ms_per_step'],3))" | tee -a $O/bench.txt
done
