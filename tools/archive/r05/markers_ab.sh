# matcher stage markers on (base) vs off (nomarks), the bench's stage events outside the timed region: headline, C3, C5, latency
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/mk; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
lib() { if [ $1 = base ]; then echo $GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else echo $V/$1.so; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_matcher.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity failed"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for v in base nomarks base nomarks base; do
  ORB_AMD_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --no-cpu --host-frames 0 > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), 'C3', round(d['C3_stereo_pairs_per_s']['value']), 'C5', round(d['C5_problems_per_s']['value']), round(d['C5_problems_per_s']['match_only_problems_per_s']), 'lat', round(d['C4_latency']['frames_per_call_1']['serial_ms_per_call'],4), round(d['C4_latency']['frames_per_call_8']['serial_ms_per_call'],4))" | tee -a $O/sum.txt
done
