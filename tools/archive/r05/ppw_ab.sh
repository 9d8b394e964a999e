# k_orient_desc keypoint pairs per wave 4 (base) / 8 / 16: stage times and bench, interleaved
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ppw; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
lib() { if [ $1 = base ]; then echo $GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else echo $V/$1.so; fi; }
ORB_AMD_LIB=$V/ppw16.so timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_headline.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity failed"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for v in base ppw8 ppw16; do
  ORB_AMD_LIB=$(lib $v) timeout -k 10 120 python3 tools/probe/stage_times.py --batch 1024 --calls 20 > $O/st_${v}.txt 2>&1 || exit 1
  echo "$v: $(grep B= $O/st_${v}.txt)" | tee -a $O/stages.txt
done
for v in base ppw8 ppw16 base ppw8 ppw16 base ppw8 ppw16; do
  ORB_AMD_LIB=$(lib $v) timeout -k 10 200 python3 bench.py --no-cpu --no-secondary --host-frames 0 > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); k=d['kernels']['k_orient_desc']; print('$v', round(d['value']), round(k['ms_per_call_isolated'],4), round(k['ms_per_call_pipelined'],4))" | tee -a $O/bench.txt
done
