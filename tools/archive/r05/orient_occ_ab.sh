# k_orient_desc: 5 waves per SIMD (DESC_MIN_WAVES=5, 96 VGPRs) and 2 / 8 keypoint pairs per wave vs 4: parity, stage times, bench
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/oocc; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
lib() { if [ $1 = base ]; then echo $GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else echo $V/$1.so; fi; }
for v in dw5 ppw2 ppw8; do
ORB_AMD_LIB=$V/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py -m gpu -x -q --timeout 120 --timeout-method thread -k "batch" > $O/parity_$v.log 2>&1 || { echo "parity $v failed"; tail -30 $O/parity_$v.log; exit 1; }
tail -1 $O/parity_$v.log
done
for r in 1 2; do for v in base dw5 ppw2 ppw8; do
  ORB_AMD_LIB=$(lib $v) timeout -k 10 120 python3 tools/probe/stage_times.py --batch 1024 --calls 20 > $O/st_${v}_$r.txt 2>&1 || exit 1
  echo "$v: $(grep B= $O/st_${v}_$r.txt)" | tee -a $O/stages.txt
done; done
for v in base dw5 base dw5; do
  ORB_AMD_LIB=$(lib $v) timeout -k 10 200 python3 bench.py --no-cpu --no-secondary --host-frames 0 > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']))" | tee -a $O/bench.txt
done
