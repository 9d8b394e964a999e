# k_pyr_resize images per workgroup from a target workgroup count (PYR_TARGET_WGS; told = 16 always, the old shape)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ipwt; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
lib() { if [ $1 = t2k ]; then echo $GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else echo $V/$1.so; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_headline.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity failed"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for v in told t2k t1k t4k; do
  for cfg in "--batch 16 --width 1920 --height 1080 --features 4000 --calls 50" "--batch 256 --features 2000 --calls 20"; do
    ORB_AMD_LIB=$(lib $v) timeout -k 10 120 python3 tools/probe/stage_times.py $cfg 2>/dev/null | sed "s/^/$v /" | tee -a $O/stages.txt || exit 1
  done
done
for v in told t2k t1k t4k told t2k t1k t4k; do
  ORB_AMD_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --no-cpu --host-frames 0 > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); c=d['C5_problems_per_s']; print('$v', round(d['value']), 'C3', round(d['C3_stereo_pairs_per_s']['value']), 'C5', round(c['value']), round(c['match_only_problems_per_s']))" | tee -a $O/bench.txt
done
