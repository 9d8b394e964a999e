# k_octree memory-resident key sweeps, 4 keys per thread per step (base = OCT_SWEEP_UNROLL 4; sw2, sw8) vs one at a time (sw1): parity, stages, bench
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/octs; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
lib() { if [ $1 = base ]; then echo $GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else echo $V/$1.so; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_headline.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity failed"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for v in base sw1 sw2 sw8 base sw1; do
  ORB_AMD_LIB=$(lib $v) timeout -k 10 120 python3 tools/probe/stage_times.py --batch 1024 --calls 20 > $O/b_$v.txt 2>&1 || exit 1
  ORB_AMD_LIB=$(lib $v) timeout -k 10 120 python3 tools/probe/stage_times.py --batch 1 --calls 300 > $O/s_$v.txt 2>&1 || exit 1
  echo "$v B1024: $(tail -1 $O/b_$v.txt)" | tee -a $O/sum.txt
  echo "$v B1: $(tail -1 $O/s_$v.txt)" | tee -a $O/sum.txt
done
for v in base sw1 base sw1; do
  ORB_AMD_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --no-cpu --host-frames 0 > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); k=d['kernels']['k_octree']; c=d['C5_problems_per_s']; print('$v', round(d['value']), 'oct', round(k['ms_per_call_isolated'],4), round(k['ms_per_call_pipelined'],4), 'C3', round(d['C3_stereo_pairs_per_s']['value']), 'C5', round(c['value']), 'lat', round(d['C4_latency']['frames_per_call_1']['serial_ms_per_call'],4))" | tee -a $O/sum.txt
done
