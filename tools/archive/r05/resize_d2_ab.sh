# k_pyr_resize: two source windows in flight (PYR_DEPTH2) and 8 images per workgroup on the small levels: parity, per-level trace, bench
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/rd2; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
ORB_AMD_LIB=$V/d2r8.so timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_headline.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity failed"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for v in base d2 d2r8 r8; do
  if [ $v = base ]; then L=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else L=$V/$v.so; fi
  ORB_AMD_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr_$v -o run --output-format csv -- python3 tools/probe/serial_stages.py --batch 1024 > $O/ser_$v.txt 2>&1 || exit 1
  python3 tools/trace_summary.py $O/tr_$v/run_kernel_trace.csv | grep pyr_resize > $O/lv_$v.txt
  rm -rf $O/tr_$v
done
for v in base d2 d2r8 r8 base d2 d2r8 r8; do
  if [ $v = base ]; then L=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else L=$V/$v.so; fi
  ORB_AMD_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu --no-secondary --host-frames 0 > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), d['kernels']['k_pyr_resize']['ms_per_call_isolated'], d['kernels']['k_pyr_resize']['ms_per_call_pipelined'])" | tee -a $O/bench.txt
done
