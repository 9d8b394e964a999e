# k_pyr_resize XCD-contiguous tile order (default now) vs grid order (noxcd), + 8 images per workgroup on small levels (xr8)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/rxcd; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
lib() { if [ $1 = xcd ]; then echo $GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else echo $V/$1.so; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_headline.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity failed"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for v in noxcd xcd xr8; do
  ORB_AMD_LIB=$(lib $v) timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr_$v -o run --output-format csv -- python3 tools/probe/serial_stages.py --batch 1024 > $O/ser_$v.txt 2>&1 || exit 1
  python3 tools/trace_summary.py $O/tr_$v/run_kernel_trace.csv | grep pyr_resize > $O/lv_$v.txt
  rm -rf $O/tr_$v
  ORB_AMD_LIB=$(lib $v) timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/pf_$v -o run --output-format csv -- python3 tools/probe/serial_stages.py --batch 1024 --calls 3 > $O/pf_$v.txt 2>&1 || exit 1
done
for v in noxcd xcd xr8 noxcd xcd xr8; do
  ORB_AMD_LIB=$(lib $v) timeout -k 10 200 python3 bench.py --no-cpu --no-secondary --host-frames 0 > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), d['kernels']['k_pyr_resize']['ms_per_call_isolated'], d['kernels']['k_pyr_resize']['ms_per_call_pipelined'])" | tee -a $O/bench.txt
done
