# k_pyr_resize images per workgroup on the smaller levels (PYR_SMALL_IPW for levels launching < 4096 workgroups at 16)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ripw; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
for v in base r8 r4 r2; do
  if [ $v = base ]; then L=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else L=$V/$v.so; fi
  ORB_AMD_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr_$v -o run --output-format csv -- python3 tools/probe/serial_stages.py --batch 1024 > $O/ser_$v.txt 2>&1 || exit 1
  python3 tools/trace_summary.py $O/tr_$v/run_kernel_trace.csv | grep pyr_resize > $O/lv_$v.txt
  rm -rf $O/tr_$v
  ORB_AMD_LIB=$L timeout -k 10 120 python3 tools/probe/stage_times.py --batch 1024 --calls 20 > $O/st_$v.txt 2>&1 || exit 1
done
for v in base r8 r4 r2 base r8 r4 r2; do
  if [ $v = base ]; then L=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else L=$V/$v.so; fi
  ORB_AMD_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu --no-secondary --host-frames 0 > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), d['kernels']['k_pyr_resize']['ms_per_call_isolated'], d['kernels']['k_pyr_resize']['ms_per_call_pipelined'])" | tee -a $O/bench.txt
done
