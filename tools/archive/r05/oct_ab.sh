# k_octree batch workgroup size (OCT_BATCH_THREADS 128 vs 256) and LDS budget (ORB_OCTREE_LDS_KB 32 vs 52): parity, serial stages, bench
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/oct; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
lib() { if [ $1 = base ]; then echo $GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else echo $V/$1.so; fi; }
for v in o128 o128s; do
ORB_AMD_LIB=$V/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_headline.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity_$v.log 2>&1 || { echo "parity $v failed"; tail -30 $O/parity_$v.log; exit 1; }
tail -1 $O/parity_$v.log
done
for r in 1 2; do for v in base o128 o128s o256s; do
  ORB_AMD_LIB=$(lib $v) timeout -k 10 120 python3 tools/probe/serial_stages.py --batch 1024 > $O/ser_${v}_$r.txt 2>&1 || exit 1
  echo "$v: $(tr '\n' ' ' < $O/ser_${v}_$r.txt)" | tee -a $O/serial.txt
done; done
for v in base o128 o128s o256s base o128 o128s o256s; do
  ORB_AMD_LIB=$(lib $v) timeout -k 10 200 python3 bench.py --no-cpu --no-secondary --host-frames 0 > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); k=d['kernels']['k_octree']; print('$v', round(d['value']), round(k['ms_per_call_isolated'],4), round(k['ms_per_call_pipelined'],4))" | tee -a $O/bench.txt
done
