# k_fast_cells: the wave's cell descriptors prefetched in one vector load (FC_DESC_PREFETCH) and cells per wave 4 / 8 / 16
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fdesc; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
lib() { if [ $1 = base ]; then echo $GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else echo $V/$1.so; fi; }
for v in dp dp8 dp16; do
ORB_AMD_LIB=$V/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_headline.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity_$v.log 2>&1 || { echo "parity $v failed"; tail -30 $O/parity_$v.log; exit 1; }
tail -1 $O/parity_$v.log
done
ORB_AMD_LIB=$V/dpst.so timeout -k 10 200 python3 tools/probe/fc_stamps.py 1024 > $O/stamps_dp.txt 2>&1 || exit 1
cat $O/stamps_dp.txt
for r in 1 2; do for v in base dp dp8 dp16 c8; do
  ORB_AMD_LIB=$(lib $v) timeout -k 10 120 python3 tools/probe/serial_stages.py --batch 1024 > $O/ser_${v}_$r.txt 2>&1 || exit 1
  echo "$v: $(grep -h 'k_fast_cells\|extract_total' $O/ser_${v}_$r.txt | tr '\n' ' ')" | tee -a $O/serial.txt
done; done
for v in base dp dp8 dp16 base dp dp8 dp16; do
  ORB_AMD_LIB=$(lib $v) timeout -k 10 200 python3 bench.py --no-cpu --no-secondary --host-frames 0 > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); k=d['kernels']['k_fast_cells']; print('$v', round(d['value']), round(k['ms_per_call_isolated'],4), round(k['ms_per_call_pipelined'],4))" | tee -a $O/bench.txt
done
