# candidate scan without the LDS staging of the frame grid (PROJ_DIRECT=1) in the pipelined headline: frees LDS for FAST / orient?
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pdir; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
lib() { if [ $1 = base ]; then echo $GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else echo $V/$1.so; fi; }
ORB_AMD_LIB=$V/pdirect.so timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity failed"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for v in base pdirect base pdirect; do
  ORB_AMD_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --no-cpu --no-secondary --host-frames 0 > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); k=d['kernels']['k_proj_candidates']; print('$v', round(d['value']), round(k['ms_per_call_isolated'],4), round(k['ms_per_call_pipelined'],4))" | tee -a $O/bench.txt
done
