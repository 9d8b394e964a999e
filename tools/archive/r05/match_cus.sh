# headline with the match stream CU-masked to n of 256 CUs (every (256/n)-th CU; n = 256: all CUs, a queue of its own) vs default
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/mcu; mkdir -p $O
for n in 0 256 192 128 64 0 256 128; do
  ORB_BENCH_CUS_MATCH=$n timeout -k 10 300 python3 bench.py --no-cpu --host-frames 0 --no-secondary > $O/b_$n.json 2> $O/b_$n.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$n.json').read().strip().splitlines()[-1]); k=d['kernels']; print('cus $n', round(d['value']), round(d['ms_per_step'],3), 'cand pipelined', round(k['k_proj_candidates']['ms_per_call_pipelined'],3))" | tee -a $O/sum.txt
done
