# bench headline with the per-stage HIP events inside the timed region on the extractor (ext), the matcher (match), both (the
# round-4 / round-5 layout) or neither (off: the events go in a profiled pass after the timed region)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/tev2; mkdir -p $O
for v in off both ext match off both ext match; do
  timeout -k 10 300 python3 bench.py --no-cpu --host-frames 0 --no-secondary --timed-events $v > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$v', round(d['value']), round(d['ms_per_step'],3), 'pipelined fast', round(k['k_fast_cells']['ms_per_call_pipelined'],3), 'orient', round(k['k_orient_desc']['ms_per_call_pipelined'],3), 'cand', round(k['k_proj_candidates']['ms_per_call_pipelined'],3))" | tee -a $O/sum.txt
done
