# GPU box (round 5): headline A/B of the match stream's priority (bench.py --steps 20, in order)
set -o pipefail
O=gpurun_out/r05_prio.jsonl; : > $O
B="timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-dropin --no-cpu --no-secondary --host-frames 0"
for p in greatest normal least greatest normal least; do
  ORB_BENCH_PRIO_MATCH=$p $B > gpurun_out/r05_prio.json 2>> gpurun_out/r05_prio.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r05_prio.json').read().strip().splitlines()[-1]);print(json.dumps({'match_prio':'$p','value':d['value'],'parity':d['parity_sample']['bit_exact'],'cand_pipe':d['kernels']['k_proj_candidates'].get('ms_per_call_pipelined')}))" >> $O
done
cat $O
