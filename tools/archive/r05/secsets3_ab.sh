# C5 / C3 with every match stream at normal priority: 4 / 6 / 8 rotating buffer sets (ORB_BENCH_SEC_SETS)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ss3; mkdir -p $O
for n in 4 6 8 4 6 8; do
  ORB_BENCH_SEC_SETS=$n timeout -k 10 300 python3 bench.py --no-cpu --host-frames 0 > $O/b_$n.json 2> $O/b_$n.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$n.json').read().strip().splitlines()[-1]); c5=d['C5_problems_per_s']; print('sets $n', round(d['value']), 'C3', round(d['C3_stereo_pairs_per_s']['value']), 'C5', round(c5['value']), round(c5['match_only_problems_per_s']), 'one', round(c5['one_match_stream']['problems_per_s']))" | tee -a $O/sum.txt
done
