# C5 two-match-stream pipeline with 4 / 6 / 8 buffer sets
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/secsets2; mkdir -p $O
for n in 4 6 8 4 6 8; do
  ORB_BENCH_SEC_SETS=$n timeout -k 10 300 python3 bench.py --no-cpu > $O/b$n.json 2> $O/b$n.err || { echo "sets $n failed"; tail -5 $O/b$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b$n.json').read().strip().splitlines()[-1]); c=d['C5_problems_per_s']; print('sets $n', round(d['value']), 'C3', round(d['C3_stereo_pairs_per_s']['value']), 'C5', round(c['value']), round(c['match_only_problems_per_s']), 'one', round(c['one_match_stream']['problems_per_s']))" | tee -a $O/bench.txt
done
