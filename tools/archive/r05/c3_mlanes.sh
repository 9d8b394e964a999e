# C3 with a matcher handle per buffer set: one match stream (m1) vs two (m2, ORB_BENCH_C3_MATCH_LANES=2)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/c3m; mkdir -p $O
for v in m1 m2 m1 m2; do
  ORB_BENCH_C3_MATCH_LANES=${v:1:1} timeout -k 10 300 python3 bench.py --no-cpu --host-frames 0 > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); c3=d['C3_stereo_pairs_per_s']; c5=d['C5_problems_per_s']; print('$v', round(d['value']), 'C3', round(c3['value']), round(c3['stereo_match_only_ms_per_step'],3), 'C5', round(c5['value']))" | tee -a $O/sum.txt
done
