# C5 / C3 vs the second match stream's priority (match1: greatest = current, normal, least) and match least
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pc5; mkdir -p $O
for c in ng nn nl ln ng nn nl ln; do
  m() { case $1 in n) echo normal;; g) echo greatest;; l) echo least;; esac; }
  ORB_BENCH_PRIO_MATCH=$(m ${c:0:1}) ORB_BENCH_PRIO_MATCH1=$(m ${c:1:1}) \
    timeout -k 10 300 python3 bench.py --no-cpu --host-frames 0 > $O/b_$c.json 2> $O/b_$c.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$c.json').read().strip().splitlines()[-1]); c5=d['C5_problems_per_s']; print('$c', round(d['value']), 'C3', round(d['C3_stereo_pairs_per_s']['value']), 'C5', round(c5['value']), round(c5['match_only_problems_per_s']), 'one', round(c5['one_match_stream']['problems_per_s']))" | tee -a $O/sum.txt
done
