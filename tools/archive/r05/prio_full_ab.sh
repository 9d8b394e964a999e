# full bench keys with the match stream at normal priority (mn) vs greatest (mg; the previous setting), stage events outside the timed region
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/priof; mkdir -p $O
for v in mn mg mn mg; do
  if [ $v = mn ]; then p=normal; else p=greatest; fi
  ORB_BENCH_PRIO_MATCH=$p timeout -k 10 300 python3 bench.py --no-cpu --host-frames 0 > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); c5=d['C5_problems_per_s']; print('$v', round(d['value']), 'C3', round(d['C3_stereo_pairs_per_s']['value']), 'C5', round(c5['value']), round(c5['match_only_problems_per_s']), 'one', round(c5['one_match_stream']['problems_per_s']), 'lat', round(d['C4_latency']['frames_per_call_1']['serial_ms_per_call'],4))" | tee -a $O/sum.txt
done
