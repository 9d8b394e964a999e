# extraction lanes 2 vs 3 vs 4 with the round-5 stream layout (library streams least priority, CU-masked side stream)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/lanes; mkdir -p $O
for n in 2 3 4 2 3 4; do
  ORB_BENCH_LANES=$n timeout -k 10 200 python3 bench.py --no-cpu --no-secondary --host-frames 0 > $O/b$n.json 2> $O/b$n.err || { echo "lanes $n failed"; tail -5 $O/b$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b$n.json').read().strip().splitlines()[-1]); print('lanes $n', round(d['value']), d['config']['extraction_lanes'][:60])" | tee -a $O/lanes.txt
done
