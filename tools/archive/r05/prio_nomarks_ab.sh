# no stage markers: match stream priority greatest (the bench's) / normal / least, headline only
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prio; mkdir -p $O
L=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants/nomarks.so
for p in greatest normal least greatest normal least; do
  ORB_AMD_LIB=$L ORB_BENCH_PRIO_MATCH=$p timeout -k 10 300 python3 bench.py --no-cpu --host-frames 0 --no-secondary > $O/b_$p.json 2> $O/b_$p.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$p.json').read().strip().splitlines()[-1]); print('$p', round(d['value']), round(d['ms_per_step'],3))" | tee -a $O/sum.txt
done
