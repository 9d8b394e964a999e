# headline bimodality: host queueing unbounded (free) vs at most one launch per buffer set in flight (bounded), stage events off
# (default) and on inside the timed region (prof)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/bnd; mkdir -p $O
for v in free bounded prof bprof free bounded prof bprof free bounded; do
  F=""
  case $v in bounded) F="--bounded";; prof) F="--timed-events match";; bprof) F="--bounded --timed-events match";; esac
  timeout -k 10 300 python3 bench.py --no-cpu --host-frames 0 --no-secondary $F > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],3))" | tee -a $O/sum.txt
done
