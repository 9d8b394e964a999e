# headline lanes / match placement with normal-priority match streams and no events in the timed region
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ln2; mkdir -p $O
for c in l2s l3s l2i l1s l2s l3s l2i; do
  case $c in l2s) F="--lanes 2";; l3s) F="--lanes 3";; l2i) F="--lanes 2 --lane-match inlane";; l1s) F="--lanes 1";; esac
  timeout -k 10 300 python3 bench.py --no-cpu --host-frames 0 --no-secondary $F > $O/b_$c.json 2> $O/b_$c.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$c.json').read().strip().splitlines()[-1]); print('$c', round(d['value']), round(d['ms_per_step'],3))" | tee -a $O/sum.txt
done
