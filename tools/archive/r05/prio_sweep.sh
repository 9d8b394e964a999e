# headline vs stream priorities (extract lane 0 / lane 1 / match), no events in the timed region
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/psw; mkdir -p $O
for c in nnn ggn nnl gnn ngn nnn ggn nnl gnn ngn; do
  pe=${c:0:1}; p1=${c:1:1}; pm=${c:2:1}
  m() { case $1 in n) echo normal;; g) echo greatest;; l) echo least;; esac; }
  ORB_BENCH_PRIO_EXTRACT=$(m $pe) ORB_BENCH_PRIO_EXTRACT1=$(m $p1) ORB_BENCH_PRIO_MATCH=$(m $pm) \
    timeout -k 10 300 python3 bench.py --no-cpu --host-frames 0 --no-secondary > $O/b_$c.json 2> $O/b_$c.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$c.json').read().strip().splitlines()[-1]); print('$c', round(d['value']), round(d['ms_per_step'],3))" | tee -a $O/sum.txt
done
