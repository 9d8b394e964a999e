# matcher stream markers: untimed events after each stage (mm1), timed events after each stage (mm2), timed before and after (mm3),
# none (base), against the profiled matcher inside the timed region (base, --timed-events match)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/mmk; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
lib() { if [ $1 = base ] || [ $1 = prof ]; then echo $GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else echo $V/$1.so; fi; }
for v in base prof mm1 mm2 mm3 base prof mm1 mm2 mm3; do
  if [ $v = prof ]; then F="--timed-events match"; else F=""; fi
  ORB_AMD_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --no-cpu --host-frames 0 --no-secondary $F > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$v', round(d['value']), round(d['ms_per_step'],3))" | tee -a $O/sum.txt
done
