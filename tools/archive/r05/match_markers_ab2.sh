# matcher stream markers, repeated: timed events before and after each stage (mm3), the same plus call begin / end (mm4: the
# profiler's eight records), none (base), the profiler inside the timed region (prof)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/mmk2; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
lib() { if [ $1 = base ] || [ $1 = prof ]; then echo $GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else echo $V/$1.so; fi; }
for v in mm4 mm3 base prof mm4 mm3 base mm4 mm3 prof mm4; do
  if [ $v = prof ]; then F="--timed-events match"; else F=""; fi
  ORB_AMD_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --no-cpu --host-frames 0 --no-secondary $F > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],3))" | tee -a $O/sum.txt
done
