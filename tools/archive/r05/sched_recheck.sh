# schedule constants re-checked under the closing stream setup: FAST side levels 1 / 2 (base) / 3, octree 128 threads + 32 KB (o128s)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/sched; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
lib() { if [ $1 = base ]; then echo $GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else echo $V/$1.so; fi; }
for v in base fsl1 fsl3 o128s base fsl1 fsl3 o128s; do
  ORB_AMD_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --no-cpu --host-frames 0 --no-secondary > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],3))" | tee -a $O/sum.txt
done
