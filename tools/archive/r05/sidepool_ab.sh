# two CU-masked side streams per device handed to extractor handles in turn (sp2) vs one shared (base)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/sp2; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
lib() { if [ $1 = base ]; then echo $GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else echo $V/$1.so; fi; }
for v in base sp2 base sp2; do
  ORB_AMD_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --no-cpu --host-frames 0 > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); c5=d['C5_problems_per_s']; print('$v', round(d['value']), 'C3', round(d['C3_stereo_pairs_per_s']['value']), 'C5', round(c5['value']), round(c5['match_only_problems_per_s']))" | tee -a $O/sum.txt
done
