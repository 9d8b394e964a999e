# PYR_TARGET_WGS=2048 under the round-5 secondary schedule (4 sets, C5 on two match streams)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/t2kc5; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
lib() { if [ $1 = base ]; then echo $GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else echo $V/$1.so; fi; }
for v in base t2k base t2k; do
  ORB_AMD_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --no-cpu > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); c=d['C5_problems_per_s']; print('$v', round(d['value']), 'C3', round(d['C3_stereo_pairs_per_s']['value']), 'C5', round(c['value']), round(c['match_only_problems_per_s']), 'one', round(c['one_match_stream']['problems_per_s']))" | tee -a $O/bench.txt
done
