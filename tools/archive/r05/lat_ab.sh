# one-frame latency (B = 1): resolve schedules and the unstaged candidate scan (PROJ_DIRECT=1)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/lat; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
for r in 0 1 2 3; do
  timeout -k 10 180 python3 tools/probe/latency_probe.py --calls 200 --resolve $r --tag base >> $O/lat.jsonl 2> $O/err_$r.txt || exit 1
done
ORB_AMD_LIB=$V/pdirect.so timeout -k 10 180 python3 tools/probe/latency_probe.py --calls 200 --tag pdirect >> $O/lat.jsonl 2> $O/err_pd.txt || exit 1
timeout -k 10 180 python3 tools/probe/latency_probe.py --calls 200 --tag base >> $O/lat.jsonl 2> $O/err_b2.txt || exit 1
python3 -c "
import json
for l in open('$O/lat.jsonl'):
    d=json.loads(l); print(d['tag'], d['resolve'], round(d['extract_ms'],4), round(d['match_ms'],4), round(d['both_ms'],4), {k:round(v,4) for k,v in d['stage_ms'].items()})
"
