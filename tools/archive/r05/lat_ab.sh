# one-frame latency: default vs PROJ_DIRECT (candidate scan over the staged grid in global memory, no LDS copy)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/lat; mkdir -p $O
V=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/variants
for v in base pdirect base pdirect; do
  if [ $v = base ]; then L=$GRAFT_REPO_ROOT/orb_slam2-chinese-annotation_amd/lib/liborb_amd.so; else L=$V/$v.so; fi
  ORB_AMD_LIB=$L timeout -k 10 200 python3 tools/probe/latency_probe.py --calls 300 --tag $v >> $O/lat.jsonl 2> $O/lat_$v.err || exit 1
done
cat $O/lat.jsonl
