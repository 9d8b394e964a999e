# occupancy control: register staging with the GLDS variant's LDS (3 workgroups per CU) vs GLDS vs base
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/glds; mkdir -p $O
V=orb_slam2-chinese-annotation_amd/lib/variants
for r in 1 2; do
  timeout -k 10 120 python tools/probe/stage_times.py --batch 1024 --calls 20 > $O/b2base_$r.txt 2>&1 || exit 1
  ORB_AMD_LIB=$V/opad.so timeout -k 10 120 python tools/probe/stage_times.py --batch 1024 --calls 20 > $O/b2pad_$r.txt 2>&1 || exit 1
  ORB_AMD_LIB=$V/oglds.so timeout -k 10 120 python tools/probe/stage_times.py --batch 1024 --calls 20 > $O/b2glds_$r.txt 2>&1 || exit 1
done
for f in $O/b2*_*.txt; do echo "== $f"; grep B= $f; done
