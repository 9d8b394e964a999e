# k_fast_cells occupancy control: one / two unused byte tiles per wave (the LDS of an LDS-DMA ring) vs base
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fpad; mkdir -p $O
V=orb_slam2-chinese-annotation_amd/lib/variants
for r in 1 2; do
  timeout -k 10 120 python tools/probe/stage_times.py --batch 1024 --calls 20 > $O/base_$r.txt 2>&1 || exit 1
  ORB_AMD_LIB=$V/fpad1.so timeout -k 10 120 python tools/probe/stage_times.py --batch 1024 --calls 20 > $O/pad1_$r.txt 2>&1 || exit 1
  ORB_AMD_LIB=$V/fpad2.so timeout -k 10 120 python tools/probe/stage_times.py --batch 1024 --calls 20 > $O/pad2_$r.txt 2>&1 || exit 1
done
for f in $O/*_*.txt; do echo "== $f"; grep B= $f; done
