# k_orient_desc LDS-DMA staging (DESC_GLDS=1) vs the register staging: parity, then stage times A/B/A/B
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/glds; mkdir -p $O
V=orb_slam2-chinese-annotation_amd/lib/variants
ORB_AMD_LIB=$V/oglds.so timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_headline.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
for r in 1 2; do
  timeout -k 10 120 python tools/probe/stage_times.py --batch 1024 --calls 20 > $O/base_$r.txt 2>&1 || exit 1
  ORB_AMD_LIB=$V/oglds.so timeout -k 10 120 python tools/probe/stage_times.py --batch 1024 --calls 20 > $O/glds_$r.txt 2>&1 || exit 1
done
for f in $O/base_1.txt $O/glds_1.txt $O/base_2.txt $O/glds_2.txt; do echo "== $f"; cat $f; done
