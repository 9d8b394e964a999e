# GPU box (round 5): full GPU suite, then bench default vs pooled side stream
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_t6.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; tail -3 gpurun_out/r05_t6.log
[ $rc -eq 0 ] || exit 1
B="timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-dropin --cpu-seconds 3 --cpu-all-seconds 0"
$B > gpurun_out/r05_b4.json 2> gpurun_out/r05_b4.err || exit 1
ORB_AMD_LIB=orb_slam2-chinese-annotation_amd/lib/variants/sidepool.so $B > gpurun_out/r05_b4p.json 2> gpurun_out/r05_b4p.err || exit 1
$B > gpurun_out/r05_b4b.json 2> gpurun_out/r05_b4b.err || exit 1
echo done
