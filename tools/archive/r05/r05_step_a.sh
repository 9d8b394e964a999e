# GPU box (round 5): contention probes, concurrency tests, one-frame latency per variant, short bench
set -o pipefail
bash tools/probe/contention_probe.sh
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_concurrency.py > gpurun_out/r05_t5.log 2>&1; echo "conc rc=$?"; tail -4 gpurun_out/r05_t5.log
V=orb_slam2-chinese-annotation_amd/lib/variants
O=gpurun_out/r05_latency.jsonl; : > $O
L="timeout -k 10 120 python tools/probe/latency_probe.py"
$L --tag default >> $O || exit 1
ORB_AMD_LIB=$V/oct256.so $L --tag oct256 >> $O || exit 1
ORB_AMD_LIB=$V/oct128.so $L --tag oct128 >> $O || exit 1
$L --tag default_b8 --batch 8 >> $O || exit 1
cat $O
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-dropin --cpu-seconds 3 --cpu-all-seconds 0 > gpurun_out/r05_b3.json 2> gpurun_out/r05_b3.err; echo "bench rc=$?"
