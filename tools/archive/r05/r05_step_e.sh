# GPU box (round 5): one-frame latency with per-stage times, octree workgroup variants
set -o pipefail
V=orb_slam2-chinese-annotation_amd/lib/variants
O=gpurun_out/r05_latency3.jsonl; : > $O
L="timeout -k 10 120 python tools/probe/latency_probe.py"
$L --tag default >> $O || exit 1
ORB_AMD_LIB=$V/oct1024.so $L --tag oct1024 >> $O || exit 1
$L --tag default_b8 --batch 8 >> $O || exit 1
cat $O
