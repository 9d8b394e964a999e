# GPU box (round 5): one-frame latency with the cell FAST kernel instead of bands
set -o pipefail
V=orb_slam2-chinese-annotation_amd/lib/variants
O=gpurun_out/r05_latency5.jsonl; : > $O
L="timeout -k 10 120 python tools/probe/latency_probe.py"
$L --tag default >> $O || exit 1
for v in cells1 cells4 cells1inl; do ORB_AMD_LIB=$V/$v.so $L --tag $v >> $O || exit 1; done
$L --tag default_again >> $O || exit 1
cat $O
