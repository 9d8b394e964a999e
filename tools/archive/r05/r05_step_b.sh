# GPU box (round 5): idle / busy batch rates and one-frame latency per library variant
set -o pipefail
V=orb_slam2-chinese-annotation_amd/lib/variants
O=gpurun_out/r05_contention8.jsonl; : > $O
P="timeout -k 10 120 python tools/probe/contention_probe.py"
$P --tag default >> $O || exit 1
$P --tag default_pre_two --pre two >> $O || exit 1
ORB_AMD_LIB=$V/fcdesc0.so $P --tag fcdesc0 >> $O || exit 1
ORB_AMD_LIB=$V/ownnormal.so $P --tag ownnormal >> $O || exit 1
ORB_AMD_LIB=$V/ownnormal.so $P --tag ownnormal_pre_two --pre two >> $O || exit 1
cat $O
O=gpurun_out/r05_latency2.jsonl; : > $O
L="timeout -k 10 120 python tools/probe/latency_probe.py"
$L --tag default >> $O || exit 1
$L --tag default_b8 --batch 8 >> $O || exit 1
ORB_AMD_LIB=$V/ownnormal.so $L --tag ownnormal_b8 --batch 8 >> $O || exit 1
cat $O
