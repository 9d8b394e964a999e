# GPU box: batch rate with busy caller streams after various pre-steps
set -o pipefail
O=gpurun_out/r05_contention5.jsonl; : > $O
P="timeout -k 10 120 python tools/probe/contention_probe.py"
V=orb_slam2-chinese-annotation_amd/lib/variants
$P --tag base >> $O || exit 1
$P --tag pre_two --pre two >> $O || exit 1
$P --tag pre_twoseq --pre twoseq >> $O || exit 1
$P --tag pre_one --pre one >> $O || exit 1
$P --tag pre_handles --pre handles >> $O || exit 1
$P --tag torch_base --workload torch >> $O || exit 1
$P --tag torch_pre_two --workload torch --pre two >> $O || exit 1
$P --tag pre_two_tf --pre two --torch-first >> $O || exit 1
ORB_AMD_LIB=$V/l0inline.so $P --tag l0_pre_two --pre two >> $O || exit 1
cat $O
