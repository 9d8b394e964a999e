# GPU box: batch / torch rate with busy caller streams after various pre-steps
set -o pipefail
O=gpurun_out/r05_contention7.jsonl; : > $O
P="timeout -k 10 120 python tools/probe/contention_probe.py"
$P --tag ext_pre_two_lowown --pre two >> $O || exit 1
$P --tag ext_pre_handles_lowown --pre handles >> $O || exit 1
$P --tag torch_pre_two_lowown --workload torch --pre two >> $O || exit 1
$P --tag torch_raw3 --workload torch --pre raw3 >> $O || exit 1
cat $O
