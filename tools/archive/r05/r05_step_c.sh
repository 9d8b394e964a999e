# GPU box (round 5): side / own stream queue variants, idle and busy-caller batch rates
set -o pipefail
V=orb_slam2-chinese-annotation_amd/lib/variants
O=gpurun_out/r05_contention9.jsonl; : > $O
P="timeout -k 10 120 python tools/probe/contention_probe.py"
for v in l0inline sidemask sidemask_ownnormal; do
  ORB_AMD_LIB=$V/$v.so $P --tag $v >> $O || exit 1
  ORB_AMD_LIB=$V/$v.so $P --tag ${v}_pre_two --pre two >> $O || exit 1
done
cat $O
