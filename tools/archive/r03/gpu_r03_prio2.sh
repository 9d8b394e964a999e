#!/bin/bash
# Round 3: C5 alternation per pipelined() call vs the extractor side stream's priority
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
OUT=$O/prio2.txt; : > "$OUT"
for set in "X=0" "ORB_STREAM2_PRIO=greatest" "ORB_STREAM2_PRIO=least"; do
  echo "== $set" >> "$OUT"
  env $set timeout -k 10 200 python "$R/tools/probe/c5_swap.py" --repeat 2>/dev/null >> "$OUT" || exit 1
done
cat "$OUT"
