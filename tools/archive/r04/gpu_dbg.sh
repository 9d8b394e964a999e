#!/bin/bash
# bench segfault hunt (Python stack of the faulting call) + Jacobi round counts
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
timeout -k 10 400 python -X faulthandler -u bench.py > "$O/d_bench.json" 2> "$O/d_bench.err"
echo "bench rc $?"
tail -40 "$O/d_bench.err"
for R in 8 16; do ORB_JACOBI_ROUNDS=$R timeout -k 10 200 python -u tools/r04/c5_stages.py 16 >> "$O/d_c5.log" 2>&1; done
cat "$O/d_c5.log"
