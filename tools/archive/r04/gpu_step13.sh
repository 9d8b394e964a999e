#!/bin/bash
# round-4 step 13: C5 matcher counters (candidates, Jacobi rounds, windowed
# resolve): kernel trace + one SQ pass, B = 16
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/c5pmc; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
ORB_RESOLVE_JACOBI=1 ORB_JACOBI_ROUNDS=6 timeout -k 10 150 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 "$R/tools/r04/c5_stages.py" 16 > "$O/trace.log" 2>&1
ORB_RESOLVE_JACOBI=1 ORB_JACOBI_ROUNDS=6 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
  -d "$O/pmcA" -o run --output-format csv -- python3 "$R/tools/r04/c5_stages.py" 16 > "$O/pmcA.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
  -d "$O/pmcB" -o run --output-format csv -- python3 "$R/tools/r04/c5_stages.py" 16 > "$O/pmcB.log" 2>&1
cd "$R"
grep C5 "$O/trace.log"
python3 tools/pmc_table.py "$O/pmcA" | cut -c1-220
python3 tools/pmc_table.py "$O/pmcB" | cut -c1-220
