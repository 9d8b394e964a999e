#!/bin/bash
# Round-4 profile set (GPU box, repo root): rocprofv3 kernel trace of the
# bench (its pipelined region and its isolated table), the two HBM PMC passes
# (FETCH_SIZE, WRITE_SIZE: separate runs) and the two SQ passes, each pass
# over the bench at 1024 frames per launch, two launches (one per lane) per step.
set -eo pipefail
TAG=${1:-r04}
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/prof$TAG; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
SMALL="--no-cpu --no-secondary --no-dropin --host-frames 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv \
  -- python3 "$R/bench.py" $SMALL --steps 20 > "$O/trace.json" 2> "$O/trace.err"
python3 "$R/tools/r04/trace_summary.py" "$O/trace/run_kernel_trace.csv" > "$O/trace_summary.jsonl"
PM="$SMALL --frames 2048 --steps 1 --warmup 1 --iso-launches 2"
ORB_FAST_L0_INLINE=1 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$O/pmcf" -o run --output-format csv \
  -- python3 "$R/bench.py" $PM > "$O/pmcf.json" 2> "$O/pmcf.err"
ORB_FAST_L0_INLINE=1 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$O/pmcw" -o run --output-format csv \
  -- python3 "$R/bench.py" $PM > "$O/pmcw.json" 2> "$O/pmcw.err"
ORB_FAST_L0_INLINE=1 timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH GRBM_GUI_ACTIVE \
  -d "$O/pmcA" -o run --output-format csv -- python3 "$R/bench.py" $PM > "$O/pmcA.log" 2>&1
ORB_FAST_L0_INLINE=1 timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU \
  -d "$O/pmcB" -o run --output-format csv -- python3 "$R/bench.py" $PM > "$O/pmcB.log" 2>&1
echo done
