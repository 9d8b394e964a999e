#!/bin/bash
# Round profile recipe (run on the GPU box through gpurun from the repo root):
#   the default bench line, a rocprofv3 kernel-trace/stats pass, two HBM PMC
#   passes (FETCH_SIZE and WRITE_SIZE cannot share a pass), the FETCH_SIZE
#   calibration probe, and the two SQ passes of tools/gpu_pmc.sh.  The PMC
#   passes run FAST as one launch per call (the l0inline variant, built by
#   tools/build_variant.sh l0inline -DFAST_L0_INLINE=1 before the call; counters
#   are per dispatch and the level-0 split changes no instruction or byte counts).
# Usage: tools/gpu_profile.sh <tag>
set -eo pipefail
TAG=${1:-r03}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
L0LIB=$R/orb_slam2-chinese-annotation_amd/lib/variants/l0inline.so
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python bench.py > "$O/bench_$TAG.json" 2> "$O/bench_$TAG.err"
cd /tmp && export TMPDIR=/tmp
# the kernel-trace pass runs the bench's own timed workload (8192 resident
# frames, two lanes, 60 steps) without the side legs, so its per-kernel averages
# compare with the line's HIP-event times
SMALL="--no-cpu --no-secondary --host-frames 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$TAG" -o run --output-format csv \
  -- python3 "$R/bench.py" $SMALL > "$O/prof_$TAG.json" 2> "$O/prof_$TAG.err"
ORB_AMD_LIB=$L0LIB timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$O/pmcf_$TAG" -o run --output-format csv \
  -- python3 "$R/bench.py" --no-cpu --no-secondary --frames 512 --steps 2 --warmup 1 --host-frames 0 > "$O/pmcf_$TAG.json" 2> "$O/pmcf_$TAG.err"
ORB_AMD_LIB=$L0LIB timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$O/pmcw_$TAG" -o run --output-format csv \
  -- python3 "$R/bench.py" --no-cpu --no-secondary --frames 512 --steps 2 --warmup 1 --host-frames 0 > "$O/pmcw_$TAG.json" 2> "$O/pmcw_$TAG.err"
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d "$O/calib_$TAG" -o run --output-format csv \
  -- "$R/tools/probe/fetch_calib" > "$O/calib_$TAG.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d "$O/calibw_$TAG" -o run --output-format csv \
  -- "$R/tools/probe/fetch_calib" > "$O/calibw_$TAG.log" 2>&1
cd "$R"
bash tools/gpu_pmc.sh "$TAG" --frames 512 --no-secondary
echo done
