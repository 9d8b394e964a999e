#!/bin/bash
# A/B: extraction lanes (two extractor handles on streams of their own) against
# the one-lane pipeline; each variant one bench run without the extra legs.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
Q="--no-cpu --no-secondary --host-frames 0"
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 python bench.py $Q > "$O/lanes_$tag.json" 2> "$O/lanes_$tag.err"
  python - "$O/lanes_$tag.json" "$tag" <<'P'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["value"]), round(d["ms_per_step"], 3), flush=True)
P
}
if [ "$1" = "sec" ]; then  # secondary configs (C3 / C5) with one and two lanes, and resize images per workgroup
  Q="--no-cpu --host-frames 0 --frames 2048 --steps 20"
  runs() {  # tag, env...
    local tag=$1; shift
    env "$@" timeout -k 10 300 python bench.py $Q > "$O/sec_$tag.json" 2> "$O/sec_$tag.err"
    python - "$O/sec_$tag.json" "$tag" <<'P'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["value"]), "C3", round(d["C3_stereo_pairs_per_s"]["value"]), "C5", round(d["C5_problems_per_s"]["value"]), flush=True)
P
  }
  runs l1 ORB_BENCH_LANES=1
  runs l2 ORB_BENCH_LANES=2
  runs l1r ORB_BENCH_LANES=1
  runs l2r ORB_BENCH_LANES=2
  Q="--no-cpu --no-secondary --host-frames 0"
  run d ORB_BENCH_LANES=2
  run rs16 ORB_RESIZE_IMAGES_PER_WG=16
  run rs12 ORB_RESIZE_IMAGES_PER_WG=12
  run rs24 ORB_RESIZE_IMAGES_PER_WG=24
  run d_r ORB_BENCH_LANES=2
  run rs16_r ORB_RESIZE_IMAGES_PER_WG=16
  exit 0
fi
if [ "$1" = "sweep4" ]; then  # launch-shape knobs and FAST cells-per-wave builds under two lanes
  V=$R/orb_slam2-chinese-annotation_amd/lib/variants
  run d ORB_BENCH_LANES=2
  run rs4 ORB_RESIZE_IMAGES_PER_WG=4
  run rs16 ORB_RESIZE_IMAGES_PER_WG=16
  run olds32 ORB_OCTREE_LDS_KB=32
  run olds80 ORB_OCTREE_LDS_KB=80
  run cpw6 ORB_AMD_LIB=$V/cpw6.so
  run cpw8 ORB_AMD_LIB=$V/cpw8.so
  run d_r ORB_BENCH_LANES=2
  exit 0
fi
if [ "$1" = "sweep3" ]; then  # schedule knobs under two lanes
  run l2 ORB_BENCH_LANES=2
  run l2_side1 ORB_BENCH_LANES=2 ORB_FAST_SIDE_LEVELS=1
  run l2_side3 ORB_BENCH_LANES=2 ORB_FAST_SIDE_LEVELS=3
  run l2_side0 ORB_BENCH_LANES=2 ORB_FAST_SIDE_LEVELS=0
  run l2_s2norm ORB_BENCH_LANES=2 ORB_STREAM2_PRIO=normal
  run l2_q8 ORB_BENCH_LANES=2 GPU_MAX_HW_QUEUES=8
  run l3_q8 ORB_BENCH_LANES=3 GPU_MAX_HW_QUEUES=8
  run l2_r ORB_BENCH_LANES=2
  exit 0
fi
if [ "$1" = "sweep2" ]; then
  run base ORB_BENCH_LANES=1
  run l2s ORB_BENCH_LANES=2
  run l3s ORB_BENCH_LANES=3
  run l4s ORB_BENCH_LANES=4
  Q="$Q --batch 512"
  run l2s_b512 ORB_BENCH_LANES=2
  run l3s_b512 ORB_BENCH_LANES=3
  run l4s_b512 ORB_BENCH_LANES=4
  Q="${Q% --batch 512}"
  run l2s_r ORB_BENCH_LANES=2
  run base_r ORB_BENCH_LANES=1
  exit 0
fi
run base ORB_BENCH_LANES=1
run l2s ORB_BENCH_LANES=2 ORB_BENCH_LANE_MATCH=stream
run l2i ORB_BENCH_LANES=2 ORB_BENCH_LANE_MATCH=inlane
run l2i_ss0 ORB_BENCH_LANES=2 ORB_BENCH_LANE_MATCH=inlane ORB_SIDE_SHARED=0
run l2s_ss0 ORB_BENCH_LANES=2 ORB_BENCH_LANE_MATCH=stream ORB_SIDE_SHARED=0
run base2 ORB_BENCH_LANES=1
