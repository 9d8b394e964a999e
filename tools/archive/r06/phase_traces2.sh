#!/bin/bash
# kernel traces: ppw8fcw2 (always the slow mode in r06_ab24) and ppw8 (both modes), for tools/probe/lane_phase.py
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
for i in 1 2 3; do for v in ppw8fcw2 ppw8; do
  export ORB_AMD_LIB=orb_slam2-chinese-annotation_amd/lib/variants/$v.so
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06_phase2/$v.$i -- python3 -u bench.py --no-cpu --no-dropin --no-secondary > gpurun_out/r06_phase2/$v.$i.json 2> gpurun_out/r06_phase2/$v.$i.err || { echo FAIL $v $i; exit 1; }
  echo "$v $i $(grep -o '"value": [0-9.]*' gpurun_out/r06_phase2/$v.$i.json | head -1)"
done; done
