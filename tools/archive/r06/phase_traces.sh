#!/bin/bash
# kernel traces of 4 headline runs (slow / high modes) for tools/probe/lane_phase.py
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
for i in 1 2 3 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06_phase/t$i -- python3 -u bench.py --no-cpu --no-dropin --no-secondary > gpurun_out/r06_phase/b$i.json 2> gpurun_out/r06_phase/b$i.err || { echo FAIL $i; exit 1; }
  echo "run $i $(grep -o '"value": [0-9.]*' gpurun_out/r06_phase/b$i.json | head -1)"
done
