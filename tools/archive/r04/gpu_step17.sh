#!/bin/bash
# round-4 step 17: frames per extraction launch (1024 default vs 2048 / 512 /
# 1536), interleaved, headline only
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
for b in 1024 2048 512 1024 2048 1536; do
  timeout -k 10 300 python bench.py --no-cpu --no-dropin --no-secondary --host-frames 0 --steps 40 --batch $b > "$O/s17_b.json" 2> "$O/s17_b.err" || { tail -20 "$O/s17_b.err"; exit 1; }
  python3 -c "import json; r=json.loads(open('$O/s17_b.json').read().strip().splitlines()[-1]); print('batch $b', round(r['value']), round(r['ms_per_step'], 3))"
done
