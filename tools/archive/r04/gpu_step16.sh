#!/bin/bash
# round-4 step 16: the default bench line with the C4 latency-shaped key, and smoke()
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"; cd "$R"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/s16_smoke.log" 2>&1 || { tail -20 "$O/s16_smoke.log"; exit 1; }
tail -1 "$O/s16_smoke.log"
t0=$(date +%s)
timeout -k 10 600 python -u bench.py > "$O/s16_bench.json" 2> "$O/s16_bench.err" || { tail -20 "$O/s16_bench.err"; exit 1; }
echo "bench wall $(( $(date +%s) - t0 )) s"
python3 -c "
import json; r=json.loads(open('$O/s16_bench.json').read().strip().splitlines()[-1])
print(round(r['value']), r['roofline']['frac'], json.dumps(r['C4_latency']), round(r['C5_problems_per_s']['value']), round(r['C3_stereo_pairs_per_s']['value']))
print(json.dumps(r['dropin']['gpu_stereo_build']))"
