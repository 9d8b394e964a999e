#!/bin/bash
# Round 3: k_proj_candidates in XCD-contiguous order (default) vs the plain
# grid order (variant projnox): matcher parity, bench A/B, FETCH_SIZE per variant.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  "$R/tests/test_gpu_matcher.py" "$R/tests/test_gpu_matchers_more.py" > "$O/xcd_parity.log" 2>&1 || exit 1
"$R/tools/ab_variants.sh" xcd projnox || exit 1
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu --no-secondary --steps 2 --warmup 1 --host-frames 0"
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d "$O/xcdF_base" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$O/xcdF_base.log" 2>&1 || exit 1
ORB_AMD_LIB=$R/orb_slam2-chinese-annotation_amd/lib/variants/projnox.so timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d "$O/xcdF_nox" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$O/xcdF_nox.log" 2>&1 || exit 1
echo done
