#!/bin/bash
# Round 6 A/B driver (GPU box).  ab.sh OUT "PARITY_VARIANTS" "STAGE_VARIANTS" "BENCH_VARIANTS" [REPS]
# variant "product" = lib/liborb_amd.so, else lib/variants/NAME.so.  Parity: the
# extractor, headline and stream-order tests against the oracle; stages: each
# extraction stage alone (profile mode 2) + one-frame latency; bench: the
# headline without the CPU / secondary / drop-in legs, variants interleaved.
O=$1; PV=$2; SV=$3; BV=$4; REPS=${5:-2}
mkdir -p "$O"
lib() { if [ "$1" = product ]; then unset ORB_AMD_LIB; else export ORB_AMD_LIB=orb_slam2-chinese-annotation_amd/lib/variants/$1.so; fi; }
for v in $PV; do
  lib $v
  timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_headline.py tests/test_gpu_stream_order.py -x -q --timeout 120 --timeout-method thread > "$O/parity_$v.log" 2>&1 || { echo "PARITY FAIL $v"; tail -30 "$O/parity_$v.log"; exit 1; }
  echo "parity ok $v"
done
for v in $SV; do
  lib $v
  timeout -k 10 120 python -u tools/probe/serial_stages.py --batch 1024 --calls 10 > "$O/stages_$v.txt" 2>&1 || exit 1
  timeout -k 10 120 python -u tools/probe/latency_probe.py --calls 300 --tag $v > "$O/latency_$v.json" 2>&1 || exit 1
  echo "stages $v: $(grep -h 'ms per call' "$O/stages_$v.txt" | tr '\n' ' ' | head -c 600)"
done
for r in $(seq 1 $REPS); do
  for v in $BV; do
    lib $v
    timeout -k 10 240 python -u bench.py --no-secondary --no-cpu --no-dropin > "$O/bench_${v}_$r.log" 2>&1 || exit 1
    echo "bench $v $r: $(grep -o '"value": [0-9.]*' "$O/bench_${v}_$r.log" | head -1)"
  done
done
