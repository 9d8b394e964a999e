#!/bin/bash
# k_proj_resolve_fp window size, smaller windows: 1024 (product) vs 512 / 256 points (one per thread) and 1024 on 512 threads
O=${AB_OUT:-gpurun_out/r06_ab22}; mkdir -p $O
for v in w512 w256 t512w1024; do
  ORB_AMD_LIB=orb_slam2-chinese-annotation_amd/lib/variants/$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_matcher.py tests/test_gpu_headline.py > $O/$v.tests.log 2>&1 || { echo "TESTS FAIL $v"; tail -5 $O/$v.tests.log; exit 1; }
  echo "tests $v: $(tail -1 $O/$v.tests.log)"
done
for r in 1 2; do for v in product w512 w256 t512w1024; do
  if [ $v = product ]; then unset ORB_AMD_LIB; else export ORB_AMD_LIB=orb_slam2-chinese-annotation_amd/lib/variants/$v.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-dropin > $O/$v.$r.json 2> $O/$v.$r.err || { echo FAIL $v; exit 1; }
  python -c "import json;d=json.load(open('$O/$v.$r.json'));c=d['C5_problems_per_s'];print('$v $r', round(d['value']), round(c['value']), round(c['match_only_problems_per_s']), round(c['one_match_stream']['match_only_problems_per_s']), round(d['C4_latency']['frames_per_call_1']['serial_ms_per_call'],4), round(d['C4_latency']['frames_per_call_8']['serial_ms_per_call'],4))"
done; done
