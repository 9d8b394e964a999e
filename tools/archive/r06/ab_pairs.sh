#!/bin/bash
# level pairs only for calls of <= 8 images (product) vs pairs for every call (pairsall = the round-6 pyramid before this change): full bench, 4 reps
O=${AB_OUT:-gpurun_out/r06_ab30}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_extractor.py tests/test_gpu_headline.py tests/test_gpu_dropin.py > $O/tests.log 2>&1 || { echo "TESTS FAIL"; tail -8 $O/tests.log; exit 1; }
echo "tests product: $(tail -1 $O/tests.log)"
for r in 1 2 3 4; do for v in product pairsall; do
  if [ $v = product ]; then unset ORB_AMD_LIB; else export ORB_AMD_LIB=orb_slam2-chinese-annotation_amd/lib/variants/$v.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-dropin > $O/$v.$r.json 2> $O/$v.$r.err || { echo FAIL $v; exit 1; }
  python -c "import json;d=json.load(open('$O/$v.$r.json'));c=d['C5_problems_per_s'];c3=d['C3_stereo_pairs_per_s'];l=d['C4_latency'];k=d['kernels']['k_pyr_resize'];print('$v $r', round(d['value']), 'C3', round(c3['value'] if isinstance(c3,dict) else c3), 'C5', round(c['value']), 'lat1 %.4f lat8 %.4f'%(l['frames_per_call_1']['serial_ms_per_call'], l['frames_per_call_8']['serial_ms_per_call']), 'resize', k['launches_per_call'], round(k['ms_per_call_isolated'],3))"
done; done
