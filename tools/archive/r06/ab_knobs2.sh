#!/bin/bash
# second pass, 4 reps interleaved: orient/desc 8 slot pairs per wave (ppw8), FAST 2 waves per workgroup (fcw2), both
O=${AB_OUT:-gpurun_out/r06_ab24}; mkdir -p $O
for v in ppw8 ppw8fcw2; do
  ORB_AMD_LIB=orb_slam2-chinese-annotation_amd/lib/variants/$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_extractor.py tests/test_gpu_headline.py > $O/$v.tests.log 2>&1 || { echo "TESTS FAIL $v"; tail -5 $O/$v.tests.log; exit 1; }
  echo "tests $v: $(tail -1 $O/$v.tests.log)"
done
for r in 1 2 3 4; do for v in product ppw8 fcw2 ppw8fcw2; do
  if [ $v = product ]; then unset ORB_AMD_LIB; else export ORB_AMD_LIB=orb_slam2-chinese-annotation_amd/lib/variants/$v.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-dropin --no-secondary > $O/$v.$r.json 2> $O/$v.$r.err || { echo FAIL $v; exit 1; }
  python -c "import json;d=json.load(open('$O/$v.$r.json'));k=d['kernels'];print('$v $r', round(d['value']), ' '.join('%s=%.3f/%.3f'%(n[2:8],k[n]['ms_per_call_isolated'],k[n]['ms_per_call_pipelined']) for n in ('k_fast_cells','k_octree','k_orient_desc')))"
done; done
