#!/bin/bash
# candidate scan vs k_orient_desc co-residency: PROJ_DIRECT=1 (no LDS), 256-thread workgroups with 2 points per thread (1 wave per SIMD: fits beside 4 orient workgroups per CU), 256-thread workgroups; 4 reps
O=${AB_OUT:-gpurun_out/r06_ab26}; mkdir -p $O
for t in direct wg256ppt2; do ORB_AMD_LIB=orb_slam2-chinese-annotation_amd/lib/variants/$t.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_matcher.py tests/test_gpu_headline.py > $O/$t.tests.log 2>&1 || { echo "TESTS FAIL $t"; tail -5 $O/$t.tests.log; exit 1; }; echo "tests $t: $(tail -1 $O/$t.tests.log)"; done
for r in 1 2 3 4; do for v in product direct wg256ppt2 wg256; do
  if [ $v = product ]; then unset ORB_AMD_LIB; else export ORB_AMD_LIB=orb_slam2-chinese-annotation_amd/lib/variants/$v.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-dropin --no-secondary > $O/$v.$r.json 2> $O/$v.$r.err || { echo FAIL $v; exit 1; }
  python -c "import json;d=json.load(open('$O/$v.$r.json'));k=d['kernels'];print('$v $r', round(d['value']), ' '.join('%s=%.3f/%.3f'%(n[2:8],k[n]['ms_per_call_isolated'],k[n]['ms_per_call_pipelined']) for n in ('k_octree','k_orient_desc','k_proj_candidates')))"
done; done
