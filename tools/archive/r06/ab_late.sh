#!/bin/bash
# late re-checks on the closing code: the headline's resolve as k_proj_resolve<4> (rw4) or the fixed-point kernel (rfp) instead of <1>; per-level resize with 8 images per workgroup (ipw8) instead of 16; 4 reps
O=${AB_OUT:-gpurun_out/r06_ab31}; mkdir -p $O
for r in 1 2 3 4; do for v in product rw4 rfp ipw8; do
  if [ $v = product ]; then unset ORB_AMD_LIB; else export ORB_AMD_LIB=orb_slam2-chinese-annotation_amd/lib/variants/$v.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-dropin > $O/$v.$r.json 2> $O/$v.$r.err || { echo FAIL $v; exit 1; }
  python -c "import json;d=json.load(open('$O/$v.$r.json'));c=d['C5_problems_per_s'];c3=d['C3_stereo_pairs_per_s'];k=d['kernels'];print('$v $r', round(d['value']), 'C3', round(c3['value'] if isinstance(c3,dict) else c3), 'C5', round(c['value']), 'resize %.3f resolve %.3f/%.3f'%(k['k_pyr_resize']['ms_per_call_isolated'], k['k_proj_resolve']['ms_per_call_isolated'], k['k_proj_resolve']['ms_per_call_pipelined']))"
done; done
