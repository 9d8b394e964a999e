#!/bin/bash
# headline with the level-pair pyramid (product) vs one launch per level (PYR_FUSE2=0), 6 reps interleaved
O=${AB_OUT:-gpurun_out/r06_ab29}; mkdir -p $O
for r in 1 2 3 4 5 6; do for v in product nofuse2; do
  if [ $v = product ]; then unset ORB_AMD_LIB; else export ORB_AMD_LIB=orb_slam2-chinese-annotation_amd/lib/variants/$v.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-dropin --no-secondary > $O/$v.$r.json 2> $O/$v.$r.err || { echo FAIL $v; exit 1; }
  python -c "import json;d=json.load(open('$O/$v.$r.json'));k=d['kernels'];print('$v $r', round(d['value']), 'resize %.3f/%.3f'%(k['k_pyr_resize']['ms_per_call_isolated'],k['k_pyr_resize']['ms_per_call_pipelined']))"
done; done
