#!/bin/bash
# extraction knobs re-swept on the round-6 pipeline: batch octree workgroup 128 threads, orient/desc slot pairs per wave 2 / 8, FAST waves per workgroup 2
O=${AB_OUT:-gpurun_out/r06_ab23}; mkdir -p $O
for r in 1 2; do for v in product oct128 ppw2 ppw8 fcw2; do
  if [ $v = product ]; then unset ORB_AMD_LIB; else export ORB_AMD_LIB=orb_slam2-chinese-annotation_amd/lib/variants/$v.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-dropin --no-secondary > $O/$v.$r.json 2> $O/$v.$r.err || { echo FAIL $v; exit 1; }
  python -c "import json;d=json.load(open('$O/$v.$r.json'));k=d['kernels'];print('$v $r', round(d['value']), ' '.join('%s=%.3f/%.3f'%(n[2:8],k[n]['ms_per_call_isolated'],k[n]['ms_per_call_pipelined']) for n in ('k_fast_cells','k_octree','k_orient_desc')))"
done; done
