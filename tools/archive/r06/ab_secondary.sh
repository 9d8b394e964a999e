#!/bin/bash
O=${AB_OUT:-gpurun_out/r06_ab7}; mkdir -p $O
for r in 1 2 3; do for v in product listcall; do
  if [ $v = product ]; then unset ORB_AMD_LIB; else export ORB_AMD_LIB=orb_slam2-chinese-annotation_amd/lib/variants/$v.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-dropin > $O/$v.$r.json 2> $O/$v.$r.err || { echo FAIL $v; exit 1; }
  python -c "import json;d=json.load(open('$O/$v.$r.json'));c=d['C5_problems_per_s'];print('$v $r', round(d['value']), round(c['value']), round(c['match_only_problems_per_s']), round(c['one_match_stream']['match_only_problems_per_s']), d['C4_latency']['frames_per_call_1']['serial_ms_per_call'], d['kernels']['k_proj_resolve']['ms_per_launch_isolated'])"
done; done
