#!/bin/bash
# k_proj_candidates scoring batch (PROJ_QB: window candidates whose descriptor loads go out together): 4 (product) vs 6 / 8
O=${AB_OUT:-gpurun_out/r06_ab20}; mkdir -p $O
for r in 1 2; do for v in product qb8 qb6; do
  if [ $v = product ]; then unset ORB_AMD_LIB; else export ORB_AMD_LIB=orb_slam2-chinese-annotation_amd/lib/variants/$v.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-dropin > $O/$v.$r.json 2> $O/$v.$r.err || { echo FAIL $v; exit 1; }
  python -c "import json;d=json.load(open('$O/$v.$r.json'));c=d['C5_problems_per_s'];k=d['kernels']['k_proj_candidates'];print('$v $r', round(d['value']), round(c['value']), round(c['match_only_problems_per_s']), round(c['one_match_stream']['match_only_problems_per_s']), round(d['C4_latency']['frames_per_call_1']['serial_ms_per_call'],4), round(d['C4_latency']['frames_per_call_8']['serial_ms_per_call'],4), round(k['ms_per_launch_isolated'],4), round(k['ms_per_call_pipelined'],4))"
done; done
