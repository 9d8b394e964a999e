#!/bin/bash
# C5 (1920x1080) and C3 with the level-pair pyramid (product) vs one launch per level (PYR_FUSE2=0), 3 reps
O=${AB_OUT:-gpurun_out/r06_ab28}; mkdir -p $O
for r in 1 2 3; do for v in product nofuse2; do
  if [ $v = product ]; then unset ORB_AMD_LIB; else export ORB_AMD_LIB=orb_slam2-chinese-annotation_amd/lib/variants/$v.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-dropin > $O/$v.$r.json 2> $O/$v.$r.err || { echo FAIL $v; exit 1; }
  python -c "import json;d=json.load(open('$O/$v.$r.json'));c=d['C5_problems_per_s'];c3=d['C3_stereo_pairs_per_s'];print('$v $r', round(d['value']), 'C3', round(c3['value'] if isinstance(c3,dict) else c3), 'C5', round(c['value']), round(c['one_match_stream']['problems_per_s']), round(c['match_only_problems_per_s']))"
done; done
