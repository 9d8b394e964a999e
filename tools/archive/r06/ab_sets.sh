#!/bin/bash
# buffer sets (launch g waits for set g % NS's previous match): 4 (2 per lane, default) vs 6 / 8, 4 reps
# (ran against a bench.py patch reading NS from ORB_BENCH_SETS, not kept)
O=${AB_OUT:-gpurun_out/r06_ab27}; mkdir -p $O
for r in 1 2 3 4; do for v in 4 6 8; do
  ORB_BENCH_SETS=$v timeout -k 10 300 python -u bench.py --no-cpu --no-dropin --no-secondary > $O/s$v.$r.json 2> $O/s$v.$r.err || { echo FAIL $v; exit 1; }
  python -c "import json;d=json.load(open('$O/s$v.$r.json'));k=d['kernels'];print('sets=$v $r', round(d['value']), ' '.join('%s=%.3f'%(n[2:8],k[n]['ms_per_call_pipelined']) for n in ('k_octree','k_orient_desc','k_proj_candidates')))"
done; done
