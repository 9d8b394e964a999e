#!/bin/bash
# lane stagger at the start of the timed region (ORB_BENCH_STAGGER=1, bench default) vs both lanes starting together (0), 6 reps interleaved
# (ran against a bench.py prologue patch that was not kept: the second lane's first timed launch waited on extracted[first lane's set])
O=${AB_OUT:-gpurun_out/r06_ab25}; mkdir -p $O
for r in 1 2 3 4 5 6; do for v in 1 0; do
  ORB_BENCH_STAGGER=$v timeout -k 10 300 python -u bench.py --no-cpu --no-dropin --no-secondary > $O/s$v.$r.json 2> $O/s$v.$r.err || { echo FAIL $v; exit 1; }
  python -c "import json;d=json.load(open('$O/s$v.$r.json'));k=d['kernels'];print('stagger=$v $r', round(d['value']), ' '.join('%s=%.3f'%(n[2:8],k[n]['ms_per_call_pipelined']) for n in ('k_octree','k_orient_desc','k_proj_candidates')))"
done; done
