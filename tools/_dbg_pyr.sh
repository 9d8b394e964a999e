for v in 0 1 2 3; do ORB_PYR_DBG=$v timeout -k 10 200 python bench.py --no-cpu --steps 10 > gpurun_out/pyrd_$v.json 2>/dev/null || exit 1; done
