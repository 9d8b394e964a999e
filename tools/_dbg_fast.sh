for v in 0 1 2 3 4; do ORB_FAST_DBG=$v timeout -k 10 200 python bench.py --no-cpu --steps 10 > gpurun_out/dbg_$v.json 2>/dev/null || exit 1; done
