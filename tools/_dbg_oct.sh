for v in 150 96 64 52 40; do ORB_OCTREE_LDS_KB=$v timeout -k 10 200 python bench.py --no-cpu --steps 10 > gpurun_out/oct_$v.json 2>/dev/null || exit 1; done
