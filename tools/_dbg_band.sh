for v in 4096 6144 8192 10240 14336; do ORB_BAND_BYTES=$v timeout -k 10 200 python bench.py --no-cpu --steps 10 > gpurun_out/band_$v.json 2>/dev/null || exit 1; done
