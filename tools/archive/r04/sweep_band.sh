set -e
for b in ${BANDS:-5120 5632 6144 6656 7168 8192}; do
  ORB_BAND_BYTES=$b timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/sw_$b.json 2>/dev/null
  python3 -c "import json; d=json.load(open('gpurun_out/sw_$b.json')); print($b, round(d['ms_per_step'],3), round(d['kernels_ms_per_step']['k_fast_band'],3))"
done
