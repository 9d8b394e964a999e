O=gpurun_out/r06_ab18; mkdir -p $O
for r in 1 2 3; do for v in base skipgrid; do
  if [ $v = base ]; then unset ORB_AMD_LIB; else export ORB_AMD_LIB=orb_slam2-chinese-annotation_amd/lib/variants/$v.so; fi
  timeout -k 10 240 python -u bench.py --no-secondary --no-dropin > $O/$v.$r.log 2>&1
  echo "$v $r $(grep -o '"value": [0-9.]*' $O/$v.$r.log | head -1)"
done; done
