# headline schedule A/B: one match stream (base) vs two (a matcher handle per stream), 2 / 3 lanes
O=gpurun_out/r06_ab19; mkdir -p $O
for r in 1 2 3; do for v in base ms2 l3ms2; do
  case $v in base) a="";; ms2) a="--match-streams 2";; l3ms2) a="--match-streams 2 --lanes 3";; esac
  timeout -k 10 240 python -u bench.py --no-secondary --no-dropin $a > $O/$v.$r.log 2>&1 || exit 1
  echo "$v $r $(grep -o '"value": [0-9.]*' $O/$v.$r.log | head -1)"
done; done
