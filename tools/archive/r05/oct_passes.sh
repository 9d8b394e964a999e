# k_octree time against its pass bound (ORB_OCTREE_MAX_PASSES test hook: the distribution stops after k passes; results flagged, timing only)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/octp; mkdir -p $O
for k in 1 2 3 4 5 6 8 10 14 512; do
  ORB_OCTREE_MAX_PASSES=$k timeout -k 10 120 python3 tools/probe/stage_times.py --batch 1024 --calls 10 > $O/b_$k.txt 2>&1 || exit 1
  ORB_OCTREE_MAX_PASSES=$k timeout -k 10 120 python3 tools/probe/stage_times.py --batch 1 --calls 200 > $O/s_$k.txt 2>&1 || exit 1
  echo "passes<=$k B1024: $(grep -o 'k_octree [0-9.]*' $O/b_$k.txt)  B1: $(grep -o 'k_octree [0-9.]*' $O/s_$k.txt)" | tee -a $O/sum.txt
done
