# C5 shape (16 x 1920x1080, 4000 features): extraction stages alone, and the C5 keys of the bench
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/c5st; mkdir -p $O
timeout -k 10 180 python3 tools/probe/stage_times.py --batch 16 --calls 50 --width 1920 --height 1080 --features 4000 > $O/st16.txt 2>&1 || exit 1
timeout -k 10 180 python3 tools/probe/stage_times.py --batch 32 --calls 50 --width 1920 --height 1080 --features 4000 >> $O/st16.txt 2>&1 || exit 1
cat $O/st16.txt
