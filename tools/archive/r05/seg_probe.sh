# exit-time segfault under rocprofv3 --kernel-trace: no-CU-mask variant first, then the default library
set -u
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/seg
mkdir -p $O
A="--no-cpu --no-secondary --host-frames 0 --frames 64 --steps 2 --warmup 1"
ORB_AMD_LIB=$R/orb_slam2-chinese-annotation_amd/lib/variants/nocumask.so timeout -k 10 200 rocprofv3 --kernel-trace -d $O/b -o run --output-format csv -- python3 $R/bench.py $A > $O/b.json 2> $O/b.err
echo "nocumask rc=$?"
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/a -o run --output-format csv -- python3 $R/bench.py $A > $O/a.json 2> $O/a.err
echo "default rc=$?"
