# device-side kernel durations of one kbench mode (host overhead excluded): bash tools/gpu_kprof.sh <tag> <mode> [ENV=..]
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
env ${3:-KB_DUMMY=1} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/tools/kbench.py $2 > $O/log 2>&1
echo done
