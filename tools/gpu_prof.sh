set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-prof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --profile --steps 5 --warmup 2 > $O/prof.log 2>&1
echo done
