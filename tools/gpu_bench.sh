set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-b}
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --profile --steps 5 --warmup 2 > $O/prof.log 2>&1
echo done
