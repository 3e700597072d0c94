set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --profile --steps 5 --warmup 2 > $R/gpurun_out/prof.log 2>&1
