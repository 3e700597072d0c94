# c5 bf16 vs fp8 at the default 24 views, and a hip-API trace of the cbox frame (which calls issue the
# small rocclr copyBuffer blits).  usage: bash tools/gpu_r2_c5.sh <tag>
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-c5}
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py --workload c5 --steps 3 --warmup 1 > $O/c5bf16.json 2> $O/c5.err
timeout -k 10 400 python bench.py --workload c5 --fp8 --steps 3 --warmup 1 > $O/c5fp8.json 2>> $O/c5.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace -d $O/trace -o run -- python3 $R/bench.py --profile --steps 2 --warmup 1 > $O/trace.log 2>&1
echo done
