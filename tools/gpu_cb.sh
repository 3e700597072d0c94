set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-cb}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_parity_gpu.py -k "conv or dpt or pipeline or padding" -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo done
