set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-gm}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "gemm" -x -q --timeout 120 --timeout-method thread > $O/t_gemm.log 2>&1
KB_VARIANTS=blaslt,auto timeout -k 10 300 python tools/kbench.py gemm > $O/kb_gemm.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo done
