set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-tex}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_parity_gpu.py -k "texture or scene or pos or pipeline or forward or padding" -x -v --timeout 120 --timeout-method thread > $O/t.log 2>&1
for i in 1 2; do
RF_TEX_FAST=0 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_slow$i.json 2> $O/bench.err
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_fast$i.json 2> $O/bench.err
done
echo done
