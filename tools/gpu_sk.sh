# stream-K attention check: attention + parity GPU tests, attention kbench, one bench run.
# usage: bash tools/gpu_sk.sh <tag>
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-sk}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention or swin" -x -v --timeout 120 --timeout-method thread > $O/t_attn.log 2>&1
timeout -k 10 200 python tools/kbench.py attn > $O/kb_attn.log 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo done
